#!/usr/bin/env python3
"""Print per-kernel average PMC values from tools/gpu_pmc.sh outputs."""
import glob
import os
import sqlite3
import sys

d = sys.argv[1]
for db in sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True)):
    c = sqlite3.connect(db)
    for kname, ctr, n, avg, dur in c.execute(
            "select kernel_name, counter_name, count(*), avg(value), avg(duration) from counters_collection "
            "group by kernel_name, counter_name"):
        if "rocclr" in kname:
            continue
        print(f"{kname[:60]:60s} {ctr:28s} n={n:3d} avg={avg:.6g} dur_ns={dur:.0f}")
