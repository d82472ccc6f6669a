#!/usr/bin/env python3
"""Kernel + memory-copy timeline of a rocprofv3 --kernel-trace
--memory-copy-trace run (rocpd database), around the last passes of a fill
kernel: start, duration, the idle gap before each operation, stream.

    python tools/timeline.py RUN_DIR [--kernel fill_pk] [--passes 2]"""
import argparse
import glob
import os
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run")
    ap.add_argument("--kernel", default="fill_pk")
    ap.add_argument("--passes", type=int, default=2)
    a = ap.parse_args()
    c = sqlite3.connect(glob.glob(os.path.join(a.run, "**", "*.db"), recursive=True)[0])
    ev = [(s, e, "K " + n[:48], st) for n, s, e, st in c.execute("select name, start, end, stream_id from kernels")]
    ev += [(s, e, f"C {n} {sz} B", st) for n, s, e, st, sz in
           c.execute("select name, start, end, stream_id, size from memory_copies")]
    ev.sort()
    fills = [x for x in ev if a.kernel in x[2]]
    t0 = fills[-1 - a.passes][0]
    t1 = fills[-1][0]
    prev = None
    for s, e, name, st in ev:
        if t0 <= s < t1:
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:7.1f}  s{st}  {name}")
            prev = e if prev is None else max(prev, e)


if __name__ == "__main__":
    main()
