"""GPU box: the single-pair config records of bench.py (BASELINE configs 2
and 3, untracked and tracked) without the headline batch, one JSON line each.
Usage: python3 tools/config_lines.py [steps] [which ...]  (which: c2 c3 c2t c3t)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
import bench  # noqa: E402
import gxamd as gx  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
which = sys.argv[2:] or ["c2", "c3", "c2t", "c3t"]
ctx = gx.Context(0)
for w in which:
    rec = bench.config_record(gx, ctx, "covid" if w.startswith("c2") else "brca2", steps, tracked=w.endswith("t"))
    fl = rec["fill_launch"]
    print(json.dumps({"which": w, "gcups": rec["gcups"], "ms_per_step": rec["ms_per_step"],
                      "fill_ms_avg": rec["fill_ms_avg"], "layout": fl.get("layout"), "W": fl.get("band_waves"),
                      "parity": rec["parity"]["bit_exact"]}), flush=True)
ctx.close()
