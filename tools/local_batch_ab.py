"""GPU: bench.py's local_batch record (32 related 30k pairs, local SW, planes +
traceback, parity against the oracle digests) under the current environment;
prints one JSON line.  tools/local_batch_ab.py [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "genomics-rs_amd")]
import bench  # noqa: E402
import gxamd as gx  # noqa: E402

ctx = gx.Context(0)
rec = bench.local_batch_record(gx, ctx, int(sys.argv[1]) if len(sys.argv) > 1 else 3)
rec["env"] = {k: v for k, v in os.environ.items() if k.startswith("GX_")}
print(json.dumps(rec), flush=True)
ctx.close()
