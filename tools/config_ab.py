"""GPU: bench.py's config2 / config3 record (the single-pair align calls,
parity against tests/golden/large_digests.json) under the current
environment; one JSON line per config.  tools/config_ab.py covid|brca2 [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "genomics-rs_amd")]
import bench  # noqa: E402
import gxamd as gx  # noqa: E402

ctx = gx.Context(0)
for which in sys.argv[1].split(","):
    rec = bench.config_record(gx, ctx, which, int(sys.argv[2]) if len(sys.argv) > 2 else 5)
    rec["env"] = {k: v for k, v in os.environ.items() if k.startswith("GX_")}
    print(json.dumps(rec), flush=True)
ctx.close()
