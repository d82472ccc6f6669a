"""Time StagedPairs.run calls (host wall) next to the library's GX_LOG=debug phase lines."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
import bench  # noqa: E402  (synthetic pairs)
import gxamd as gx  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 16
pairs = [bench.synth_pair(p, 30000) for p in range(P)]
st = gx.StagedPairs(pairs)
for k in range(4):
    t0 = time.perf_counter()
    res, fms = st.run(gx.Scores(*bench.SCORES), False, True)
    t1 = time.perf_counter()
    print(f"call {k}: wall {1e3 * (t1 - t0):.3f} ms fill {fms:.3f} ms", file=sys.stderr, flush=True)
