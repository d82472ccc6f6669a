"""Time StagedPairs.run calls (host wall) next to the library's GX_LOG=debug phase lines.
    python tools/time_staged.py [pairs] [length]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
import bench  # noqa: E402  (synthetic pairs)
import gxamd as gx  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 16
L = int(sys.argv[2]) if len(sys.argv) > 2 else 30000
pairs = [bench.synth_pair(p, L) for p in range(P)]
st = gx.StagedPairs(pairs)
for k in range(5):
    t0 = time.perf_counter()
    res, fms = st.run(gx.Scores(*bench.SCORES), False, True)
    t1 = time.perf_counter()
    got = [(r.score, r.n_steps, r.matches) for r in res]
    t2 = time.perf_counter()
    print(f"call {k}: run {1e3 * (t1 - t0):.3f} ms (fill {fms:.3f}) + results {1e3 * (t2 - t1):.3f} ms",
          file=sys.stderr, flush=True)
