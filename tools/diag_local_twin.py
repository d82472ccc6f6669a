"""Diagnostic (GPU): local twin fill vs the scalar local fill vs the oracle on
planted-core pairs -- per pair, which plane sums, score and alignment agree."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "genomics-rs_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import gxamd as gx  # noqa: E402
import oracle  # noqa: E402
from test_gpu_twin_local import _planted  # noqa: E402

os.environ["GX_LAYOUT"] = "0"
scores = (1, -2, -1, -5)
rng = random.Random(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
shapes = [(900, 700, 300), (700, 900, 250), (1500, 400, 200), (333, 1200, 150), (257, 256, 256), (129, 3000, 100)]
pairs = [_planted(rng, n, m, c) for n, m, c in shapes]
ctx = gx.Context(0)
for twin in ("1", "0"):
    os.environ["GX_TWIN"] = twin
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*scores), True, keep_planes=True, steps=1, plane_sums=True)
    sums = st.plane_sums()
    print("GX_TWIN", twin, ctx.fill_info())
    for p, (a, b) in enumerate(pairs):
        o = oracle.align_lean(a, b, scores, is_local=True)
        ok = [int(sums[0, p][k]) == o.extra["plane_sums"][k] for k in range(3)]
        al = [(c, i, j) for c, i, j in zip(st.steps(p)["choice"], st.steps(p)["i"], st.steps(p)["j"])]
        print(p, len(a), len(b), "sums I/D/S ok", ok, "score", res[p].score, o.score, "nsteps", res[p].n_steps,
              len(o.choices), "start", al[0][1:] if al else None, o.alignment()[0][1:] if o.alignment() else None)
ctx.close()
