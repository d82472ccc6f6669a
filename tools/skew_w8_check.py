"""Repeat the layout-3 W = 8 staged check (tests/test_gpu_skew.py
test_skew_staged_steps[w8-global]) and report which pass / pair / plane
differs from the oracle, plus whether scores and alignments agree."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gxamd as gx  # noqa: E402
import oracle  # noqa: E402

oracle.build()
oracle.load()
ctx = gx.Context(0)
sc = (1, -2, -1, -5)
for W in sys.argv[1:] or ["2"]:
    os.environ["GX_LAYOUT"] = "3"
    os.environ["GX_BAND_WAVES"] = W
    for is_local in (False, True):
        rng = random.Random(909 + is_local)
        pairs = [(bytes(rng.choice(b"ACGT") for _ in range(n)), bytes(rng.choice(b"ACGT") for _ in range(m)))
                 for n, m in [(1500, 1400), (700, 900)]]
        want = [oracle.align_lean(a, b, sc, is_local=is_local) for a, b in pairs]
        for rep in range(4):
            st = gx.StagedPairs(pairs, ctx=ctx)
            res, _ = st.run(gx.Scores(*sc), is_local, keep_planes=True, steps=3, plane_sums=True)
            sums = st.plane_sums()
            passes = st.pass_results()
            bad = []
            for p, o in enumerate(want):
                for k in range(3):
                    got = [int(x) for x in sums[k, p]]
                    if got != o.extra["plane_sums"]:
                        bad.append((p, k, [g == w for g, w in zip(got, o.extra["plane_sums"])]))
                    if (passes[k][p].score, passes[k][p].n_steps) != (o.score, len(o.choices)):
                        bad.append((p, k, "result"))
            print(f"W={W} local={is_local} rep {rep}: info {ctx.fill_info()} bad {bad}", flush=True)
        # single-pass and table form of pair 0
        for p, (a, b) in enumerate(pairs):
            cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
            t, _ = gx.alignment_table(cont, gx.Scores(*sc), is_local, False, ctx=ctx, max_cell=False)
            print(f"  table pair {p}: sums ok {t.plane_sums() == want[p].extra['plane_sums']}", flush=True)
            t.free()
ctx.close()
