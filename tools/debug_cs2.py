"""GPU debug: first plane mismatches of the split column step (GX_CS2) on one table."""
import os, random, sys
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", d) for d in ("oracle", "genomics-rs_amd")]
import oracle as o
import gxamd as gx
o.load()
ctx = gx.Context(0)
rng = random.Random(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
scores = (1, -2, -1, -5)
for n, m in [(127, 130), (200, 40), (65, 17)]:
    a = bytes(rng.choice(b"ACGT") for _ in range(n))
    b = bytes(rng.choice(b"ACGT") for _ in range(m))
    r = o.align(a, b, scores, want_planes=True)
    cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
    for cs2 in ("1", "0"):
        os.environ["GX_CS2"] = cs2
        os.environ["GX_LAYOUT"] = "1"
        t, _ = gx.alignment_table(cont, gx.Scores(*scores), False, False, ctx=ctx, max_cell=False)
        print("shape", n, m, "cs2", cs2, ctx.fill_info())
        for k in range(3):
            p = t.plane(k)
            bad = np.argwhere(p != r.planes[k])
            if len(bad):
                i, j = bad[0]
                print("  plane", k, "bad", len(bad), "first", (int(i), int(j)), "got", int(p[i, j]), "want",
                      int(r.planes[k][i, j]), "rows", sorted(set(int(x) for x in bad[:, 0]))[:8])
                print("   got row", [int(x) for x in p[i, :12]])
                print("  want row", [int(x) for x in r.planes[k][i, :12]])
        al = gx.retrace(cont, t, False)
        print("  score", al.score, "want", r.score)
