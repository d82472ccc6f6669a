"""Debug helper: a table filled by the twin fill (GX_TABLE_TWIN=1) vs the oracle, plane by plane, row by row."""
import os, sys, random
sys.path.insert(0, 'genomics-rs_amd'); sys.path.insert(0, 'oracle')
import numpy as np
import gxamd as gx, oracle as o
os.environ["GX_LAYOUT"] = "0"
os.environ["GX_TABLE_TWIN"] = "1"
ctx = gx.Context(0)
rng = random.Random(3)
for n, m in [(129, 16), (200, 40)]:
    a = bytes(rng.choice(b"ACGT") for _ in range(n)); b = bytes(rng.choice(b"ACGT") for _ in range(m))
    cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
    t, _ = gx.alignment_table(cont, gx.Scores(1, -2, -1, -5), False, False, ctx=ctx, max_cell=False)
    print((n, m), ctx.fill_info())
    oo = o.align(a, b, want_planes=True)
    for k in range(3):
        pl = t.plane(k)
        bad = np.argwhere(pl != oo.planes[k])
        print(" plane", k, "bad cells", len(bad), bad[:6].tolist())
        if len(bad):
            i, j = bad[0]
            print("   row", i, "got", pl[i, max(0, j - 2):j + 6].tolist(), "want", oo.planes[k][i, max(0, j - 2):j + 6].tolist())
    t.free()
