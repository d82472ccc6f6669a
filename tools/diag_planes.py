"""Diagnostics: first cells where the device planes differ from the oracle."""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "genomics-rs_amd")]
import gxamd as gx  # noqa: E402
import oracle  # noqa: E402

ctx = gx.Context(0)
cases = [(int(a), int(b)) for a, b in (x.split("x") for x in sys.argv[1:])] or [(3302, 3843), (700, 900), (300, 1000)]
for n, m in cases:
    rng = random.Random(n * 7 + m)
    a = bytes(rng.choice(b"ACGT") for _ in range(n))
    b = bytes(rng.choice(b"ACGT") for _ in range(m))
    o = oracle.align(a, b, (1, -2, -1, -5), is_local=False, want_planes=True)
    cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
    t, mam = gx.alignment_table(cont, gx.Scores(1, -2, -1, -5), False, False, ctx=ctx)
    for k, name in enumerate(("I", "D", "S")):
        p = t.plane(k)
        bad = np.argwhere(p != o.planes[k])
        print(f"{n}x{m} plane {name}: {len(bad)} bad cells", end="")
        if len(bad):
            rows = sorted(set(int(x) for x in bad[:, 0]))
            print(f"; first {bad[:5].tolist()} rows {rows[:10]}{'...' if len(rows) > 10 else ''} "
                  f"strips {sorted(set((r - 1) // 64 for r in rows))[:10]}; "
                  f"dev {[int(p[i, j]) for i, j in bad[:3]]} ora {[int(o.planes[k][i, j]) for i, j in bad[:3]]}")
        else:
            print()
    aln = gx.retrace(cont, t, False)
    print("  alignment equal:", [(c.name, i, j) for c, i, j in aln.alignment] == o.alignment(), flush=True)
