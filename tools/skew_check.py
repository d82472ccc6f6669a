"""Layout-3 plane check on the GPU: fill untracked alignment tables of a few
shapes on layout 3 and report, per plane, the first cells that differ from
the oracle (strip, row in strip, column) and how many differ.

    python tools/skew_check.py [W ...]        (default W = 2)
"""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gxamd as gx  # noqa: E402
import oracle  # noqa: E402

oracle.build()
oracle.load()
ctx = gx.Context(0)
sc = (1, -2, -1, -5)
os.environ["GX_LAYOUT"] = "3"
for W in sys.argv[1:] or ["2"]:
    os.environ["GX_BAND_WAVES"] = W
    for is_local in (False, True):
        rng = random.Random(31 + is_local)
        for n, m in [(640, 641), (1000, 1300), (1000, 300), (300, 1300)]:
            a = bytes(rng.choice(b"ACGT") for _ in range(n))
            b = bytes(rng.choice(b"ACGT") for _ in range(m))
            o = oracle.align(a, b, sc, is_local=is_local, want_planes=True)
            cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
            for rep in range(3):
                table, _ = gx.alignment_table(cont, gx.Scores(*sc), is_local, False, ctx=ctx, max_cell=False)
                msg = []
                for k in range(3):
                    d = np.argwhere(table.plane(k) != o.planes[k])
                    if len(d):
                        first = [(int(i) - 1) // 64 for i, j in d[:1]], [tuple(int(x) for x in c) for c in d[:4]]
                        msg.append(f"plane {k}: {len(d)} cells differ, first strip/cells {first}")
                print(f"W={W} local={is_local} {n}x{m} rep {rep}: {ctx.fill_info()['layout']} "
                      f"{'OK' if not msg else '; '.join(msg)}", flush=True)
                table.free()
ctx.close()
