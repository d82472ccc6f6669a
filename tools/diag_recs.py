"""Diagnostics: compare strip-0 pushed records and strip-1 consumed records
(GX_DEBUG_RECS dump) with the oracle's row 64."""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "genomics-rs_amd")]
import gxamd as gx  # noqa: E402
import oracle  # noqa: E402

n, m = [int(x) for x in sys.argv[1].split("x")]
rng = random.Random(n * 7 + m)
a = bytes(rng.choice(b"ACGT") for _ in range(n))
b = bytes(rng.choice(b"ACGT") for _ in range(m))
path = "gpurun_out/recs.bin"
os.environ["GX_DEBUG_RECS"] = path
ctx = gx.Context(0)
cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
t, _ = gx.alignment_table(cont, gx.Scores(1, -2, -1, -5), False, False, ctx=ctx)
t.free()
d = np.fromfile(path, dtype=np.int32).reshape(2, m + 1, 4)
o = oracle.align(a, b, (1, -2, -1, -5), want_planes=True, want_lcs=True)
I, D, S = o.planes
r = 64
g, h = -1, -5
exp_dd = np.maximum(np.maximum(I[r], S[r]) + h + g, D[r] + g)
exp_sm = np.maximum(np.maximum(I[r], S[r]), D[r])
for kind, arr in (("pushed", d[0]), ("consumed", d[1])):
    bad = [c for c in range(1, m + 1) if arr[c, 0] != exp_dd[c] or arr[c, 1] != exp_sm[c] or arr[c, 2] != o.lcs[r, c]
           or arr[c, 3] != b[c - 1]]
    print(kind, "bad columns:", len(bad), bad[:20])
    for c in bad[:4]:
        print("   col", c, "got", arr[c].tolist(), "want", [int(exp_dd[c]), int(exp_sm[c]), int(o.lcs[r, c]), b[c - 1]])
