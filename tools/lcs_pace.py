"""GPU box: pace of the LCS sweep alone (GX_LCS_ALONE: the tracked layout-3
launch with its LCS workgroups only) on n x 30,000 random pairs, n from one
strip to Covid size: time = chain steps x pace, chain = 72 (S - 1) + T steps
(gx_lcs.h).  One JSON line per n.  Usage: python3 tools/lcs_pace.py [m]"""
import json
import os
import random
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
import gxamd as gx

m = int(sys.argv[1]) if len(sys.argv) > 1 else 30000
os.environ["GX_LAYOUT"] = "3"
os.environ["GX_LCS_ALONE"] = "1"
ctx = gx.Context(0)
rng = random.Random(1)
b = "".join(rng.choice("ACGT") for _ in range(m))
for n in (64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 30000):
    a = "".join(rng.choice("ACGT") for _ in range(n))
    cont = gx.SequenceContainer([gx.Sequence("a", a), gx.Sequence("b", b)])
    fills = []
    for _ in range(4):
        t, _mam = gx.alignment_table(cont, gx.Scores(1, -2, -1, -5), False, False, ctx=ctx, max_cell=True)
        fills.append(t.info()["fill_us"] / 1e3)
        t.free()
    S, wd = -(-n // 64), -(-m // 64)
    T = (wd + 64 + 31) & ~31
    ms = statistics.median(fills[1:])
    chain = 72 * (S - 1) + T
    print(json.dumps({"n": n, "m": m, "layout": ctx.fill_info()["layout"], "fill_ms": round(ms, 4),
                      "strips": S, "steps_T": T, "chain_steps": chain, "ns_per_chain_step": round(ms * 1e6 / chain, 1)}),
          flush=True)
ctx.close()
