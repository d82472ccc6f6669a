"""GPU box: per-strip timing of the LCS sweep (GX_LCS_TRACE stamps, 100 MHz
s_memrealtime) on a random 30,000 x 30,000 pair, alone (GX_LCS_ALONE) and
beside the tracked fill: each strip's pace (ns a step between its first
group and its end), its lag behind the strip above (first group to first
group), and whether its input crossed workgroups (HBM) or waves (LDS).
Usage: python3 tools/lcs_trace.py [n] [m]"""
import json
import os
import random
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
import gxamd as gx

n = int(sys.argv[1]) if len(sys.argv) > 1 else 30000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 30000
os.environ["GX_LAYOUT"] = "3"
ctx = gx.Context(0)
rng = random.Random(2)
a = "".join(rng.choice("ACGT") for _ in range(n))
b = "".join(rng.choice("ACGT") for _ in range(m))
cont = gx.SequenceContainer([gx.Sequence("a", a), gx.Sequence("b", b)])
wd = -(-m // 64)
T = (wd + 64 + 31) & ~31
for alone in (True, False):
    if alone:
        os.environ["GX_LCS_ALONE"] = "1"
    else:
        os.environ.pop("GX_LCS_ALONE", None)
    t, _ = gx.alignment_table(cont, gx.Scores(1, -2, -1, -5), False, False, ctx=ctx, max_cell=True)   # warm
    t.free()
    path = f"/tmp/lcs_trace_{int(alone)}.csv"
    if os.path.exists(path):
        os.remove(path)
    os.environ["GX_LCS_TRACE"] = path
    t, _ = gx.alignment_table(cont, gx.Scores(1, -2, -1, -5), False, False, ctx=ctx, max_cell=True)
    fill_ms = t.info()["fill_us"] / 1e3
    t.free()
    os.environ.pop("GX_LCS_TRACE")
    rows = [list(map(int, l.split(","))) for l in open(path)]
    rows = [r for r in rows if r[0] == 0]
    st, fi, en, ww = ([r[k] for r in rows] for k in (2, 3, 4, 5))
    S = len(rows)
    t0 = min(st)
    pace = [(en[s] - fi[s]) * 10.0 / (T - 8) for s in range(S)]
    lag = [(fi[s] - fi[s - 1]) * 10.0 for s in range(1, S)]
    cross = [ww[s] // 64 != ww[s - 1] // 64 for s in range(1, S)]
    lag_h = [x for x, c in zip(lag, cross) if c]
    lag_l = [x for x, c in zip(lag, cross) if not c]
    med = lambda v: round(statistics.median(v), 1) if v else None
    print(json.dumps({"alone": alone, "n": n, "m": m, "T": T, "strips": S, "fill_ms": round(fill_ms, 3),
                      "sweep_ms": round((max(en) - t0) * 1e-5, 3), "first_strip_start_us": round((st[0] - t0) * 1e-2, 2),
                      "pace_ns_step_median": med(pace), "pace_ns_step_min": round(min(pace), 1),
                      "lag_ns_lds_median": med(lag_l), "lag_ns_hbm_median": med(lag_h),
                      "lag_steps_lds": round(med(lag_l) / med(pace), 1) if lag_l else None,
                      "wait_first_group_ns_median": med([(fi[s] - st[s]) * 10.0 for s in range(S)])}), flush=True)
ctx.close()
