"""GPU box: fill time of the drop-in alignment_table on BASELINE config 2 / 3
pairs, tracked (max cell + matches_at_max) vs untracked, and tracked without
the LCS workgroups (GX_LCS=0, diagnostics: matches_at_max not computed).
Usage: python3 tools/tracked_ab.py [reps]; one JSON line per variant."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
    sys.path.insert(0, ROOT)
    import bench
    import gxamd as gx
    which, tracked, reps = sys.argv[2], sys.argv[3] == "1", int(sys.argv[4])
    a, b = bench.fasta_pair(gx, which)
    ctx = gx.Context(0)
    cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
    fills, mams = [], set()
    for _ in range(reps + 1):
        t, mam = gx.alignment_table(cont, gx.Scores(1, -2, -1, -5), which == "brca2", False, ctx=ctx,
                                    max_cell=tracked)
        fills.append(t.info()["fill_us"] / 1e3)
        mams.add(mam)
        t.free()
    env = {k: v for k, v in os.environ.items() if k in ("GX_LCS", "GX_LCS_ALONE", "GX_LIB")}
    print(json.dumps({"pair": which, "tracked": tracked, "env": env,
                      "layout": ctx.fill_info()["layout"], "fill_ms_median": round(statistics.median(fills[1:]), 3),
                      "fill_ms": [round(x, 3) for x in fills[1:]], "matches_at_max": sorted(mams)}), flush=True)
    ctx.close()
    sys.exit(0)

reps = sys.argv[1] if len(sys.argv) > 1 else "5"
extra = sys.argv[2] if len(sys.argv) > 2 else ""   # a variant library (GX_LIB) for the last two lines
for which in ("covid", "brca2"):
    variants = [("0", {}), ("1", {}), ("1", {"GX_LCS": "0"}), ("1", {"GX_LCS_ALONE": "1"})]
    if extra:
        variants += [("1", {"GX_LIB": extra}), ("1", {"GX_LIB": extra, "GX_LCS": "0"})]
    for tracked, env in variants:
        e = dict(os.environ, **env)
        r = subprocess.run([sys.executable, __file__, "--child", which, tracked, reps], env=e, timeout=300)
        if r.returncode:
            sys.exit(r.returncode)
