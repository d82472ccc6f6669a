#!/usr/bin/env python3
"""Summarise tools/gpu_local_pmc.sh into profiles/<tag>_local_fill.json: the
bench line of the local batch (64 related 30k pairs, Smith-Waterman), the
local twin fill's rocprofv3 --kernel-trace --stats row, and its issue
counters per cell, averaged over the fill dispatches after the first (cold).

    python tools/local_fill_summary.py gpurun_out/local_<tag> <tag>
"""
import glob
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, tag = sys.argv[1], sys.argv[2]
    with open(os.path.join(src, "kt.json")) as f:
        bench = json.loads(f.read().strip().splitlines()[-1])
    # kernel trace (rocpd database): the local fill's launches, the first (cold) one apart
    kdb = sqlite3.connect(glob.glob(os.path.join(src, "kt", "**", "*.db"), recursive=True)[0])
    ks = [(n, d, g, vg, sg) for n, d, g, vg, sg in kdb.execute(
        "select name, duration, grid_x, vgpr_count, sgpr_count from kernels order by start") if "fill_pk_kernel" in n]
    durs = [d for _, d, _, _, _ in ks]
    kt = {"kernel": ks[0][0][:60], "launches": len(ks), "first_ms": round(durs[0] / 1e6, 4),
          "avg_ms_after_first": round(sum(durs[1:]) / max(len(durs) - 1, 1) / 1e6, 4),
          "min_ms": round(min(durs) / 1e6, 4), "max_ms": round(max(durs) / 1e6, 4),
          "grid_x": sorted({g for _, _, g, _, _ in ks}), "vgpr": ks[0][3], "sgpr": ks[0][4]}
    db = glob.glob(os.path.join(src, "pmc", "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    per = {}
    for kname, disp, ctr, val, dur in c.execute(
            "select kernel_name, dispatch_id, counter_name, value, duration from counters_collection"):
        if "fill_pk_kernel" in kname:
            per.setdefault(disp, {"duration_ns": dur})[ctr] = val
    disps = sorted(per)[1:]
    keys = [k for k in per[disps[0]]]
    v = {k: sum(per[x][k] for x in disps) / len(disps) for k in keys}
    cells = bench["config"]["cells_per_step"]
    groups = bench["fill_launch"].get("groups", 1)
    cells_launch = cells / groups   # (the overlapped pipeline: two launches a pass)
    out = {"source": "tools/gpu_local_pmc.sh: bench.py --local --related --pairs-per-gpu 64 --steps 3; "
                     "rocprofv3 --kernel-trace --stats, one --pmc pass",
           "bench": {k: bench[k] for k in ("value", "ms_per_step", "fill_launch", "fill_gcups_per_gpu", "config")},
           "kernel_stats": kt, "pmc_dispatches_averaged": len(disps), "cells_per_launch_avg": cells_launch,
           "pmc_fill_ms": round(v["duration_ns"] / 1e6, 4),
           "valu_per_cell": round(v["SQ_INSTS_VALU"] * 64 / cells_launch, 3),
           "salu_per_cell": round(v["SQ_INSTS_SALU"] * 64 / cells_launch, 3),
           "lds_per_cell": round(v["SQ_INSTS_LDS"] * 64 / cells_launch, 3),
           "dual_issue_frac": round(v["SQ_ACTIVE_INST_VALU2"] / max(v["SQ_INSTS_VALU"], 1), 4),
           "wait_frac_of_active": round(v["SQ_WAIT_INST_ANY"] / max(v["SQ_ACTIVE_INST_ANY"], 1), 4),
           "raw_pmc": v}
    p = os.path.join(ROOT, "profiles", f"{tag}_local_fill.json")
    with open(p, "w") as f:
        json.dump(out, f, indent=1)
    print({k: out[k] for k in ("pmc_fill_ms", "valu_per_cell", "dual_issue_frac", "wait_frac_of_active")},
          bench["value"], bench["fill_launch"])
    print("wrote", p)


if __name__ == "__main__":
    main()
