#!/usr/bin/env python3
"""Summarise tools/gpu_single_pair.sh (configs 2 and 3 on the layout the host
picks and on layout 3 forced) into profiles/<tag>_single_pair.json: the bench
line, the fill kernel's rocprofv3 --kernel-trace --stats row, and its issue
counters per DP step of the critical path (n + m + 63 anti-diagonal steps)
and per cell, averaged over the fill dispatches after the first.

    python tools/single_pair_summary.py gpurun_out/sp_<tag> <tag>
"""
import csv
import glob
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZES = {"covid": (29903, 29882), "brca2": (11382, 10346)}


def fill_row(path):
    with open(path) as f:
        rows = [r for r in csv.DictReader(f) if "gx::fill" in r["Name"]]
    r = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    return {"kernel": r["Name"][:100], "calls": int(r["Calls"]), "avg_ms": round(float(r["AverageNs"]) / 1e6, 4),
            "min_ms": round(float(r["MinNs"]) / 1e6, 4), "max_ms": round(float(r["MaxNs"]) / 1e6, 4)}


def pmc(d):
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    per = {}
    for kname, disp, ctr, val, dur in c.execute(
            "select kernel_name, dispatch_id, counter_name, value, duration from counters_collection"):
        if "gx::fill" in kname:   # (not the runtime's __amd_rocclr_fillBufferAligned memsets)
            per.setdefault(disp, {"duration_ns": dur, "kernel": kname})[ctr] = val
    disps = sorted(per)[1:] or sorted(per)
    keys = [k for k in per[disps[0]] if k != "kernel"]
    return {k: sum(per[x][k] for x in disps) / len(disps) for k in keys}, len(disps)


def main():
    src, tag = sys.argv[1], sys.argv[2]
    out = {"source": "tools/gpu_single_pair.sh: rocprofv3 --kernel-trace --stats and one --pmc pass per case, "
                     "bench.py --workload covid|brca2 --steps 5 --warmup 2",
           "cases": {}}
    for wl in ("covid", "brca2"):
        n, m = SIZES[wl]
        for lay in ("auto", "3"):
            name = f"{wl}_{lay}"
            with open(os.path.join(src, f"kt_{name}.json")) as f:
                bench = json.loads(f.read().strip().splitlines()[-1])
            k = fill_row(glob.glob(os.path.join(src, f"kt_{name}", "**", "*kernel_stats.csv"), recursive=True)[0])
            v, nd = pmc(os.path.join(src, f"pmc_{name}"))
            steps = n + m + 63
            case = {"layout": bench["fill_launch"]["layout"], "band_waves": bench["fill_launch"]["band_waves"],
                    "gcups": bench["value"], "ms_per_step": bench["ms_per_step"],
                    "fill_gcups": bench.get("fill_gcups_per_gpu"), "kernel_stats": k,
                    "pmc_dispatches_averaged": nd, "pmc_fill_ms": round(v["duration_ns"] / 1e6, 4)}
            for ctr in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
                case[ctr.lower() + "_per_cell"] = round(v[ctr] * 64 / (n * m), 3)
            case["sq_wait_inst_any_frac"] = round(v["SQ_WAIT_INST_ANY"] / max(v["SQ_WAVE_CYCLES"], 1), 4)
            case["sq_active_inst_any_frac"] = round(v["SQ_ACTIVE_INST_ANY"] / max(v["SQ_WAVE_CYCLES"], 1), 4)
            case["ns_per_critical_step"] = round(k["avg_ms"] * 1e6 / steps, 2)
            case["raw_pmc"] = v
            out["cases"][name] = case
            print(name, case["layout"], case["gcups"], "fill", k["avg_ms"], "ms", case["ns_per_critical_step"],
                  "ns/step  VALU/cell", case["sq_insts_valu_per_cell"], "wait", case["sq_wait_inst_any_frac"])
    p = os.path.join(ROOT, "profiles", f"{tag}_single_pair.json")
    with open(p, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", p)


if __name__ == "__main__":
    main()
