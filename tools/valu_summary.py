#!/usr/bin/env python3
"""Summarise tools/gpu_valu.sh (rocprofv3 --pmc SQ_INSTS_VALU ... GRBM_GUI_ACTIVE)
into profiles/valu_fill_<tag>.json: VALU instructions per cell and the VALU
issue fraction of the batch fill, with and without score planes.

    python tools/valu_summary.py gpurun_out/valu_<tag> <tag>

issue_frac = SQ_INSTS_VALU x 4 cycles (a wave64 VALU op occupies a 16-lane
SIMD for 4 cycles) / (kernel cycles x 1024 SIMDs), kernel cycles =
GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs; MI355X_MICROARCH.md "DVFS").
SQ_WAVE_CYCLES counts quad-cycles (its ratio to the kernel cycles is the
resident waves / 4)."""
import glob
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 256 * 4


def counters(d):
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    out = {}
    for kname, ctr, avg, dur in c.execute(
            "select kernel_name, counter_name, avg(value), avg(duration) from counters_collection "
            "group by kernel_name, counter_name"):
        if "fill_kernel" in kname:
            out.setdefault(kname, {"duration_ns": dur})[ctr] = avg
    # the batch fill: the longest fill launch
    k = max(out, key=lambda n: out[n]["duration_ns"])
    return k, out[k]


def main():
    src, tag = sys.argv[1], sys.argv[2]
    res = {"source": "rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS "
                     "GRBM_GUI_ACTIVE, bench.py --steps 2 --warmup 1 (tools/gpu_valu.sh)"}
    for case in ("planes", "noplanes"):
        k, v = counters(os.path.join(src, case))
        with open(os.path.join(src, f"{case}.json")) as f:
            bench = json.loads(f.read().strip().splitlines()[-1])
        cells = bench["config"]["cells_per_step"] // bench["n_gpus"]
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        res[case] = {
            "workload": bench["config"]["workload"], "kernel": k,
            "duration_ms": round(v["duration_ns"] / 1e6, 3),
            "clock_ghz": round(cyc / v["duration_ns"], 3),
            "valu_insts_per_cell": round(v["SQ_INSTS_VALU"] * 64 / cells, 2),
            "salu_insts_per_cell": round(v["SQ_INSTS_SALU"] * 64 / cells, 2),
            "lds_insts_per_cell": round(v["SQ_INSTS_LDS"] * 64 / cells, 2),
            "valu_issue_frac": round(v["SQ_INSTS_VALU"] * 4 / (cyc * SIMDS), 4),
            "resident_waves": round(v["SQ_WAVE_CYCLES"] * 4 / cyc, 1),
            "raw": v,
        }
    p = os.path.join(ROOT, "profiles", f"valu_fill_{tag}.json")
    with open(p, "w") as f:
        json.dump(res, f, indent=1)
    for case in ("planes", "noplanes"):
        r = res[case]
        print(case, r["duration_ms"], "ms", r["clock_ghz"], "GHz VALU/cell", r["valu_insts_per_cell"],
              "issue", r["valu_issue_frac"], "waves", r["resident_waves"])


if __name__ == "__main__":
    main()
