#!/usr/bin/env python3
"""Summarise tools/gpu_valu.sh into profiles/valu_fill_<tag>.json: the batch
fill's VALU instructions per cell, and how close it runs to the VALU issue
ceiling MEASURED on this chip (tools/valu_probe.hip), with and without score
planes.

    python tools/valu_summary.py gpurun_out/valu_<tag> <tag> [profiles/isa_mix_*.json] [waves per SIMD]

(the twin fill, gx_fill_pk.hip: profiles/isa_mix_twin_r02.json at its 8-strip
bands' 9 waves per CU, ~2 per SIMD)

Ceiling.  valu_probe times independent streams of one instruction form at 1,
2, 4 and 8 waves per SIMD over the whole chip (kernel wall time x clock x
SIMDs / instructions).  At the fill's occupancy (a 15 + 1-wave workgroup per
CU = 4 waves per SIMD) a SIMD retires one wave64 v_max_i32 / v_cndmask_b32 /
v_cmp / DPP / SDWA / v_bfe / v_pk_* per ~4.3 cycles, and one VOP2 v_add_u32 /
v_sub_u32 per ~2.4 (the dual-issue rate, SQ_ACTIVE_INST_VALU2).  The fill's
steady-state mix (tools/isa_mix.py) weights the two:
    cpi = f_dual x cpi(v_add_u32) + (1 - f_dual) x cpi(rest)
    issue_frac = SQ_INSTS_VALU x cpi / (kernel cycles x 1024 SIMDs)
kernel cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs).  The VALU
roofline in lane-operations: peak = 1024 SIMDs x 64 lanes x clock / cpi,
achieved = SQ_INSTS_VALU x 64 / kernel time."""
import glob
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 256 * 4
FILL_WAVES_PER_SIMD = 4


def counters(d, skip=1):
    """Per-launch averages of the batch fill's counters, the process's first
    pass excluded (`skip` dispatches: its first launch is cold, code object
    load and page faults, 903 ms against 24 in the r04 trace; a pass of the
    overlapped pipeline is two launches of unequal size, so whole passes are
    averaged)."""
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    rows = {}
    for kname, disp, ctr, val, dur in c.execute(
            "select kernel_name, dispatch_id, counter_name, value, duration from counters_collection"):
        if "fill_kernel" in kname or "fill_pk_kernel" in kname:
            rows.setdefault(kname, {}).setdefault(disp, {"duration_ns": dur})[ctr] = val
    k = max(rows, key=lambda n: sum(v["duration_ns"] for v in rows[n].values()))   # the batch fill
    disps = sorted(rows[k])
    if len(disps) > skip:
        disps = disps[skip:]
    out = {}
    for ctr in rows[k][disps[0]]:
        out[ctr] = sum(rows[k][x][ctr] for x in disps) / len(disps)
    out["launches_averaged"] = len(disps)
    return k, out


def probe_cpi(probe, waves=FILL_WAVES_PER_SIMD):
    """(cpi of the dual-rate forms, cpi of the rest, names of the dual-rate
    forms): a form is dual-rate when the probe retires it in < 3 cycles."""
    dual, rest, names = [], [], set()
    for r in probe["results"]:
        if r["waves_per_simd"] != waves or "alternating" in r["op"]:
            continue
        x = r["chip_cycles_per_inst_per_simd"]
        if x < 3.0:
            dual.append(x)
            names.add(r["op"])
        else:
            rest.append(x)
    return sum(dual) / len(dual), sum(rest) / len(rest), names


def main():
    src, tag = sys.argv[1], sys.argv[2]
    mix_path = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles", "isa_mix_fill_r02.json")
    with open(os.path.join(src, "valu_probe.json")) as f:
        probe = json.load(f)
    with open(mix_path) as f:
        mix = json.load(f)
    waves = int(sys.argv[4]) if len(sys.argv) > 4 else FILL_WAVES_PER_SIMD
    cpi_dual, cpi_rest, dual_names = probe_cpi(probe, waves)
    n_dual = sum(n for op, n in mix["valu"].items()
                 if op.replace("_e32", "").replace("_e64", "").replace("subrev", "sub") in dual_names)
    f_dual = n_dual / mix["valu_total"]
    cpi = f_dual * cpi_dual + (1 - f_dual) * cpi_rest
    res = {"source": "rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_WAVE_CYCLES "
                     "SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE, bench.py --steps 2 "
                     "--warmup 1 (tools/gpu_valu.sh); ceiling from tools/valu_probe.hip",
           "ceiling": {"waves_per_simd": waves, "cpi_dual_rate_ops": round(cpi_dual, 3),
                       "cpi_other_ops": round(cpi_rest, 3), "dual_rate_forms": sorted(dual_names),
                       "dual_rate_fraction_of_fill_valu": round(f_dual, 4),
                       "cpi_fill_mix": round(cpi, 3), "isa_mix": os.path.relpath(mix_path, ROOT),
                       "probe": "valu_probe (chip wall time x clock x SIMDs / instructions)"}}
    cases = [c for c in ("planes", "noplanes") if os.path.isdir(os.path.join(src, c))]
    for case in cases:
        with open(os.path.join(src, f"{case}.json")) as f:
            bench = json.loads(f.read().strip().splitlines()[-1])
        k, v = counters(os.path.join(src, case), int(bench.get("fill_launch", {}).get("groups", 1) or 1))
        # a pass may be two fill launches: the counters are per
        # launch (rocprofv3 --pmc serialises dispatches), so per launch cells
        groups = int(bench.get("fill_launch", {}).get("groups", 1) or 1)
        cells = bench["config"]["cells_per_step"] // bench["n_gpus"] // groups
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        dur = v["duration_ns"] * 1e-9
        clk = cyc / dur
        insts = v["SQ_INSTS_VALU"]
        res[case] = {
            "workload": bench["config"]["workload"], "kernel": k,
            "duration_ms": round(dur * 1e3, 3),
            "clock_ghz": round(clk / 1e9, 3),
            "valu_insts_per_cell": round(insts * 64 / cells, 2),
            "valu_insts_per_cell_note": "wave64 instructions x 64 lanes / cells (a packed twin instruction covers two cells)",
            "salu_insts_per_cell": round(v["SQ_INSTS_SALU"] * 64 / cells, 2),
            "valu_issue_frac": round(insts * cpi / (cyc * SIMDS), 4),
            "valu_issue_frac_at_4_cycles": round(insts * 4 / (cyc * SIMDS), 4),
            "dual_issued_fraction": round(v["SQ_ACTIVE_INST_VALU2"] / insts, 4),
            "valu_lane_ops_achieved_tops": round(insts * 64 / dur / 1e12, 3),
            "valu_lane_ops_peak_tops": round(SIMDS * 64 * clk / cpi / 1e12, 3),
            "fill_gcups": round(cells / dur / 1e9, 1),
            "fill_gcups_ceiling_at_this_mix": round(SIMDS * 64 * clk / cpi / (insts * 64 / cells) / 1e9, 1),
            "resident_waves": round(v["SQ_WAVE_CYCLES"] * 4 / cyc, 1),
            "raw": v,
        }
    p = os.path.join(ROOT, "profiles", f"valu_fill_{tag}.json")
    with open(p, "w") as f:
        json.dump(res, f, indent=1)
    print("cpi", res["ceiling"])
    for case in cases:
        r = res[case]
        print(case, r["duration_ms"], "ms", r["clock_ghz"], "GHz VALU/cell", r["valu_insts_per_cell"],
              "issue", r["valu_issue_frac"], "dual", r["dual_issued_fraction"], "ceiling GCUPS",
              r["fill_gcups_ceiling_at_this_mix"], "fill", r["fill_gcups"])


if __name__ == "__main__":
    main()
