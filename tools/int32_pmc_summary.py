#!/usr/bin/env python3
"""Summarise tools/gpu_int32_pmc.sh into profiles/pmc_int32_<tag>.json: HBM
bytes of the int32-plane batch fill (bench.py's int32_planes record) from
WRITE_SIZE and FETCH_SIZE (separate passes; MI355X_MICROARCH.md 'HBM':
WRITE_SIZE KiB x 1024, FETCH_SIZE KiB x 1024 x 2 on gfx950), per pass (the
chunk launches of one pass summed) against 12 B per cell, and the fill's
launch times from the kernel trace of the same command.

    python tools/int32_pmc_summary.py gpurun_out/i32_<tag> <tag>
"""
import csv
import glob
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(d, ctr):
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    out = {}
    for kname, disp, val, dur in c.execute(
            "select kernel_name, dispatch_id, value, duration from counters_collection where counter_name = ?", (ctr,)):
        if "gx::fill_kernel" in kname:
            out.setdefault(disp, [kname, 0.0, dur])[1] += val
    return [out[k] for k in sorted(out)]


def main():
    src, tag = sys.argv[1], sys.argv[2]
    with open(os.path.join(src, "kt_bench.json")) as f:
        bench = json.loads(f.read().strip().splitlines()[-1])
    chunks = int(bench["fill_launch"]["chunks"])
    cells = bench["config"]["cells_per_step"]
    w = per_dispatch(os.path.join(src, "pw"), "WRITE_SIZE")
    r = per_dispatch(os.path.join(src, "pf"), "FETCH_SIZE")
    # the process's passes: warmup 1 + 2 timed, each `chunks` launches; the last pass's launches
    wl, rl = w[-chunks:], r[-chunks:]
    wr = sum(x[1] for x in wl) * 1024
    rd = sum(x[1] for x in rl) * 1024 * 2
    with open(glob.glob(os.path.join(src, "kt", "**", "*kernel_trace.csv"), recursive=True)[0]) as f:
        kt = [row for row in csv.DictReader(f) if "gx::fill_kernel" in row["Kernel_Name"]]
    kt.sort(key=lambda x: int(x["Start_Timestamp"]))
    last = kt[-chunks:]
    launch_ms = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6 for x in last]
    alg = 12 * cells
    out = {
        "workload": bench["config"]["workload"],
        "kernel": wl[-1][0][:100],
        "chunks_per_pass": chunks,
        "write_bytes_per_pass": int(wr),
        "fetch_bytes_per_pass_corrected": int(rd),
        "hbm_bytes_per_pass": int(wr + rd),
        "algorithmic_bytes_per_pass": alg,
        "hbm_over_algorithmic": round((wr + rd) / alg, 4),
        "write_over_algorithmic": round(wr / alg, 4),
        "kernel_ms_per_pass": round(sum(launch_ms), 3),
        "kernel_ms_per_launch": [round(x, 3) for x in launch_ms],
        "write_tb_s_over_kernel_time": round(wr / (sum(launch_ms) * 1e-3) / 1e12, 3),
        "algorithmic_tb_s_over_kernel_time": round(alg / (sum(launch_ms) * 1e-3) / 1e12, 3),
        "bench_fill_ms_avg": bench["roofline"].get("fill_ms_avg"),
        "source": "tools/gpu_int32_pmc.sh: GX_PLANES32=1 bench.py --steps 2 --warmup 1, rocprofv3 --kernel-trace "
                  "--stats and --pmc WRITE_SIZE / FETCH_SIZE in separate passes; the last pass's chunk launches",
        "correction": "WRITE_SIZE KiB x1024, FETCH_SIZE KiB x1024 x2 (MI355X_MICROARCH.md 'HBM')",
    }
    p = os.path.join(ROOT, "profiles", f"pmc_int32_{tag}.json")
    with open(p, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
