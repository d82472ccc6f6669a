#!/usr/bin/env python3
"""Summarise a tools/gpu_profile.sh run (rocprofv3 rocpd SQLite outputs) into
committed files under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
                                    (name, calls, total_ns, avg_ns, pct)
  profiles/pmc_fill_<tag>.json      WRITE_SIZE / FETCH_SIZE of the fill kernel
                                    per launch -> HBM bytes (bench.py "traffic")
  profiles/<tag>_bench.json         the bench line of the same run

    python tools/rocpd_summary.py gpurun_out/prof_<tag> <tag>

HBM bytes follow MI355X_MICROARCH.md "HBM": WRITE_SIZE is exact for 16-B/lane
stores (KiB -> x1024); FETCH_SIZE reports half the bytes of wide coalesced
reads on gfx950, so it is doubled (an upper bound for the fill's narrow reads).
"""
import csv
import glob
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one_db(d):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if not dbs:
        raise SystemExit(f"no rocpd database under {d}")
    return sqlite3.connect(dbs[0])


def main():
    src, tag = sys.argv[1], sys.argv[2]
    out_dir = os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)

    ks = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)
    if ks:   # (tools/gpu_evidence.sh: the kernel-trace pass writes csv)
        with open(ks[0]) as f:
            rows = [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3,
                     float(r["Percentage"])) for r in csv.DictReader(f)]   # (ns -> us, as top_kernels)
    else:
        c = one_db(os.path.join(src, "kt"))
        rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    stats = os.path.join(out_dir, f"{tag}_kernel_stats.csv")
    with open(stats, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for r in rows:
            w.writerow([r[0], r[1], round(r[2], 1), round(r[3], 1), round(r[4], 3)])
    print("wrote", stats)
    for r in rows[:4]:
        print(f"  {r[0][:70]:70s} calls {r[1]:4d} avg {r[3] / 1e3:10.3f} ms  {r[4]:.1f}%")

    pmc = {}
    for sub, name in (("pw", "WRITE_SIZE"), ("pf", "FETCH_SIZE")):
        c = one_db(os.path.join(src, sub))
        for kname, n, avg, dur in c.execute(
                "select kernel_name, count(*), avg(value), avg(duration) from counters_collection "
                "where counter_name = ? group by kernel_name", (name,)):
            # the batch fill (the bench's timed kernel): the fill launch writing
            # the most; FETCH_SIZE of that same kernel (the bench also runs a
            # no-plane variant of the batch, which fetches as much)
            if name == "FETCH_SIZE" and "WRITE_SIZE" in pmc:
                if kname == pmc["WRITE_SIZE"]["kernel"]:
                    pmc[name] = {"kernel": kname, "launches": n, "avg_kib": avg, "avg_duration_ns": dur}
            elif ("fill_kernel" in kname or "fill_pk_kernel" in kname) and (name not in pmc or avg > pmc[name]["avg_kib"]):
                pmc[name] = {"kernel": kname, "launches": n, "avg_kib": avg, "avg_duration_ns": dur}
    bj = os.path.join(src, "bench.json")
    with open(bj if os.path.exists(bj) else os.path.join(src, "kt_bench.json")) as f:
        bench = json.loads(f.read().strip().splitlines()[-1])
    workload = bench["config"]["workload"]
    # a pass may be two fill launches (the overlapped batch):
    # the per-pass figures are the launch average times the launches per pass
    groups = int(bench.get("fill_launch", {}).get("groups", 1) or 1)
    pwb = os.path.join(src, "pw_bench.json")   # (the PMC pass's own launch shape, if it differs)
    if os.path.exists(pwb):
        with open(pwb) as f:
            groups = int(json.loads(f.read().strip().splitlines()[-1]).get("fill_launch", {}).get("groups", 1) or 1)
    wr = pmc["WRITE_SIZE"]["avg_kib"] * 1024 * groups
    rd = pmc["FETCH_SIZE"]["avg_kib"] * 1024 * 2 * groups
    out = {
        "workload": workload,
        "kernel": pmc["WRITE_SIZE"]["kernel"],
        "write_bytes_per_launch": int(wr),
        "fetch_bytes_per_launch_corrected": int(rd),
        "hbm_bytes_per_launch": int(wr + rd),
        "algorithmic_bytes_per_launch": bench["roofline"].get("hbm", bench["roofline"])["algorithmic_bytes_per_launch"],
        "correction": "WRITE_SIZE KiB x1024 (exact for 16-B/lane stores); FETCH_SIZE KiB x1024 x2 (gfx950 "
                      "reports half of wide coalesced reads; MI355X_MICROARCH.md 'HBM'); per pass = the launch "
                      "average x fill launches per pass",
        "fill_launches_per_pass": groups,
        "raw": pmc,
        "source": f"rocprofv3 --pmc WRITE_SIZE / --pmc FETCH_SIZE, separate passes, bench.py --steps 2 --warmup 1",
    }
    p = os.path.join(out_dir, f"pmc_fill_{tag}.json")
    with open(p, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", p, "hbm/alg = %.4f" % ((wr + rd) / out["algorithmic_bytes_per_launch"]))
    with open(os.path.join(out_dir, f"{tag}_bench.json"), "w") as f:
        json.dump(bench, f, indent=1)


if __name__ == "__main__":
    main()
