"""Per-pass summary of a fill pipeline from a rocprofv3 kernel trace, so that
the bench line's fill time (fill_ms_avg: HIP events around the fill
pipeline of the K timed passes, bench.py) can be recomputed from a tracked
file.

    python tools/pass_summary.py KERNEL_TRACE.csv --passes K [--kernel fill_pk_kernel]
                                 [--cells CELLS_PER_PASS] [--out profiles/x.json]

The profiled command must end its fill launches with the K timed passes
(bench.py ... --no-verify --int32-steps 0 --no-plane-steps 0
--single-pair-steps 0 --config-steps 0 --local-batch-steps 0): the timed
launches are the last K x G of the kernel (G = launches per pass, read off
the streams that ran them: 2 for the overlapped two-group pipeline).  The
first launch of the process (cold: code object load, page faults) is
reported apart and never part of the timed set."""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--passes", type=int, required=True)
    ap.add_argument("--kernel", default="fill_pk_kernel")
    ap.add_argument("--cells", type=float, default=0.0, help="DP cells per pass (GCUPS column)")
    ap.add_argument("--skip", type=int, default=-1,
                    help="fill launches before the timed call (default: all but the last passes x G)")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if not rows:
        raise SystemExit(f"no {a.kernel} dispatches in {a.trace}")
    streams = sorted({r["Stream_Id"] for r in rows})
    # launches per pass: the streams among the last launches
    tail = rows[-2 * a.passes:]
    G = 2 if len({r["Stream_Id"] for r in tail}) >= 2 else 1
    timed = rows[a.skip:a.skip + G * a.passes] if a.skip >= 0 else rows[-G * a.passes:]
    t0 = int(timed[0]["Start_Timestamp"])
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6   # ns -> ms
    per_stream = {}
    for r in timed:
        per_stream.setdefault(r["Stream_Id"], []).append(r)
    span = (max(int(r["End_Timestamp"]) for r in timed) - t0) / 1e6
    out = {
        "trace": a.trace, "kernel": a.kernel, "passes": a.passes, "launches_per_pass": G,
        "cold_first_launch_ms": round(dur(rows[0]), 3), "dispatches_in_trace": len(rows),
        "timed_launches": [{"stream": r["Stream_Id"], "start_ms": round((int(r["Start_Timestamp"]) - t0) / 1e6, 3),
                            "duration_ms": round(dur(r), 3), "name": r["Kernel_Name"][:80]} for r in timed],
        "per_stream_mean_ms": {s: round(statistics.mean(dur(r) for r in v), 3) for s, v in per_stream.items()},
        "pipeline_ms_per_pass": round(span / a.passes, 3),
        "note": "pipeline_ms_per_pass = (last timed fill end - first timed fill start) / passes: the bench's "
                "fill_ms_avg (HIP events ev0..ev1 around the same launches)",
    }
    if G == 2:   # pass period from the second group's launch starts
        b = per_stream[sorted(per_stream, key=lambda s: int(per_stream[s][0]["Start_Timestamp"]))[-1]]
        st = [int(r["Start_Timestamp"]) for r in b]
        if len(st) > 1:
            out["pass_period_ms"] = round(statistics.mean((st[k + 1] - st[k]) / 1e6 for k in range(len(st) - 1)), 3)
    if a.cells:
        out["fill_gcups_per_pass"] = round(a.cells / (out["pipeline_ms_per_pass"] * 1e-3) / 1e9, 1)
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
