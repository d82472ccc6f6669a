"""Layout-3 (gx_skew.hip) diagnostics on the GPU: fill time and the per-strip
timeline (GX_TRACE_FILE) of single pairs of growing height, so that a
strip's own pace (ns per step), the lag between consecutive strips inside a
band and across a band hand-off, and the input waits can be read apart.

    python tools/skew_diag.py [W ...]     (default W = 4)
"""
import csv
import os
import statistics
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import gxamd as gx  # noqa: E402
import make_golden  # noqa: E402


def summarize(path, m, W):
    rows = list(csv.DictReader(open(path)))
    t0 = min(int(r["t_start"]) for r in rows)
    us = lambda x: (int(x) - t0) / 100.0   # s_memrealtime ticks are 10 ns
    first = [us(r["t_first"]) for r in rows]
    dur = [us(r["t_end"]) - us(r["t_first"]) for r in rows]
    lags = [first[k + 1] - first[k] for k in range(len(first) - 1)]
    intra = [lags[k] for k in range(len(lags)) if (k + 1) % W] or [0.0]
    inter = [lags[k] for k in range(len(lags)) if (k + 1) % W == 0] or [0.0]
    clk = [int(r["clk"]) / max(d, 1e-9) for r, d in zip(rows, dur)]
    ramp = [(us(r["q1"]) - us(r["t_first"])) * 1e3 / 64 for r in rows if int(r["q1"]) > 0]
    steps = m + 64
    print(f"    strips {len(rows)}: pace {statistics.mean(dur) * 1e3 / steps:.1f} ns/step "
          f"(min {min(dur) * 1e3 / steps:.1f}, max {max(dur) * 1e3 / steps:.1f}); "
          f"ramp-up {statistics.mean(ramp) if ramp else 0:.1f} ns/step; "
          f"lag intra {statistics.mean(intra):.2f} us = {statistics.mean(intra) * 1e3 / (statistics.mean(dur) * 1e3 / steps):.0f} steps, "
          f"inter {statistics.mean(inter):.2f} us; clock {statistics.mean(clk):.0f} MHz; "
          f"core waits: input {statistics.mean(int(r['wait_in']) for r in rows):.0f} hand-off space "
          f"{statistics.mean(int(r['q6']) for r in rows):.0f}; side waits {statistics.mean(int(r['wait_out']) for r in rows):.0f}, "
          f"side ends {statistics.mean(us(r['q7']) - us(r['t_end']) for r in rows):.1f} us after the core; "
          f"last strip first input at {first[-1]:.0f} us, "
          f"end {max(us(r['t_end']) for r in rows):.0f} us")


def main():
    widths = [int(x) for x in sys.argv[1:]] or [4]
    ctx = gx.Context(0)
    sc = gx.Scores(1, -2, -1, -5)
    a30, b30 = make_golden.synth_pair(0, 30000)
    cases = [("64x30000", a30[:64], b30), ("256x30000", a30[:256], b30), ("1024x30000", a30[:1024], b30),
             ("30000x30000", a30, b30)]
    if os.environ.get("SKEW_DIAG_QUICK"):
        cases = cases[:2]
    if os.environ.get("SKEW_DIAG_LONE"):   # (a lone strip: for experiment builds without pushes)
        cases = cases[:1]
    if os.environ.get("SKEW_DIAG_FULL"):   # (the full 30k pair only)
        cases = cases[-1:]
    modes = (False,) if os.environ.get("SKEW_DIAG_GLOBAL") else (False, True)
    keep = os.environ.get("SKEW_DIAG_OUT")  # (a directory: keep the trace CSVs)
    os.environ["GX_LAYOUT"] = "3"
    for W in widths:
        os.environ["GX_BAND_WAVES"] = str(W)
        for name, a, b in cases:
            for local in modes:
                # (int32 score planes, as the drop-in table call and bench.py's
                # config records keep them: the traced instantiation has planes)
                st = gx.StagedPairs([(a, b)], ctx=ctx)
                for _ in range(2):
                    res, fms = st.run(sc, local, True)
                r = res[0]
                tr = os.path.join(tempfile.gettempdir(), f"skew_{W}_{name}_{int(local)}.csv")
                os.environ["GX_TRACE_FILE"] = tr
                _, fms2 = st.run(sc, local, True)
                del os.environ["GX_TRACE_FILE"]
                cells = len(a) * len(b)
                fus = fms * 1e3
                print(f"W={W} {name} {'local' if local else 'global'}: fill {fus:.0f} us "
                      f"({cells / max(fus, 1) / 1e3:.1f} GCUPS), traced fill {fms2 * 1e3:.0f} us, "
                      f"retrace {r.retrace_us} us; {ctx.fill_info()}", flush=True)
                summarize(tr, len(b), W)
                if keep:
                    os.makedirs(keep, exist_ok=True)
                    import shutil
                    shutil.copy(tr, keep)
    ctx.close()


if __name__ == "__main__":
    main()
