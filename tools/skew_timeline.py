"""Where a layout-3 single-pair fill's time goes, from a GX_TRACE_FILE
timeline (tools/skew_diag.py SKEW_DIAG_OUT=...): per strip its first input,
pace and end; the chain decomposition T = (last strip's start) + (its
duration), the start being the sum of the strip-to-strip lags, each lag
split into its 64-step minimum (a strip's lane 0 needs the row above's
column j, which lane 63 of the strip above computes 63 steps after its own
lane 0) and the excess, by hand-off kind (inside a band: LDS ring; across
bands: HBM feed granules through the I/O waves).

    python tools/skew_timeline.py TRACE.csv [W]
"""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["strip"]))
    t0 = min(int(r["t_start"]) for r in rows)
    us = lambda x: (int(x) - t0) / 100.0          # s_memrealtime: 100 MHz ticks
    first = [us(r["t_first"]) for r in rows]
    end = [us(r["t_end"]) for r in rows]
    S = len(rows)
    # steps a strip runs: m + 64 (its lane 63 reaches column m at step m + 62)
    fill_ms = float(rows[0]["fill_ms"])
    m = None
    # the dense timeline tl0.. (a stamp every 1024 steps) gives the pace
    paces = []
    for r in rows:
        tl = [us(r[f"tl{k}"]) for k in range(64) if f"tl{k}" in r and int(r[f"tl{k}"]) > 0]
        if len(tl) >= 3:
            paces.append((tl[-1] - tl[1]) / (1024 * (len(tl) - 2)) * 1e3)
        m = m or (1024 * len(tl))
    pace = statistics.mean(paces)
    dur = [e - f for e, f in zip(end, first)]
    steps = statistics.mean(dur) * 1e3 / pace
    lags = [first[k + 1] - first[k] for k in range(S - 1)]
    intra = [lags[k] for k in range(S - 1) if (k + 1) % W]
    inter = [lags[k] for k in range(S - 1) if (k + 1) % W == 0]
    lag_min = 64 * pace / 1e3
    print(f"trace {path}: {S} strips, W = {W}, traced fill {fill_ms:.3f} ms "
          f"(untraced runs are faster: the stamps cost the core wave issue slots)")
    print(f"  strip pace {pace:.1f} ns/step (steady; mean over strips), a strip runs {statistics.mean(dur):.0f} us "
          f"= {steps:.0f} steps")
    print(f"  last strip's first input at {first[-1]:.0f} us, last end at {max(end):.0f} us")
    print(f"  lags: inside a band {statistics.mean(intra):.2f} us = {statistics.mean(intra) * 1e3 / pace:.0f} steps "
          f"({len(intra)}), across bands {statistics.mean(inter) if inter else 0:.2f} us = "
          f"{(statistics.mean(inter) if inter else 0) * 1e3 / pace:.0f} steps ({len(inter)}); minimum 64 steps = "
          f"{lag_min:.2f} us")
    chain = sum(lags)
    ex_intra = sum(l - lag_min for l in intra)
    ex_inter = sum(l - lag_min for l in inter)
    print(f"  T = chain of lags {chain:.0f} us + last strip {dur[-1]:.0f} us = {chain + dur[-1]:.0f} us; "
          f"of the chain: {lag_min * (S - 1):.0f} us the 64-step minimum, {ex_intra:.0f} us excess inside bands, "
          f"{ex_inter:.0f} us excess across bands")
    print(f"  with every lag at its minimum the fill would take {lag_min * (S - 1) + dur[-1]:.0f} us at this pace")


if __name__ == "__main__":
    main()
