"""Summarise a GX_TRACE_FILE per-strip timeline (diagnostics)."""
import csv
import sys

for f in sys.argv[1:]:
    rows = list(csv.DictReader(open(f)))
    t0 = min(int(r["t_start"]) for r in rows)
    us = lambda x: (int(x) - t0) / 100.0
    P0 = [r for r in rows if r["pair"] == "0"]
    W = int(rows[0]["W"])
    firsts = [us(r["t_first"]) for r in P0]
    lags = [firsts[k + 1] - firsts[k] for k in range(len(firsts) - 1)]
    intra = [lags[k] for k in range(len(lags)) if (k + 1) % W != 0] or [0]
    inter = [lags[k] for k in range(len(lags)) if (k + 1) % W == 0] or [0]
    durs = [us(r["t_end"]) - us(r["t_first"]) for r in rows]
    m_steps = 30064
    print(f"{f}: fill_ms {rows[0]['fill_ms']} strips {len(rows)} W {W}")
    print(f"  lag intra-band {sum(intra)/len(intra):.2f} us, inter-band {sum(inter)/len(inter):.2f} us")
    print(f"  strip compute {sum(durs)/len(durs):.0f} us avg (min {min(durs):.0f}, max {max(durs):.0f}) -> "
          f"{sum(durs)/len(durs)*1000/m_steps:.1f} ns/step")
    print(f"  last strip of pair 0 starts {firsts[-1]:.0f} us; last end {max(us(r['t_end']) for r in rows):.0f} us")
