"""Summarise a GX_TRACE_FILE per-strip timeline (diagnostics)."""
import csv
import sys

for f in [a for a in sys.argv[1:] if not a.startswith("--")]:
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
    if "clk" in rows[0]:
        mhz = [int(r["clk"]) / max(us(r["t_end"]) - us(r["t_first"]), 1e-9) for r in rows]
        print(f"  shader clock while computing: {sum(mhz)/len(mhz):.0f} MHz avg (min {min(mhz):.0f}, max {max(mhz):.0f})")
    print(f"  last strip of pair 0 starts {firsts[-1]:.0f} us; last end {max(us(r['t_end']) for r in rows):.0f} us")

    # timeline: active strips and implied plane-store bandwidth per 1 ms bin
    # (1.5 KiB per strip per step: 3 int32 planes x 128 rows)
    if "--bins" in sys.argv or True:
        end = max(us(r["t_end"]) for r in rows)
        nb = int(end // 1000) + 1
        act = [0.0] * nb
        bw = [0.0] * nb
        for r in rows:
            a, b = us(r["t_first"]), us(r["t_end"])
            rate = 1536.0 * m_steps / max(b - a, 1e-9) / 1e3   # GB/s while active (bytes/us / 1e3)
            for k in range(nb):
                lo, hi = 1000.0 * k, 1000.0 * (k + 1)
                ov = max(0.0, min(b, hi) - max(a, lo)) / 1000.0
                act[k] += ov
                bw[k] += ov * rate
        print("  ms  active  GB/s(planes)")
        for k in range(nb):
            print(f"  {k:3d} {act[k]:7.0f} {bw[k]:8.0f}")
