"""Single-pair fill times on the latency layouts (untraced, several runs each):
the synthetic 30k pair and BASELINE configs 2 (Covid, global) and 3 (BRCA2,
local), per band width / layout, min and median of the fill's HIP-event time.

    python tools/skew_bench.py [runs] [W ...]     (default 7 runs, W = 2)
    env SKEW_BENCH_LAYOUTS="3 1" picks the layouts (default: 3); SKEW_BENCH_TRACK=1 times
    the tracked fill (max cell + matches_at_max) with int32 score planes instead
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import gxamd as gx  # noqa: E402
import make_golden  # noqa: E402


def fasta(name):
    c = gx.SequenceContainer()
    c.from_fasta(os.path.join(ROOT, "tests", "golden", *name))
    return c.sequences[0].sequence.encode(), c.sequences[1].sequence.encode()


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    widths = [int(x) for x in sys.argv[2:]] or [2]
    layouts = os.environ.get("SKEW_BENCH_LAYOUTS", "3").split()
    ctx = gx.Context(0)
    sc = gx.Scores(1, -2, -1, -5)
    a30, b30 = make_golden.synth_pair(0, 30000)
    cw = gx.SequenceContainer()
    cw.from_fasta(os.path.join(ROOT, "tests", "golden", "comparison_data", "Covid_Wuhan.fasta"))
    cw.from_fasta(os.path.join(ROOT, "tests", "golden", "comparison_data", "Covid_USA-CA4.fasta"))
    covid = (cw.sequences[0].sequence.encode(), cw.sequences[1].sequence.encode())
    brca2 = fasta(("fasta", "Human-Mouse-BRCA2-cds.fasta"))
    cases = [("synthetic 30k", a30, b30, False), ("covid", covid[0], covid[1], False),
             ("brca2 local", brca2[0], brca2[1], True)]
    if os.environ.get("SKEW_BENCH_SMALL"):   # a lone strip and 16 strips of the synthetic pair
        cases = [("64 x 30k", a30[:64], b30, False), ("1024 x 30k", a30[:1024], b30, False)] + cases[:1]
    for lay in layouts:
        os.environ["GX_LAYOUT"] = lay
        for W in widths:
            os.environ["GX_BAND_WAVES"] = str(W)
            for name, a, b, local in cases:
                t = []
                if os.environ.get("SKEW_BENCH_TRACK"):   # tracked fill with int32 planes (the drop-in table call)
                    st = gx.StagedPairs([(a, b)], ctx=ctx)
                    for _ in range(runs + 1):
                        _, fms = st.run(sc, local, True, max_cell=True)
                        t.append(int(fms * 1e3))
                    del st
                else:
                    for _ in range(runs + 1):
                        _, r = gx.align_raw(a, b, sc, local, ctx=ctx, max_cell=False)
                        t.append(r.fill_us)
                t = t[1:]
                cells = len(a) * len(b)
                info = ctx.fill_info()
                print(f"layout {lay} (ran {info['layout']}) W={W} {name}: fill min {min(t)} med "
                      f"{statistics.median(t)} us ({cells / min(t) / 1e3:.1f} / "
                      f"{cells / statistics.median(t) / 1e3:.1f} GCUPS)", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
