"""GPU diagnostics: the sweep pace of the split column step on synthetic
pairs of few strips (n = 64 .. 640 rows, m = 30,000 columns): fill time per
column of one strip alone and of short chains, beside the one-wave layout 1.
    python tools/cs_pace2.py"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "genomics-rs_amd")]
import gxamd as gx  # noqa: E402

ctx = gx.Context(0)
rng = random.Random(3)
m = 30000
b = bytes(rng.choice(b"ACGT") for _ in range(m))
for n in (64,):
    a = bytes(rng.choice(b"ACGT") for _ in range(n))
    c = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
    row = [n]
    for cs2 in ("1", "0"):
        os.environ["GX_CS2"] = cs2
        os.environ["GX_LAYOUT"] = "1"
        best = 1e9
        for _ in range(3):
            t, _ = gx.alignment_table(c, gx.Scores(), False, False, ctx=ctx, max_cell=False)
            best = min(best, t.info()["fill_us"])
            t.free()
        row += [cs2, best, round(best * 1000 / m, 1)]
    print("n", row, flush=True)
# diagnostics: the same single strips with the side reduced to consuming
# (GX_CS2_DIAG=1: the core's pace) and with the core reduced (=2: the side's)
for diag in ("1", "2", "3", "4", "5", "6", "7", "8", "9"):
    os.environ["GX_CS2_DIAG"] = diag
    os.environ["GX_CS2"] = "1"
    for n in (64,):
        a = bytes(rng.choice(b"ACGT") for _ in range(n))
        c = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
        best = 1e9
        for _ in range(3):
            try:
                t, _ = gx.alignment_table(c, gx.Scores(), False, False, ctx=ctx, max_cell=False)
                best = min(best, t.info()["fill_us"])
                t.free()
            except gx.GxError as e:
                print("diag", diag, n, "error", e)
                break
        print("diag", diag, "n", n, best, round(best * 1000 / m, 1), flush=True)
os.environ.pop("GX_CS2_DIAG")
