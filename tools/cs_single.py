"""One single-strip table fill (64 x 30,000, global, int32 planes) per call
through the split column step: the target of PMC profiles (tools/pmc_cs2.sh)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "genomics-rs_amd")]
import gxamd as gx  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ctx = gx.Context(0)
rng = random.Random(3)
a = "".join(rng.choice("ACGT") for _ in range(n))
b = "".join(rng.choice("ACGT") for _ in range(30000))
c = gx.SequenceContainer([gx.Sequence("a", a), gx.Sequence("b", b)])
os.environ.setdefault("GX_LAYOUT", "1")
for _ in range(3):
    t, _ = gx.alignment_table(c, gx.Scores(), False, False, ctx=ctx, max_cell=False)
    print("fill_us", t.info()["fill_us"], ctx.fill_info(), flush=True)
    t.free()
