"""A fixed layout-3 workload for rocprofv3 --pmc passes (tools/gpu_skew_pmc.sh):
a lone 64 x 30,000 strip (one core + one side wave) and the Covid-sized
synthetic pair, global, untracked, each aligned a few times."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import gxamd as gx  # noqa: E402
import make_golden  # noqa: E402

os.environ.setdefault("GX_LAYOUT", "3")
ctx = gx.Context(0)
sc = gx.Scores(1, -2, -1, -5)
a, b = make_golden.synth_pair(0, 30000)
which = sys.argv[1] if len(sys.argv) > 1 else "strip"
pair = (a[:64], b) if which == "strip" else (a, b)
for _ in range(3):
    _, r = gx.align_raw(pair[0], pair[1], sc, False, ctx=ctx, max_cell=False)
print(which, r.fill_us, flush=True)
ctx.close()
