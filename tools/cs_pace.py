"""Column-step (layout 1) pace: fill time of one m = 30000 pair cut to
1, 3, 9, 30 64-row strips, per column, for the library in GX_LIB (diagnostic
builds drop store kinds: GX_DIAG_NO_PLANES / _SKEL / _CODES).
    GX_LAYOUT=1 python tools/cs_pace.py [strips ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
import bench  # noqa: E402
import gxamd as gx  # noqa: E402

M = 30000
sc = gx.Scores(*bench.SCORES)
lib = os.environ.get("GX_LIB", "default").split("/")[-1] + " W=" + os.environ.get("GX_BAND_WAVES", "auto")
a, b = bench.synth_pair(0, M)
for ns in [int(x) for x in (sys.argv[1:] or ["1", "3", "9", "30"])]:
    st = gx.StagedPairs([(a[:64 * ns], b)])
    fs = []
    for k in range(4):
        _, fms = st.run(sc, False, os.environ.get("PLANES", "1") == "1")
        if k:
            fs.append(fms)
    f = min(fs)
    print(f"{lib} strips {ns:3d}: fill {f:.3f} ms  {f * 1e6 / M:.1f} ns/column (incl. lag)", flush=True)
