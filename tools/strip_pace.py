"""Strip pace: fill time of one m=30000 pair with a few 128-row strips (no
planes of other pairs around), per anti-diagonal step, for the library in
GX_LIB (diagnostic builds drop store kinds: GX_DIAG_NO_PLANES / _SKEL /
_CODES).  pace = fill / (T + (strips - 1) * 74 lag steps)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
import bench  # noqa: E402
import gxamd as gx  # noqa: E402

M = 30000
sc = gx.Scores(*bench.SCORES)
lib = os.environ.get("GX_LIB", "default").split("/")[-1] + " W=" + os.environ.get("GX_BAND_WAVES", "auto") + \
    " planes=" + os.environ.get("PLANES", "1")
strips_list = [int(x) for x in (sys.argv[1:] or ["1", "3", "9", "30", "117"])]
a, b = bench.synth_pair(0, M)
for ns in strips_list:
    rows = 128 * ns
    st = gx.StagedPairs([(a[:rows], b)])
    fs = []
    planes = os.environ.get("PLANES", "1") == "1"
    for k in range(4):
        _, fms = st.run(sc, False, planes)
        if k:
            fs.append(fms)
    f = min(fs)
    steps = M + 64 + (ns - 1) * 74
    print(f"{lib:28s} strips {ns:4d} fill {f:7.3f} ms  pace {f * 1e6 / steps:6.1f} ns/step", flush=True)
