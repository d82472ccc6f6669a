# round 6: LCS mask loads as 16-B runs (GX_LCS_B128 build) vs 8-B, alternating on one box
set -o pipefail
mkdir -p gpurun_out
GX_LIB=genomics-rs_amd/build_var/libgx_amd_b128.so timeout -k 10 600 python -u -m pytest -q --maxfail=3 --timeout 300 --timeout-method thread tests/test_gpu_skew.py -k "lcs" -m gpu > gpurun_out/r06b128_tests.log 2>&1 || { echo TESTS_FAIL; tail -5 gpurun_out/r06b128_tests.log; exit 1; }
tail -1 gpurun_out/r06b128_tests.log
for r in 1 2; do
  for V in b8 b128; do
    if [ $V = b128 ]; then export GX_LIB=genomics-rs_amd/build_var/libgx_amd_b128.so; else unset GX_LIB; fi
    echo "$V"; timeout -k 10 120 python3 tools/lcs_trace.py 2>&1 | cut -c1-200 || exit 1
  done
done
