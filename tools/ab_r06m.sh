# round-6 A/B: tracked LCS (checkpoint rows) parity + timing, then the headline 12-bit vs round-5 library
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread tests/test_gpu_skew.py tests/test_gpu_atsize.py -k "tracked or lcs or short_pipeline" -m gpu > gpurun_out/r06m_tests.log 2>&1 || exit 1
(GX_LCS_ALONE=1 timeout -k 10 120 python3 tools/tracked_ab.py --child covid 1 3 && timeout -k 10 400 python3 tools/tracked_ab.py 5) > gpurun_out/r06m_lcs.log 2>&1 || exit 1
B="--steps 10 --warmup 2 --no-cpu-baseline --config-steps 0 --single-pair-steps 0 --int32-steps 0 --no-plane-steps 0 --local-batch-steps 0"
for r in 1 2; do
 timeout -k 10 300 python3 bench.py $B > gpurun_out/r06m_bench_new$r.json 2> gpurun_out/r06m_bench_new$r.err || exit 1
 GX_LIB=genomics-rs_amd/build_var/libgx_amd_r05.so timeout -k 10 300 python3 bench.py $B > gpurun_out/r06m_bench_r05_$r.json 2> gpurun_out/r06m_bench_r05_$r.err || exit 1
done
