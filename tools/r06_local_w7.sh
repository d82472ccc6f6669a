# round 6: local twin fill at 123 VGPRs -- parity, then local_batch at 8-wave bands (one a CU) vs 7 (two a CU)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_twin_local.py -m gpu > gpurun_out/r06w_tests.log 2>&1 || { echo TESTS_FAIL; tail -5 gpurun_out/r06w_tests.log; exit 1; }
tail -1 gpurun_out/r06w_tests.log
A="--steps 1 --warmup 1 --no-cpu-baseline --config-steps 0 --single-pair-steps 0 --int32-steps 0 --no-plane-steps 0 --no-verify"
for r in 1 2; do
  for W in auto 7; do
    if [ "$W" = auto ]; then unset GX_BAND_WAVES; else export GX_BAND_WAVES=$W; fi
    timeout -k 10 300 python3 bench.py $A > gpurun_out/r06w_${W}_${r}.json 2> gpurun_out/r06w_${W}_$r.err || { echo BENCH_FAIL; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r06w_${W}_${r}.json'));lb=d['local_batch'];print('$W',lb['gcups'],lb['fill_ms_avg'],lb['fill_launch'],lb['parity']['pairs_checked'])"
  done
done
