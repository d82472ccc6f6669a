# round 6: reductions beside the next fill -- the pipelined batch tests, tracked parity, config lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --maxfail=3 --timeout 300 --timeout-method thread tests/test_gpu_atsize.py tests/test_gpu_skew.py tests/test_gpu_twin.py -m gpu > gpurun_out/r06pa_tests.log 2>&1 || { echo TESTS_FAIL; tail -5 gpurun_out/r06pa_tests.log; exit 1; }
tail -1 gpurun_out/r06pa_tests.log
timeout -k 10 300 python3 tools/config_lines.py 10 > gpurun_out/r06pa_lines.log 2>&1 || exit 1
cat gpurun_out/r06pa_lines.log
