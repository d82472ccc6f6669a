# round 6: tracked-path parity, then the four single-pair config lines (c2, c3, c2t, c3t)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread tests/test_gpu_skew.py tests/test_gpu_atsize.py -k "tracked or lcs or max_cell" -m gpu > gpurun_out/r06n_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/config_lines.py 10 > gpurun_out/r06n_lines.log 2>&1 || exit 1
