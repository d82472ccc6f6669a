set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "untracked_table_planes or staged or random_pairs_batched or exported_planes" > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 200 python bench.py --no-cpu-baseline --single-pair-steps 0 --steps 5 > gpurun_out/b_d8.json && python3 -c "import json;d=json.load(open('gpurun_out/b_d8.json'));print('d8',d['value'],d['roofline']['fill_ms_avg'])"
GX_PLANES32=1 timeout -k 10 200 python bench.py --no-cpu-baseline --single-pair-steps 0 --steps 5 > gpurun_out/b_32.json && python3 -c "import json;d=json.load(open('gpurun_out/b_32.json'));print('i32',d['value'],d['roofline']['fill_ms_avg'])"
