set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "untracked_table_planes or staged or random_pairs_batched or untracked_batch" > gpurun_out/t2.log 2>&1 || { tail -30 gpurun_out/t2.log; exit 1; }
tail -1 gpurun_out/t2.log
NO_TESTS=1 bash tools/gpu_libsweep.sh "genomics-rs_amd/libgx_amd.so var/libgx_sbdesc.so genomics-rs_amd/libgx_amd.so var/libgx_sbdesc.so" "64|"
