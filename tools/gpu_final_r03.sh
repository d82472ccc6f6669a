# GPU box: the round's closing evidence in one call -- every GPU test, the
# default bench line, a kernel trace of the local batch, and gx_align_batch on
# the local batch with and without the local twin fill.
#   gpurun --timeout 1200 -- 'bash tools/gpu_final_r03.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/final
rm -rf "$O" && mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1 || { echo TESTS_FAIL; exit 1; }
echo tests ok
timeout -k 10 400 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo BENCH_FAIL; exit 1; }
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/lkt" -o lkt --output-format csv -- python3 tools/local_batch_ab.py 3 \
    > "$O/lkt.json" 2> "$O/lkt.err" || { echo LKT_FAIL; exit 1; }
echo lkt ok
timeout -k 10 300 python -u tools/align_batch_local.py 3 > "$O/abl_twin.json" 2> "$O/abl_twin.err" || { echo ABL_FAIL; exit 1; }
GX_TWIN=0 timeout -k 10 300 python -u tools/align_batch_local.py 3 > "$O/abl_scalar.json" 2> "$O/abl_scalar.err" || { echo ABLS_FAIL; exit 1; }
echo FINAL_DONE
