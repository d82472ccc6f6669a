# GPU box: the GPU tests, then (unless they crashed or timed out: pytest exit
# codes 0 / 1 only) a short headline bench.  Output under gpurun_out/$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-check}; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$O/tests.log" 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
GX_LOG=${BENCH_LOG:-} timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --config-steps 0 --int32-steps 0 \
    --no-plane-steps 0 --single-pair-steps 0 > "$O/bench.json" 2> "$O/bench.err"
echo "bench rc=$?"
