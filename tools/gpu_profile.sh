# GPU box: parity tests, the default bench line (with cpu_baseline), a
# rocprofv3 kernel-trace/stats pass and two separate PMC passes (WRITE_SIZE,
# FETCH_SIZE) for the fill kernel's HBM traffic.  Outputs under gpurun_out/.
#   gpurun --timeout 1200 -- 'bash tools/gpu_profile.sh [TAG]'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
O=gpurun_out/prof_$TAG
rm -rf "$O" && mkdir -p "$O"
BENCH_ARGS=${BENCH_ARGS:-}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo TESTS_FAIL; tail -30 "$O/gpu_tests.log"; exit 1; }
tail -1 "$O/gpu_tests.log"
timeout -k 10 600 python bench.py $BENCH_ARGS > "$O/bench.json" 2> "$O/bench.err" || { echo BENCH_FAIL; tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt -- python3 bench.py $BENCH_ARGS --no-cpu-baseline \
    > "$O/kt_bench.json" 2> "$O/kt.err" || { echo KT_FAIL; tail -20 "$O/kt.err"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$O/pw" -o pw -- python3 bench.py $BENCH_ARGS --no-cpu-baseline --steps 2 --warmup 1 --int32-steps 0 --no-plane-steps 0 --single-pair-steps 0 --no-verify \
    > "$O/pw_bench.json" 2> "$O/pw.err" || { echo PMCW_FAIL; tail -20 "$O/pw.err"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$O/pf" -o pf -- python3 bench.py $BENCH_ARGS --no-cpu-baseline --steps 2 --warmup 1 --int32-steps 0 --no-plane-steps 0 --single-pair-steps 0 --no-verify \
    > "$O/pf_bench.json" 2> "$O/pf.err" || { echo PMCF_FAIL; tail -20 "$O/pf.err"; exit 1; }
find "$O" -name "*.csv" | head -20
echo PROFILE_DONE
