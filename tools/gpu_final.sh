# GPU box: the round's closing evidence from the final build in one session:
# GPU tests, the default bench line, then tools/gpu_evidence.sh (VALU probe,
# kernel stats, PMC traffic, VALU counters).  Output under gpurun_out/fin_$TAG
# and gpurun_out/ev_$TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03}
O=gpurun_out/fin_$TAG; rm -rf "$O"; mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; tail -1 "$O/tests.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo BENCH_FAIL; tail -5 "$O/bench.err"; exit 1; }
echo bench ok
bash tools/gpu_evidence.sh "$TAG"
