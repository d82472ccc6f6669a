# GPU box: run selected GPU tests, then optional bench invocations.
#   gpurun -- 'bash tools/gpu_quick.sh "<pytest selection>" ["<bench args>" ...]'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/quick
rm -rf "$O" && mkdir -p "$O"
SEL=$1; shift
if [ -n "$SEL" ]; then
  eval "timeout -k 10 600 python -u -m pytest $SEL -x -v --timeout 300 --timeout-method thread" > "$O/tests.log" 2>&1 \
    || { echo TESTS_FAIL; tail -40 "$O/tests.log"; exit 1; }
  tail -3 "$O/tests.log"
fi
k=0
for B in "$@"; do
  k=$((k+1))
  timeout -k 10 400 python bench.py $B > "$O/bench$k.json" 2> "$O/bench$k.err" || { echo BENCH_FAIL $k; tail -20 "$O/bench$k.err"; exit 1; }
  cat "$O/bench$k.json"
done
echo QUICK_DONE
