# GPU box: one rocprofv3 PMC pass per argument group over a short bench run.
#   gpurun -- 'bash tools/gpu_pmc.sh "<bench args>" "CTR1 CTR2 ..." ["CTR ..." ...]'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ARGS=$1; shift
O=gpurun_out/pmc
rm -rf "$O" && mkdir -p "$O"
k=0
for CTRS in "$@"; do
  k=$((k+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS -d "$O/p$k" -o p$k -- python3 bench.py $ARGS --steps 1 --warmup 1 --no-cpu-baseline \
      > "$O/p$k.json" 2> "$O/p$k.err" || { echo PMC_FAIL $k; tail -20 "$O/p$k.err"; exit 1; }
done
python3 tools/pmc_dump.py "$O"
