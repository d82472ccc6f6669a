# GPU box: per-strip fill timelines (GX_TRACE_FILE) for each "P|flags" case.
#   gpurun -- 'bash tools/gpu_trace.sh "1| 8|"'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for C in ${1:-"1| 8|"}; do
  P=${C%%|*}; F=${C#*|}
  GX_TRACE_FILE=gpurun_out/trace_p$P.csv timeout -k 10 300 python bench.py --pairs-per-gpu $P --steps 1 --warmup 1 \
      --no-cpu-baseline --single-pair-steps 0 $F > gpurun_out/trace_p$P.json 2>&1 || { echo FAIL $C; exit 1; }
done
python3 tools/trace_summary.py gpurun_out/trace_p*.csv
