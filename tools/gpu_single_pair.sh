#!/bin/bash
# GPU box: the single-pair fills that ship (configs 2 and 3: the layout
# fill_layout picks; and layout 3 forced) under rocprofv3 --kernel-trace
# --stats, then one --pmc pass of issue counters per run.  Outputs under
# gpurun_out/sp_$TAG.
#   gpurun --timeout 1200 -- 'bash tools/gpu_single_pair.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r04}
O=gpurun_out/sp_$TAG
rm -rf "$O" && mkdir -p "$O"
A="--no-cpu-baseline --int32-steps 0 --no-plane-steps 0 --steps 5 --warmup 2"
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
for wl in covid brca2; do
  for lay in auto 3; do
    if [ $lay = auto ]; then unset GX_LAYOUT; else export GX_LAYOUT=$lay; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_${wl}_$lay" -o kt --output-format csv -- python3 bench.py --workload $wl $A \
        > "$O/kt_${wl}_$lay.json" 2> "$O/kt_${wl}_$lay.err" || { echo KT_FAIL $wl $lay; tail -20 "$O/kt_${wl}_$lay.err"; exit 1; }
    timeout -s KILL 240 rocprofv3 --pmc $CTRS -d "$O/pmc_${wl}_$lay" -o pmc -- python3 bench.py --workload $wl $A --no-verify \
        > "$O/pmc_${wl}_$lay.json" 2> "$O/pmc_${wl}_$lay.err" || { echo PMC_FAIL $wl $lay; tail -20 "$O/pmc_${wl}_$lay.err"; exit 1; }
    echo "$wl $lay ok"
  done
done
unset GX_LAYOUT
echo SP_DONE
