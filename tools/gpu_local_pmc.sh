#!/bin/bash
# GPU box: the local twin fill (gx_fill_pk.hip LOCAL) on the bench's local
# batch shape (64 related 30k pairs, Smith-Waterman, twin plane codes): one
# rocprofv3 --kernel-trace --stats run and one --pmc pass of issue counters.
#   gpurun -- 'bash tools/gpu_local_pmc.sh TAG'  ->  gpurun_out/local_TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r04}
O=gpurun_out/local_$TAG
rm -rf "$O" && mkdir -p "$O"
ARGS="--local --related --pairs-per-gpu 64 --steps 3 --warmup 1 --no-cpu-baseline --single-pair-steps 0 --no-plane-steps 0 --int32-steps 0 --no-verify"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt -- python3 bench.py $ARGS > "$O/kt.json" 2> "$O/kt.err" || { echo KT_FAIL; tail -20 "$O/kt.err"; exit 1; }
CTRS="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $CTRS -d "$O/pmc" -o pmc -- python3 bench.py $ARGS > "$O/pmc.json" 2> "$O/pmc.err" || { echo PMC_FAIL; tail -20 "$O/pmc.err"; exit 1; }
echo LOCAL_PMC_DONE
