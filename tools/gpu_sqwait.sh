#!/bin/bash
# GPU box: where the batch fill's wave cycles go (SQ wait/issue split), compact planes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/sqwait
rm -rf "$O" && mkdir -p "$O"
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --single-pair-steps 0 --no-plane-steps 0"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  -d "$O/p" -o p -- python3 bench.py $ARGS > "$O/p.json" 2> "$O/p.err" || { echo PMC_FAIL; tail -20 "$O/p.err"; exit 1; }
python3 tools/pmc_dump.py "$O" | grep "fill_kernel<8"
