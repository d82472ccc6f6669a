#!/bin/bash
# GPU box: issue counters of the layout-3 fill (tools/skew_pmc.py) per
# dispatch, one rocprofv3 --pmc pass per counter set (<= 8 SQ counters).
#   gpurun -- 'bash tools/gpu_skew_pmc.sh TAG [strip|pair]'  ->  gpurun_out/skewpmc_TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-x}
W=${2:-strip}
O=gpurun_out/skewpmc_$TAG
rm -rf "$O" && mkdir -p "$O"
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
B="SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT"
timeout -s KILL 90 rocprofv3 --pmc $A -d "$O/a" -o a -- python3 tools/skew_pmc.py $W > "$O/a.log" 2>&1 || { echo PMC_A_FAIL; tail -5 "$O/a.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc $B -d "$O/b" -o b -- python3 tools/skew_pmc.py $W > "$O/b.log" 2>&1 || { echo PMC_B_FAIL; tail -5 "$O/b.log"; exit 1; }
python3 tools/pmc_dump.py "$O" | grep -i skew
echo PMC_DONE
