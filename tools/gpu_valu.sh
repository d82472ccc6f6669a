#!/bin/bash
# GPU box: the VALU issue probe (tools/valu_probe.hip: cycles per wave64
# instruction per SIMD, by instruction form and waves per SIMD) and the issue
# counters of the batch fill (the bench's headline kernel), with compact
# planes and without planes, one rocprofv3 --pmc pass each (<= 8 SQ counters).
#   gpurun -- 'bash tools/gpu_valu.sh TAG'  ->  gpurun_out/valu_TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02}
O=gpurun_out/valu_$TAG
rm -rf "$O" && mkdir -p "$O"
if [ -x tools/valu_probe ]; then
  timeout -k 10 120 ./tools/valu_probe > "$O/valu_probe.json" 2> "$O/valu_probe.err" || { echo PROBE_FAIL; exit 1; }
fi
CTRS="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --single-pair-steps 0 --no-plane-steps 0 --no-verify"
timeout -s KILL 240 rocprofv3 --pmc $CTRS -d "$O/planes" -o planes -- python3 bench.py $ARGS > "$O/planes.json" 2> "$O/planes.err" || { echo PMC_FAIL; tail -20 "$O/planes.err"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc $CTRS -d "$O/noplanes" -o noplanes -- python3 bench.py $ARGS --no-planes > "$O/noplanes.json" 2> "$O/noplanes.err" || { echo PMC_FAIL2; tail -20 "$O/noplanes.err"; exit 1; }
python3 tools/pmc_dump.py "$O" | grep fill_kernel
echo VALU_DONE
