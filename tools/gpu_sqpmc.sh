# GPU box: SQ stall counters of the fill kernel for a lone layout-1 strip
#   gpurun -- 'bash tools/gpu_sqpmc.sh [layout]'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp GX_LAYOUT=${1:-1}
O=gpurun_out/sqpmc
rm -rf "$O" && mkdir -p "$O"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS \
   -d "$O/p1" -o p1 -- python3 tools/cs_pace.py 1 > "$O/p1.log" 2>&1 || { echo PMC_FAIL; tail -20 "$O/p1.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INSTS_SMEM \
   -d "$O/p2" -o p2 -- python3 tools/cs_pace.py 1 > "$O/p2.log" 2>&1 || { echo PMC_FAIL2; tail -20 "$O/p2.log"; exit 1; }
python3 tools/pmc_dump.py "$O" | grep fill_kernel
