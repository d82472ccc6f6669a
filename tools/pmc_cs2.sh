# GPU box: PMC counters of the split column step on one strip (tools/cs_single.py).
#   gpurun -- 'bash tools/pmc_cs2.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pmc_cs2
rm -rf "$O" && mkdir -p "$O"
timeout -k 5 60 rocprofv3 -L > "$O/avail.txt" 2>&1 || true
k=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_SMEM"; do
  k=$((k+1))
  timeout -s KILL 90 rocprofv3 --pmc $SET -d "$O/p$k" -o run --output-format csv -- python3 tools/cs_single.py > "$O/p$k.log" 2>&1 \
    || { echo "PMC pass $k failed"; tail -5 "$O/p$k.log"; }
done
echo PMC_DONE
