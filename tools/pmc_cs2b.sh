# GPU box: instruction-fetch / wait counters of the core loop alone (GX_CS2_DIAG=5)
# against the register-only probe (gpurun_exp/lat_probe2, kernel probe<10>).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pmc_cs2b
rm -rf "$O" && mkdir -p "$O"
SET="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS SQ_INSTS_BRANCH"
GX_CS2_DIAG=5 timeout -s KILL 90 rocprofv3 --pmc $SET -d "$O/k" -o run --output-format csv -- python3 tools/cs_single.py > "$O/k.log" 2>&1 || echo "kernel pass failed"
timeout -s KILL 90 rocprofv3 --pmc $SET -d "$O/p" -o run --output-format csv -- ./gpurun_exp/lat_probe2 > "$O/p.log" 2>&1 || echo "probe pass failed"
echo PMC_DONE
