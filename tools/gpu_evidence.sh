# GPU box: the evidence for the headline fill in one session -- the VALU issue
# probe, a kernel-trace/stats pass of the headline bench, the HBM traffic
# (WRITE_SIZE and FETCH_SIZE, separate passes) and the VALU issue counters,
# each its own rocprofv3 run.  Outputs under gpurun_out/ev_$TAG.
#   gpurun --timeout 1200 -- 'bash tools/gpu_evidence.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r04}
O=gpurun_out/ev_$TAG
rm -rf "$O" && mkdir -p "$O"
A="--no-cpu-baseline --config-steps 0 --int32-steps 0 --no-plane-steps 0 --single-pair-steps 0 --local-batch-steps 0"
timeout -k 10 120 ./tools/valu_probe > "$O/valu_probe.json" 2> "$O/valu_probe.err" || { echo PROBE_FAIL; exit 1; }
echo probe ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py $A --steps 5 --warmup 1 \
    > "$O/kt_bench.json" 2> "$O/kt.err" || { echo KT_FAIL; tail -20 "$O/kt.err"; exit 1; }
echo kt ok
# (the PMC passes run the timed configuration itself, the overlapped two-group
# pipeline; rocprofv3 --pmc serialises the dispatches, so the counters are per
# launch of each group and a pass is the sum of its two launches)
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/pw" -o pw -- python3 bench.py $A --steps 2 --warmup 1 --no-verify \
    > "$O/pw_bench.json" 2> "$O/pw.err" || { echo PMCW_FAIL; tail -20 "$O/pw.err"; exit 1; }
echo pw ok
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/pf" -o pf -- python3 bench.py $A --steps 2 --warmup 1 --no-verify \
    > "$O/pf_bench.json" 2> "$O/pf.err" || { echo PMCF_FAIL; tail -20 "$O/pf.err"; exit 1; }
echo pf ok
CTRS="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
mkdir -p "$O/valu"
cp "$O/valu_probe.json" "$O/valu/valu_probe.json"
timeout -s KILL 240 rocprofv3 --pmc $CTRS -d "$O/valu/planes" -o planes -- python3 bench.py $A --steps 2 --warmup 1 --no-verify \
    > "$O/valu/planes.json" 2> "$O/valu/planes.err" || { echo PMCV_FAIL; tail -20 "$O/valu/planes.err"; exit 1; }
echo EVIDENCE_DONE
