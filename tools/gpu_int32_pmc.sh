#!/bin/bash
# GPU box: HBM traffic of the int32-plane batch fill (bench.py's int32_planes
# record: the same 80 x 30k batch with GX_PLANES32=1, 12 B/cell, in chunks),
# WRITE_SIZE and FETCH_SIZE in separate rocprofv3 --pmc passes, plus a
# kernel-trace/stats pass for its launch times.  Outputs under gpurun_out/i32_$TAG.
#   gpurun --timeout 900 -- 'bash tools/gpu_int32_pmc.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05}
O=gpurun_out/i32_$TAG
rm -rf "$O" && mkdir -p "$O"
export GX_PLANES32=1
A="--no-cpu-baseline --config-steps 0 --int32-steps 0 --no-plane-steps 0 --single-pair-steps 0 --local-batch-steps 0 --no-verify --steps 2 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py $A \
    > "$O/kt_bench.json" 2> "$O/kt.err" || { echo KT_FAIL; tail -20 "$O/kt.err"; exit 1; }
echo kt ok
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pw" -o pw -- python3 bench.py $A \
    > "$O/pw_bench.json" 2> "$O/pw.err" || { echo PMCW_FAIL; tail -20 "$O/pw.err"; exit 1; }
echo pw ok
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pf" -o pf -- python3 bench.py $A \
    > "$O/pf_bench.json" 2> "$O/pf.err" || { echo PMCF_FAIL; tail -20 "$O/pf.err"; exit 1; }
echo I32_DONE
