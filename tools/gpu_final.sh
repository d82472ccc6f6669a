#!/bin/bash
# GPU box: the closing checks of a round in one session -- the full -m gpu
# suite, smoke(), the default bench line, the local fill's profile
# (tools/gpu_local_pmc.sh) and the 1024 x 1k band/grid sweep.
#   gpurun --timeout 1200 -- 'bash tools/gpu_final.sh TAG'  ->  gpurun_out/fin_TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04}
O=gpurun_out/fin_$TAG
rm -rf "$O" && mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu.log" 2>&1 || { echo TESTS_FAIL; tail -30 "$O/gpu.log"; exit 1; }
tail -1 "$O/gpu.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > "$O/smoke.log" 2>&1 || { echo SMOKE_FAIL; tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo BENCH_FAIL; tail -20 "$O/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));lb=d.get('local_batch',{});print('bench',d['value'],d['ms_per_step'],'local',lb.get('gcups'),lb.get('fill_launch'),lb.get('parity',{}).get('pairs_checked'))"
timeout -k 10 500 bash tools/gpu_local_pmc.sh "$TAG" || exit 1
bash tools/k1_grid_sweep.sh
