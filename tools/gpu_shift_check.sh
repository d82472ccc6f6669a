#!/bin/bash
# Full GPU parity suite + headline / all-vs-all / 16k bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/ -m gpu > gpurun_out/t6.log 2>&1 || { tail -30 gpurun_out/t6.log; exit 1; }
tail -1 gpurun_out/t6.log
run() {
  local lab=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --single-pair-steps 0 --steps 3 "$@" > gpurun_out/w.json 2>gpurun_out/w.err || { echo FAIL $lab; tail -5 gpurun_out/w.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/w.json'));r=d['roofline'];f=d['fill_launch'];print('$lab',d['value'],r['fill_ms_avg'],f['layout'],f['band_waves'],d.get('no_plane_fill'))"
}
run p64 || exit 1
run ava --workload allvsall || exit 1
run 16k --pairs-per-gpu 128 --length 16384 || exit 1
run p64 || exit 1
