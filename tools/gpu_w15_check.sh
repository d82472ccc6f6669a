#!/bin/bash
# Automatic band width after the deep-queue 15-strip rule: headline, all-vs-all, 16 x 30k, 128 x 16k.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
run() {
  local lab=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --single-pair-steps 0 --no-plane-steps 0 --steps 3 "$@" > gpurun_out/w.json 2>gpurun_out/w.err || { echo FAIL $lab; tail -5 gpurun_out/w.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/w.json'));r=d['roofline'];f=d['fill_launch'];print('$lab',d['value'],r['fill_ms_avg'],f['layout'],f['band_waves'])"
}
run p64 || exit 1
run ava --workload allvsall || exit 1
run p16 --pairs-per-gpu 16 || exit 1
run 16k --pairs-per-gpu 128 --length 16384 || exit 1
run p64 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "staged or random_pairs_batched or untracked" > gpurun_out/t4.log 2>&1 || { tail -20 gpurun_out/t4.log; exit 1; }
tail -1 gpurun_out/t4.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
