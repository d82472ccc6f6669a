#!/bin/bash
# Band queue order A/B (GX_BAND_ORDER=pair vs the default band-major order) + parity.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/t3.log 2>&1 || { tail -30 gpurun_out/t3.log; exit 1; }
tail -1 gpurun_out/t3.log
run() {  # label env... -- bench args
  local lab=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --single-pair-steps 0 --no-plane-steps 0 --steps 3 "$@" > gpurun_out/o.json 2>gpurun_out/o.err || { echo FAIL $lab "${envs[@]}"; tail -5 gpurun_out/o.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/o.json'));r=d['roofline'];print('$lab','${envs[*]}',d['value'],r['fill_ms_avg'])"
}
for O in pair round; do run p64 GX_BAND_ORDER=$O -- || exit 1; done
for O in pair round; do run p16 GX_BAND_ORDER=$O -- --pairs-per-gpu 16 || exit 1; done
for O in pair round; do run ava GX_BAND_ORDER=$O -- --workload allvsall || exit 1; done
for O in pair round; do run 4k GX_BAND_ORDER=$O -- --pairs-per-gpu 1024 --length 4096 || exit 1; done
for O in pair round; do run 16k GX_BAND_ORDER=$O -- --pairs-per-gpu 128 --length 16384 || exit 1; done
for O in pair round; do run p64 GX_BAND_ORDER=$O -- || exit 1; done
