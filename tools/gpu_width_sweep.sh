#!/bin/bash
# Band-width sweep for queued batches (more strips than one band per CU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
run() {  # label env... -- bench args
  local lab=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --single-pair-steps 0 --steps 3 "$@" > gpurun_out/w.json 2>/dev/null || { echo FAIL $lab "${envs[@]}"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/w.json'));r=d['roofline'];print('$lab','${envs[*]}',d['value'],r['fill_ms_avg'])"
}
for W in 8; do run ava GX_LAYOUT=0 GX_BAND_WAVES=$W -- --workload allvsall || exit 1; done
for W in 8 15; do run 30k16 GX_LAYOUT=0 GX_BAND_WAVES=$W -- --pairs-per-gpu 16 --length 30000 || exit 1; done
for W in 8 15; do run 30k20 GX_LAYOUT=0 GX_BAND_WAVES=$W -- --pairs-per-gpu 20 --length 30000 || exit 1; done
for W in 8 15; do run 16k GX_LAYOUT=0 GX_BAND_WAVES=$W -- --pairs-per-gpu 64 --length 16384 || exit 1; done
for W in 4 8 15; do run nop GX_LAYOUT=0 GX_BAND_WAVES=$W -- --no-planes --pairs-per-gpu 64 --length 30000 || exit 1; done
