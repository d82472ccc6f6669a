#!/bin/bash
# Band widths with compact planes (d8) vs without planes, 16 x 30k global.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
run() {  # label env... -- bench args
  local lab=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --single-pair-steps 0 --steps 5 "$@" > gpurun_out/w.json 2>/dev/null || { echo FAIL $lab "${envs[@]}"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/w.json'));r=d['roofline'];print('$lab','${envs[*]}',d['value'],r['fill_ms_avg'])"
}
for W in 4 6 8 11 15; do run d8 GX_BAND_WAVES=$W -- || exit 1; done
for W in 8 15; do run nop GX_BAND_WAVES=$W -- --no-planes || exit 1; done
for W in 8 15; do run d8x32 GX_BAND_WAVES=$W -- --pairs-per-gpu 32 || exit 1; done
run d8_1k -- --pairs-per-gpu 1024 --length 1024 || exit 1
run d8_4k -- --pairs-per-gpu 256 --length 4096 || exit 1
run d8_16k -- --pairs-per-gpu 64 --length 16384 || exit 1
