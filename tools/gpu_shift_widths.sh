#!/bin/bash
# Band widths 8 vs 15 after the value shift (section 4.3).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
run() {  # label env... -- bench args
  local lab=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --single-pair-steps 0 --no-plane-steps 0 --steps 3 "$@" > gpurun_out/r.json 2>gpurun_out/r.err || { echo FAIL $lab "${envs[@]}"; tail -5 gpurun_out/r.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r.json'));r=d['roofline'];f=d['fill_launch'];print('$lab','${envs[*]}',d['value'],r['fill_ms_avg'],f['layout'],f['band_waves'])"
}
for W in 8 15; do run p16 GX_BAND_WAVES=$W -- --pairs-per-gpu 16 || exit 1; done
for W in 8 11 15; do run 16k GX_BAND_WAVES=$W -- --pairs-per-gpu 128 --length 16384 || exit 1; done
for W in 8 15; do run 4k GX_BAND_WAVES=$W -- --pairs-per-gpu 1024 --length 4096 || exit 1; done
for W in 8 15; do run 64k GX_BAND_WAVES=$W -- --pairs-per-gpu 12 --length 65536 || exit 1; done
for W in 8 11 15; do run p64 GX_BAND_WAVES=$W -- || exit 1; done
for W in 8 15; do run p32 GX_BAND_WAVES=$W -- --pairs-per-gpu 32 || exit 1; done
