#!/bin/bash
# Under band-major order: band widths, batch sizes, int32 planes, layouts for small batches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
run() {  # label env... -- bench args
  local lab=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --single-pair-steps 0 --no-plane-steps 0 --steps 3 "$@" > gpurun_out/r.json 2>gpurun_out/r.err || { echo FAIL $lab "${envs[@]}"; tail -5 gpurun_out/r.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r.json'));r=d['roofline'];print('$lab','${envs[*]}',d['value'],r['fill_ms_avg'],d['fill_launch'])"
}
for W in 4 6 11 15; do run p64 GX_BAND_WAVES=$W -- || exit 1; done
run p64nop -- --no-planes || exit 1
run p16_i32 GX_PLANES32=1 -- --pairs-per-gpu 16 || exit 1
run p48 -- --pairs-per-gpu 48 || exit 1
for L in 0 1; do run p4 GX_LAYOUT=$L -- --pairs-per-gpu 4 || exit 1; done
for L in 0 1; do run p8 GX_LAYOUT=$L -- --pairs-per-gpu 8 || exit 1; done
run 1k -- --pairs-per-gpu 1024 --length 1024 || exit 1
