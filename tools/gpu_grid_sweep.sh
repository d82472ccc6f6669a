#!/bin/bash
# Band width x persistent grid (several bands per CU) for the compact-plane batch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
run() {  # label env... -- bench args
  local lab=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --single-pair-steps 0 --no-plane-steps 0 --steps 3 "$@" > gpurun_out/g.json 2>gpurun_out/g.err || { echo FAIL $lab "${envs[@]}"; tail -5 gpurun_out/g.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/g.json'));r=d['roofline'];print('$lab','${envs[*]}',d['value'],r['fill_ms_avg'])"
}
run p64 GX_BAND_WAVES=8 GX_FILL_GRID=256 -- || exit 1
run p64 GX_BAND_WAVES=4 GX_FILL_GRID=512 -- || exit 1
run p64 GX_BAND_WAVES=3 GX_FILL_GRID=768 -- || exit 1
run p64 GX_BAND_WAVES=6 GX_FILL_GRID=512 -- || exit 1
run p64 GX_BAND_WAVES=4 GX_FILL_GRID=256 -- || exit 1
run p64 GX_BAND_WAVES=3 GX_FILL_GRID=512 -- || exit 1
