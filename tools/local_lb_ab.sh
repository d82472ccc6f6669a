#!/bin/bash
# GPU box: the local twin at <= 128 VGPRs (variant gpurun_exp/lb4: launch bound of 4 waves a SIMD) against the
# in-tree build, 8-wave bands (one workgroup a CU) and 7-wave bands (two), the bench's local_batch line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/llb
V=$GRAFT_REPO_ROOT/gpurun_exp/lb4/libgx_amd.so
k=0
for cfg in "tree X=1" "tree7 GX_BAND_WAVES=7" "lb4 GX_LIB=$V" "lb4_7 GX_LIB=$V GX_BAND_WAVES=7"; do
  set -- $cfg; name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --single-pair-steps 0 --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 \
      --config-steps 0 > gpurun_out/llb/$name.json 2> gpurun_out/llb/$name.err || { echo "FAIL $name"; tail -3 gpurun_out/llb/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/llb/$name.json'));lb=d['local_batch'];print('$name', 'head', d['value'], 'local', lb['gcups'], lb['ms_per_step'], lb['fill_ms_avg'], lb['fill_launch'], lb.get('parity',{}).get('bit_exact'), flush=True)"
done
