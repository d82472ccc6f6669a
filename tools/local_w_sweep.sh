#!/bin/bash
# GPU box: the local twin's band width (GX_BAND_WAVES; workgroups per CU follow it), the bench's local_batch line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/lw
for W in 8 4 3; do
  GX_BAND_WAVES=$W timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --single-pair-steps 0 --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 \
      --config-steps 0 --no-verify > gpurun_out/lw/W$W.json 2> gpurun_out/lw/W$W.err || { echo "FAIL W$W"; tail -3 gpurun_out/lw/W$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/lw/W$W.json'));lb=d['local_batch'];print('W$W', lb['gcups'], lb['ms_per_step'], lb['fill_ms_avg'], lb['fill_launch'], lb.get('parity',{}).get('bit_exact'), flush=True)"
done
