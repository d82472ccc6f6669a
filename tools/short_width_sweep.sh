#!/bin/bash
# GPU box: band width (GX_BAND_WAVES) of the twin fill on short batches, one bench line each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sw
for L in 1024 4096; do
  for W in 8 7 4 3; do
    GX_BAND_WAVES=$W timeout -k 10 150 python3 bench.py --length $L --pairs-per-gpu 1024 --steps 20 --single-pair-steps 0 --no-cpu-baseline \
        --int32-steps 0 --no-plane-steps 0 --local-batch-steps 0 --config-steps 0 --no-verify > gpurun_out/sw/L${L}_W$W.json 2> gpurun_out/sw/L${L}_W$W.err \
        || { echo "FAIL L$L W$W"; tail -3 gpurun_out/sw/L${L}_W$W.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/sw/L${L}_W$W.json'));print('L$L W$W', d['value'], d['ms_per_step'], d['roofline'].get('fill_ms_avg'), d['fill_launch'], flush=True)"
  done
done
