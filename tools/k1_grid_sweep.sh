#!/bin/bash
# GPU box: 1024 x 1k synthetic pairs (config 5 at 1k) by twin band width and
# fill grid (GX_BAND_WAVES, GX_FILL_GRID), one bench line each -> gpurun_out/sw/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sw
for cfg in "8 256" "8 512" "4 512" "4 768" "4 1024" "3 768" "3 1024" "7 512"; do
  set -- $cfg
  GX_BAND_WAVES=$1 GX_FILL_GRID=$2 timeout -k 10 120 python bench.py --length 1024 --pairs-per-gpu 1024 --single-pair-steps 0 --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 --local-batch-steps 0 --steps 10 --no-verify > gpurun_out/sw/w$1_g$2.json 2> gpurun_out/sw/w$1_g$2.err || { echo FAIL $cfg; tail -5 gpurun_out/sw/w$1_g$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sw/w$1_g$2.json'));print('W',$1,'grid',$2,d['value'],d['ms_per_step'],d['roofline'].get('fill_ms_avg'),d['fill_launch'])"
done
