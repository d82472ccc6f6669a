#!/bin/bash
# GPU box: the headline batch (80 x 30k global, twin plane codes) under
# launch-shaping environment settings, one bench line each -> gpurun_out/hs/.
#   tools/headline_sweep.sh "GX_FILL_GRID=512" "GX_OVERLAP=0" ...   ("" = defaults)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/hs
k=0
for cfg in "$@"; do
  k=$((k + 1))
  env $cfg timeout -k 10 150 python bench.py --single-pair-steps 0 --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 \
      --local-batch-steps 0 --config-steps 0 --steps 10 --warmup 2 --no-verify > gpurun_out/hs/r$k.json 2> gpurun_out/hs/r$k.err \
      || { echo "FAIL [$cfg]"; tail -5 gpurun_out/hs/r$k.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/hs/r$k.json'));print('[' + sys.argv[1] + ']', d['value'], d['ms_per_step'], d['roofline'].get('fill_ms_avg'), d['fill_launch'], flush=True)" "$cfg"
done
