#!/bin/bash
# GPU box: twin fill band width x workgroups per CU (GX_BAND_WAVES, GX_FILL_GRID = CUs x per-CU), one bench line each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/gw
one() {   # name env -- bench args
  local name=$1 envv=$2; shift 2
  env $envv timeout -k 10 200 python3 bench.py "$@" --single-pair-steps 0 --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 \
      --config-steps 0 --local-batch-steps 0 > gpurun_out/gw/$name.json 2> gpurun_out/gw/$name.err || { echo "FAIL $name"; tail -3 gpurun_out/gw/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/gw/$name.json'));p=d.get('parity',{});print('$name', d['value'], d['ms_per_step'], d['roofline'].get('fill_ms_avg'), d['fill_launch'].get('band_waves'), p.get('pairs_checked'), p.get('bit_exact'), flush=True)"
}
one head_def X=1 --steps 10
one head_w8g512 "GX_BAND_WAVES=8 GX_FILL_GRID=512" --steps 10
one head_w4g1024 "GX_BAND_WAVES=4 GX_FILL_GRID=1024" --steps 10
one head_w7g512 "GX_BAND_WAVES=7 GX_FILL_GRID=512" --steps 10
one avsa_def X=1 --workload allvsall --planes --steps 10
one avsa_w8g512 "GX_BAND_WAVES=8 GX_FILL_GRID=512" --workload allvsall --planes --steps 10
one k4_def X=1 --length 4096 --pairs-per-gpu 1024 --steps 20
one k4_w8g512 "GX_BAND_WAVES=8 GX_FILL_GRID=512 GX_TB_OWN_STREAM=0" --length 4096 --pairs-per-gpu 1024 --steps 20
