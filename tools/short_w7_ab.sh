#!/bin/bash
# GPU box: short batches, 8-wave bands with the walk on its own stream (default) against 7-wave bands
# (two workgroups per CU) with the walk on the fill's stream, one bench line each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sw7
for L in 2048 4096 8192; do
  for cfg in "def X=1" "w7same GX_BAND_WAVES=7 GX_TB_OWN_STREAM=0" "w8same GX_TB_OWN_STREAM=0"; do
    set -- $cfg; name=$1; shift
    env "$@" timeout -k 10 150 python3 bench.py --length $L --pairs-per-gpu 1024 --steps 20 --single-pair-steps 0 --no-cpu-baseline \
        --int32-steps 0 --no-plane-steps 0 --local-batch-steps 0 --config-steps 0 > gpurun_out/sw7/L${L}_$name.json 2> gpurun_out/sw7/L${L}_$name.err \
        || { echo "FAIL L$L $name"; tail -3 gpurun_out/sw7/L${L}_$name.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/sw7/L${L}_$name.json'));p=d.get('parity',{});print('L$L $name', d['value'], d['ms_per_step'], d['roofline'].get('fill_ms_avg'), d['fill_launch'].get('band_waves'), p.get('pairs_checked'), p.get('bit_exact'), flush=True)"
  done
done
