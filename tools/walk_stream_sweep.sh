#!/bin/bash
# GPU box: short batches (config 5) with the walk on the fill's stream (default)
# and on a stream of its own (GX_WALK_STREAM=1), alternating, 3 runs each.
set -o pipefail
mkdir -p gpurun_out/ws
run() {   # name L P env...
  n=$1; L=$2; P=$3; shift 3
  env "$@" timeout -k 10 150 python3 bench.py --length $L --pairs-per-gpu $P --steps 10 --single-pair-steps 0 --no-cpu-baseline \
      --int32-steps 0 --no-plane-steps 0 --local-batch-steps 0 --config-steps 0 --no-verify > gpurun_out/ws/$n.json \
      2> gpurun_out/ws/$n.err || { echo FAIL $n; tail -3 gpurun_out/ws/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ws/$n.json'));print('$n', d['value'], d['ms_per_step'], d['roofline'].get('fill_ms_avg'), flush=True)"
}
for r in 1 2 3; do
  run k1_base_$r 1024 1024 GX_WALK_STREAM=0 && run k1_ws_$r 1024 1024 GX_WALK_STREAM=1 || exit 1
done
for r in 1 2; do
  run k4_base_$r 4096 1024 GX_WALK_STREAM=0 && run k4_ws_$r 4096 1024 GX_WALK_STREAM=1 || exit 1
  run k16_base_$r 16384 128 GX_WALK_STREAM=0 && run k16_ws_$r 16384 128 GX_WALK_STREAM=1 || exit 1
done
