#!/bin/bash
# Host phase times of the pipelined staged path (GX_LOG=debug) for short- and long-pair batches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for C in "1024 1024" "1024 4096" "64 30000"; do
  set -- $C
  GX_LOG=debug timeout -k 10 200 python bench.py --no-cpu-baseline --single-pair-steps 0 --no-plane-steps 0 --steps 10 --warmup 1 --pairs-per-gpu $1 --length $2 > gpurun_out/ph.json 2>gpurun_out/ph.err || { tail -5 gpurun_out/ph.err; exit 1; }
  grep "pipelined" gpurun_out/ph.err | tail -1 || true
  python3 -c "import json;d=json.load(open('gpurun_out/ph.json'));print('$1 x $2',d['value'],d['ms_per_step'],d['roofline']['fill_ms_avg'])"
done
