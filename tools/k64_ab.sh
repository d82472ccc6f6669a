#!/bin/bash
# GPU box: 1024 x 64k (config 5) under several library builds (GX_LIB), one bench line each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/k64ab
k=0
for lib in "$@"; do
  k=$((k + 1))
  if [ "$lib" != "-" ]; then export GX_LIB=$GRAFT_REPO_ROOT/$lib; else unset GX_LIB; fi
  timeout -k 10 300 python bench.py --length 65536 --pairs-per-gpu 1024 --single-pair-steps 0 --steps 2 --warmup 1 \
      --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 --local-batch-steps 0 --config-steps 0 --no-verify \
      > gpurun_out/k64ab/r$k.json 2> gpurun_out/k64ab/r$k.err || { echo "FAIL $lib"; tail -3 gpurun_out/k64ab/r$k.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/k64ab/r$k.json'));print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline'].get('fill_ms_avg'), flush=True)" "$lib"
done
