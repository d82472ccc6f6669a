#!/bin/bash
# GPU box: one bench configuration under several library builds (GX_LIB):
#   tools/lib_sweep.sh "BENCH ARGS" lib1 lib2 ...   ("" = the in-tree build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ls
ARGS=$1; shift
k=0
for lib in "$@"; do
  k=$((k + 1))
  if [ -n "$lib" ]; then export GX_LIB=$lib; else unset GX_LIB; fi
  timeout -k 10 150 python bench.py $ARGS --single-pair-steps 0 --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 \
      --local-batch-steps 0 --config-steps 0 --no-verify > gpurun_out/ls/r$k.json 2> gpurun_out/ls/r$k.err \
      || { echo "FAIL [$lib]"; tail -5 gpurun_out/ls/r$k.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/ls/r$k.json'));print('[' + sys.argv[1] + ']', d['value'], d['ms_per_step'], d['roofline'].get('fill_ms_avg'), flush=True)" "$lib"
done
