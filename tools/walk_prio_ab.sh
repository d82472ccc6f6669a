#!/bin/bash
# GPU box: the walker wave's priority (default build vs gpurun_exp/noprio,
# built with -DGX_TB_NOPRIO) and the walk's own stream (GX_TB_OWN_STREAM=0:
# on the fill's stream), one bench line each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/wp
one() {   # name env... -- bench args
  local name=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 150 python3 bench.py "$@" --single-pair-steps 0 --no-cpu-baseline --int32-steps 0 \
      --no-plane-steps 0 --config-steps 0 > gpurun_out/wp/$name.json 2> gpurun_out/wp/$name.err \
      || { echo "FAIL $name"; tail -5 gpurun_out/wp/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/wp/$name.json'));p=d.get('parity',{});lb=d.get('local_batch',{});print('$name', d['value'], d['ms_per_step'], d['roofline'].get('fill_ms_avg'), p.get('pairs_checked'), p.get('bit_exact'), 'local', lb.get('gcups'), flush=True)"
}
NP=$GRAFT_REPO_ROOT/gpurun_exp/noprio/libgx_amd.so
for L in 1024 4096; do
  A="--length $L --pairs-per-gpu 1024 --steps 20 --local-batch-steps 0"
  one def$L X=1 -- $A
  one noprio$L GX_LIB=$NP -- $A
  one samestream$L GX_TB_OWN_STREAM=0 -- $A
done
one def_head X=1 -- --steps 10
one noprio_head GX_LIB=$NP -- --steps 10
one def_avsa X=1 -- --workload allvsall --planes --steps 10 --local-batch-steps 0
one noprio_avsa GX_LIB=$NP -- --workload allvsall --planes --steps 10 --local-batch-steps 0
