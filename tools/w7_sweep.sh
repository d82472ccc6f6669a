#!/bin/bash
# GPU box: the twin fill at 7-wave bands (two workgroups per CU) against the default width, one bench line each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/w7
one() {   # name env -- bench args
  local name=$1 envv=$2; shift 2
  env $envv timeout -k 10 200 python3 bench.py "$@" --single-pair-steps 0 --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 \
      --config-steps 0 > gpurun_out/w7/$name.json 2> gpurun_out/w7/$name.err || { echo "FAIL $name"; tail -3 gpurun_out/w7/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/w7/$name.json'));p=d.get('parity',{});lb=d.get('local_batch',{});print('$name', d['value'], d['ms_per_step'], d['roofline'].get('fill_ms_avg'), d['fill_launch'].get('band_waves'), p.get('pairs_checked'), p.get('bit_exact'), 'local', lb.get('gcups'), lb.get('fill_launch',{}).get('band_waves'), flush=True)"
}
one head_def X=1 --steps 10
one head_w7 GX_BAND_WAVES=7 --steps 10
one avsa_def X=1 --workload allvsall --planes --steps 10 --local-batch-steps 0
one avsa_w7 GX_BAND_WAVES=7 --workload allvsall --planes --steps 10 --local-batch-steps 0
one k16_def X=1 --length 16384 --pairs-per-gpu 1024 --steps 3 --warmup 1 --local-batch-steps 0
one k16_w7 GX_BAND_WAVES=7 --length 16384 --pairs-per-gpu 1024 --steps 3 --warmup 1 --local-batch-steps 0
one k4_w7b GX_BAND_WAVES=7 --length 4096 --pairs-per-gpu 1024 --steps 20 --local-batch-steps 0
one k2_def X=1 --length 2048 --pairs-per-gpu 1024 --steps 20 --local-batch-steps 0
one k2_w7 GX_BAND_WAVES=7 --length 2048 --pairs-per-gpu 1024 --steps 20 --local-batch-steps 0
