#!/bin/bash
# GPU box: one bench line per workload on the in-tree build (headline, 1024 x 1k / 4k / 64k, all-vs-all with planes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ql
one() {
  local name=$1; shift
  timeout -k 10 300 python3 bench.py "$@" --single-pair-steps 0 --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 \
      --config-steps 0 > gpurun_out/ql/$name.json 2> gpurun_out/ql/$name.err || { echo "FAIL $name"; tail -3 gpurun_out/ql/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ql/$name.json'));p=d.get('parity',{});lb=d.get('local_batch',{});print('$name', d['value'], d['ms_per_step'], d['roofline'].get('fill_ms_avg'), p.get('pairs_checked'), p.get('bit_exact'), 'local', lb.get('gcups'), flush=True)"
}
one head --steps 10
one k1 --length 1024 --pairs-per-gpu 1024 --steps 20 --local-batch-steps 0
one k4 --length 4096 --pairs-per-gpu 1024 --steps 20 --local-batch-steps 0
one avsa --workload allvsall --planes --steps 10 --local-batch-steps 0
one k64 --length 65536 --pairs-per-gpu 1024 --steps 2 --warmup 1 --local-batch-steps 0
