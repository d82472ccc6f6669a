#!/bin/bash
# Fill time of the 64-pair batch: one step vs pipelined steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for S in 1 5 1 5; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --single-pair-steps 0 --no-plane-steps 0 --steps $S --warmup 1 > gpurun_out/s.json 2>gpurun_out/s.err || { echo FAIL; tail -5 gpurun_out/s.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/s.json'));r=d['roofline'];print('steps',$S,d['value'],d['ms_per_step'],r['fill_ms_avg'])"
done
