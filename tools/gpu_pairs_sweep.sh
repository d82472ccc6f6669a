#!/bin/bash
# Pairs per GPU with compact planes (automatic band width), 30k global.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for P in 32 48 64; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --single-pair-steps 0 --steps 3 --pairs-per-gpu $P > gpurun_out/p.json 2>gpurun_out/p.err || { echo FAIL $P; tail -5 gpurun_out/p.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/p.json'));r=d['roofline'];print($P,d['value'],d['ms_per_step'],r['fill_ms_avg'])"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --single-pair-steps 0 --steps 3 --pairs-per-gpu 64 --no-planes > gpurun_out/p.json 2>gpurun_out/p.err && python3 -c "import json;d=json.load(open('gpurun_out/p.json'));r=d['roofline'];print('nop64',d['value'],d['ms_per_step'],r['fill_ms_avg'])"
