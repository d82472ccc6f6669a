#!/bin/bash
# Larger headline batches (HBM sizing): 64 vs 72 vs 80 pairs of 30k.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for P in 64 72 80 64 80; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --single-pair-steps 0 --no-plane-steps 0 --steps 3 --pairs-per-gpu $P > gpurun_out/p.json 2>gpurun_out/p.err || { echo FAIL $P; tail -5 gpurun_out/p.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/p.json'));r=d['roofline'];f=d['fill_launch'];print($P,d['value'],d['ms_per_step'],r['fill_ms_avg'],f['band_waves'])"
done
python3 -c "import torch;f,t=torch.cuda.mem_get_info();print('HBM total bytes',t)"
