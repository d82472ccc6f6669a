#!/bin/bash
# GPU box: group A's pair count (GX_OVERLAP_A) for all-vs-all with planes (45 pairs), one bench line each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/aa
for A in 22 8 10 12 14 22; do
  GX_OVERLAP_A=$A timeout -k 10 150 python3 bench.py --workload allvsall --planes --steps 10 --single-pair-steps 0 --no-cpu-baseline --int32-steps 0 \
      --no-plane-steps 0 --config-steps 0 --local-batch-steps 0 > gpurun_out/aa/A$A.json 2> gpurun_out/aa/A$A.err || { echo "FAIL A$A"; tail -3 gpurun_out/aa/A$A.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/aa/A$A.json'));p=d.get('parity',{});print('A$A', d['value'], d['ms_per_step'], d['roofline'].get('fill_ms_avg'), d['fill_launch'].get('band_waves'), p.get('pairs_checked'), p.get('bit_exact'), flush=True)"
done
