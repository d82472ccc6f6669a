#!/bin/bash
# GPU box: group A's pair count (GX_OVERLAP_A) of the headline's overlapped pipeline at 7-wave bands, one bench line each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/oa
for A in 40 36 44 48 40; do
  GX_OVERLAP_A=$A timeout -k 10 150 python3 bench.py --steps 10 --single-pair-steps 0 --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 \
      --config-steps 0 --local-batch-steps 0 --no-verify > gpurun_out/oa/A$A.json 2> gpurun_out/oa/A$A.err || { echo "FAIL A$A"; tail -3 gpurun_out/oa/A$A.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/oa/A$A.json'));print('A$A', d['value'], d['ms_per_step'], d['roofline'].get('fill_ms_avg'), d['fill_launch'], flush=True)"
done
