#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/ -m gpu -k "staged or random_pairs_batched or untracked or allvsall" > gpurun_out/t5.log 2>&1 || { tail -20 gpurun_out/t5.log; exit 1; }
tail -1 gpurun_out/t5.log
bash tools/gpu_phase_1k.sh
