# GPU box: fill rate of the headline batch against its size (pairs per GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pairs_sweep; mkdir -p "$O"
for P in ${SWEEP:-80 40 56 24}; do
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --pairs-per-gpu $P --no-cpu-baseline --config-steps 0 \
      --int32-steps 0 --no-plane-steps 0 --single-pair-steps 0 --no-verify > "$O/p$P.json" 2> "$O/p$P.err" || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/p$P.json').read().strip().splitlines()[-1]); print($P, d['value'], d['ms_per_step'], d['fill_gcups_per_gpu'], d['fill_launch'])"
done
