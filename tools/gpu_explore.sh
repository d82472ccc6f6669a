set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -f gpurun_out/explore.jsonl
run() { # label, env..., args
  local label=$1; shift
  echo "== $label" >> gpurun_out/explore.err
  env "$@" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $EXTRA >> gpurun_out/explore.tmp 2>> gpurun_out/explore.err || { echo FAIL $label; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/explore.tmp').read().strip().splitlines()[-1]); r=d['roofline']; print('$label', d['config']['pairs_per_gpu'], 'fill_ms', r['fill_ms_avg'], 'fillGCUPS', d['fill_gcups_per_gpu'], 'step_ms', d['ms_per_step'])" >> gpurun_out/explore.txt
}
rm -f gpurun_out/explore.txt
for P in 1 8; do
  EXTRA="--pairs-per-gpu $P" run "planes_W4" GX_BAND_WAVES=4
  EXTRA="--pairs-per-gpu $P --no-planes" run "noplanes_W4" GX_BAND_WAVES=4
  EXTRA="--pairs-per-gpu $P" run "planes_W2" GX_BAND_WAVES=2
  EXTRA="--pairs-per-gpu $P" run "planes_W1" GX_BAND_WAVES=1
done
EXTRA="--pairs-per-gpu 8" run "planes_W4_grid256" GX_BAND_WAVES=4 GX_FILL_GRID=256
EXTRA="--pairs-per-gpu 8" run "planes_W4_grid512" GX_BAND_WAVES=4 GX_FILL_GRID=512
EXTRA="--pairs-per-gpu 16" run "planes_W4_p16" GX_BAND_WAVES=4
cat gpurun_out/explore.txt
