# GPU box: BASELINE config 5 shapes -- synthetic random-DNA pairs of length L,
# P pairs per launch (HBM-resident, score planes + traceback), one bench line per L.
#   gpurun -- 'bash tools/gpu_sweep.sh "1024:1024 4096:256 16384:32 65536:2" [extra bench args]'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sweep
rm -rf "$O" && mkdir -p "$O"
SPEC=$1; shift
for LP in $SPEC; do
  L=${LP%%:*}; P=${LP##*:}
  echo "L=$L P=$P"
  timeout -k 10 300 python bench.py --length $L --pairs-per-gpu $P --steps 3 --warmup 1 --no-cpu-baseline \
      --single-pair-steps 0 "$@" > "$O/L$L.json" 2> "$O/L$L.err" || { echo SWEEP_FAIL $L; tail -20 "$O/L$L.err"; exit 1; }
  python -c "import json,sys;d=json.load(open('$O/L$L.json'));print(d['value'],d['roofline']['frac'],d['roofline']['fill_ms_avg'],d['ms_per_step'])"
done
