set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
rm -f gpurun_out/sweep.jsonl gpurun_out/trace_p1.csv gpurun_out/trace_p8.csv
for P in ${SWEEP:-1 8}; do
  for PL in "" "--no-planes"; do
    timeout -k 10 300 python bench.py --pairs-per-gpu $P --steps 3 --warmup 1 --no-cpu-baseline $PL >> gpurun_out/sweep.jsonl 2>> gpurun_out/sweep.err || { echo BENCH_FAIL $P; exit 1; }
  done
done
GX_TRACE_FILE=gpurun_out/trace_p1.csv timeout -k 10 300 python bench.py --pairs-per-gpu 1 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2>&1
GX_TRACE_FILE=gpurun_out/trace_p8.csv timeout -k 10 300 python bench.py --pairs-per-gpu 8 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2>&1
python - <<'PY'
import json
for l in open("gpurun_out/sweep.jsonl"):
    d=json.loads(l); r=d["roofline"]
    print(d["config"]["pairs_per_gpu"], "planes" if r["achieved"] else "noplanes", "GCUPS", d["value"], "fill_ms", r["fill_ms_avg"], "fillGCUPS", d["fill_gcups_per_gpu"], "GB/s", r["achieved"], "tb_us", d["traceback_us_pair0"])
PY
