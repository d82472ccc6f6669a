set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
for P in 1 2 4 8; do
  timeout -k 10 300 python bench.py --pairs-per-gpu $P --steps 3 --warmup 1 --no-cpu-baseline >> gpurun_out/sweep.jsonl 2>> gpurun_out/sweep.err || { echo BENCH_FAIL $P; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --pairs-per-gpu 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof1.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
