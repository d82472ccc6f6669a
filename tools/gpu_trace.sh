set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
GX_TRACE_FILE=gpurun_out/trace_p1.csv timeout -k 10 300 python bench.py --pairs-per-gpu 1 --steps 1 --warmup 1 --no-cpu-baseline --no-planes > gpurun_out/trace_p1.json 2>&1 || { echo FAIL1; exit 1; }
GX_TRACE_FILE=gpurun_out/trace_p8.csv timeout -k 10 300 python bench.py --pairs-per-gpu 8 --steps 1 --warmup 1 --no-cpu-baseline --no-planes > gpurun_out/trace_p8.json 2>&1 || { echo FAIL8; exit 1; }
echo OK
