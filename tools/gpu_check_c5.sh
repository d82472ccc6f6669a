set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh r03n || exit $?
timeout -k 10 600 python -u bench.py --pairs-per-gpu 1024 --length 65536 --steps 2 --warmup 1 --no-cpu-baseline --config-steps 0 --int32-steps 0 --no-plane-steps 0 --single-pair-steps 0 > gpurun_out/r03n/c5_64k.json 2> gpurun_out/r03n/c5_64k.err
echo c5 rc=$?
