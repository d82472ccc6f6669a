set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/prof_r03b; rm -rf $O; mkdir -p $O
GX_LOG=debug timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --config-steps 0 --int32-steps 0 --no-plane-steps 0 --single-pair-steps 0 > $O/bench.json 2> $O/bench.err
