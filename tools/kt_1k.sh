set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/kt1k; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/kt -o kt --output-format csv -- python3 bench.py --pairs-per-gpu 1024 --length 1024 --steps 10 --warmup 2 --no-cpu-baseline --config-steps 0 --int32-steps 0 --no-plane-steps 0 --single-pair-steps 0 --no-verify > $O/b.json 2> $O/b.err
