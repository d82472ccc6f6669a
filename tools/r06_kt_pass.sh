# round 6: a kernel trace whose last fill launches are the K timed passes (tools/pass_summary.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/kt06
rm -rf "$O" && mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O" -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 1 \
  --no-verify --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 --single-pair-steps 0 --config-steps 0 --local-batch-steps 0 \
  > "$O/kt_bench.json" 2> "$O/kt.err" || { echo KT_FAIL; tail -20 "$O/kt.err"; exit 1; }
echo KT_DONE
