set -o pipefail
mkdir -p gpurun_out/ov
one() { n=$1; shift; env $ENVV timeout -k 10 300 python3 bench.py "$@" --single-pair-steps 0 --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 --local-batch-steps 0 --config-steps 0 --no-verify > gpurun_out/ov/$n.json 2> gpurun_out/ov/$n.err || { echo FAIL $n; tail -3 gpurun_out/ov/$n.err; exit 1; }; python3 -c "import json;d=json.load(open('gpurun_out/ov/$n.json'));print('$n', d['value'], d['ms_per_step'], d['roofline'].get('fill_ms_avg'), d['fill_launch'])"; }
ENVV="" one k16_new --length 16384 --pairs-per-gpu 1024 --steps 3 --warmup 1
ENVV="GX_OVERLAP_A=50" one k16_old --length 16384 --pairs-per-gpu 1024 --steps 3 --warmup 1
ENVV="" one avsa_new --workload allvsall --planes --steps 5
ENVV="GX_OVERLAP_A=8" one avsa_old --workload allvsall --planes --steps 5
ENVV="" one loc_new --local --related --pairs-per-gpu 64 --steps 5
ENVV="GX_OVERLAP_A=12" one loc_old --local --related --pairs-per-gpu 64 --steps 5
