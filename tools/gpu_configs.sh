# GPU box: one bench line per BASELINE config (2: Covid pair, 3: BRCA2 local,
# 4: all-vs-all, 5: synthetic length sweep) into gpurun_out/configs/.
#   gpurun -- 'bash tools/gpu_configs.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/configs
rm -rf "$O" && mkdir -p "$O"
run() {   # name, bench args
  timeout -k 10 300 python bench.py "${@:2}" --no-cpu-baseline > "$O/$1.json" 2> "$O/$1.err" || { echo BENCH_FAIL $1; tail -20 "$O/$1.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$O/$1.json'));r=d['roofline'];print('$1',d['value'],'GCUPS','fill_ms',r['fill_ms_avg'],'ms/step',d['ms_per_step'],'frac',r['frac'],'B/cell',r.get('algorithmic_bytes_per_cell'))"
}
run config2_covid --workload covid
run config3_brca2 --workload brca2
run config4_allvsall --workload allvsall
run config4_allvsall_planes --workload allvsall --planes
# config 5: 1024 pairs per length; one GPU holds all 1024 at 1k and 4k, and at
# 16k the 128 that each of 8 GPUs holds (compact planes, 103 GB); at 64k 12
# pairs (155 GB of planes; 1024 such pairs exceed any node's HBM)
run config5_L1024 --length 1024 --pairs-per-gpu 1024 --single-pair-steps 0
run config5_L4096 --length 4096 --pairs-per-gpu 1024 --single-pair-steps 0
run config5_L16384 --length 16384 --pairs-per-gpu 128 --single-pair-steps 0
run config5_L65536 --length 65536 --pairs-per-gpu 12 --single-pair-steps 0
echo CONFIGS_DONE
