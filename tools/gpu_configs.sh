# GPU box: one bench line per BASELINE config (2: Covid pair, 3: BRCA2 local,
# 4: all-vs-all, 5: 1024 synthetic pairs at each length) into gpurun_out/configs/.
#   gpurun -- 'bash tools/gpu_configs.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/configs
rm -rf "$O" && mkdir -p "$O"
run() {   # name, bench args
  timeout -k 10 400 python bench.py "${@:2}" --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 \
      > "$O/$1.json" 2> "$O/$1.err" || { echo BENCH_FAIL $1; tail -20 "$O/$1.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$O/$1.json'))
if 'roofline' not in d: print('$1', d.get('predicted'), 'parity', d.get('parity', {}).get('pair_passes_checked')); sys.exit()
r=d['roofline'];h=r.get('hbm',r);print('$1',d['value'],'GCUPS','fill_ms',r['fill_ms_avg'],'ms/step',d['ms_per_step'],'frac',r['frac'],r['unit'],'hbm',h['frac'],'chunks',d['fill_launch'].get('chunks'),'parity',d.get('parity',{}).get('pairs_checked'))"
}
run config2_covid --workload covid
run config3_brca2 --workload brca2
run config4_allvsall --workload allvsall
run config4_allvsall_planes --workload allvsall --planes
# config 4 on 8 GPUs, predicted from this GPU: each simulated rank's LPT share
# timed alone (bench.py --simulate-world)
run config4_sim8 --workload allvsall --simulate-world 8
# config 5 as stated: 1024 pairs per length (batches beyond the free HBM run
# in chunks through the same buffers; 16k: 825 GB, 64k: 13 TB of compact planes)
run config5_L1024 --length 1024 --pairs-per-gpu 1024 --single-pair-steps 0 --steps 20
run config5_L4096 --length 4096 --pairs-per-gpu 1024 --single-pair-steps 0 --steps 20
run config5_L16384 --length 16384 --pairs-per-gpu 1024 --single-pair-steps 0 --steps 3 --warmup 1
run config5_L65536 --length 65536 --pairs-per-gpu 1024 --single-pair-steps 0 --steps 2 --warmup 1
echo CONFIGS_DONE
