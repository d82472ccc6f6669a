# round 6: local_batch, the opaque row-max (123 VGPRs) vs round 5's reassociable one (149), alternating; then 7-wave bands
set -o pipefail
mkdir -p gpurun_out
A="--steps 3 --warmup 1 --no-cpu-baseline --config-steps 0 --single-pair-steps 0 --int32-steps 0 --no-plane-steps 0 --no-verify"
for r in 1 2; do
  for V in new old; do
    if [ "$V" = old ]; then export GX_LIB=genomics-rs_amd/build_var/libgx_amd_lbold.so; else unset GX_LIB; fi
    timeout -k 10 300 python3 bench.py $A > gpurun_out/r06x_${V}_${r}.json 2> gpurun_out/r06x_${V}_${r}.err || { echo BENCH_FAIL; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r06x_${V}_${r}.json'));lb=d['local_batch'];print('$V',lb['gcups'],lb['fill_ms_avg'],lb['fill_launch'],lb['parity']['pairs_checked'])"
  done
done
unset GX_LIB
GX_LOG=debug GX_BAND_WAVES=7 GX_OVERLAP=1 timeout -k 10 300 python3 bench.py $A > gpurun_out/r06x_w7.json 2> gpurun_out/r06x_w7.err || { echo BENCH_FAIL; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r06x_w7.json'));lb=d['local_batch'];print('w7',lb['gcups'],lb['fill_ms_avg'],lb['fill_launch'])"
