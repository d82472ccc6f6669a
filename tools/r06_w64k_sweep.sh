# round 6: config 5 at 1024 x 64k, band width sweep (auto = the planner's choice) -> gpurun_out/w64k/
set -o pipefail
O=gpurun_out/w64k
rm -rf "$O" && mkdir -p "$O"
for W in auto 7 8 4; do
  if [ "$W" = auto ]; then unset GX_BAND_WAVES; else export GX_BAND_WAVES=$W; fi
  GX_LOG=debug timeout -k 10 400 python3 bench.py --length 65536 --pairs-per-gpu 1024 --single-pair-steps 0 --steps 2 --warmup 1 \
     --no-cpu-baseline --int32-steps 0 --no-plane-steps 0 --config-steps 0 --local-batch-steps 0 \
     > "$O/w$W.json" 2> "$O/w$W.err" || { echo FAIL $W; tail -5 "$O/w$W.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/w$W.json'));r=d['roofline'];print('$W',d['value'],d['ms_per_step'],d['fill_launch'],r.get('frac'),r.get('hbm',r).get('frac'))"
done
echo SWEEP_DONE
