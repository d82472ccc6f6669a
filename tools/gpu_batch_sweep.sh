set -o pipefail
cd "$GRAFT_REPO_ROOT"
for C in "16 15" "16 11" "16 8" "12 15" "14 15" "18 15"; do
  set -- $C
  GX_LAYOUT=0 GX_BAND_WAVES=$2 timeout -k 10 200 python bench.py --pairs-per-gpu $1 --no-cpu-baseline --single-pair-steps 0 --steps 3 > gpurun_out/s.json 2>/dev/null || { echo FAIL $C; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/s.json'));r=d['roofline'];print('P',$1,'W',$2,d['value'],r['fill_ms_avg'],r['frac'])"
done
