# GPU box: A/B of fill launch settings on the headline bench (one env setting per line)
#   gpurun -- 'bash tools/gpu_ab.sh "name:ENV=V ENV2=V2" ...'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; rm -rf $O; mkdir -p $O
for cfg in "$@"; do
  n=${cfg%%:*}; e=${cfg#*:}
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $O/$n.json 2> $O/$n.err || { echo BFAIL $n; tail -20 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));r=d['roofline'];print('$n',d['value'],d['ms_per_step'],r['fill_ms_avg'],d['fill_launch'],d.get('parity',{}).get('pairs_checked'))"
done
