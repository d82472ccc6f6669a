# GPU box: the same bench lines under fill layout 0 (anti-diagonal) and 1
# (column step), for picking the host's layout heuristic.
#   gpurun -- 'bash tools/gpu_layouts.sh "<bench args>|<bench args>|..."'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/layouts
rm -rf "$O" && mkdir -p "$O"
IFS='|' read -ra CASES <<< "$1"
k=0
for C in "${CASES[@]}"; do
  for LAY in 0 1; do
    k=$((k+1))
    GX_LAYOUT=$LAY timeout -k 10 300 python bench.py $C --no-cpu-baseline --single-pair-steps 0 --steps 3 --warmup 2 \
        > "$O/b$k.json" 2> "$O/b$k.err" || { echo BENCH_FAIL "$C" $LAY; tail -20 "$O/b$k.err"; exit 1; }
    python3 - "$O/b$k.json" "$C" $LAY <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d["roofline"]
print(f"layout {sys.argv[3]} [{sys.argv[2]}] GCUPS {d['value']} fill_ms {r['fill_ms_avg']} ms/step {d['ms_per_step']} "
      f"frac {r['frac']}")
PY
  done
done
