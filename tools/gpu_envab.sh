# GPU box: interleaved timing of environment settings over "P|flags" cases.
#   gpurun -- 'bash tools/gpu_envab.sh "GX_FILL_GRID=1024 GX_FILL_GRID=256" "8| 16|" 3'
# (settings joined by commas within one variant; flags joined by commas within one case)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/envab
rm -rf "$O" && mkdir -p "$O"
R=${3:-3}
for r in $(seq 1 "$R"); do
  for C in $2; do
    for E in $1; do
      P=${C%%|*}; F=${C#*|}
      env ${E//,/ } timeout -k 10 300 python bench.py --pairs-per-gpu $P --steps 4 --warmup 1 --no-cpu-baseline ${F//,/ } \
          > "$O/b.json" 2>> "$O/err.log" || { echo BENCH_FAIL $E $C; tail -20 "$O/err.log"; exit 1; }
      python3 - "$E" "$C" >> "$O/ab.tsv" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/envab/b.json").read().strip().splitlines()[-1])
print(sys.argv[1], sys.argv[2], d["roofline"]["fill_ms_avg"], d["ms_per_step"], sep="\t")
PY
    done
  done
done
python3 - <<'PY'
import collections, statistics
rows = [l.rstrip("\n").split("\t") for l in open("gpurun_out/envab/ab.tsv")]
g = collections.defaultdict(list)
for e, case, f, s in rows:
    g[(case, e)].append((float(f), float(s)))
for (case, e), v in sorted(g.items()):
    fs = [x for x, _ in v]; ss = [y for _, y in v]
    print(f"{case:8s} {e:40s} fill min {min(fs):7.3f} med {statistics.median(fs):7.3f}  step med {statistics.median(ss):7.3f}")
PY
