# GPU box: parity tests on the default library, then bench lines for each
# library given (GX_LIB) x each "P planes-flag" case.
#   gpurun -- 'bash tools/gpu_libsweep.sh "lib1 lib2" "8| 8|--no-planes 16|"'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/libsweep
rm -rf "$O" && mkdir -p "$O"
if [ -z "$NO_TESTS" ]; then
timeout -k 10 500 python -m pytest tests -m gpu -x -q > "$O/gpu_tests.log" 2>&1 || { echo TESTS_FAIL; tail -30 "$O/gpu_tests.log"; exit 1; }
tail -1 "$O/gpu_tests.log"
fi
for L in $1; do
  for C in $2; do
    P=${C%%|*}; F=${C#*|}
    GX_LIB=$L timeout -k 10 300 python bench.py --pairs-per-gpu $P --steps 3 --warmup 1 --no-cpu-baseline $F > "$O/b.json" 2>> "$O/err.log" || { echo BENCH_FAIL $L $C; tail -20 "$O/err.log"; exit 1; }
    python3 - "$L" "$P" "$F" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/libsweep/b.json").read().strip().splitlines()[-1]); r = d["roofline"]
print(sys.argv[1].split("/")[-1], "P", sys.argv[2], sys.argv[3] or "planes", "GCUPS", d["value"], "fill_ms", r["fill_ms_avg"],
      "fillGCUPS", d["fill_gcups_per_gpu"], "GB/s", r["achieved"], "tb_us", d["traceback_us_pair0"], "ms/step", d["ms_per_step"])
PY
  done
done
