#!/bin/bash
# Kernel-time breakdown of the 1024 x 1k batch (BASELINE config 5, shortest length).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/kt1k
rm -rf "$O" && mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt -- python3 bench.py --length 1024 --pairs-per-gpu 1024 --steps 10 --warmup 2 --no-cpu-baseline --single-pair-steps 0 --no-plane-steps 0 > "$O/b.json" 2> "$O/err" || { tail -20 "$O/err"; exit 1; }
python3 - <<'PY'
import glob, sqlite3, json
db = glob.glob("gpurun_out/kt1k/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
for r in c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"):
    print(f"{r[0][:60]:60s} calls {r[1]:5d} total_ms {r[2]/1e6:9.3f} avg_us {r[3]/1e3:9.1f}")
d = json.loads(open("gpurun_out/kt1k/b.json").read().strip().splitlines()[-1])
print("bench", d["value"], d["ms_per_step"], d["roofline"]["fill_ms_avg"])
PY
