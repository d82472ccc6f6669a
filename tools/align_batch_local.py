"""GPU: gx_align_batch (the drop-in batch call, steps returned to the host) on
bench.py's local batch (32 related 30k pairs, local SW), wall-clock per call
after one warm-up call, under the current environment; one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "genomics-rs_amd")]
import bench  # noqa: E402
import gxamd as gx  # noqa: E402

ctx = gx.Context(0)
pairs = [bench.related_pair(k, 30000) for k in range(bench.LOCAL_BATCH_PAIRS)]
sc = gx.Scores(*bench.SCORES)
gx.align_batch(pairs, sc, True, ctx=ctx, max_cell=False)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
t0 = time.perf_counter()
for _ in range(reps):
    out = gx.align_batch(pairs, sc, True, ctx=ctx, max_cell=False)
el = (time.perf_counter() - t0) / reps
cells = sum(len(a) * len(b) for a, b in pairs)
with open(os.path.join(ROOT, "tests", "golden", "synthetic_related_local_L30000.json")) as f:
    gold = {c["k"]: c for c in json.load(f)["cases"]}
ok = all((r.score, [r.matches, r.mismatches, r.gap_extensions, r.opening_gaps], r.n_steps) ==
         (gold[p]["score"], gold[p]["stats"], gold[p]["n_steps"]) for p, (_, r) in enumerate(out))
print(json.dumps({"call": "gx_align_batch", "pairs": len(pairs), "ms_per_call": round(el * 1e3, 2),
                  "gcups": round(cells / el / 1e9, 1), "fill_launch": ctx.fill_info(), "matches_oracle_digests": ok,
                  "env": {k: v for k, v in os.environ.items() if k.startswith("GX_")}}), flush=True)
ctx.close()
