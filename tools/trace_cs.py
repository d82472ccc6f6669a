"""GPU diagnostics: strip timelines (GX_TRACE_FILE) of the single-pair fills
(BASELINE configs 2 and 3) -> gpurun_out/trace_<name>.csv + summary.
    python tools/trace_cs.py [extra env k=v ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "genomics-rs_amd")]
for kv in sys.argv[1:]:
    k, v = kv.split("=", 1)
    os.environ[k] = v
import gxamd as gx  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
out = os.path.join(ROOT, "gpurun_out")
os.makedirs(out, exist_ok=True)
ctx = gx.Context(0)
import random  # noqa: E402
rng = random.Random(3)
syn = os.path.join(out, "syn64.fasta")
with open(syn, "w") as f:
    f.write(">a\n" + "".join(rng.choice("ACGT") for _ in range(64)) + "\n>b\n" +
            "".join(rng.choice("ACGT") for _ in range(30000)) + "\n")
cases = [("syn64", syn, None, False), ("covid", os.path.join(G, "comparison_data", "Covid_Wuhan.fasta"),
          os.path.join(G, "comparison_data", "Covid_USA-CA4.fasta"), False),
         ("brca2", os.path.join(G, "fasta", "Human-Mouse-BRCA2-cds.fasta"), None, True)]
tag = os.environ.get("GX_TRACE_TAG", "")
for name, f1, f2, local in cases:
    c = gx.SequenceContainer()
    c.from_fasta(f1)
    if f2:
        c.from_fasta(f2)
    c = gx.SequenceContainer(c.sequences[:2])
    os.environ.pop("GX_TRACE_FILE", None)
    for _ in range(2):   # warm-up: the table with its int32 score planes, then the traceback
        t, _ = gx.alignment_table(c, gx.Scores(), local, False, ctx=ctx, max_cell=False)
        gx.retrace(c, t, local)
    path = os.path.join(out, f"trace_{name}{tag}.csv")
    os.environ["GX_TRACE_FILE"] = path
    t, _ = gx.alignment_table(c, gx.Scores(), local, False, ctx=ctx, max_cell=False)
    os.environ.pop("GX_TRACE_FILE")
    al = gx.retrace(c, t, local)
    print(name, len(c.sequences[0].sequence), len(c.sequences[1].sequence), "fill_us", al.fill_us,
          "retrace_us", al.retrace_us, ctx.fill_info(), flush=True)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_summary.py"), path])
    import csv
    rows = list(csv.DictReader(open(path)))
    m = len(c.sequences[1].sequence)
    for k in sorted(set(k for k in (0, 1, len(rows) // 2, len(rows) - 1) if 0 <= k < len(rows))):
        r = rows[k]
        dur = (int(r["t_end"]) - int(r["t_first"])) / 100.0
        print(f"  strip {k}: {dur:.0f} us = {dur * 1000 / m:.1f} ns/col, clk/col {int(r['clk']) / m:.0f}, "
              f"core input waits {r['wait_in']}, core staging waits {r['wait_out']}, side waits {r['q7']}")
