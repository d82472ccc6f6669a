"""GPU: BASELINE config 4 -- all-vs-all global NW of the 10 comparison_data
genomes (55 pairs i <= j, files in name order), through the Python mirror
(gxamd.all_vs_all, one batched launch) and the gx-align CLI (`all-vs-all`,
the reference compare writer's TSV layout), against oracle digests
(tests/golden/allvsall_digests.json, tests/golden/make_golden.py --allvsall).
Also the CLI `align` mode on a small pair: its stdout is the reference's
print_alignment_table text followed by the AlignedSequences Display."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import COMPARISON, FASTA, GOLDEN, ROOT

pytestmark = pytest.mark.gpu

CLI = os.path.join(ROOT, "genomics-rs_amd", "gx-align")


def _golden():
    with open(os.path.join(GOLDEN, "allvsall_digests.json")) as f:
        return json.load(f)


def _container(gx):
    cont = gx.SequenceContainer()
    for f in sorted(os.listdir(COMPARISON)):
        if f.endswith(".fasta"):
            cont.from_fasta(os.path.join(COMPARISON, f))
    return cont


def _digest(steps):
    h = hashlib.sha256()
    h.update(bytes(steps["choice"].astype(np.uint8)))
    h.update(steps["i"].astype("<u8").tobytes())
    h.update(steps["j"].astype("<u8").tobytes())
    return h.hexdigest()


def _golden_result(g):
    pairs = [(c["i"], c["j"]) for c in g["cases"]]
    recs = [[c["score"]] + c["stats"] + [c["n_steps"]] for c in g["cases"]]
    return pairs, recs


def test_all_vs_all_stats_match_oracle(gx, ctx):
    g = _golden()
    cont = _container(gx)
    assert [s.name for s in cont.sequences] == g["names"]
    res = gx.all_vs_all(cont, gx.Scores(*g["scores"]), is_local=False, with_self=True, ctx=ctx)
    pairs, recs = _golden_result(g)
    assert res["pairs"] == pairs
    assert res["records"] == recs


def test_all_vs_all_alignments_match_oracle(gx, ctx):
    """Full traceback vectors of all 55 pairs in one batched launch."""
    g = _golden()
    seqs = [s.sequence.encode() for s in _container(gx).sequences]
    out = gx.align_batch([(seqs[c["i"]], seqs[c["j"]]) for c in g["cases"]], gx.Scores(*g["scores"]), False,
                         ctx=ctx, max_cell=False)
    for c, (steps, r) in zip(g["cases"], out):
        assert r.score == c["score"], (c["i"], c["j"])
        assert len(steps) == c["n_steps"], (c["i"], c["j"])
        assert _digest(steps) == c["alignment_sha256"], (c["i"], c["j"])


def test_cli_all_vs_all_tsv(gx, tmp_path):
    g = _golden()
    cfg = tmp_path / "config.toml"
    cfg.write_text("[scores]\ns_match = %d\ns_mismatch = %d\ng = %d\nh = %d\n" % tuple(g["scores"]))
    tsv = tmp_path / "similarity_matrix.tsv"
    p = subprocess.run([CLI, "-c", str(cfg), "all-vs-all", "-d", COMPARISON, "-o", str(tsv)],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    pairs, recs = _golden_result(g)
    want = {"names": g["names"], "lengths": [0] * len(g["names"]), "pairs": pairs, "records": recs}
    assert tsv.read_text() == gx.similarity_tsv(want)
    assert p.stdout.startswith("Similarity TSV:\n" + gx.similarity_tsv(want, blank_header=True))
    assert "\nMatches TSV:\n" + gx.similarity_tsv(want, "matches", blank_header=True) in p.stdout


@pytest.mark.parametrize("mode", ["global", "local"])
def test_cli_align_small_prints_table_and_display(gx, oracle, tmp_path, mode):
    """gx-align align on test1.fasta: stdout == print_alignment_table text
    (display.rs:131-220, via retrace, algo.rs:438) + Display (display.rs:9-127),
    both rendered from the oracle's table and alignment."""
    from conftest import read_fasta_records
    path = os.path.join(FASTA, "test1.fasta")
    recs = read_fasta_records(path)
    a, b = recs[0][1], recs[1][1]
    assert len(a) < 200 and len(b) < 2000
    o = oracle.align(a, b, (1, -2, -1, -5), is_local=mode == "local", want_planes=True)
    aln = gx.AlignedSequences(gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode()),
                              [(gx.AlignmentChoice[c], i, j) for c, i, j in o.alignment()], o.score,
                              o.matches, o.mismatches, o.gap_extensions, o.opening_gaps)
    want = gx.format_alignment_table(aln, [o.planes[k] for k in range(3)], False) + str(aln)
    cfg = os.path.join(GOLDEN, "config.toml")
    p = subprocess.run([CLI, "-c", cfg, "align", "-a", mode, "-f", path], capture_output=True, text=True,
                       timeout=120, env=dict(os.environ, NO_COLOR="1"))
    assert p.returncode == 0, p.stderr
    assert p.stdout == want
