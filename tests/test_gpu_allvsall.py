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


@pytest.mark.parametrize("shards", [2, 4])
def test_cli_all_vs_all_sharded_on_one_gpu(gx, tmp_path, shards):
    """The CLI's multi-GPU path (one context and thread per shard, LPT split,
    results merged into one matrix) with `shards` logical shards mapped onto
    device 0 (GX_DEVICE_MAP): the TSV equals the oracle digests'."""
    g = _golden()
    cfg = tmp_path / "config.toml"
    cfg.write_text("[scores]\ns_match = %d\ns_mismatch = %d\ng = %d\nh = %d\n" % tuple(g["scores"]))
    tsv = tmp_path / "similarity_matrix.tsv"
    p = subprocess.run([CLI, "-c", str(cfg), "all-vs-all", "-d", COMPARISON, "-o", str(tsv), "-g", str(shards)],
                       capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, GX_DEVICE_MAP=",".join(["0"] * shards)))
    assert p.returncode == 0, p.stderr
    assert f"on {shards} shard(s)" in p.stderr
    assert sum(f"[INFO] shard {k}: device 0" in p.stderr for k in range(shards)) == shards
    pairs, recs = _golden_result(g)
    want = {"names": g["names"], "lengths": [0] * len(g["names"]), "pairs": pairs, "records": recs}
    assert tsv.read_text() == gx.similarity_tsv(want)


def _avsa_rank(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), GX_DEVICE_MAP="0")
    import torch.distributed as dist
    import gxamd as gx
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cont = _container(gx) if rank == 0 else gx.SequenceContainer()
    g = _golden()
    res = gx.all_vs_all(cont, gx.Scores(*g["scores"]), is_local=False, with_self=True, dist=dist, device="cpu")
    q.put((rank, res["pairs"], res["records"], res["names"]))
    dist.barrier()
    dist.destroy_process_group()


def test_all_vs_all_two_ranks_on_one_gpu():
    """gxamd.all_vs_all's distributed path with the real GPU aligner: two
    ranks (gloo for the broadcast / all-gather, both on device 0 through
    GX_DEVICE_MAP) each align their LPT share; every rank ends with the
    oracle's records for all 55 pairs."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_avsa_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = sorted(q.get(timeout=240) for _ in range(2))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    g = _golden()
    pairs, recs = _golden_result(g)
    for rank, prs, records, names in out:
        assert prs == pairs and records == recs and names == g["names"], rank


@pytest.mark.parametrize("twin", ["auto", "off"])
def test_all_vs_all_planes_match_oracle(gx, ctx, monkeypatch, twin):
    """The 55 comparison pairs at size through the staged path with compact
    score planes: every pair's I/D/S plane checksums (the weighted sums of
    make_golden.py) and alignment.  By default the batch takes the twin fill,
    whose twins here differ in shape; "off" pins the scalar fill."""
    if twin == "off":
        monkeypatch.setenv("GX_TWIN", "0")
    g = _golden()
    cont = _container(gx)
    seqs = [s.sequence.encode() for s in cont.sequences]
    pairs = [(seqs[c["i"]], seqs[c["j"]]) for c in g["cases"]]
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*g["scores"]), False, keep_planes=True, steps=1, plane_sums=True)
    info = ctx.fill_info()
    assert info["plane_bytes_per_cell"] == (1.5 if twin == "auto" else 3) and info["twin"] == (1 if twin == "auto" else 0), info
    sums = st.plane_sums()
    for p, c in enumerate(g["cases"]):
        assert [int(x) for x in sums[0, p]] == c["plane_sums"], (c["i"], c["j"])
        assert res[p].score == c["score"] and res[p].n_steps == c["n_steps"]
        assert _digest(st.steps(p)) == c["alignment_sha256"], (c["i"], c["j"])


@pytest.mark.parametrize("nctx", [2, 4])
def test_align_batch_multi_contexts_on_one_gpu(gx, nctx, monkeypatch):
    """gx_align_batch_multi (the C ABI's multi-GPU batch: LPT shares, one host
    thread and context per device) with `nctx` contexts mapped onto device 0
    (GX_DEVICE_MAP=0,0,..): all 55 comparison pairs' scores, statistics and
    alignment digests against the oracle's."""
    monkeypatch.setenv("GX_DEVICE_MAP", ",".join(["0"] * nctx))
    g = _golden()
    seqs = [s.sequence.encode() for s in _container(gx).sequences]
    ctxs = [gx.Context(gx.device_for_rank(k)) for k in range(nctx)]
    try:
        out = gx.align_batch_multi([(seqs[c["i"]], seqs[c["j"]]) for c in g["cases"]], gx.Scores(*g["scores"]),
                                   False, ctxs, max_cell=False)
    finally:
        for c in ctxs:
            c.close()
    for c, (steps, r) in zip(g["cases"], out):
        assert [r.score, r.matches, r.mismatches, r.gap_extensions, r.opening_gaps, r.n_steps] == \
               [c["score"]] + c["stats"] + [c["n_steps"]], (c["i"], c["j"])
        assert _digest(steps) == c["alignment_sha256"], (c["i"], c["j"])
