"""GPU parity at the sizes the product runs: the score matrix and the
alignment of BASELINE configs 2, 3 and 5 and of the bench's own launch,
against oracle digests (tests/golden/make_golden.py --large / --synthetic).

The score planes of a 30k x 30k table (9e8 cells, 2.7 GB compact or 10.8 GB
int32 on the device, 21.6 GB as the reference's int64 planes) are compared
through weighted checksums: for each of the I, D, S planes the sum over the
interior cells of value * (1 + i*0x9E3779B1 + j*0x85EBCA77) mod 2^64, which
oracle_align_lean (oracle/gx_oracle.c) folds while it fills.  The device
computes them from the stored planes with the exports' decode
(gx_table_plane_sums / GX_STAGED_PLANE_SUMS); test_plane_sums_host_fold pins
that kernel against a host fold of exported rows.  Alignments are compared
by the sha256 of the step vector, plus score, statistics and length.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import COMPARISON, CONFIG_SCORES, FASTA, GOLDEN, read_fasta_records

pytestmark = pytest.mark.gpu

W_I, W_J = 0x9E3779B1, 0x85EBCA77


def _digest(steps):
    h = hashlib.sha256()
    h.update(bytes(steps["choice"].astype(np.uint8)))
    h.update(steps["i"].astype("<u8").tobytes())
    h.update(steps["j"].astype("<u8").tobytes())
    return h.hexdigest()


def _synth(L):
    with open(os.path.join(GOLDEN, f"synthetic_L{L}.json")) as f:
        return json.load(f)["cases"]


def _synth_pair(k, L):
    import sys
    sys.path.insert(0, GOLDEN)
    import make_golden
    return make_golden.synth_pair(k, L)


def _large_inputs():
    brca = read_fasta_records(os.path.join(FASTA, "Human-Mouse-BRCA2-cds.fasta"))
    wuhan = read_fasta_records(os.path.join(COMPARISON, "Covid_Wuhan.fasta"))[0][1]
    usa = read_fasta_records(os.path.join(COMPARISON, "Covid_USA-CA4.fasta"))[0][1]
    return {"brca2": (brca[0][1], brca[1][1]), "covid_wuhan_usa": (wuhan, usa)}


def _large_cases():
    with open(os.path.join(GOLDEN, "large_digests.json")) as f:
        return json.load(f)["cases"]


def _check_result(r, steps, c, tag):
    assert r.score == c["score"], tag
    assert [r.matches, r.mismatches, r.gap_extensions, r.opening_gaps] == c["stats"], tag
    assert r.n_steps == c["n_steps"], tag
    if steps is not None:
        assert len(steps) == c["n_steps"] and _digest(steps) == c["alignment_sha256"], tag


@pytest.mark.parametrize("layout", ["auto", "lay0", "cs1", "cs2", "skew"])
@pytest.mark.parametrize("tracked", [True, False], ids=["tracked", "untracked"])
@pytest.mark.parametrize("case", range(4), ids=[c["name"] for c in _large_cases()])
def test_large_table_plane_sums(gx, ctx, monkeypatch, case, tracked, layout):
    """BASELINE configs 2 (Covid 29,903 x 29,882) and 3 (BRCA2 11,382 x
    10,346), both modes: the whole score matrix (three planes) of
    alignment_table equals the oracle's, then retrace's alignment.  auto =
    the single-pair layout (column step, int32 planes); lay0 = the
    anti-diagonal layout, whose untracked tables keep compact byte planes;
    cs1 / cs2 = the column step as one wave per strip / as the split core +
    side waves (gx_cs2.hip, untracked fills only); skew = layout 3
    (gx_skew.hip; tracked fills carry the first maximum and the LCS values in
    the side waves)."""
    if layout == "lay0":
        monkeypatch.setenv("GX_LAYOUT", "0")
    if layout in ("cs1", "cs2"):
        monkeypatch.setenv("GX_LAYOUT", "1")
        monkeypatch.setenv("GX_CS2", "1" if layout == "cs2" else "0")
    if layout == "skew":
        monkeypatch.setenv("GX_LAYOUT", "3")
    c = _large_cases()[case]
    a, b = _large_inputs()[c["name"].split("/")[0]]
    cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
    table, mam = gx.alignment_table(cont, gx.Scores(*c["scores"]), c["is_local"], False, ctx=ctx, max_cell=tracked)
    info = ctx.fill_info()
    if layout == "lay0":
        assert info["layout"] == 0 and info["plane_bytes_per_cell"] == (12 if tracked else 3), info
    if layout in ("cs1", "cs2"):
        assert info["layout"] == (2 if layout == "cs2" and not tracked else 1), info
    if layout == "skew":
        assert info["layout"] == 3, info   # (tracked fills too, since round 5)
    assert table.plane_sums() == [int(x) for x in c["plane_sums"]], (c["name"], info)
    if tracked:
        assert mam == c["matches_at_max"] and table.info()["max_cell"] == tuple(c["max_cell"])
    aln = gx.retrace(cont, table, c["is_local"])
    assert aln.score == c["score"] and list(aln.start) == c["start"]
    assert [aln.matches, aln.mismatches, aln.gap_extensions, aln.opening_gaps] == c["stats"]
    assert len(aln.alignment) == c["n_steps"] and _digest(aln._steps) == c["alignment_sha256"]


@pytest.mark.parametrize("case", range(4), ids=[c["name"] for c in _large_cases()])
def test_large_tracked_lcs_rows(gx, ctx, oracle, case):
    """The drop-in alignment_table with max_cell / matches_at_max and the
    full-cell export flag at configs 2 and 3 (round 6): the default launch
    puts them on layout 3, whose max_matches are LCS bit rows beside the fill
    (gx_lcs.h).  matches_at_max and max_cell against large_digests.json, the
    score matrix against its checksums, and max_matches of row slices (first
    rows, the middle, the last rows, every column) against the LCS recurrence
    (algo.rs:250-256) restated row by row in numpy (oracle.lcs_rows)."""
    c = _large_cases()[case]
    a, b = _large_inputs()[c["name"].split("/")[0]]
    n, m = len(a), len(b)
    cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
    table, mam = gx.alignment_table(cont, gx.Scores(*c["scores"]), c["is_local"], False, ctx=ctx, max_cell=True,
                                    flags=gx.GX_TABLE_MATCHES)
    info = ctx.fill_info()
    assert info["layout"] == 3, info
    assert mam == c["matches_at_max"] and table.info()["max_cell"] == tuple(c["max_cell"])
    assert table.plane_sums() == [int(x) for x in c["plane_sums"]]
    slices = [(0, 40), (n // 2 - 20, 41), (n - 39, 40)]
    want = set()
    for r0, k in slices:
        want.update(range(r0, r0 + k))
    want.add(c["max_cell"][0])
    L = oracle.lcs_rows(a, b, want)
    for r0, k in slices:
        got = table.rows(3, r0, k)
        for r in range(k):
            assert np.array_equal(got[r], L[r0 + r]), (c["name"], r0 + r)
    assert L[c["max_cell"][0]][c["max_cell"][1]] == mam
    aln = gx.retrace(cont, table, c["is_local"])
    assert aln.score == c["score"] and len(aln.alignment) == c["n_steps"]
    assert _digest(aln._steps) == c["alignment_sha256"]


def _host_fold(table, n, m, chunk=1024):
    """Weighted plane sums folded on the host from exported int64 rows."""
    sums = [np.uint64(0)] * 3
    jw = np.arange(m + 1, dtype=np.uint64) * np.uint64(W_J)
    for r0 in range(1, n + 1, chunk):
        rows = min(chunk, n + 1 - r0)
        iw = np.uint64(1) + np.arange(r0, r0 + rows, dtype=np.uint64)[:, None] * np.uint64(W_I)
        w = (iw + jw[None, :])[:, 1:]
        for k in range(3):
            v = table.rows(k, r0, rows)[:, 1:].view(np.uint64)
            with np.errstate(over="ignore"):   # the checksum wraps mod 2^64 by design
                sums[k] = sums[k] + np.sum(v * w, dtype=np.uint64)
    return [int(x) for x in sums]


@pytest.mark.parametrize("variant", ["local_compact", "global_compact", "global_int32"])
def test_plane_sums_host_fold(gx, ctx, monkeypatch, variant):
    """The device checksum kernel against a host fold of the exported rows
    (gx_table_export_rows, row-chunked), and both against the oracle's
    plane_sums for BASELINE config 3's pair (1.2e8 cells per plane)."""
    is_local = variant.startswith("local")
    if variant.endswith("compact"):
        monkeypatch.setenv("GX_LAYOUT", "0")
    c = [x for x in _large_cases() if x["name"] == f"brca2/{'local' if is_local else 'global'}"][0]
    a, b = _large_inputs()["brca2"]
    cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
    table, _ = gx.alignment_table(cont, gx.Scores(*c["scores"]), is_local, False, ctx=ctx,
                                  max_cell=variant.endswith("int32"))
    assert ctx.fill_info()["plane_bytes_per_cell"] == (12 if variant.endswith("int32") else 3)
    want = [int(x) for x in c["plane_sums"]]
    assert table.plane_sums() == want
    assert _host_fold(table, len(a), len(b)) == want
    # a row slice also carries the analytic boundary column (algo.rs:195-220)
    r = table.rows(1, 5, 3)
    g, h = c["scores"][2], c["scores"][3]
    assert list(r[:, 0]) == [h + i * g for i in range(5, 8)]
    table.free()


def _staged_check(gx, ctx, pairs, cases, steps=2, **kw):
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, fill_ms = st.run(gx.Scores(*CONFIG_SCORES), False, keep_planes=True, steps=steps, plane_sums=True, **kw)
    assert fill_ms > 0
    sums = st.plane_sums()
    assert sums.shape == (steps, len(pairs), 3)
    passes = st.pass_results()
    assert len(passes) == steps
    for p, c in enumerate(cases):
        want = [int(x) for x in c["plane_sums"]]
        for k in range(steps):   # every pass of the pipelined run, not just the last
            assert [int(x) for x in sums[k, p]] == want, (p, c["k"], "pass", k)
            _check_result(passes[k][p], None, c, (p, c["k"], "pass", k))
        _check_result(res[p], st.steps(p), c, (p, c["k"]))
    return ctx.fill_info()


LAUNCHES = {
    # the scalar fill's headline instantiation: 15-strip bands, compact byte planes, band-major queue;
    # a grid of 8 workgroups makes the 64 bands run in 8 rounds with HBM hand-offs between them
    "w15_grid8": ({"GX_TWIN": "0", "GX_BAND_WAVES": "15", "GX_FILL_GRID": "8"}, (0, 15, 3)),
    # the bench's headline launch: the twin fill at 8-strip bands, 12-bit twin plane codes
    "twin_w8_grid8": ({"GX_TWIN": "1", "GX_BAND_WAVES": "8", "GX_FILL_GRID": "8"}, (0, 8, 1.5)),
    # the twin fill with per-pair byte planes (the table format)
    "twin_w8_bytes": ({"GX_TWIN": "1", "GX_BAND_WAVES": "8", "GX_PLANES_W16": "0"}, (0, 8, 3)),
    "auto": ({}, None),
    "int32_planes": ({"GX_PLANES32": "1"}, (0, None, 12)),
    # every buffer the pool hands out is poisoned on its new user's stream: a pass that read the previous pass's data would fail
    "w15_poison": ({"GX_BAND_WAVES": "15", "GX_FILL_GRID": "16", "GX_POOL_POISON": "1"}, (0, 15, None)),
    "twin_poison": ({"GX_TWIN": "1", "GX_BAND_WAVES": "15", "GX_FILL_GRID": "16", "GX_POOL_POISON": "1"}, (0, 15, 1.5)),
}


@pytest.mark.parametrize("launch", sorted(LAUNCHES))
def test_bench_launch_synthetic_30k(gx, ctx, monkeypatch, launch):
    """The bench's own staged, untracked, pipelined launch on four of its
    synthetic 30,000 x 30,000 pairs (pairs 0-3 of bench.py rank 0), three
    passes: every pass's score matrix, and the last pass's alignments, equal
    the oracle's."""
    env, expect = LAUNCHES[launch]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cases = _synth(30000)[:4]
    pairs = [_synth_pair(c["k"], 30000) for c in cases]
    info = _staged_check(gx, ctx, pairs, cases, steps=3)
    if expect:
        lay, W, pb = expect
        assert info["layout"] == lay and (pb is None or info["plane_bytes_per_cell"] == pb), info
        if W:
            assert info["band_waves"] == W, info


@pytest.mark.parametrize("npairs,env", [(20, {"GX_TWIN": "1"}), (80, {})], ids=["20_twin", "80_default"])
def test_overlapped_bench_launch_30k(gx, ctx, monkeypatch, npairs, env):
    """The launch the headline times: synthetic 30k pairs through the
    overlapped two-group pipeline (gx_api_batch.cpp batch_core_overlap), three
    passes -- 20 pairs with the twin fill forced (group A's 4 pairs alone
    would not fill the grid and take the scalar fill, so the pipeline would
    not run by default) and the bench's whole 80-pair batch under the default
    environment.  Every pass's plane checksums and results, the last pass's
    alignments, against the oracle digests; groups == 2."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cases = _synth(30000)[:npairs]
    pairs = [_synth_pair(c["k"], 30000) for c in cases]
    info = _staged_check(gx, ctx, pairs, cases, steps=3)
    assert info["groups"] == 2 and info["twin"] == 1 and info["plane_bytes_per_cell"] == 1.5, info


@pytest.mark.parametrize("poison", [True, False], ids=["poison", "plain"])
def test_overlapped_alternating_sets(gx, ctx, monkeypatch, poison):
    """The headline's overlapped two-group pipeline (groups == 2, twin plane
    codes) over two different sets of 20 synthetic 30k pairs that alternate
    pass by pass (GX_STAGED_ALTERNATE: pass k runs set k % 2), so that every
    device buffer a pass takes from the pool last held the other set's planes
    and records: a walk that read a later pass's planes, or a fill that
    overwrote planes a walk still reads (the wait of group B's next fill on
    the previous walk, gx_api_batch.cpp batch_core_overlap), gives wrong results
    here, where repeating one set would hide it.  With GX_POOL_POISON every
    buffer is also filled with garbage on its new user's stream before use.
    Every pass's plane checksums and results, and each set's last
    alignments, against the oracle digests."""
    monkeypatch.setenv("GX_TWIN", "1")
    if poison:
        monkeypatch.setenv("GX_POOL_POISON", "1")
    cases = _synth(30000)[:40]
    pairs = [_synth_pair(c["k"], 30000) for c in cases]
    H = len(pairs) // 2
    steps = 4
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, fill_ms = st.run(gx.Scores(*CONFIG_SCORES), False, keep_planes=True, steps=steps, plane_sums=True,
                          alternate=True)
    info = ctx.fill_info()
    assert info["groups"] == 2 and info["twin"] == 1 and info["plane_bytes_per_cell"] == 1.5, info
    assert fill_ms > 0
    sums = st.plane_sums()
    passes = st.pass_results()
    assert sums.shape == (steps, len(pairs), 3) and len(passes) == steps
    for k in range(steps):
        for q in range(H):
            p = (k % 2) * H + q
            c = cases[p]
            assert [int(x) for x in sums[k, p]] == [int(x) for x in c["plane_sums"]], (p, "pass", k)
            _check_result(passes[k][p], None, c, (p, "pass", k))
            other = passes[k][(1 - k % 2) * H + q]
            assert other.score == 0 and other.n_steps == 0, (p, "pass", k, "the other set's row is empty")
    for p, c in enumerate(cases):   # each set's last pass
        _check_result(res[p], st.steps(p), c, (p, "last"))


SHORT_PIPELINES = {
    # 2 x 512 pairs of 1k: the walk on its own stream beside the next passes' fills (fill buffers held
    # until the walk is collected, gx_api_batch.cpp trace_dev)
    "1k_walk_stream": (1024, 512, lambda W: W != 7),
    # the same on a 64-workgroup fill grid: most CUs stay free, so a walk that did not wait for its
    # fill (or read a buffer handed back too early) would run while the fill still writes
    "1k_walk_stream_grid64": (1024, 512, lambda W: W != 7),
    # 2 x 32 pairs of 4k on the twin fill at 7-wave bands (forced: 32 pairs alone take the scalar
    # fill), two workgroups a CU as at 1024 x 4k, so the walk stays on the fill's stream
    "4k_w7_fill_stream": (4096, 32, lambda W: W == 7),
}


@pytest.mark.parametrize("poison", [False, True], ids=["plain", "poison"])
@pytest.mark.parametrize("shape", sorted(SHORT_PIPELINES))
def test_short_pipeline_alternating_sets(gx, ctx, monkeypatch, shape, poison):
    """The three-slot short-batch pipeline (gx_api_batch.cpp, global
    untracked batches too short for the overlapped two-group launch: three
    passes in flight, the walk on its own stream when it fits) over two
    different sets of synthetic pairs that alternate pass by pass
    (GX_STAGED_ALTERNATE), five passes: every buffer a pass takes from the
    pool -- planes, records, descriptors, pinned staging -- last held the
    other set's data, so a walk that ran before its fill finished (no wait on
    the slot's fdone event), or a fill buffer returned to the pool while its
    walk still reads it, gives wrong results here (with GX_POOL_POISON the
    buffers are also filled with garbage on their new user's stream).  Every
    pass's plane checksums and results, and each set's last alignments,
    against the oracle digests (tests/golden/synthetic_L{1024,4096}.json)."""
    L, H, w_ok = SHORT_PIPELINES[shape]
    if shape.endswith("grid64"):
        monkeypatch.setenv("GX_FILL_GRID", "64")
    if L == 4096:
        monkeypatch.setenv("GX_TWIN", "1")
        monkeypatch.setenv("GX_BAND_WAVES", "7")
    if poison:
        monkeypatch.setenv("GX_POOL_POISON", "1")
    cases = _synth(L)[:2 * H]
    assert len(cases) == 2 * H
    pairs = [_synth_pair(c["k"], L) for c in cases]
    # (the grid-64 case runs more passes: the early ones allocate pool
    # buffers, and an allocation orders the device work behind it)
    steps = 9 if shape.endswith("grid64") else 5
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, fill_ms = st.run(gx.Scores(*CONFIG_SCORES), False, keep_planes=True, steps=steps, plane_sums=True,
                          alternate=True)
    info = ctx.fill_info()
    assert info.get("groups", 1) == 1 and w_ok(info["band_waves"]), info
    assert fill_ms > 0
    sums = st.plane_sums()
    passes = st.pass_results()
    assert sums.shape == (steps, len(pairs), 3) and len(passes) == steps
    for k in range(steps):
        for q in range(H):
            p = (k % 2) * H + q
            c = cases[p]
            assert [int(x) for x in sums[k, p]] == [int(x) for x in c["plane_sums"]], (shape, p, "pass", k)
            _check_result(passes[k][p], None, c, (shape, p, "pass", k))
    for p, c in enumerate(cases):   # each set's last pass
        _check_result(res[p], st.steps(p), c, (shape, p, "last"))


def test_alternating_sets_rejects_shapes(gx, ctx):
    """GX_STAGED_ALTERNATE needs pair p and p + P/2 of one shape."""
    st = gx.StagedPairs([(b"ACGT" * 10, b"ACGA" * 10), (b"ACGT" * 11, b"ACGA" * 10)], ctx=ctx)
    with pytest.raises(gx.GxError):
        st.run(gx.Scores(*CONFIG_SCORES), False, keep_planes=True, steps=2, alternate=True)


@pytest.mark.parametrize("L", [1024, 4096, 16384])
def test_config5_batches(gx, ctx, L):
    """BASELINE configs[4]: 1024 x 1k pairs in one batch, and samples of the
    4k (64 pairs) and 16k (8 pairs) batches, through the staged pipelined
    path with score planes: every pair's planes and alignment."""
    cases = _synth(L)
    pairs = [_synth_pair(c["k"], L) for c in cases]
    _staged_check(gx, ctx, pairs, cases, steps=2)


@pytest.mark.parametrize("layout", ["auto", "lay0"])
def test_config5_64k_pair(gx, ctx, monkeypatch, layout):
    """One 65,536 x 65,536 pair of configs[4] (4.3e9 cells): column-step
    layout with int32 planes (auto) and the anti-diagonal layout with compact
    planes."""
    if layout == "lay0":
        monkeypatch.setenv("GX_LAYOUT", "0")
    cases = _synth(65536)
    pairs = [_synth_pair(c["k"], 65536) for c in cases]
    info = _staged_check(gx, ctx, pairs, cases, steps=1)
    assert info["plane_bytes_per_cell"] == (3 if layout == "lay0" else 12), info   # one pair: no twin


@pytest.mark.parametrize("variant", ["compact", "int32"])
def test_chunked_bench_launch(gx, ctx, monkeypatch, variant):
    """A staged batch larger than its device budget runs as chunks of pairs
    through the same buffers (GX_CHUNK_BYTES forces two pairs per chunk):
    every pass's planes and the last pass's alignments still equal the
    oracle's."""
    monkeypatch.setenv("GX_CHUNK_BYTES", "7e9" if variant == "compact" else "25e9")
    monkeypatch.setenv("GX_LAYOUT", "0")   # two-pair chunks would otherwise take the single-pair layout
    if variant == "int32":
        monkeypatch.setenv("GX_PLANES32", "1")
    cases = _synth(30000)[4:8]
    pairs = [_synth_pair(c["k"], 30000) for c in cases]
    info = _staged_check(gx, ctx, pairs, cases, steps=2)
    assert info["chunks"] == 2, info
    assert info["plane_bytes_per_cell"] in ((1.5, 3) if variant == "compact" else (12,)), info


def test_config5_1k_chunked(gx, ctx, monkeypatch):
    """1024 x 1k in uneven chunks (staged path with planes, and the
    traceback-only gx_align_batch)."""
    monkeypatch.setenv("GX_CHUNK_BYTES", "1.5e9")
    cases = _synth(1024)
    pairs = [_synth_pair(c["k"], 1024) for c in cases]
    info = _staged_check(gx, ctx, pairs, cases, steps=2)
    assert info["chunks"] >= 3, info
    monkeypatch.setenv("GX_CHUNK_BYTES", "0.2e9")
    out = gx.align_batch(pairs, gx.Scores(*CONFIG_SCORES), False, ctx=ctx, max_cell=False)
    assert ctx.fill_info()["chunks"] >= 3
    for (steps, r), c in zip(out, cases):
        _check_result(r, steps, c, c["k"])


def test_chunks_keep_twins(gx, ctx, monkeypatch):
    """A budget of 5.5 pairs: 5-pair chunks; twin_table forms the twins by
    shape inside each chunk (one pair twinned with itself per odd chunk), so
    every chunk keeps the twin fill."""
    pdb = (1024 + 128) * (1024 + 64) * 3.25 + 64 * (1024 + 64) * (1024 // 64 + 2) / 8 + 65536   # pair_device_bytes
    monkeypatch.setenv("GX_CHUNK_BYTES", str(5.5 * pdb))
    monkeypatch.setenv("GX_LAYOUT", "0")
    monkeypatch.setenv("GX_TWIN", "1")   # 4-pair chunks: a short queue would take the scalar fill
    cases = _synth(1024)[:40]
    pairs = [_synth_pair(c["k"], 1024) for c in cases]
    info = _staged_check(gx, ctx, pairs, cases, steps=1)
    assert info["chunks"] == 8 and info["twin"] == 1, info


@pytest.mark.parametrize("twin", ["1", "0"])
def test_related_30k_batch(gx, ctx, monkeypatch, twin):
    """SURVEY 8(d) M1's related variant (s2 = s1 with ~10 % substitutions and
    ~1 % indels, so the path winds through the whole table and the pair
    lengths differ): eight pairs through the staged launch with planes, with
    and without the twin fill, against the oracle's digests
    (tests/golden/synthetic_related_L30000.json)."""
    import sys
    sys.path.insert(0, GOLDEN)
    import make_golden
    monkeypatch.setenv("GX_TWIN", twin)
    monkeypatch.setenv("GX_LAYOUT", "0")
    with open(os.path.join(GOLDEN, "synthetic_related_L30000.json")) as f:
        cases = json.load(f)["cases"][:8]
    pairs = [make_golden.related_pair(c["k"], 30000) for c in cases]
    assert any(len(a) != len(b) for a, b in pairs)
    info = _staged_check(gx, ctx, pairs, cases, steps=2)
    assert info["twin"] == int(twin), info
