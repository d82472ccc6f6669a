"""GPU parity of layout 3, the latency fill (genomics-rs_amd/csrc/gx_skew.hip):
64-row strips on the anti-diagonal skew with one row per lane, the default
for untracked single pairs (gx_align without max-cell tracking, untracked
alignment tables, staged runs of a few pairs).  Global fills keep V - (i+j) g
and fold the gap opening onto score_max (exact for h <= 0; h > 0 must fall
back to the column step); local fills keep plain values with the 0 floor.
Every result against the oracle (oracle/gx_oracle.c): alignments, statistics,
start cells, every exported plane value, plane checksums; at strip and band
edges, with bands queued for a one- or two-workgroup grid (every band
hand-off through HBM) and every instantiated band width."""
import random

import numpy as np
import pytest

from conftest import CONFIG_SCORES, TEST_SCORES

pytestmark = pytest.mark.gpu

NAMES = ["Match", "Mismatch", "Insert", "Delete", "OpenInsert", "OpenDelete"]
LAUNCH = {"w2": {"GX_LAYOUT": "3"}, "w3": {"GX_LAYOUT": "3", "GX_BAND_WAVES": "3"},
          "w2_grid1": {"GX_LAYOUT": "3", "GX_BAND_WAVES": "2", "GX_FILL_GRID": "1"},
          "w3_grid2": {"GX_LAYOUT": "3", "GX_BAND_WAVES": "3", "GX_FILL_GRID": "2"},
          "w1_grid1": {"GX_LAYOUT": "3", "GX_BAND_WAVES": "1", "GX_FILL_GRID": "1"}}
SIZES = [(1, 1), (1, 7), (7, 1), (2, 70), (63, 64), (64, 63), (64, 64), (65, 65), (127, 3), (3, 127), (128, 128),
         (129, 200), (255, 40), (256, 257), (257, 256), (300, 17), (17, 300), (513, 70), (640, 641), (1000, 1300)]


@pytest.fixture(params=sorted(LAUNCH))
def launch(request, monkeypatch):
    for k, v in LAUNCH[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param


def _steps_list(steps):
    return [(NAMES[int(c)], int(i), int(j)) for c, i, j in zip(steps["choice"], steps["i"], steps["j"])]


def _same(steps, r, o, tag):
    assert _steps_list(steps) == o.alignment(), tag
    assert (r.score, r.matches, r.mismatches, r.gap_extensions, r.opening_gaps) == \
           (o.score, o.matches, o.mismatches, o.gap_extensions, o.opening_gaps), tag
    assert (r.start_i, r.start_j) == o.start, tag


@pytest.mark.parametrize("is_local", [False, True], ids=["global", "local"])
def test_skew_edge_sizes(gx, ctx, oracle, launch, is_local):
    """gx_align without max-cell tracking (main.rs:143-150 discards it): every
    size around the 64-row strip and 16-step sub-block edges, two alphabets
    (AC: dense ties), both scoring configurations."""
    rng = random.Random(31 + is_local)
    for n, m in SIZES:
        for alpha in (b"ACGT", b"AC"):
            a = bytes(rng.choice(alpha) for _ in range(n))
            b = bytes(rng.choice(alpha) for _ in range(m))
            for t in (CONFIG_SCORES, TEST_SCORES):
                steps, r = gx.align_raw(a, b, gx.Scores(*t), is_local, ctx=ctx, max_cell=False)
                assert ctx.fill_info()["layout"] == 3, ctx.fill_info()
                _same(steps, r, oracle.align(a, b, t, is_local=is_local), (n, m, alpha, t))


@pytest.mark.parametrize("is_local", [False, True], ids=["global", "local"])
def test_skew_tracked(gx, ctx, oracle, launch, is_local):
    """Tracked fills on layout 3 (round 5): alignment_table's max_cell -- the
    FIRST maximum of score_max in row-major order, strict < (algo.rs:258-262)
    -- and matches_at_max, the max_matches field there (algo.rs:250-256, 279,
    carried by the side waves and, across bands, by the I/O waves' LCS
    granules), with the alignment, at every edge size, two alphabets (AC:
    dense ties between maxima), both scoring configurations."""
    rng = random.Random(71 + is_local)
    for n, m in SIZES:
        for alpha in (b"ACGT", b"AC"):
            a = bytes(rng.choice(alpha) for _ in range(n))
            b = bytes(rng.choice(alpha) for _ in range(m))
            for t in (CONFIG_SCORES, TEST_SCORES):
                steps, r = gx.align_raw(a, b, gx.Scores(*t), is_local, ctx=ctx, max_cell=True)
                assert ctx.fill_info()["layout"] == 3, ctx.fill_info()
                o = oracle.align(a, b, t, is_local=is_local)
                _same(steps, r, o, (n, m, alpha, t))
                assert (r.max_cell_i, r.max_cell_j, r.matches_at_max) == (*o.max_cell, o.matches_at_max), \
                    (n, m, alpha, t)


def test_skew_tracked_table(gx, ctx, oracle, monkeypatch):
    """alignment_table (the drop-in call with max_cell / matches_at_max, as
    INTEGRATION.md binds it) on layout 3: every exported cell value and the
    tracked outputs against the oracle, reverse_sequences both ways.  With
    GX_TABLE_MATCHES (round 6) the full 48-B cells: the *_matches fields come
    from the LCS bit rows of the launch's leading workgroups (gx_lcs.h),
    insert = LM(i, j-1), delete = LM(i-1, j), sub = LM(i-1, j-1) + is_match on
    the processed bytes (algo.rs:250-256, sequence.rs:102-115)."""
    monkeypatch.setenv("GX_LAYOUT", "3")
    rng = random.Random(5)
    for n, m, rev in ((200, 333, False), (333, 200, True), (129, 640, False), (70, 129, True)):
        a = "".join(rng.choice("ACGT") for _ in range(n))
        b = "".join(rng.choice("ACGT") for _ in range(m))
        for is_local in (False, True):
            for flags in (0, gx.GX_TABLE_PLANES | gx.GX_TABLE_MATCHES):
                cont = gx.SequenceContainer([gx.Sequence("a", a), gx.Sequence("b", b)])
                table, mam = gx.alignment_table(cont, gx.Scores(*CONFIG_SCORES), is_local, rev, ctx=ctx,
                                                max_cell=True, flags=flags or gx.GX_TABLE_PLANES)
                assert ctx.fill_info()["layout"] == 3, ctx.fill_info()
                o = oracle.align(a.encode(), b.encode(), CONFIG_SCORES, is_local=is_local, rev=rev, want_planes=True,
                                 want_lcs=True)
                tag = (n, m, rev, is_local, flags)
                assert mam == o.matches_at_max and table.info()["max_cell"] == o.max_cell, tag
                for k in range(3):
                    assert np.array_equal(table.plane(k), o.planes[k]), (tag, k)
                if flags:
                    cells = table.export()
                    L = o.lcs.astype(np.int64)
                    c1, c2 = oracle.processed_bytes(a.encode(), b.encode(), rev)
                    mt = (c1[:, None] == c2[None, :]).astype(np.int64)
                    assert np.array_equal(cells["insert_matches"][1:, 1:], L[1:, :-1]), tag
                    assert np.array_equal(cells["delete_matches"][1:, 1:], L[:-1, 1:]), tag
                    assert np.array_equal(cells["sub_matches"][1:, 1:], L[:-1, :-1] + mt), tag
                    for f in ("insert_matches", "delete_matches", "sub_matches"):
                        assert not cells[f][0, :].any() and not cells[f][:, 0].any(), (tag, f)
                    assert np.array_equal(table.rows(3, 0, n + 1), L), tag
                table.free()


# rows / columns around the LCS units' edges (128 words = 8,192 columns a
# unit, 2W + 1 units a workgroup: 40,960 columns at W = 2) and the 32-row
# carry hand-offs between units
LCS_SHAPES = [(1, 8193), (31, 8192), (32, 8191), (33, 16385), (64, 24577), (65, 40961), (40, 50000), (97, 100)]


@pytest.mark.parametrize("n,m", LCS_SHAPES)
def test_skew_lcs_rows(gx, ctx, oracle, monkeypatch, n, m):
    """max_matches of every cell (table rows, which = 3) and matches_at_max
    of tracked layout-3 tables whose LCS rows span several units and LCS
    workgroups, for DNA (score tables in the core), a 6-letter alphabet and
    reverse_sequences (None == None past the ends), at band widths 2 and 1
    (1: three units a workgroup)."""
    rng = random.Random(n * 7 + m)
    for alpha, rev, bw in ((b"ACGT", False, "2"), (b"ACDEFG", True, "2"), (b"AC", False, "1")):
        monkeypatch.setenv("GX_LAYOUT", "3")
        monkeypatch.setenv("GX_BAND_WAVES", bw)
        a = bytes(rng.choice(alpha) for _ in range(n))
        b = bytes(rng.choice(alpha) for _ in range(m))
        cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
        table, mam = gx.alignment_table(cont, gx.Scores(*CONFIG_SCORES), False, rev, ctx=ctx, max_cell=True,
                                        flags=gx.GX_TABLE_MATCHES)
        assert ctx.fill_info()["layout"] == 3, ctx.fill_info()
        o = oracle.align(a, b, CONFIG_SCORES, rev=rev)
        tag = (n, m, alpha, rev, bw)
        assert mam == o.matches_at_max and table.info()["max_cell"] == o.max_cell, tag
        L = oracle.lcs_rows(a, b, range(n + 1), rev=rev)
        got = table.rows(3, 0, n + 1)
        for i in range(n + 1):
            assert np.array_equal(got[i], L[i]), (tag, i)
        table.free()


LCS_SWEEPS = [("1", "1"), ("1", "3"), ("2", "2"), ("3", "2"), ("4", "1"), ("4", "3")]


@pytest.mark.parametrize("waves,wgs", LCS_SWEEPS, ids=[f"w{w}g{g}" for w, g in LCS_SWEEPS])
def test_skew_lcs_strip_handoffs(gx, ctx, oracle, monkeypatch, waves, wgs):
    """The LCS sweep's strip-to-strip hand-offs (gx_lcs.h) on pairs of 5-24
    strips, with the sweeping waves a workgroup and the workgroups forced
    (GX_LCS_WAVES / GX_LCS_WGS): one wave a workgroup sends every bottom row
    through HBM, several waves hand off through the LDS ring and reuse it
    block after block (counters across blocks), several workgroups pass
    blocks between them.  Every row with GX_TABLE_MATCHES (each row kept) and
    matches_at_max without it (only the strips' last rows kept; the max
    cell's strip re-swept by lcs_matches), against the oracle."""
    monkeypatch.setenv("GX_LAYOUT", "3")
    monkeypatch.setenv("GX_LCS_WAVES", waves)
    monkeypatch.setenv("GX_LCS_WGS", wgs)
    rng = random.Random(int(waves) * 10 + int(wgs))
    for n, m, alpha, rev in ((300, 1000, b"ACGT", False), (700, 200, b"AC", True), (1500, 5000, b"ACGT", False)):
        a = bytes(rng.choice(alpha) for _ in range(n))
        b = bytes(rng.choice(alpha) for _ in range(m))
        cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
        o = oracle.align(a, b, CONFIG_SCORES, rev=rev)
        tag = (n, m, rev, waves, wgs)
        table, mam = gx.alignment_table(cont, gx.Scores(*CONFIG_SCORES), False, rev, ctx=ctx, max_cell=True,
                                        flags=gx.GX_TABLE_MATCHES)
        assert ctx.fill_info()["layout"] == 3, ctx.fill_info()
        assert mam == o.matches_at_max and table.info()["max_cell"] == o.max_cell, tag
        L = oracle.lcs_rows(a, b, range(n + 1), rev=rev)
        got = table.rows(3, 0, n + 1)
        for i in range(n + 1):
            assert np.array_equal(got[i], L[i]), (tag, i)
        table.free()
        table, mam = gx.alignment_table(cont, gx.Scores(*CONFIG_SCORES), False, rev, ctx=ctx, max_cell=True)
        assert mam == o.matches_at_max and table.info()["max_cell"] == o.max_cell, (tag, "last rows only")
        table.free()


@pytest.mark.parametrize("scores,layout", [((1, -2, -1, -5), 3), ((2, -3, -2, -4), 3), ((5, -4, 0, -10), 3),
                                           ((1, -1, -1, 0), 3), ((3, 1, -1, -2), 3), ((1, -2, 1, -3), 3),
                                           ((2, -1, -1, 3), 1), ((1, -1, 0, 2), 1)])
@pytest.mark.parametrize("is_local", [False, True], ids=["global", "local"])
def test_skew_scoring_variants(gx, ctx, oracle, monkeypatch, scores, layout, is_local):
    """Scores with g = 0, g > 0, h = 0, a positive mismatch: layout 3; h > 0
    falls back to the column step (the folded gap opening needs h <= 0).
    Alignments and every exported plane value of the untracked table."""
    monkeypatch.setenv("GX_LAYOUT", "3")
    rng = random.Random(hash(scores) & 0xffff)
    for n, m in [(1, 1), (50, 130), (129, 70), (200, 200), (333, 257)]:
        for alpha in (b"ACGT", b"A"):
            a = bytes(rng.choice(alpha) for _ in range(n))
            b = bytes(rng.choice(alpha) for _ in range(m))
            o = oracle.align(a, b, scores, is_local=is_local, want_planes=True)
            cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
            table, _ = gx.alignment_table(cont, gx.Scores(*scores), is_local, False, ctx=ctx, max_cell=False)
            # (the fallback: the column step, as one wave per strip or split, gx_cs2.hip)
            assert ctx.fill_info()["layout"] in ((3,) if layout == 3 else (1, 2)), (scores, ctx.fill_info())
            for k in range(3):
                assert np.array_equal(table.plane(k), o.planes[k]), (scores, n, m, alpha, "plane", k)
            aln = gx.retrace(cont, table, is_local)
            assert [(x[0].name, x[1], x[2]) for x in aln.alignment] == o.alignment(), (scores, n, m)
            assert aln.score == o.score


@pytest.mark.parametrize("is_local", [False, True], ids=["global", "local"])
def test_skew_table_planes(gx, ctx, oracle, launch, is_local):
    """Untracked alignment tables on layout 3: every plane value (the
    step-indexed int32 planes decoded by export_kernel, with the shift undone
    for global fills) and the plane checksums (plane_sums_kernel)."""
    rng = random.Random(77 + is_local)
    for n, m in [(65, 64), (200, 333), (700, 257), (1024, 100)]:
        a = bytes(rng.choice(b"ACGT") for _ in range(n))
        b = bytes(rng.choice(b"ACGT") for _ in range(m))
        o = oracle.align(a, b, CONFIG_SCORES, is_local=is_local, want_planes=True)
        cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
        table, _ = gx.alignment_table(cont, gx.Scores(*CONFIG_SCORES), is_local, False, ctx=ctx, max_cell=False)
        assert ctx.fill_info()["layout"] == 3
        for k in range(3):
            assert np.array_equal(table.plane(k), o.planes[k]), (n, m, "plane", k)
        assert table.plane_sums() == oracle.align_lean(a, b, CONFIG_SCORES, is_local=is_local).extra["plane_sums"]
        aln = gx.retrace(cont, table, is_local)
        assert [(x[0].name, x[1], x[2]) for x in aln.alignment] == o.alignment()


@pytest.mark.parametrize("is_local", [False, True], ids=["global", "local"])
def test_skew_batch_and_reverse(gx, ctx, oracle, is_local, monkeypatch):
    """A few pairs per launch (gx_align_batch, untracked) and reverse_sequences
    (sequence.rs:102-115) on layout 3; five symbols (no score table)."""
    monkeypatch.setenv("GX_LAYOUT", "3")
    rng = random.Random(5 + is_local)
    pairs = [(bytes(rng.choice(b"ACGTN") for _ in range(rng.randint(1, 400))),
              bytes(rng.choice(b"ACGTN") for _ in range(rng.randint(1, 400)))) for _ in range(12)]
    out = gx.align_batch(pairs, gx.Scores(*CONFIG_SCORES), is_local, ctx=ctx, max_cell=False)
    assert ctx.fill_info()["layout"] == 3
    for (a, b), (steps, r) in zip(pairs, out):
        _same(steps, r, oracle.align(a, b, CONFIG_SCORES, is_local=is_local), (len(a), len(b)))
    for a, b in pairs[:6]:
        steps, r = gx.align_raw(a, b, gx.Scores(*CONFIG_SCORES), is_local, reverse_sequences=True, ctx=ctx,
                                max_cell=False)
        _same(steps, r, oracle.align(a, b, CONFIG_SCORES, is_local=is_local, rev=True), (len(a), len(b), "rev"))


@pytest.mark.parametrize("is_local", [False, True], ids=["global", "local"])
def test_skew_staged_steps(gx, ctx, oracle, launch, is_local):
    """The staged, pipelined path (config records of bench.py) on layout 3:
    three passes, every pass's plane checksums and results, the last pass's
    alignments."""
    rng = random.Random(909 + is_local)
    pairs = [(bytes(rng.choice(b"ACGT") for _ in range(n)), bytes(rng.choice(b"ACGT") for _ in range(m)))
             for n, m in [(1500, 1400), (700, 900)]]
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*CONFIG_SCORES), is_local, keep_planes=True, steps=3, plane_sums=True)
    assert ctx.fill_info()["layout"] == 3 and ctx.fill_info()["plane_bytes_per_cell"] == 12
    sums = st.plane_sums()
    passes = st.pass_results()
    for p, (a, b) in enumerate(pairs):
        o = oracle.align_lean(a, b, CONFIG_SCORES, is_local=is_local)
        for k in range(3):
            assert [int(x) for x in sums[k, p]] == o.extra["plane_sums"], (p, k)
            assert (passes[k][p].score, passes[k][p].n_steps) == (o.score, len(o.choices)), (p, k)
        assert _steps_list(st.steps(p)) == o.alignment(), p
