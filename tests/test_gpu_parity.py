"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle, bit-exact.

Covers the reference's own golden vectors (tests/test_alignment.rs), the
committed oracle fixtures, seeded random pairs around the 128-row strip and
band edges, exported score planes and full AlignmentCell tables,
reverse_sequences, batched pairs, and the large pairs of BASELINE configs 2
and 3 through digests.  Every test runs under each fill launch shape: the
automatic band width, forced 7-strip (tracked variants) and 8-strip bands,
and 15-strip bands on a 2-workgroup grid (bands wait in the queue for a
workgroup, hand-offs cross launch order), for the three fill layouts (0: the
anti-diagonal sweep of 128-row strips; 1: the column step over 64-row
strips; 3: the anti-diagonal sweep of 64-row strips, one row per lane) and
the automatic layout choice.
"""
import hashlib
import json
import os
import random

import numpy as np
import pytest

from conftest import COMPARISON, CONFIG_SCORES, FASTA, GOLDEN, TEST_SCORES, read_fasta_records

pytestmark = pytest.mark.gpu

LAUNCH_SHAPES = {"auto": {},
                 # layout 0: anti-diagonal fill over 128-row strips
                 "lay0": {"GX_LAYOUT": "0"}, "w7": {"GX_LAYOUT": "0", "GX_BAND_WAVES": "7"},
                 "w8": {"GX_LAYOUT": "0", "GX_BAND_WAVES": "8"},
                 "w15_grid2": {"GX_LAYOUT": "0", "GX_BAND_WAVES": "15", "GX_FILL_GRID": "2"},
                 # layout 3: the skewed 64-row strips (gx_skew.hip, the default for untracked
                 # single pairs), two-strip bands queued for one workgroup (every hand-off through HBM)
                 "skew": {"GX_LAYOUT": "3"},
                 "skew_w1_grid1": {"GX_LAYOUT": "3", "GX_BAND_WAVES": "1", "GX_FILL_GRID": "1"},
                 # layout 1: column-step fill over 64-row strips (gx_internal.h), as
                 # the split core + side waves (gx_cs2.hip, GX_CS2=1; the default for
                 # local fills); one-band bands queued on a 2-workgroup grid (every
                 # hand-off through HBM)
                 "cs": {"GX_LAYOUT": "1", "GX_CS2": "1"},
                 "cs_w7": {"GX_LAYOUT": "1", "GX_CS2": "1", "GX_BAND_WAVES": "7"},
                 "cs_w1_grid2": {"GX_LAYOUT": "1", "GX_CS2": "1", "GX_BAND_WAVES": "1", "GX_FILL_GRID": "2"},
                 # layout 1's one-wave strips (GX_CS2=0; the default for global fills)
                 "cs1": {"GX_LAYOUT": "1", "GX_CS2": "0"},
                 "cs1_w15_grid2": {"GX_LAYOUT": "1", "GX_CS2": "0", "GX_BAND_WAVES": "15", "GX_FILL_GRID": "2"}}


@pytest.fixture(autouse=True, params=sorted(LAUNCH_SHAPES))
def launch_shape(request, monkeypatch):
    for k, v in LAUNCH_SHAPES[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param

NAMES = ["Match", "Mismatch", "Insert", "Delete", "OpenInsert", "OpenDelete"]


def steps_list(steps):
    return [(NAMES[int(c)], int(i), int(j)) for c, i, j in zip(steps["choice"], steps["i"], steps["j"])]


def assert_same(gx_steps, gx_res, o, tag=""):
    assert steps_list(gx_steps) == o.alignment(), tag
    assert gx_res.score == o.score, tag
    assert (gx_res.matches, gx_res.mismatches, gx_res.gap_extensions, gx_res.opening_gaps) == \
           (o.matches, o.mismatches, o.gap_extensions, o.opening_gaps), tag
    assert (gx_res.start_i, gx_res.start_j) == o.start, tag
    assert (gx_res.max_cell_i, gx_res.max_cell_j) == o.max_cell, tag
    assert gx_res.matches_at_max == o.matches_at_max, tag


def sc(gx, t):
    return gx.Scores(*t)


def test_reference_golden_vectors(gx, ctx):
    """tests/test_alignment.rs:24-139 through the mirrored Rust API."""
    with open(os.path.join(GOLDEN, "reference_vectors.json")) as f:
        data = json.load(f)
    scores = gx.Scores(*data["scores"])
    for c in data["cases"]:
        cont = gx.SequenceContainer([gx.Sequence("s1", c["s1"]), gx.Sequence("s2", c["s2"])])
        table, _ = gx.alignment_table(cont, scores, False, False, ctx=ctx)
        a = gx.retrace(cont, table, False)
        if c["score"] is not None:
            assert a.score == c["score"]
        assert (a.matches, a.mismatches, a.opening_gaps, a.gap_extensions) == \
               (c["matches"], c["mismatches"], c["opening_gaps"], c["gap_extensions"])
        assert [(x[0].name, x[1], x[2]) for x in a.alignment] == [tuple(x) for x in c["alignment"]]


def test_committed_oracle_vectors(gx, ctx):
    with open(os.path.join(GOLDEN, "oracle_vectors.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        steps, r = gx.align_raw(c["s1"].encode("latin-1"), c["s2"].encode("latin-1"), gx.Scores(*c["scores"]),
                                c["is_local"], ctx=ctx)
        assert steps_list(steps) == [tuple(x) for x in c["alignment"]], c["name"]
        assert r.score == c["score"], c["name"]
        assert [r.matches, r.mismatches, r.gap_extensions, r.opening_gaps] == c["stats"], c["name"]
        assert [r.start_i, r.start_j] == c["start"] and [r.max_cell_i, r.max_cell_j] == c["max_cell"], c["name"]
        assert r.matches_at_max == c["matches_at_max"], c["name"]


EDGE_SIZES = [(0, 0), (0, 5), (5, 0), (1, 1), (1, 7), (7, 1), (63, 64), (64, 63), (64, 64), (65, 65), (127, 3),
              (3, 127), (255, 40), (256, 257), (257, 256), (300, 17), (17, 300), (513, 70), (640, 641)]


@pytest.mark.parametrize("is_local", [False, True], ids=["global", "local"])
def test_edge_sizes(gx, ctx, oracle, is_local):
    rng = random.Random(11)
    for n, m in EDGE_SIZES:
        for alpha in (b"ACGT", b"AC"):
            a = bytes(rng.choice(alpha) for _ in range(n))
            b = bytes(rng.choice(alpha) for _ in range(m))
            for t in (CONFIG_SCORES, TEST_SCORES):
                steps, r = gx.align_raw(a, b, sc(gx, t), is_local, ctx=ctx)
                assert_same(steps, r, oracle.align(a, b, t, is_local=is_local), (n, m, alpha, t))


@pytest.mark.parametrize("is_local", [False, True], ids=["global", "local"])
def test_random_pairs_batched(gx, ctx, oracle, is_local):
    """300 seeded random pairs per mode in one batched launch (ties are
    frequent under +1/-2 scoring and exercise the tie rules)."""
    rng = random.Random(1234 + is_local)
    pairs = []
    for _ in range(300):
        n, m = rng.randint(0, 200), rng.randint(0, 200)
        alpha = rng.choice([b"ACGT", b"AC", b"ACGTN"])
        pairs.append((bytes(rng.choice(alpha) for _ in range(n)), bytes(rng.choice(alpha) for _ in range(m))))
    out = gx.align_batch(pairs, sc(gx, CONFIG_SCORES), is_local, ctx=ctx)
    for (a, b), (steps, r) in zip(pairs, out):
        assert_same(steps, r, oracle.align(a, b, CONFIG_SCORES, is_local=is_local), (len(a), len(b)))


@pytest.mark.parametrize("scores", [(1, -2, -1, -5), (2, -3, -2, -4), (5, -4, 0, -10), (1, -1, -1, 0), (3, 1, -1, -2),
                                    (1, -2, 1, -3)])
def test_scoring_variants(gx, ctx, oracle, scores):
    rng = random.Random(hash(scores) & 0xffff)
    for _ in range(20):
        n, m = rng.randint(1, 150), rng.randint(1, 150)
        a = bytes(rng.choice(b"ACGT") for _ in range(n))
        b = bytes(rng.choice(b"ACGT") for _ in range(m))
        for loc in (False, True):
            steps, r = gx.align_raw(a, b, sc(gx, scores), loc, ctx=ctx)
            assert_same(steps, r, oracle.align(a, b, scores, is_local=loc), (n, m, scores, loc))


@pytest.mark.parametrize("n,m", [(1, 1), (5, 9), (63, 65), (64, 64), (130, 70), (257, 300), (300, 1000)])
@pytest.mark.parametrize("is_local", [False, True], ids=["global", "local"])
def test_exported_planes_and_cells(gx, ctx, oracle, n, m, is_local):
    """The score matrix: every plane value and full AlignmentCell (incl. the
    *_matches fields) equals the oracle's table, in the reference's
    column-major layout."""
    rng = random.Random(n * 1000 + m)
    a = bytes(rng.choice(b"ACGT") for _ in range(n))
    b = bytes(rng.choice(b"ACGT") for _ in range(m))
    o = oracle.align(a, b, CONFIG_SCORES, is_local=is_local, want_planes=True, want_lcs=True)
    cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
    table, mam = gx.alignment_table(cont, sc(gx, CONFIG_SCORES), is_local, False,
                                    flags=gx.GX_TABLE_PLANES | gx.GX_TABLE_MATCHES, ctx=ctx)
    assert mam == o.matches_at_max
    for k in range(3):
        assert np.array_equal(table.plane(k), o.planes[k]), ("plane", k)
    cells = table.export()
    assert cells.shape == (n + 1, m + 1) and cells.flags["F_CONTIGUOUS"]
    assert np.array_equal(cells["insert_score"], o.planes[0])
    assert np.array_equal(cells["delete_score"], o.planes[1])
    assert np.array_equal(cells["sub_score"], o.planes[2])
    # max_matches(cell) == oracle LCS plane
    mm = np.maximum(np.maximum(cells["insert_matches"], cells["sub_matches"]), cells["delete_matches"])
    assert np.array_equal(mm, o.lcs)
    # full cell fidelity against the ref_layout oracle (48-B cells, column-major)
    aln = gx.retrace(cont, table, is_local)
    assert [(x[0].name, x[1], x[2]) for x in aln.alignment] == o.alignment()


@pytest.mark.parametrize("scores", [(1, -2, -1, -5), (1, -2, -2, -5), (2, -3, -2, -4), (5, -4, 0, -10),
                                    (10, -10, -5, -20), (1, -1, 0, 0), (30, -30, -10, -40), (3, 1, -1, -2),
                                    (1, -2, 1, -3), (2, -1, 1, -4)])
@pytest.mark.parametrize("is_local", [False, True], ids=["global", "local"])
def test_untracked_table_planes(gx, ctx, oracle, scores, is_local):
    """Tables built without the max-cell tracking: on layout 0 their
    score planes are stored as per-cell byte differences when the scores pass
    the range proof (gx_api_plan.cpp d8_planes_ok; (30, -30, -10, -40) does not and
    (1, -2, 1, -3), (2, -1, 1, -4) have g > 0, all keep int32 planes).  On
    layout 1 a local fill with g > 0 must not take the split column step
    (gx_api_plan.cpp cs2_enabled: its 0 floor is applied after the delete chain's
    prefix max, exact only for g <= 0), even where GX_CS2=1 asks for it.  Every exported plane
    value equals the oracle's, including dense-tie and long-match inputs that
    push the differences towards the proof's bounds."""
    rng = random.Random(hash(scores) & 0xffff)
    for n, m in [(1, 1), (5, 9), (127, 130), (129, 300), (300, 1000), (700, 257)]:
        for alpha in (b"ACGT", b"AC", b"A"):
            a = bytes(rng.choice(alpha) for _ in range(n))
            b = bytes(rng.choice(alpha) for _ in range(m))
            o = oracle.align(a, b, scores, is_local=is_local, want_planes=True)
            cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
            table, mam = gx.alignment_table(cont, sc(gx, scores), is_local, False, ctx=ctx, max_cell=False)
            assert mam == 0
            for k in range(3):
                assert np.array_equal(table.plane(k), o.planes[k]), (n, m, alpha, "plane", k)
            aln = gx.retrace(cont, table, is_local)
            assert [(x[0].name, x[1], x[2]) for x in aln.alignment] == o.alignment(), (n, m, alpha)
            assert aln.score == o.score


def test_full_cells_match_reference_fields(gx, ctx, oracle):
    """Each *_matches field individually (algo.rs:250-255)."""
    a, b = b"ACGGATAAAAAAAATC", b"ACGGATAAAATC"
    cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
    table, _ = gx.alignment_table(cont, sc(gx, TEST_SCORES), False, False,
                                  flags=gx.GX_TABLE_PLANES | gx.GX_TABLE_MATCHES, ctx=ctx)
    cells = table.export()
    o = oracle.align(a, b, TEST_SCORES, want_lcs=True)
    L = o.lcs.astype(np.int64)
    n, m = len(a), len(b)
    for i in range(1, n + 1):
        for j in range(1, m + 1):
            mt = 1 if a[i - 1] == b[j - 1] else 0
            assert cells[i, j]["insert_matches"] == L[i, j - 1]
            assert cells[i, j]["delete_matches"] == L[i - 1, j]
            assert cells[i, j]["sub_matches"] == L[i - 1, j - 1] + mt
    table.free()


def test_reverse_sequences(gx, ctx, oracle):
    """is_match(.., true) index mapping (sequence.rs:102-115), incl. the
    None == None matches past the ends."""
    rng = random.Random(5)
    for _ in range(40):
        n, m = rng.randint(1, 90), rng.randint(1, 90)
        a = bytes(rng.choice(b"ACGT") for _ in range(n))
        b = bytes(rng.choice(b"ACGT") for _ in range(m))
        for loc in (False, True):
            steps, r = gx.align_raw(a, b, sc(gx, CONFIG_SCORES), loc, reverse_sequences=True, ctx=ctx)
            assert_same(steps, r, oracle.align(a, b, CONFIG_SCORES, is_local=loc, rev=True), (n, m, loc))


def test_test_data_files(gx, ctx, oracle):
    """Every multi-record FASTA fixture, as the CLI would align it."""
    for f in ("test1", "test2_short", "test3_short", "test4", "Opsin1_colorblindness_gene"):
        recs = read_fasta_records(os.path.join(FASTA, f + ".fasta"))
        for loc in (False, True):
            for t in (CONFIG_SCORES, TEST_SCORES):
                steps, r = gx.align_raw(recs[0][1], recs[1][1], sc(gx, t), loc, ctx=ctx)
                assert_same(steps, r, oracle.align(recs[0][1], recs[1][1], t, is_local=loc), (f, loc, t))


def test_errors(gx, ctx):
    with pytest.raises(gx.GxError) as e:
        gx.alignment_table(gx.SequenceContainer([gx.Sequence("a", "ACGT")]), gx.Scores(), False, False, ctx=ctx)
    assert e.value.code == 2
    # outside the exact-int32 range: computed by the int64 fill (tests/test_gpu_wide.py), not refused
    steps, r = gx.align_raw(b"ACGT", b"ACGT", gx.Scores(1 << 30, -2, -1, -5), False, ctx=ctx)
    assert r.score == 4 << 30


def _digest(steps):
    h = hashlib.sha256()
    h.update(bytes(steps["choice"].astype(np.uint8)))
    h.update(steps["i"].astype("<u8").tobytes())
    h.update(steps["j"].astype("<u8").tobytes())
    return h.hexdigest()


def test_large_pairs_digests(gx, ctx):
    """BASELINE configs 2 (Covid_Wuhan x Covid_USA-CA4, ~30k x 30k) and 3
    (Human x Mouse BRCA2), both modes, against oracle digests."""
    with open(os.path.join(GOLDEN, "large_digests.json")) as f:
        cases = json.load(f)["cases"]
    brca = read_fasta_records(os.path.join(FASTA, "Human-Mouse-BRCA2-cds.fasta"))
    wuhan = read_fasta_records(os.path.join(COMPARISON, "Covid_Wuhan.fasta"))[0][1]
    usa = read_fasta_records(os.path.join(COMPARISON, "Covid_USA-CA4.fasta"))[0][1]
    inputs = {"brca2": (brca[0][1], brca[1][1]), "covid_wuhan_usa": (wuhan, usa)}
    for c in cases:
        a, b = inputs[c["name"].split("/")[0]]
        steps, r = gx.align_raw(a, b, gx.Scores(*c["scores"]), c["is_local"], ctx=ctx)
        assert r.score == c["score"], c["name"]
        assert [r.matches, r.mismatches, r.gap_extensions, r.opening_gaps] == c["stats"], c["name"]
        assert [r.start_i, r.start_j] == c["start"], c["name"]
        assert [r.max_cell_i, r.max_cell_j] == c["max_cell"], c["name"]
        assert r.matches_at_max == c["matches_at_max"], c["name"]
        assert len(steps) == c["n_steps"], c["name"]
        assert _digest(steps) == c["alignment_sha256"], c["name"]


def test_staged_path_matches_oracle(gx, ctx, oracle):
    rng = random.Random(99)
    pairs = [(bytes(rng.choice(b"ACGT") for _ in range(rng.randint(100, 700))),
              bytes(rng.choice(b"ACGT") for _ in range(rng.randint(100, 700)))) for _ in range(6)]
    st = gx.StagedPairs(pairs, ctx=ctx)
    for keep, track, steps in ((True, True, 1), (True, False, 1), (False, True, 1), (False, False, 1),
                               (True, False, 3), (False, True, 4)):   # steps > 1: the pipelined passes
        res, fill_ms = st.run(sc(gx, CONFIG_SCORES), False, keep_planes=keep, max_cell=track, steps=steps)
        assert fill_ms > 0
        for (a, b), r in zip(pairs, res):
            o = oracle.align(a, b, CONFIG_SCORES)
            assert (r.score, r.n_steps, r.matches, r.mismatches, r.gap_extensions, r.opening_gaps) == \
                   (o.score, len(o.choices), o.matches, o.mismatches, o.gap_extensions, o.opening_gaps)
            if track:
                assert (r.max_cell_i, r.max_cell_j, r.matches_at_max) == \
                       (o.max_cell[0], o.max_cell[1], o.matches_at_max)
            else:   # main.rs discards it: not tracked on the fused path
                assert (r.max_cell_i, r.max_cell_j, r.matches_at_max) == (0, 0, 0)


@pytest.mark.parametrize("alpha,scores", [(b"ACGT", CONFIG_SCORES), (b"AC", TEST_SCORES), (b"GT", (3, -1, -2, -4)),
                                          (b"ACGTN", CONFIG_SCORES), (b"ACGT", (200, -2, -1, -5))],
                         ids=["acgt", "ac", "gt", "five_symbols", "wide_scores"])
@pytest.mark.parametrize("is_local", [False, True], ids=["global", "local"])
def test_untracked_batch_score_table(gx, ctx, oracle, alpha, scores, is_local):
    """The untracked batch path (global and local): <= 4 symbols with
    byte-sized scores take the packed score-table fill (one bit-field extract
    per cell), the rest the byte compare; both bit-exact with the oracle."""
    rng = random.Random(len(alpha) * 7 + scores[0])
    pairs = [(bytes(rng.choice(alpha) for _ in range(n)), bytes(rng.choice(alpha) for _ in range(m)))
             for n, m in [(1, 1), (5, 70), (128, 129), (300, 17), (257, 400)] + [(rng.randint(1, 300), rng.randint(1, 300))
                                                                                 for _ in range(20)]]
    out = gx.align_batch(pairs, sc(gx, scores), is_local, ctx=ctx, max_cell=False)
    for (a, b), (steps, r) in zip(pairs, out):
        o = oracle.align(a, b, scores, is_local=is_local)
        assert steps_list(steps) == o.alignment(), (len(a), len(b))
        assert (r.score, r.matches, r.mismatches, r.gap_extensions, r.opening_gaps) == \
               (o.score, o.matches, o.mismatches, o.gap_extensions, o.opening_gaps)


@pytest.mark.parametrize("scores", [(3, -2, -(1 << 22), -7), (1, -1, -(1 << 21), -(1 << 22)), (2, -3, -(1 << 23), -1)],
                         ids=["g2^22", "h2^22", "g2^23"])
def test_large_gap_scores_near_guard(gx, ctx, oracle, scores):
    """Gap scores of 2^21-2^23 on short pairs: inside the host's exact-int32
    guard, where the column-step scans offset the delete chain by up to
    64 (|g| + |h|) (layout 1 takes them while 65 (|g| + |h|) < 2^29, layout 0
    the rest); bit-exact with the oracle either way."""
    rng = random.Random(scores[2] & 0xffff)
    for _ in range(12):
        n, m = rng.randint(1, 14), rng.randint(1, 14)   # (n+m+2)(|scores|) < 2^28
        a = bytes(rng.choice(b"ACGT") for _ in range(n))
        b = bytes(rng.choice(b"ACGT") for _ in range(m))
        for loc in (False, True):
            steps, r = gx.align_raw(a, b, sc(gx, scores), loc, ctx=ctx)
            assert_same(steps, r, oracle.align(a, b, scores, is_local=loc), (n, m, scores, loc))
