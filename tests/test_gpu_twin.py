"""GPU parity of the twin fill (genomics-rs_amd/csrc/gx_fill_pk.hip): batches
run two pairs per band (of equal or different shapes), one in each 16-bit
half of every register, with values kept relative to per-block bases.  Every
result -- alignment, statistics, the compact score planes -- must equal the
oracle's, on shapes around the strip and band edges, with bands queued for
workgroups (small grids) and at every band width, and under scores near the
twin fill's admission bound."""
import random

import numpy as np
import pytest

from conftest import CONFIG_SCORES

pytestmark = pytest.mark.gpu

NAMES = ["Match", "Mismatch", "Insert", "Delete", "OpenInsert", "OpenDelete"]
SHAPES = [(1, 1), (5, 9), (63, 64), (64, 63), (128, 129), (129, 300), (257, 256), (700, 257), (300, 1000),
          (1000, 77)]
# the twin fill is a variant of the anti-diagonal layout, which small batches
# would not get by default (they take the column-step layout)
LAUNCH = {"auto": {"GX_LAYOUT": "0"}, "w4_grid2": {"GX_LAYOUT": "0", "GX_BAND_WAVES": "4", "GX_FILL_GRID": "2"},
          "w8_grid3": {"GX_LAYOUT": "0", "GX_BAND_WAVES": "8", "GX_FILL_GRID": "3"},
          "w15_grid2": {"GX_LAYOUT": "0", "GX_BAND_WAVES": "15", "GX_FILL_GRID": "2"}}


def _steps_list(steps):
    return [(NAMES[int(c)], int(i), int(j)) for c, i, j in zip(steps["choice"], steps["i"], steps["j"])]


def _twin_pairs(seed, shapes, per_shape=2, alphas=(b"ACGT", b"AC", b"ACGTN", b"A")):
    rng = random.Random(seed)
    pairs = []
    for n, m in shapes:
        for _ in range(per_shape):
            al = rng.choice(alphas)
            pairs.append((bytes(rng.choice(al) for _ in range(n)), bytes(rng.choice(al) for _ in range(m))))
    return pairs


@pytest.fixture(autouse=True)
def _force_twin(monkeypatch):
    """The batches here are small: force the twin fill (by default it runs
    only for band queues of >= 2.5 rounds, gx_api_fill.cpp run_fill)."""
    monkeypatch.setenv("GX_TWIN", "1")


@pytest.fixture(params=sorted(LAUNCH))
def launch(request, monkeypatch):
    for k, v in LAUNCH[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param


def test_twin_batch_alignments(gx, ctx, oracle, launch):
    """gx_align_batch (traceback-only twin fill): every alignment."""
    pairs = _twin_pairs(7, SHAPES)
    out = gx.align_batch(pairs, gx.Scores(*CONFIG_SCORES), False, ctx=ctx, max_cell=False)
    assert ctx.fill_info()["twin"] == 1
    for (a, b), (steps, r) in zip(pairs, out):
        o = oracle.align(a, b, CONFIG_SCORES)
        assert _steps_list(steps) == o.alignment(), (len(a), len(b))
        assert (r.score, r.matches, r.mismatches, r.gap_extensions, r.opening_gaps) == \
               (o.score, o.matches, o.mismatches, o.gap_extensions, o.opening_gaps)


@pytest.mark.parametrize("fmt", ["codes", "bytes"])
def test_twin_staged_planes(gx, ctx, oracle, launch, monkeypatch, fmt):
    """The staged, pipelined path with compact planes through the twin fill:
    every pass's plane checksums and the last pass's alignments."""
    if fmt == "bytes":
        monkeypatch.setenv("GX_PLANES_W16", "0")
    pairs = _twin_pairs(11, SHAPES, per_shape=4)
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*CONFIG_SCORES), False, keep_planes=True, steps=3, plane_sums=True)
    info = ctx.fill_info()
    assert info["twin"] == 1 and info["plane_bytes_per_cell"] == (1.5 if fmt == "codes" else 3), info
    sums = st.plane_sums()
    for p, (a, b) in enumerate(pairs):
        o = oracle.align_lean(a, b, CONFIG_SCORES)
        for k in range(3):
            assert [int(x) for x in sums[k, p]] == o.extra["plane_sums"], (p, len(a), len(b), k)
        assert res[p].score == o.score and res[p].n_steps == len(o.choices)
        assert _steps_list(st.steps(p)) == o.alignment(), (p, len(a), len(b))


@pytest.mark.parametrize("scores", [(1, -2, -2, -5), (2, -3, -2, -4), (5, -4, 0, -10), (1, -1, 0, 0), (3, -3, -1, -1),
                                    (4, -4, -2, -2)])
def test_twin_scoring_variants(gx, ctx, oracle, monkeypatch, scores):
    """Other scores: the twin fill where the admission bound holds (else the
    scalar fill), bit-exact either way; with and without planes."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    pairs = _twin_pairs(hash(scores) & 0xffff, [(200, 300), (129, 130), (700, 40)], per_shape=2)
    out = gx.align_batch(pairs, gx.Scores(*scores), False, ctx=ctx, max_cell=False)
    for (a, b), (steps, r) in zip(pairs, out):
        o = oracle.align(a, b, scores)
        assert _steps_list(steps) == o.alignment() and r.score == o.score, (scores, len(a), len(b))
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*scores), False, keep_planes=True, steps=1, plane_sums=True)
    sums = st.plane_sums()
    for p, (a, b) in enumerate(pairs):
        o = oracle.align_lean(a, b, scores)
        assert [int(x) for x in sums[0, p]] == o.extra["plane_sums"] and res[p].score == o.score, (scores, p)


def test_twin_matches_scalar_fill(gx, ctx, monkeypatch):
    """The twin and the scalar fill give identical results and planes on the same batch."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    pairs = _twin_pairs(5, [(600, 700), (333, 333)], per_shape=4, alphas=(b"ACGT",))
    st = gx.StagedPairs(pairs, ctx=ctx)
    r1, _ = st.run(gx.Scores(*CONFIG_SCORES), False, keep_planes=True, plane_sums=True)
    s1 = st.plane_sums().copy()
    assert ctx.fill_info()["twin"] == 1
    monkeypatch.setenv("GX_TWIN", "0")
    r0, _ = st.run(gx.Scores(*CONFIG_SCORES), False, keep_planes=True, plane_sums=True)
    assert ctx.fill_info()["twin"] == 0
    assert np.array_equal(s1, st.plane_sums())
    assert [(r.score, r.n_steps, r.matches) for r in r1] == [(r.score, r.n_steps, r.matches) for r in r0]


@pytest.mark.parametrize("shape", [(1, 1), (64, 16), (129, 16), (200, 40), (300, 20), (257, 300), (640, 129)])
def test_twin_table_planes(gx, ctx, oracle, monkeypatch, shape):
    """GX_TABLE_TWIN=1 fills an alignment table with the twin fill (the pair
    beside a copy of itself): every exported plane cell and the alignment."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    monkeypatch.setenv("GX_TABLE_TWIN", "1")
    monkeypatch.setenv("GX_NO_TABLE_PRINT", "1")
    n, m = shape
    rng = random.Random(n * 7919 + m)
    a = bytes(rng.choice(b"ACGT") for _ in range(n))
    b = bytes(rng.choice(b"ACGT") for _ in range(m))
    cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
    t, _ = gx.alignment_table(cont, gx.Scores(*CONFIG_SCORES), False, False, ctx=ctx, max_cell=False)
    assert ctx.fill_info()["twin"] == 1
    o = oracle.align(a, b, CONFIG_SCORES, want_planes=True)
    for k in range(3):
        assert np.array_equal(t.plane(k), o.planes[k]), (shape, k)
    al = gx.retrace(cont, t, False)
    assert _steps_list(al._steps) == o.alignment() and al.score == o.score


MIXED = [((129, 300), (300, 129)), ((1, 1), (5, 9)), ((1, 300), (300, 1)), ((700, 257), (640, 300)),
         ((64, 63), (63, 64)), ((1000, 77), (999, 80)), ((257, 256), (128, 1000))]


@pytest.mark.parametrize("odd", [False, True])
def test_twin_mixed_shapes(gx, ctx, oracle, monkeypatch, odd):
    """Twins of different shapes (the sweep covers the larger n and m, the
    shorter pair stops at its own last column) and an odd count (the last
    pair twinned with itself): every alignment, score and plane checksum."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    rng = random.Random(17 + odd)
    shapes = [s for tw in MIXED for s in tw] + ([(333, 222)] if odd else [])
    pairs = [(bytes(rng.choice(b"ACGT") for _ in range(n)), bytes(rng.choice(b"ACGT") for _ in range(m)))
             for n, m in shapes]
    out = gx.align_batch(pairs, gx.Scores(*CONFIG_SCORES), False, ctx=ctx, max_cell=False)
    assert ctx.fill_info()["twin"] == 1
    for (a, b), (steps, r) in zip(pairs, out):
        o = oracle.align(a, b, CONFIG_SCORES)
        assert _steps_list(steps) == o.alignment(), (len(a), len(b))
        assert (r.score, r.matches, r.mismatches, r.gap_extensions, r.opening_gaps) == \
               (o.score, o.matches, o.mismatches, o.gap_extensions, o.opening_gaps)
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*CONFIG_SCORES), False, keep_planes=True, steps=2, plane_sums=True)
    info = ctx.fill_info()
    assert info["twin"] == 1 and info["plane_bytes_per_cell"] == 1.5, info
    sums = st.plane_sums()
    for p, (a, b) in enumerate(pairs):
        o = oracle.align_lean(a, b, CONFIG_SCORES)
        for k in range(2):
            assert [int(x) for x in sums[k, p]] == o.extra["plane_sums"], (p, len(a), len(b), k)
        assert res[p].score == o.score
        assert _steps_list(st.steps(p)) == o.alignment(), (p, len(a), len(b))


@pytest.mark.parametrize("seed", range(6))
def test_twin_random_batches(gx, ctx, oracle, monkeypatch, seed):
    """Randomised twin batches: random shapes (1-700 x 1-700, odd and even
    counts), alphabets and admissible scores, band widths and grids; every
    alignment, score and plane checksum against the oracle."""
    rng = random.Random(1000 + seed)
    monkeypatch.setenv("GX_LAYOUT", "0")
    monkeypatch.setenv("GX_BAND_WAVES", rng.choice(["3", "4", "7", "8", "15"]))
    monkeypatch.setenv("GX_FILL_GRID", rng.choice(["1", "2", "5", "64"]))
    scores = rng.choice([CONFIG_SCORES, (1, -2, -2, -5), (2, -3, -1, -4), (1, -1, 0, -3), (3, -2, -2, -2)])
    al = rng.choice([b"ACGT", b"AC", b"ACGTN", b"ACDEFGHIKLMNPQRSTVWY"])
    shapes = [(rng.randint(1, 700), rng.randint(1, 700)) for _ in range(rng.randint(2, 9))]
    pairs = [(bytes(rng.choice(al) for _ in range(n)), bytes(rng.choice(al) for _ in range(m))) for n, m in shapes]
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*scores), False, keep_planes=True, steps=1, plane_sums=True)
    info = ctx.fill_info()
    sums = st.plane_sums()
    for p, (a, b) in enumerate(pairs):
        o = oracle.align_lean(a, b, scores)
        assert [int(x) for x in sums[0, p]] == o.extra["plane_sums"], (seed, p, len(a), len(b), info)
        assert res[p].score == o.score, (seed, p)
        assert _steps_list(st.steps(p)) == o.alignment(), (seed, p)


@pytest.mark.parametrize("skel", ["noskel", "skel"])
@pytest.mark.parametrize("m", [31920, 31921, 65536])
def test_twin_column_limit(gx, ctx, oracle, monkeypatch, m, skel):
    """With a skeleton (the per-pair byte planes, GX_PLANES_W16=0, keep code
    words and landing columns) the twin fill's landing columns are int16
    halves: twins up to 31,920 columns, the scalar fill beyond.  Without one
    (twin plane codes: no landing columns, the traceback walks the strips in
    sequence) the twin fill has no column limit: 65,536 columns.  Every pair
    checked against the oracle (plane checksums, score, alignment)."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    if skel == "skel":
        monkeypatch.setenv("GX_PLANES_W16", "0")
    rng = random.Random(m)
    shapes = [(200, m), (150, m - 7), (260, m - 1)]
    pairs = [(bytes(rng.choice(b"ACGT") for _ in range(n)), bytes(rng.choice(b"ACGT") for _ in range(mm)))
             for n, mm in shapes]
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*CONFIG_SCORES), False, keep_planes=True, steps=1, plane_sums=True)
    assert ctx.fill_info()["twin"] == (1 if m <= 31920 or skel == "noskel" else 0)
    sums = st.plane_sums()
    for p, (a, b) in enumerate(pairs):
        o = oracle.align_lean(a, b, CONFIG_SCORES)
        assert [int(x) for x in sums[0, p]] == o.extra["plane_sums"], (m, p)
        assert res[p].score == o.score and _steps_list(st.steps(p)) == o.alignment(), (m, p)


def test_twin_pairs_by_shape(gx, ctx, oracle, monkeypatch):
    """Twins are formed by shape, not by position: a batch alternating very
    different lengths (adjacent pairs 60x apart in columns, beyond the
    admission bound's column margin) still takes the twin fill, each twin
    holding two pairs of near shapes; every result against the oracle."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    rng = random.Random(77)
    shapes = []
    for k in range(5):
        shapes += [(150 + 7 * k, 6000 + 13 * k), (140 + 5 * k, 100 + 3 * k)]
    pairs = [(bytes(rng.choice(b"ACGT") for _ in range(n)), bytes(rng.choice(b"ACGT") for _ in range(m)))
             for n, m in shapes]
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*CONFIG_SCORES), False, keep_planes=True, steps=1, plane_sums=True)
    assert ctx.fill_info()["twin"] == 1
    sums = st.plane_sums()
    for p, (a, b) in enumerate(pairs):
        o = oracle.align_lean(a, b, CONFIG_SCORES)
        assert [int(x) for x in sums[0, p]] == o.extra["plane_sums"], p
        assert res[p].score == o.score and _steps_list(st.steps(p)) == o.alignment(), p


# ---- the int16 admission bound where it binds (gx_api_plan.cpp twin_width) ------
# Inputs that push the twin fill's values hardest (tests/test_twin_bound.py
# measures their spreads against the rule on the CPU) at the widest scores
# each band width admits; every plane cell of a table filled by the twin
# kernel (GX_TABLE_TWIN), and the alignment, against the oracle.
from test_twin_bound import _families  # noqa: E402

BOUND_SCORES = [(CONFIG_SCORES, 15), ((1, -1, -1, -7), 15), ((1, -1, -1, -16), 8), ((2, -2, -1, -34), 4)]


@pytest.mark.parametrize("scores,W", BOUND_SCORES)
@pytest.mark.parametrize("family", ["all_mismatch", "all_match", "gap_rows", "gap_cols", "repeat"])
def test_twin_bound_worst_inputs_table(gx, ctx, oracle, monkeypatch, scores, W, family):
    monkeypatch.setenv("GX_LAYOUT", "0")
    monkeypatch.setenv("GX_TABLE_TWIN", "1")
    monkeypatch.setenv("GX_BAND_WAVES", str(W))
    monkeypatch.setenv("GX_NO_TABLE_PRINT", "1")
    n, m = 128 * W * 2 + 300, 1400   # two full bands and a partial third
    a, b = _families(n, m)[family]
    cont = gx.SequenceContainer([gx.Sequence("a", a.decode()), gx.Sequence("b", b.decode())])
    t, _ = gx.alignment_table(cont, gx.Scores(*scores), False, False, ctx=ctx, max_cell=False)
    info = ctx.fill_info()
    assert info["twin"] == 1 and info["band_waves"] == W, info
    o = oracle.align(a, b, scores, want_planes=True)
    for k in range(3):
        assert np.array_equal(t.plane(k), o.planes[k]), (family, scores, k)
    al = gx.retrace(cont, t, False)
    assert _steps_list(al._steps) == o.alignment() and al.score == o.score


@pytest.mark.parametrize("scores,W", BOUND_SCORES)
def test_twin_bound_worst_inputs_batch(gx, ctx, oracle, monkeypatch, scores, W):
    """The same inputs as a staged twin batch (twin plane codes where w16_ok
    holds, else bytes), plus twins 1,024 columns apart where W <= 8 admits
    them: plane checksums of every pass, scores and alignments."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    monkeypatch.setenv("GX_BAND_WAVES", str(W))
    n, m = 128 * W * 2 + 300, 1400
    pairs = list(_families(n, m).values())
    if W <= 8:
        rng = random.Random(W)
        pairs += [(bytes(rng.choice(b"ACGT") for _ in range(n)), bytes(rng.choice(b"ACGT") for _ in range(mm)))
                  for mm in (3000, 1976)]
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*scores), False, keep_planes=True, steps=2, plane_sums=True)
    info = ctx.fill_info()
    assert info["twin"] == 1 and info["band_waves"] == W, info
    sums = st.plane_sums()
    for p, (a, b) in enumerate(pairs):
        o = oracle.align_lean(a, b, scores)
        for k in range(2):
            assert [int(x) for x in sums[k, p]] == o.extra["plane_sums"], (scores, p, k)
        assert res[p].score == o.score and _steps_list(st.steps(p)) == o.alignment(), (scores, p)


@pytest.mark.parametrize("m", [31920, 65536])
def test_twin_bound_column_limit_worst(gx, ctx, oracle, monkeypatch, m):
    """m = 31,920 (the int16 landing-column limit of a twin fill with a
    skeleton) and 65,536 (the fill without one) with all-mismatch and
    all-match rows: plane checksums, scores and alignments."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    pairs = [(b"A" * 200, b"C" * m), (b"A" * 150, b"A" * (m - 3)), (b"AC" * 130, b"CA" * (m // 2))]
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*CONFIG_SCORES), False, keep_planes=True, steps=1, plane_sums=True)
    assert ctx.fill_info()["twin"] == 1
    sums = st.plane_sums()
    for p, (a, b) in enumerate(pairs):
        o = oracle.align_lean(a, b, CONFIG_SCORES)
        assert [int(x) for x in sums[0, p]] == o.extra["plane_sums"], p
        assert res[p].score == o.score and _steps_list(st.steps(p)) == o.alignment(), p


@pytest.mark.parametrize("kind", ["self_twins", "deep_equal"])
def test_twin_auto_selection(gx, ctx, oracle, monkeypatch, kind):
    """GX_TWIN unset: the automatic rules of run_fill.  A batch of mostly
    unmatched shapes (column counts more than the gap cap apart, so every pair
    would be twinned with itself) stays on the scalar fill; a deep batch of
    equal shapes (>= 0.9 x CUs twin bands) takes the twin fill.  Results
    against the oracle either way."""
    monkeypatch.delenv("GX_TWIN", raising=False)
    rng = random.Random(99)
    if kind == "self_twins":
        shapes = [(300 + 13 * k, 200 + 1500 * k) for k in range(8)]
    else:
        shapes = [(1500, 1500)] * 128
    pairs = [(bytes(rng.choice(b"ACGT") for _ in range(n)), bytes(rng.choice(b"ACGT") for _ in range(m)))
             for n, m in shapes]
    out = gx.align_batch(pairs, gx.Scores(*CONFIG_SCORES), False, ctx=ctx, max_cell=False)
    assert ctx.fill_info()["twin"] == (0 if kind == "self_twins" else 1), ctx.fill_info()
    for (a, b), (steps, r) in zip(pairs, out):
        o = oracle.align_lean(a, b, CONFIG_SCORES)
        assert r.score == o.score and r.n_steps == len(o.choices)
        assert _steps_list(steps) == o.alignment()


@pytest.mark.parametrize("launch_env", ["auto", "w4_grid3"])
def test_twin_overlapped_global(gx, ctx, oracle, monkeypatch, launch_env):
    """The headline's launch shape: a long-pair global batch through the
    overlapped two-group pipeline (gx_api_batch.cpp batch_core_overlap: group A's
    fill of pass k+1 beside pass k's walk into a second A buffer, group B's
    fill of pass k+1 waiting on the device for pass k's walk before it reuses
    B's buffers).  20 mixed shapes, three passes: every pass's plane
    checksums and results (gx_staged_pass_results), the last pass's
    alignments, against the oracle; the pipeline must have run (groups == 2)."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    monkeypatch.setenv("GX_OVERLAP", "1")   # (by default from n >= 16,384)
    if launch_env == "w4_grid3":   # bands queued for three workgroups per launch: the two launches interleave
        monkeypatch.setenv("GX_BAND_WAVES", "4")
        monkeypatch.setenv("GX_FILL_GRID", "3")
    rng = random.Random(2024)
    shapes = [(1300 + 97 * k, 1100 + 61 * ((k * 7) % 20)) for k in range(20)]
    pairs = [(bytes(rng.choice(b"ACGT") for _ in range(n)), bytes(rng.choice(b"ACGT") for _ in range(m)))
             for n, m in shapes]
    steps = 3
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*CONFIG_SCORES), False, keep_planes=True, steps=steps, plane_sums=True)
    info = ctx.fill_info()
    assert info["groups"] == 2 and info["twin"] == 1 and info["plane_bytes_per_cell"] == 1.5, info
    sums = st.plane_sums()
    passes = st.pass_results()
    assert len(passes) == steps
    for p, (a, b) in enumerate(pairs):
        o = oracle.align_lean(a, b, CONFIG_SCORES)
        want = (o.score, o.matches, o.mismatches, o.gap_extensions, o.opening_gaps, len(o.choices))
        for k in range(steps):
            assert [int(x) for x in sums[k, p]] == o.extra["plane_sums"], (p, len(a), len(b), k)
            r = passes[k][p]
            assert (r.score, r.matches, r.mismatches, r.gap_extensions, r.opening_gaps, r.n_steps) == want, (p, k)
        assert _steps_list(st.steps(p)) == o.alignment(), (p, len(a), len(b))


@pytest.mark.parametrize("variant", ["twin_codes", "byte_planes", "int32", "local_twin"])
def test_staged_table_export(gx, ctx, oracle, monkeypatch, variant):
    """The batch formats handed over as tables (gx_staged_table): a staged
    run keeps its last pass's planes on the device (GX_STAGED_KEEP_PLANES)
    and each pair's table exports, row by row, the reference's I, D, S planes
    (algo.rs:172, 281) -- decoded from the twin fill's 12-bit plane codes (the
    headline's format), the byte planes, or int32 -- equal to the oracle's
    whole planes; plane checksums too.  Rows cover the strip and twin-half
    boundaries; pairs of unequal shapes so twins mix lengths."""
    env = {"twin_codes": {"GX_TWIN": "1"}, "byte_planes": {"GX_TWIN": "0"}, "int32": {"GX_PLANES32": "1"},
           "local_twin": {"GX_TWIN": "1", "GX_OVERLAP": "0"}}[variant]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    local = variant == "local_twin"
    rng = np.random.default_rng(17)
    pairs = []
    for k in range(24):
        n = int(rng.integers(200, 700)) if k % 3 else 640
        m = int(rng.integers(200, 700)) if k % 3 else 512
        a = bytes(rng.choice(list(b"ACGT"), n))
        b = bytearray(a[:m] if m <= n else a + bytes(rng.choice(list(b"ACGT"), m - n)))
        for _ in range(m // 10):   # related pairs: long local alignments for the local variant
            b[int(rng.integers(0, m))] = int(rng.choice(list(b"ACGT")))
        pairs.append((a, bytes(b)))
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*CONFIG_SCORES), local, keep_planes=True, steps=2, keep=True)
    info = ctx.fill_info()
    want_bpc = {"twin_codes": 1.5, "byte_planes": 3, "int32": 12, "local_twin": 1.5}[variant]
    assert info["plane_bytes_per_cell"] == want_bpc and info["layout"] == 0, info
    for p in (0, 1, 5, 12, 23):
        a, b = pairs[p]
        o = oracle.align(a, b, CONFIG_SCORES, is_local=local, want_planes=True)
        assert res[p].score == o.score, p
        t = st.table(p)
        for which in range(3):
            got = np.concatenate([t.rows(which, r0, min(200, len(a) + 1 - r0)) for r0 in range(0, len(a) + 1, 200)])
            assert np.array_equal(got, o.planes[which]), (variant, p, which)
        t.free()
    with pytest.raises(gx.GxError):   # the staged run's alignment is gx_staged_steps; a staged table has no retrace
        gx.retrace(gx.SequenceContainer([gx.Sequence("a", pairs[0][0].decode()), gx.Sequence("b", pairs[0][1].decode())]),
                   st.table(0), local)
