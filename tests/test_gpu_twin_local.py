"""GPU parity of the local (Smith-Waterman) twin fill (gx_fill_pk.hip LOCAL):
batches of local alignments run two pairs per band on plain 16-bit values
relative to per-block bases, with the 0 floor of algo.rs:103 in every gap recurrence and a per-row
last-max tracker (algo.rs:310-322).  Every result -- the start cell through
the score, the alignment, the statistics and the compact score planes -- must
equal the oracle's local restatement (oracle/gx_oracle.c), on shapes around
the strip and band edges, tie-heavy inputs (all-mismatch tables are all
zeros, so the last maximum is cell (n, m)), scores with and without the
small-alphabet tables, and values past 2^15 (per-block bases)."""
import random

import pytest

from conftest import CONFIG_SCORES
from test_gpu_twin import LAUNCH, SHAPES, _steps_list, _twin_pairs
from test_twin_bound import _families

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _force_twin(monkeypatch):
    """Small batches: force the twin fill (run_fill's grid-fill rule)."""
    monkeypatch.setenv("GX_TWIN", "1")


@pytest.fixture(params=sorted(LAUNCH))
def launch(request, monkeypatch):
    for k, v in LAUNCH[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param


def _check(gx, ctx, oracle, pairs, scores, steps=1, twin=1):
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*scores), True, keep_planes=True, steps=steps, plane_sums=True)
    info = ctx.fill_info()
    assert info["twin"] == twin, info
    sums = st.plane_sums()
    for p, (a, b) in enumerate(pairs):
        o = oracle.align_lean(a, b, scores, is_local=True)
        for k in range(steps):
            assert [int(x) for x in sums[k, p]] == o.extra["plane_sums"], (p, len(a), len(b), k)
        assert (res[p].score, res[p].matches, res[p].mismatches, res[p].gap_extensions, res[p].opening_gaps) == \
               (o.score, o.matches, o.mismatches, o.gap_extensions, o.opening_gaps), (p, len(a), len(b))
        assert _steps_list(st.steps(p)) == o.alignment(), (p, len(a), len(b))
    return info


def _w16_ok(scores):
    """gx_api_plan.cpp w16_ok: the twin plane codes' field ranges (DESIGN.md
    4.4): x_S in 5 signed bits, x_D in 7 (12-bit codes; the format holds no
    x_I since round 5)."""
    sm, smm, g, h = scores
    a = h + g
    U = max(0, max(sm, smm) - a)
    return (g <= 0 and h <= 0 and min(sm, smm) - U >= -16 and max(sm, smm) - 2 * a <= 15 and 2 * a - U >= -64
            and U - 2 * a <= 63)


def test_local_twin_shapes(gx, ctx, oracle, launch):
    """Shapes around the strip / band edges, every band width and small grids
    (bands queued for workgroups); two pipelined passes."""
    _check(gx, ctx, oracle, _twin_pairs(23, SHAPES), CONFIG_SCORES, steps=2)


def _planted(rng, n, m, core, al=b"ACGT"):
    """Random rows and columns sharing a planted core with ~8 % substitutions
    (a long local alignment in the middle of the table)."""
    c = bytes(rng.choice(al) for _ in range(core))
    c2 = bytes(x if rng.random() > 0.08 else rng.choice(al) for x in c)
    a = bytes(rng.choice(al) for _ in range(rng.randint(0, n - core))) + c
    b = bytes(rng.choice(al) for _ in range(rng.randint(0, m - core))) + c2
    a += bytes(rng.choice(al) for _ in range(n - len(a)))
    b += bytes(rng.choice(al) for _ in range(m - len(b)))
    return a, b


# (scores, twin fill expected): the local twin needs the twin plane codes'
# ranges (gx_api_plan.cpp w16_ok: x_S in [-16, 15], x_D in [-64, 63]);
# (2, -3, -2, -4), whose insert difference (16) overflowed the pre-round-6
# rule's 4-bit x_I field, now takes it; (5, -4, 0, -10) (x_S down to -19)
# still runs the scalar local fill
@pytest.mark.parametrize("scores,twin", [(CONFIG_SCORES, 1), ((2, -3, -1, -4), 1), ((3, -2, -1, -3), 1),
                                         ((1, -1, 0, 0), 1), ((3, -3, -1, -1), 1), ((2, -3, -2, -4), 1),
                                         ((5, -4, 0, -10), 0)])
def test_local_twin_planted_cores(gx, ctx, oracle, monkeypatch, scores, twin):
    """A planted shared core per pair (a long local alignment inside the
    table, started at the last maximum), unequal twins; several scores."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    rng = random.Random(hash(scores) & 0xffff)
    pairs = [_planted(rng, n, m, core) for n, m, core in
             [(900, 700, 300), (700, 900, 250), (1500, 400, 200), (333, 1200, 150), (257, 256, 256), (129, 3000, 100)]]
    _check(gx, ctx, oracle, pairs, scores, twin=twin)


def test_local_twin_large_alphabet(gx, ctx, oracle, monkeypatch):
    """More than four symbols: the plain match test instead of the score
    tables (cell_pk without TBL), planted cores over 20 amino-acid letters."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    rng = random.Random(5)
    al = b"ACDEFGHIKLMNPQRSTVWY"
    pairs = [_planted(rng, n, m, core, al) for n, m, core in [(800, 600, 200), (600, 800, 300), (400, 400, 100)]]
    _check(gx, ctx, oracle, pairs, CONFIG_SCORES)


@pytest.mark.parametrize("family", ["all_mismatch", "all_match", "gap_rows", "gap_cols", "repeat"])
def test_local_twin_tie_families(gx, ctx, oracle, monkeypatch, family):
    """Inputs full of ties (all-zero tables, repeats, all-match diagonals)
    at W = 15 and 8: the last maximum in row-major order must be the
    reference's."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    for W in ("15", "8"):
        monkeypatch.setenv("GX_BAND_WAVES", W)
        pair = _families(128 * int(W) + 300, 1400)[family]
        _check(gx, ctx, oracle, [pair, (pair[0][:-37], pair[1][:-11])], CONFIG_SCORES)


@pytest.mark.parametrize("seed", range(4))
def test_local_twin_random_batches(gx, ctx, oracle, monkeypatch, seed):
    """Randomised local batches: shapes, alphabets, scores, band widths and
    grids; every result against the oracle."""
    rng = random.Random(4000 + seed)
    monkeypatch.setenv("GX_LAYOUT", "0")
    monkeypatch.setenv("GX_BAND_WAVES", rng.choice(["3", "4", "7", "8", "15"]))
    monkeypatch.setenv("GX_FILL_GRID", rng.choice(["1", "2", "5", "64"]))
    scores = rng.choice([CONFIG_SCORES, (1, -2, -2, -5), (2, -3, -1, -4), (1, -1, 0, -3), (3, -2, -1, -3)])
    al = rng.choice([b"ACGT", b"AC", b"ACGTN", b"ACDEFGHIKLMNPQRSTVWY"])
    pairs = [_planted(rng, n, m, rng.randint(1, min(n, m)), al)
             for n, m in [(rng.randint(2, 700), rng.randint(2, 700)) for _ in range(rng.randint(2, 9))]]
    _check(gx, ctx, oracle, pairs, scores, twin=1 if _w16_ok(scores) else 0)


def test_local_twin_large_values(gx, ctx, oracle, monkeypatch):
    """Values past 2^15 (per-block bases, gx_fill_pk.hip LOCAL): all-match
    twins at s = 2 reach 40,000 (20,000 columns) and 32,000; the relative
    floor clamps once a base exceeds 2^15, the row maxima fold into int32 at
    every base change.  Both bit-exact against the oracle."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    scores = (2, -3, -1, -5)
    assert gx.twin_admission(gx.Scores(*scores), 15, 10, is_local=True)[0]
    _check(gx, ctx, oracle, [(b"A" * 20000, b"A" * 20000), (b"A" * 15990, b"A" * 16000)], scores, twin=1)


def test_local_twin_64k_related(gx, ctx, monkeypatch):
    """Round-3 verdict item 7: 16 related 64k pairs (SURVEY 8(d) M1 variant,
    tests/golden/make_golden.py --related-local --length 65536) aligned
    locally take the twin fill by default (local scores reach ~38,000, past
    the int16 range of a fill on fixed bases); two pipelined passes, every
    pass's plane checksums and results, and the final alignments, against
    the oracle's digests."""
    import hashlib
    import json
    import os
    import sys

    import numpy as np

    from conftest import GOLDEN
    sys.path.insert(0, GOLDEN)
    import make_golden
    monkeypatch.delenv("GX_TWIN", raising=False)
    with open(os.path.join(GOLDEN, "synthetic_related_local_L65536.json")) as f:
        cases = json.load(f)["cases"]
    assert len(cases) == 16 and max(c["score"] for c in cases) > 32767
    pairs = [make_golden.related_pair(c["k"], 65536) for c in cases]
    st = gx.StagedPairs(pairs, ctx=ctx)
    res, _ = st.run(gx.Scores(*CONFIG_SCORES), True, keep_planes=True, steps=2, plane_sums=True)
    info = ctx.fill_info()
    assert info["twin"] == 1 and info["layout"] == 0, info
    sums = st.plane_sums()
    passes = st.pass_results()
    for p, c in enumerate(cases):
        for k in range(2):
            r = passes[k][p]
            assert [int(x) for x in sums[k, p]] == [int(x) for x in c["plane_sums"]], (p, k)
            assert (r.score, [r.matches, r.mismatches, r.gap_extensions, r.opening_gaps], r.n_steps) == \
                   (c["score"], c["stats"], c["n_steps"]), (p, k)
        steps = st.steps(p)
        h = hashlib.sha256()
        h.update(bytes(steps["choice"].astype(np.uint8)))
        h.update(steps["i"].astype("<u8").tobytes())
        h.update(steps["j"].astype("<u8").tobytes())
        assert h.hexdigest() == c["alignment_sha256"], p
    ctx.trim()


def test_local_twin_overlapped(gx, ctx, oracle, monkeypatch):
    """A long-pair local batch (>= 16 pairs, n >= 16,384) takes the overlapped
    two-group pipeline (gx_api_batch.cpp batch_core_overlap): each pass's walk runs
    beside the next pass's fill and reads its start cells (the last maxima,
    finalize_kernel's PairRes) on the device.  Three passes, every result of
    every pass against the oracle."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    monkeypatch.setenv("GX_OVERLAP", "1")   # (local batches take it by default from 64 pairs)
    rng = random.Random(321)
    pairs = [_planted(rng, 4300 + 37 * k, 2500 + 53 * k, 600 + 40 * k) for k in range(18)]
    info = _check(gx, ctx, oracle, pairs, CONFIG_SCORES, steps=3)
    assert info["groups"] == 2, info


def test_local_twin_align_batch(gx, ctx, oracle, monkeypatch):
    """gx_align_batch (the drop-in batch call, no planes asked for) on local
    pairs: the local twin fill with its plane codes kept as scratch for the
    walk; every alignment and statistic against the oracle."""
    monkeypatch.setenv("GX_LAYOUT", "0")
    rng = random.Random(808)
    pairs = [_planted(rng, n, m, c) for n, m, c in [(900, 700, 300), (700, 900, 250), (1500, 400, 200),
                                                    (333, 1200, 150), (257, 256, 256), (5, 5, 1), (6, 5, 2)]]
    out = gx.align_batch(pairs, gx.Scores(*CONFIG_SCORES), True, ctx=ctx, max_cell=False)
    assert ctx.fill_info()["twin"] == 1, ctx.fill_info()
    for (a, b), (steps, r) in zip(pairs, out):
        o = oracle.align(a, b, CONFIG_SCORES, is_local=True)
        assert _steps_list(steps) == o.alignment(), (len(a), len(b))
        assert (r.score, r.matches, r.mismatches, r.gap_extensions, r.opening_gaps) == \
               (o.score, o.matches, o.mismatches, o.gap_extensions, o.opening_gaps), (len(a), len(b))
