"""CPU: the twin fill's int16 admission rule (gx_api_plan.cpp twin_width /
gx_twin_admission) against brute-force spreads measured with the oracle.

The twin fill (genomics-rs_amd/csrc/gx_fill_pk.hip) keeps every value of a
band as an int16 offset from a base taken from the band's top row: the
score_max of the first column of a 16-column block, inherited strip to strip
(each strip adopts the base of the block it consumes, so strip k's base column
lies up to 64 (k + 1) + 16 columns right of the cell).  The host
admits a band width W only when D (192 W + 16 + dm) + 2 (|a| + |smax| + |smin|)
+ 64 < 30,000, with D the largest neighbour difference of the shifted values
V'' = V - (i + j) g (the range proof of DESIGN.md 4.2).

Here, for the inputs that push values hardest (all-mismatch, all-match, long
forced gap runs either way, low-entropy repeats, random DNA) and for the widest
scores each band width still admits, the oracle's planes (algo.rs:151-282
restated) give every cell's I'', D'', S'' and score_max''; every cell of strip
k of every band is compared with every base the kernel could hold for it (the
band's top-row score_max'' over columns j - 32 .. j + 64 (k + 1) + 32 + dm),
and the largest spread must stay within the per-strip term of the rule,
D (192 (k + 1) + 16 + dm), which the admitted bound dominates.  A rule one term
short would show here as a spread above it.
"""
import numpy as np
import pytest

from conftest import CONFIG_SCORES

ROWS = 128   # rows per anti-diagonal strip (gx_internal.h kStripRows)


def _families(n, m):
    rng = np.random.default_rng(n * 31 + m)
    dna = lambda k: bytes(rng.choice(list(b"ACGT"), size=k).tolist())
    return {
        "all_mismatch": (b"A" * n, b"C" * m),
        "all_match": (b"A" * n, b"A" * m),
        "gap_rows": (dna(n), dna(max(1, m // 12))),        # n >> m: forced delete runs
        "gap_cols": (dna(max(1, n // 12)), dna(m)),        # m >> n: forced insert runs
        "repeat": ((b"AC" * n)[:n], (b"CA" * m)[:m]),
        "random": (dna(n), dna(m)),
    }


def _neighbour_d(scores):
    sm, smm, g, h = scores
    a = h + g
    smax, smin = max(sm, smm), min(sm, smm)
    U = max(0, smax - a)
    return max(abs(a - g), abs(U - g))


def _max_spread_ratio(planes, g, W, dm, local=False):
    """Largest spread of strip k over its per-strip bound term, over every
    band and strip: max |V''(i, j) - SM''(r0, c)| / (192 (k + 1) + 16 + dm).
    local: score_max carries the 0 floor (algo.rs:103), no shift (g = 0)."""
    from scipy.ndimage import maximum_filter1d, minimum_filter1d
    I, D, S = (p.astype(np.int64) for p in planes)
    n1, m1 = I.shape
    ii = np.arange(n1)[:, None]
    jj = np.arange(m1)[None, :]
    shift = (ii + jj) * g
    SM = np.maximum(np.maximum(I, D), S) - shift
    if local:
        SM = np.maximum(SM, 0)
    worst = 0.0
    band_rows = ROWS * W
    for r0 in range(0, n1 - 1, band_rows):
        top = SM[r0].copy()
        for k in range(W):
            lo_r, hi_r = r0 + ROWS * k + 1, min(r0 + ROWS * (k + 1), n1 - 1)
            if lo_r > hi_r:
                break
            sl = slice(lo_r, hi_r + 1)
            vals = [I[sl, 1:] - shift[sl, 1:], D[sl, 1:] - shift[sl, 1:], S[sl, 1:] - shift[sl, 1:],
                    SM[sl, 1:]]
            vmax = np.max(np.stack([v.max(axis=0) for v in vals]), axis=0)
            vmin = np.min(np.stack([v.min(axis=0) for v in vals]), axis=0)
            # bases over c in [j - 32, j + 64 (k + 1) + 32 + dm], clamped to [0, m]
            left, right = 32, 64 * (k + 1) + 32 + dm
            size = left + right + 1
            pad_hi = np.concatenate([top, np.full(right, top[-1])])
            pad = np.concatenate([np.full(left, top[0]), pad_hi])
            # window for column j (1..m) covers pad[j .. j + size - 1] (pad index = c + left)
            wmax = maximum_filter1d(pad, size, origin=-(size // 2))[1:m1]
            wmin = minimum_filter1d(pad, size, origin=-(size // 2))[1:m1]
            spread = max(int((vmax - wmin).max()), int((wmax - vmin).max()))
            worst = max(worst, spread / (192 * (k + 1) + 16 + dm))
    return worst


# the default scores; the widest scores each band width admits (D = 10 at
# W = 15, D = 19 at W = 8, D = 38 at W = 4: the largest neighbour differences
# the rule lets through); a wide-gap and a match-heavy scoring
SCORES = [(CONFIG_SCORES, 15), ((1, -1, -1, -7), 15), ((1, -1, -1, -16), 8), ((2, -2, -1, -34), 4),
          ((5, -4, 0, -10), 8), ((1, -2, -2, -5), 15)]


@pytest.mark.parametrize("scores,W", SCORES)
def test_admission_rule_matches_width(gx, scores, W):
    """gx_twin_admission admits exactly the widths run_fill would pick: W
    itself, and not the next wider instantiated width."""
    ok, bound = gx.twin_admission(gx.Scores(*scores), W, 0)
    assert ok and bound < 30000, (scores, W, bound)
    wider = {4: 7, 7: 8, 8: 15}.get(W)
    if wider:
        assert not gx.twin_admission(gx.Scores(*scores), wider, 0)[0], (scores, wider)
    d = _neighbour_d(scores)
    sm, smm, g, h = scores
    assert bound == d * (192 * W + 16) + 2 * (abs(h + g) + abs(max(sm, smm)) + abs(min(sm, smm))) + 64


def test_admission_column_gap(gx):
    """Twins 1,024 columns apart: admitted at W = 8, not at W = 15 (default
    scores); the gap cap twin_table applies keeps W = 15 for gaps <= 843."""
    s = gx.Scores(*CONFIG_SCORES)
    assert gx.twin_admission(s, 8, 1024)[0]
    assert not gx.twin_admission(s, 15, 1024)[0]
    assert gx.twin_admission(s, 15, 843)[0] and not gx.twin_admission(s, 15, 844)[0]


@pytest.mark.parametrize("scores,W", SCORES)
@pytest.mark.parametrize("family", ["all_mismatch", "all_match", "gap_rows", "gap_cols", "repeat", "random"])
def test_spread_within_rule(oracle, scores, W, family):
    """Brute force: every state of every strip of every band stays within the
    rule's per-strip term of every base the kernel could hold for it."""
    n = ROWS * W * 2 + 300          # two full bands and a partial third
    m = 1400
    a, b = _families(n, m)[family]
    o = oracle.align(a, b, scores, want_planes=True)
    ratio = _max_spread_ratio(o.planes, scores[2], W, 0)
    d = _neighbour_d(scores)
    assert ratio <= d, (family, scores, W, ratio, d)


def test_spread_unequal_twins(oracle):
    """A twin's shorter pair 1,024 columns narrower (the margin dm): its
    values against bases up to dm further right stay within the rule at W = 8."""
    W, dm = 8, 1024
    rng = np.random.default_rng(5)
    n, m = ROWS * W + 200, 900
    a = bytes(rng.choice(list(b"ACGT"), size=n).tolist())
    b = bytes(rng.choice(list(b"AC"), size=m).tolist())
    o = oracle.align(a, b, CONFIG_SCORES, want_planes=True)
    assert _max_spread_ratio(o.planes, CONFIG_SCORES[2], W, dm) <= _neighbour_d(CONFIG_SCORES)


# Local twins (gx_fill_pk.hip LOCAL) keep plain values relative to the same
# per-block bases: the neighbour difference of the unshifted local values is
# max(|a|, U) (d8_planes_ok's inequalities, which the 0 floor keeps), and the
# constants carry the floor's offsets (K = max(0, -s_min), |g|).
def _neighbour_d_local(scores):
    sm, smm, g, h = scores
    a = h + g
    return max(abs(a), max(0, max(sm, smm) - a), 1)


LOCAL_SCORES = [(CONFIG_SCORES, 15), ((2, -3, -1, -5), 15), ((3, -2, -1, -3), 15), ((1, -1, -1, -16), 8)]


@pytest.mark.parametrize("scores,W", LOCAL_SCORES)
def test_local_admission_rule(gx, scores, W):
    """gx_twin_admission_mode(is_local=1): the local rule's bound, admitted at W."""
    ok, bound = gx.twin_admission(gx.Scores(*scores), W, 0, is_local=True)
    sm, smm, g, h = scores
    const = 2 * (abs(h + g) + abs(max(sm, smm)) + abs(min(sm, smm))) + 64 + max(0, -min(sm, smm)) + abs(g)
    assert bound == _neighbour_d_local(scores) * (192 * W + 16) + const
    assert ok and bound < 30000, (scores, W, bound)


@pytest.mark.parametrize("scores,W", LOCAL_SCORES)
@pytest.mark.parametrize("family", ["all_mismatch", "all_match", "gap_rows", "gap_cols", "repeat", "random"])
def test_local_spread_within_rule(oracle, scores, W, family):
    """Brute force, local mode: every state of every strip of every band stays
    within the local rule's per-strip term of every base the kernel could hold
    for it (plain values: no shift)."""
    n = ROWS * W * 2 + 300
    m = 1400
    a, b = _families(n, m)[family]
    o = oracle.align(a, b, scores, is_local=True, want_planes=True)
    ratio = _max_spread_ratio(o.planes, 0, W, 0, local=True)
    assert ratio <= _neighbour_d_local(scores), (family, scores, W, ratio)
