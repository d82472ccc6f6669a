"""CPU checks of the compact plane formats' arithmetic.

The twin plane code (gx_fill_pk.hip w16_code: code = S + 32 D - 33 I mod 2^16
on the offset-binary halves the fill holds), its 12-bit records (gx_device.h
w12_pack / w12_unpack: a lane's four steps of one row for both pairs of a
twin in 12 B) and its decoder (gx_kernels.hip w16_decode: x_S =
sext5(code & 31), x_D = sext12(code - x_S) >> 5) are exact over the whole
admitted range; the format stores no x_I, so every decoder replays the insert
recurrence along the row (w16_next_I: I(i, j) = I(i, j-1) + g + max(0,
max(x_S, x_D)(i, j-1) + h), local then max(., 0); algo.rs:231-236) -- checked
here against the oracle's insert plane -- and local_col_kernel composes that
replay in chunks as maps x -> max(x + A, B) (checked against the serial
replay).  The admission bounds of gx_api_plan.cpp (d8_planes_ok, w16_ok) are
restated.  Pure integer arithmetic: no GPU, no library call."""
import random

import numpy as np
import pytest

BIAS = 0x8000   # gx_fill_pk.hip kBias2: every 16-bit half holds value + 0x8000


def _pmad(a, b, c):
    # v_pk_mad_u16 on one 16-bit half: a * b + c (mod 2^16)
    return (a * b + c) & 0xFFFF


def _encode(I, D, S):
    # w16_code: pmad(I, 0xFFDF, pmad(D, 0x0020, S)) on the biased halves
    return _pmad((I + BIAS) & 0xFFFF, 0xFFDF, _pmad((D + BIAS) & 0xFFFF, 0x0020, (S + BIAS) & 0xFFFF))


def _decode(code):
    # w16_decode: x_S = sext5(code & 31), x_D = (int)((code - x_S) << 20) >> 25 (12 significant bits)
    code = np.asarray(code, np.int64) & 0xFFF
    xS = ((code & 31) ^ 16) - 16
    t = (code - xS) & 0xFFF
    t = np.where(t >= 0x800, t - 0x1000, t)
    return xS, t >> 5


def _perm(a, b, sel):
    """v_perm_b32 a, b, sel for selectors 0-7: bytes 0-3 of b, then 4-7 of a."""
    src = [(b >> (8 * k)) & 0xFF for k in range(4)] + [(a >> (8 * k)) & 0xFF for k in range(4)]
    return sum(src[(sel >> (8 * k)) & 0xFF] << (8 * k) for k in range(4))


def _w12_pack(d):
    """gx_device.h w12_pack: the four steps' dwords (code_A | code_B << 16) -> 12 B."""
    w0 = _perm(d[1], d[0], 0x06040200)
    w1 = _perm(d[3], d[2], 0x06040200)
    n01, n23 = _perm(d[1], d[0], 0x07050301), _perm(d[3], d[2], 0x07050301)
    w2 = (n01 & 0x0F0F0F0F) | ((n23 << 4) & 0xF0F0F0F0)
    return w0, w1, w2


def _w12_unpack(w0, w1, w2):
    """gx_device.h w12_unpack."""
    n = (w2 >> 4) & 0x0F0F0F0F
    return [_perm(w2, w0, 0x05010400) & 0x0FFF0FFF, _perm(w2, w0, 0x07030602) & 0x0FFF0FFF,
            _perm(n, w1, 0x05010400), _perm(n, w1, 0x07030602)]


def test_twin_code_roundtrip_full_range():
    """Every (x_S, x_D) of the format's fields -- x_S 5 signed bits, x_D 7 --
    on random insert scores (the bias cancels: 1 + 32 - 33 = 0) decodes
    exactly from the code's low 12 bits, and those are a bijection onto the
    12-bit values."""
    xS, xD = np.meshgrid(np.arange(-16, 16), np.arange(-64, 64), indexing="ij")
    xS, xD = xS.ravel().astype(np.int64), xD.ravel().astype(np.int64)
    rng = np.random.default_rng(7)
    I = rng.integers(-30000, 30000, xS.size)   # values relative to a base (the admission bound < 30,000)
    code = _encode(I, I + xD, I + xS)
    assert len(np.unique(code & 0xFFF)) == code.size == 1 << 12
    dS, dD = _decode(code)
    assert np.array_equal(dS, xS) and np.array_equal(dD, xD)


def test_w12_records_roundtrip():
    """w12_pack / w12_unpack on random 16-bit codes of both pairs (the fill's
    dwords carry garbage above bit 11 of each half): the unpacked dwords are
    the codes' low 12 bits, so every decoder sees the codes it saw before."""
    rng = random.Random(3)
    for _ in range(20000):
        d = [rng.getrandbits(32) for _ in range(4)]
        w = _w12_pack(d)
        assert all(0 <= x < 1 << 32 for x in w)
        assert _w12_unpack(*w) == [x & 0x0FFF0FFF for x in d]


def _replay_rows(planes, h, g, local):
    """I of every interior cell from the row start and the codes' x_S, x_D
    (w16_next_I); returns the rebuilt insert plane's interior."""
    I_pl, D_pl, S_pl = planes
    n1, m1 = I_pl.shape
    xS = S_pl - I_pl
    xD = D_pl - I_pl
    out = np.zeros((n1 - 1, m1 - 1), np.int64)
    for i in range(1, n1):
        D0 = h + i * g
        I = (max(D0, 0) if local else D0) + h     # H(i, 0) + h, as the fill seeds it
        mp = 0 if local else -h                   # its max(S, D) - I
        for j in range(1, m1):
            I = I + g + max(0, mp + h)
            if local:
                I = max(I, 0)
            out[i - 1, j - 1] = I
            mp = max(xS[i, j], xD[i, j])
    return out


@pytest.mark.parametrize("scores", [(1, -2, -1, -5), (1, -2, -2, -5), (2, -3, -1, -4), (1, -1, 0, 0),
                                    (3, -3, -1, -1)])
@pytest.mark.parametrize("is_local", [False, True], ids=["global", "local"])
def test_insert_replay_matches_oracle(oracle, scores, is_local):
    """The decoders' replay of I along a row equals the oracle's insert
    plane, and x_S, x_D stay inside the format's fields, on dense-tie and
    long-match inputs (alphabets A, AC, ACGT)."""
    sm, smm, g, h = scores
    rng = random.Random(hash(scores) & 0xfff)
    for n, m, alpha in ((37, 150, b"ACGT"), (64, 90, b"AC"), (20, 200, b"A"), (90, 33, b"ACGT")):
        a = bytes(rng.choice(alpha) for _ in range(n))
        b = bytes(rng.choice(alpha) for _ in range(m))
        o = oracle.align(a, b, scores, is_local=is_local, want_planes=True)
        I_pl, D_pl, S_pl = (np.asarray(p, np.int64) for p in o.planes)
        got = _replay_rows((I_pl, D_pl, S_pl), h, g, is_local)
        assert np.array_equal(got, I_pl[1:, 1:]), (scores, n, m, alpha)
        xS = (S_pl - I_pl)[1:, 1:]
        xD = (D_pl - I_pl)[1:, 1:]
        if _w16_ok(*scores):
            assert -16 <= xS.min() and xS.max() <= 15 and -64 <= xD.min() and xD.max() <= 63
            code = _encode(I_pl[1:, 1:], D_pl[1:, 1:], S_pl[1:, 1:])
            dS, dD = _decode(code)
            assert np.array_equal(dS, xS) and np.array_equal(dD, xD)


def test_local_chunked_composition():
    """local_col_kernel: each lane's chunk of the row applies x -> max(x + A,
    B); the exclusive scan of the composed maps gives every chunk its first I
    exactly as the serial replay does (random steps, chunk sizes, 64 lanes)."""
    rng = random.Random(11)
    low = -(1 << 29)
    for _ in range(200):
        g, h = -rng.randint(0, 3), -rng.randint(0, 6)
        m = rng.randint(1, 700)
        mps = [rng.randint(-20, 20) for _ in range(m)]   # max(x_S, x_D) of each column
        # serial replay (local): I(0) = h, mp(0) = 0
        I, mp, serial = h, 0, []
        for j in range(m):
            serial.append(I)   # I before column j + 1
            I = max(I + g + max(0, mp + h), 0)
            mp = mps[j]
        C = (m + 63) // 64
        maps = []
        for lane in range(64):
            j0, j1 = lane * C, min(m, lane * C + C)
            A, B = 0, low
            mp = mps[j0 - 1] if 1 <= j0 < m else 0
            for j in range(j0, j1):
                dj = g + max(0, mp + h)
                A += dj
                B = max(B + dj, 0)
                mp = mps[j]
            maps.append((A, B))
        EA, EB = 0, low
        for lane in range(64):
            j0 = lane * C
            if j0 < m:
                assert max(h + EA, EB) == serial[j0], (lane, g, h, m)
            A, B = maps[lane]
            EA, EB = EA + A, max(EB + A, B)


def _ranges(sm, smm, g, h):
    # a = h + g, U = max(0, smax - a); shifted x_I in [0, U - a - g]
    a = h + g
    smax, smin = max(sm, smm), min(sm, smm)
    U = max(0, smax - a)
    return (0, U - a - g), (smin - U, smax - 2 * a), (2 * a - U, U - 2 * a)


def _w16_ok(sm, smm, g, h):
    """gx_api_plan.cpp w16_ok: x_S fits the code's 5 signed bits and x_D
    the other 7 of its 12 (g, h <= 0)."""
    if g > 0 or h > 0:
        return False
    _, (sl, sh), (dl, dh) = _ranges(sm, smm, g, h)
    return -16 <= sl and sh <= 15 and -64 <= dl and dh <= 63


def test_default_scores_fit_both_formats():
    rI, rS, rD = _ranges(1, -2, -1, -5)                      # config.toml
    assert (rI, rS, rD) == ((0, 14), (-9, 13), (-19, 19))
    assert _w16_ok(1, -2, -1, -5)
    assert min(-1, rS[0], rD[0]) >= -128 and max(rI[1], rS[1], rD[1]) <= 127
    # the insert difference no longer limits the code: (2, -3, -2, -4) has
    # U - a - g = 16 (the old 4-bit field) and is admitted; (5, -4, 0, -10)
    # has x_S down to -19 and is not
    assert _w16_ok(2, -3, -2, -4) and not _w16_ok(5, -4, 0, -10)


def test_shifted_score_tables_fit_a_byte():
    # gx_api_fill.cpp twin_tbl: the score tables hold s - 2g for match and mismatch
    sm, smm, g = 1, -2, -1
    assert 0 <= sm - 2 * g <= 255 and 0 <= smm - 2 * g <= 255
