"""CPU checks of the compact plane formats' arithmetic:
the twin plane code of gx_fill_pk.hip (w16_code) and its decoder in
plane_sums_kernel (mode 3) are exact over the whole admitted range, and the
admission bounds of gx_api_plan.cpp (d8_planes_ok, w16_ok) hold for the default
scores.  Pure integer arithmetic: no GPU, no library call."""
import numpy as np


def _encode(xI, xS, xD):
    # v_pk_mad_u16 twice on 16-bit lanes: x_I + 16 x_S + 512 x_D (mod 2^16)
    return (xI + 16 * xS + 512 * xD) & 0xFFFF


def _decode(code):
    # plane_sums_kernel mode 3
    xI = code & 15
    r = code >> 4
    xS = ((r << 27) & 0xFFFFFFFF).astype(np.int64)
    xS = np.where(xS >= 2 ** 31, xS - 2 ** 32, xS) >> 27
    t = ((((r - xS) & 0xFFFFFFFF) >> 5) << 25) & 0xFFFFFFFF
    xD = np.where(t >= 2 ** 31, t - 2 ** 32, t) >> 25
    return xI, xS, xD


def test_twin_code_roundtrip_full_range():
    xI, xS, xD = np.meshgrid(np.arange(0, 16), np.arange(-16, 16), np.arange(-64, 64), indexing="ij")
    xI, xS, xD = (a.ravel().astype(np.int64) for a in (xI, xS, xD))
    code = _encode(xI, xS, xD)
    assert len(np.unique(code)) == code.size == 1 << 16   # a bijection onto 16 bits
    dI, dS, dD = _decode(code.astype(np.int64))
    assert np.array_equal(dI, xI) and np.array_equal(dS, xS) and np.array_equal(dD, xD)


def _ranges(sm, smm, g, h):
    # a = h + g, U = max(0, smax - a); shifted x_I in [0, U - a - g]
    a = h + g
    smax, smin = max(sm, smm), min(sm, smm)
    U = max(0, smax - a)
    return (0, U - a - g), (smin - U, smax - 2 * a), (2 * a - U, U - 2 * a)


def test_default_scores_fit_both_formats():
    rI, rS, rD = _ranges(1, -2, -1, -5)                      # config.toml
    assert (rI, rS, rD) == ((0, 14), (-9, 13), (-19, 19))
    assert 0 <= rI[0] and rI[1] <= 15 and -16 <= rS[0] and rS[1] <= 15 and -64 <= rD[0] and rD[1] <= 63
    assert min(-1, rS[0], rD[0]) >= -128 and max(rI[1], rS[1], rD[1]) <= 127


def test_shifted_score_tables_fit_a_byte():
    # gx_api_fill.cpp twin_tbl: the score tables hold s - 2g for match and mismatch
    sm, smm, g = 1, -2, -1
    assert 0 <= sm - 2 * g <= 255 and 0 <= smm - 2 * g <= 255
