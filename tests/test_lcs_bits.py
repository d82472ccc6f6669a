"""CPU restatement of the layout-3 tracked fill's max_matches rows
(genomics-rs_amd/csrc/gx_lcs.h): the bit-parallel LCS of algo.rs:250-256
(V' = (V + (V & M)) | (V & ~M) row by row, LM(i, j) = j - popcount(V_i &
(2^j - 1))) as the GPU sweeps it -- 64-row strips on the anti-diagonal skew,
lane l advancing word w = t - l of row 64 s + l + 1 at step t, the word of the
row above from lane l - 1's previous step (lane 0: the strip above's lane 63
at step t + 63), the row's carry kept in the lane (64 columns a word), masks
zero-padded 64 words on either side, the words stored as
bits[strip][step][lane] -- checked against the oracle's LCS plane and its
numpy row recurrence (oracle.lcs_rows), including None == None matches of
reverse_sequences and shapes around strip and word boundaries; and the
hand-off of a strip's bottom row to the next wave through the LDS ring (256
slots + 8 mirrored, published / consumed counters) under random
interleavings of the waves: every read sees the step it asks for."""
import random

import numpy as np
import pytest

M64 = (1 << 64) - 1
BITS = 64  # gx_internal.h kLcsBits: columns a word
PAD = 64   # gx_internal.h kLcsMaskPad


def lcs_steps(words):
    """gx_internal.h lcs_steps."""
    return (words + 64 + 31) & ~31


def lcs_word_index(i, w, words):
    """gx_internal.h lcs_word_index: word w of row i (1-based) in [strip][step][lane]."""
    s, l = (i - 1) // 64, (i - 1) % 64
    return (s * lcs_steps(words) + w + l) * 64 + l


def skew_sweep(c1, c2):
    """The GPU's sweep (gx_lcs.h lcs_workgroup) on Python ints: returns the
    bit words in their device layout and the word count."""
    n, m = len(c1), len(c2)
    wd = -(-m // BITS)
    T = lcs_steps(wd)
    S = -(-n // 64)
    ws = wd + 2 * PAD
    masks = {}
    for j, c in enumerate(c2):   # masks[b][PAD + w] bit k: s2[63 w + k] == b
        masks.setdefault(int(c), [0] * ws)[PAD + j // BITS] |= 1 << (j % BITS)
    zero = [0] * ws
    bits = [0] * (S * T * 64)
    above = None   # the strip above's lane-63 word of each of its steps
    for s in range(S):
        row_mask = [masks.get(int(c1[s * 64 + l]), zero) if s * 64 + l < n else masks.get(0, zero) for l in range(64)]
        carry = [0] * 64
        vo = [M64] * 64   # each lane's word of the previous step
        out63 = []
        for t in range(T):
            new = [0] * 64
            for l in range(64):
                if l == 0:
                    vin = above[t + 63] if (above is not None and t + 63 < T) else (M64 if s == 0 else 0)
                else:
                    vin = vo[l - 1]
                w = t - l
                mk = row_mask[l][PAD + w] if -PAD <= w < wd + PAD else 0
                tot = vin + (vin & mk) + carry[l]   # (lcs_block4: two 32-bit adds with carry)
                carry[l] = tot >> 64
                new[l] = (tot & M64) | (vin & ~mk)
                bits[(s * T + t) * 64 + l] = new[l]
            vo = new
            out63.append(new[63])
        above = out63
    return bits, wd


@pytest.mark.parametrize("n,m,alpha,rev", [
    (1, 1, b"A", False), (7, 5, b"ACGT", False), (20, 63, b"AC", False), (9, 64, b"ACGT", True),
    (64, 65, b"ACGT", False), (65, 128, b"A", False), (130, 129, b"AC", True), (70, 300, b"ACGT", False),
    (129, 700, b"ACGTN", True), (200, 64 * 5 + 3, b"AC", False), (66, 63, b"ACGT", False), (67, 126, b"AC", True), (3, 127, b"A", False),
])
def test_skew_sweep_matches_oracle(oracle, n, m, alpha, rev):
    rng = random.Random(n * 100003 + m)
    a = bytes(rng.choice(alpha) for _ in range(n))
    b = bytes(rng.choice(alpha) for _ in range(m))
    c1, c2 = oracle.processed_bytes(a, b, rev)
    bits, wd = skew_sweep(c1, c2)
    ref = oracle.lcs_rows(a, b, range(n + 1), rev=rev)
    for i in range(1, n + 1):
        ones = 0
        row = np.zeros(m + 1, np.int64)
        for j in range(1, m + 1):
            ones += (bits[lcs_word_index(i, (j - 1) // BITS, wd)] >> ((j - 1) % BITS)) & 1
            row[j] = j - ones
        assert np.array_equal(row, ref[i]), (n, m, rev, i)
    if n * m <= 20000:
        o = oracle.align(a, b, (1, -2, -1, -5), rev=rev, want_lcs=True)
        for i in range(n + 1):
            assert np.array_equal(ref[i], o.lcs[i]), ("numpy rows vs oracle plane", n, m, rev, i)


RING = 256   # gx_lcs.h kLcsRing


@pytest.mark.parametrize("seed", range(12))
def test_lds_ring_handoff(seed):
    """gx_lcs.h lcs_workgroup's LDS hand-off, interleaved at random: the
    producer (wave k, strips q = 0, 1, ...) writes its steps' words 8 at a
    time to slots (q T + t) mod 256 (+ mirror when the group starts at slot 0)
    once the consumer's counter has passed q T + t0 + 8 - 256, then publishes
    q T + t0 + 8; the consumer's group t0 waits for q T + min(t0 + 71, T),
    reads slots (q T + t0 + 63) mod 256 + 0..7 and publishes the same
    value.  Every needed read returns the producer's word of that step and
    the two never wait on each other forever."""
    rng = random.Random(seed)
    T = rng.choice([32, 64, 96, 160, 288, 544])
    Q = rng.randint(1, 4)
    ring = [None] * (RING + 8)
    pub = con = 0

    def producer():
        nonlocal pub
        for q in range(Q):
            for t0 in range(0, T, 8):
                G = q * T + t0
                while con < G + 8 - RING:
                    yield
                r0 = G % RING
                for k in range(8):
                    ring[r0 + k] = (q, t0 + k)
                    if r0 == 0:
                        ring[RING + k] = (q, t0 + k)
                pub = G + 8
                yield

    def consumer():
        nonlocal con
        for q in range(Q):
            for t0 in range(0, T, 8):
                need = min(t0 + 71, T)
                while pub < q * T + need:
                    yield
                r0 = (q * T + t0 + 63) % RING
                for k in range(8):
                    if t0 + 63 + k < need:   # (later steps: don't care)
                        assert ring[r0 + k] == (q, t0 + 63 + k), (T, q, t0, k)
                con = q * T + need
                yield

    waves = [producer(), consumer()]
    live = [True, True]
    for _ in range(10 ** 6):
        if not any(live):
            break
        k = rng.randrange(2)
        if live[k]:
            try:
                for _ in range(rng.randint(1, 20)):
                    next(waves[k])
            except StopIteration:
                live[k] = False
    assert not any(live), "hand-off stalled"
