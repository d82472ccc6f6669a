// gx_api_plan.cpp -- launch planning on the host: the exact-int32 range
// guard and analytic boundary cells (algo.rs:193-220), the fill layout /
// band width / plane format choice, twin pairing, batch chunks, and the
// planning queries of the C ABI (gx_plan_layout, gx_twin_admission*,
// gx_plane_bytes_per_cell).
#include "gx_api.h"

// ---------------------------------------------------------------------------
// scoring: exact-int32 guard (DESIGN.md "Integer range")

static int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static int64_t wmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }

// `wide` (may be NULL): set when the job is outside the exact-int32 range of
// the main fill and must take the int64 fill (gx_wide.hip) instead; with
// wide == NULL such a job is refused with GX_ERANGE.
int check_scores(const gx_scores* s, size_t n, size_t m, HostScores* hs, Scores32* sc, int is_local,
                 bool* wide) {
    if (!s) return fail(GX_EINVAL, "scores is NULL");
    hs->sm = s->s_match; hs->smm = s->s_mismatch; hs->g = s->g; hs->h = s->h;
    const uint64_t ugh = (uint64_t)s->g + (uint64_t)s->h;   // g + h as the reference's release build adds it
    const int64_t gh = (int64_t)ugh;
    hs->neg_inf = wadd(INT64_MIN, gh < 0 ? (int64_t)(0 - ugh) : gh);
    if (wide) *wide = false;
    if (n >= (size_t)1 << 30 || m >= (size_t)1 << 30) return fail(GX_ERANGE, "sequence longer than 2^30");
    const char* why = nullptr;
    const uint64_t lim = (uint64_t)1 << 24;
    auto mag = [](int64_t v) { return v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v; };
    if (mag(s->s_match) > lim || mag(s->s_mismatch) > lim || mag(s->g) > lim || mag(s->h) > lim)
        why = "score magnitudes above 2^24 are outside the exact int32 device range";
    // The reference adds g and h+g to neg_inf at the boundary; when that
    // wraps (possible only for g < 0 < h with |g+h| < |g|) its release build
    // produces wrapped giants that the int32 path cannot reproduce.
    else if (s->g < 0 && mag(gh) < mag(s->g))
        why = "g < 0 < h with |g+h| < |g|: the reference's boundary arithmetic wraps";
    else {
        // every interior magnitude <= (n + m + 2) * (|sm| + |smm| + |g| + |h|) + |h|
        const double bound = (double)(n + m + 2) * (double)(mag(s->s_match) + mag(s->s_mismatch) + mag(s->g) +
                                                            mag(s->h)) + (double)mag(s->h);
        if (bound >= (double)(1 << 28)) why = "|score| bound exceeds 2^28: outside the exact int32 device range";
        else if (n > (size_t)1 << 26 || m > (size_t)1 << 26) why = "sequence longer than 2^26";
    }
    if (why) {
        if (!wide) return fail(GX_ERANGE, why);
        *wide = true;   // the int64 fill computes it
        return GX_OK;
    }
    sc->sm = (int)s->s_match; sc->smm = (int)s->s_mismatch; sc->g = (int)s->g; sc->h = (int)s->h;
    sc->hg = (int)(s->h + s->g);
    sc->floor_ = is_local ? 0 : kNeg;
    const char* dbg = getenv("GX_DEBUG_FLAGS");
    sc->dbg = dbg ? atoi(dbg) : 0;
    sc->shift = 0;
    for (int k = 0; k < 4; ++k) sc->sym[k] = -1;
    sc->koff = 0;
    return GX_OK;
}

// Boundary cell of the table (algo.rs:195-220), int64.
void boundary_cell(const HostScores& hs, uint64_t i, uint64_t j, int64_t* I, int64_t* D, int64_t* S) {
    if (i == 0 && j == 0) { *I = 0; *D = 0; *S = 0; }
    else if (j == 0) { *I = hs.neg_inf; *D = wadd(hs.h, wmul((int64_t)i, hs.g)); *S = hs.neg_inf; }
    else { *I = wadd(hs.h, wmul((int64_t)j, hs.g)); *D = hs.neg_inf; *S = hs.neg_inf; }
}
// score_max(cell, 0, 0, 0, is_local) (algo.rs:98-107)
int64_t smax(int64_t I, int64_t S, int64_t D, int local) {
    int64_t r = std::max(std::max(I, S), D);
    return std::max(r, local ? (int64_t)0 : INT64_MIN);
}

// Processed characters for is_match(i-1, j-1, rev) (sequence.rs:102-115).
// Without `rev` they are the bytes themselves.  With `rev`, index k of s1
// reads s1[m - k] and index k of s2 reads s2[n - k]; an index out of range
// (including a wrapped usize) is None, encoded 0xFF on both sides so that
// None == None matches.  Inputs containing 0xFF are rejected in rev mode.
int processed_chars(const uint8_t* s1, size_t n, const uint8_t* s2, size_t m, int rev,
                    std::vector<uint8_t>& c1, std::vector<uint8_t>& c2) {
    c1.assign(s1, s1 + n);
    c2.assign(s2, s2 + m);
    if (!rev) return GX_OK;
    for (size_t k = 0; k < n; ++k) if (s1[k] == 0xFF) return fail(GX_EINVAL, "byte 0xFF is reserved in reverse mode");
    for (size_t k = 0; k < m; ++k) if (s2[k] == 0xFF) return fail(GX_EINVAL, "byte 0xFF is reserved in reverse mode");
    for (size_t k = 0; k < n; ++k) {
        // i_processed = len(s2) - k
        c1[k] = (k <= m && (m - k) < n) ? s1[m - k] : 0xFF;
    }
    for (size_t k = 0; k < m; ++k) {
        // j_processed = len(s1) - k
        c2[k] = (k <= n && (n - k) < m) ? s2[n - k] : 0xFF;
    }
    return GX_OK;
}

// ---------------------------------------------------------------------------
// fill orchestration

// Persistent fill workgroups: one per CU by default (bands beyond the grid
// are taken from the queue as earlier bands finish; a band deep in a pair
// starts late anyway, so it loses little, and no CU runs two bands' waves).
int fill_grid_cap(int device) {
    if (const char* e = getenv("GX_FILL_GRID"); e && atoi(e) > 0) return atoi(e);
    static int cus = -1;
    if (cus < 0) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c < 1) c = 256;
        cus = c;
    }
    return cus;
}

// Band width: the narrowest instantiated width whose bands fit the grid
// (one band per workgroup, all strips in flight from the start) up to 8
// strips; beyond that 8-strip bands that queue for workgroups.  Measured on
// queued batches (profiles/r01i_widths.txt): 8 beats 11 and 15 everywhere
// (45 Covid pairs 845 -> 969 GCUPS, 20 x 30k 433 -> 496, 64 x 16k 485 -> 524)
// and ties 15 where 15 fits (16 x 30k).  GX_BAND_WAVES forces a width (if
// instantiated for the variant).
template <size_t N>
static int pick_width(const int (&ws)[N], int total_strips, int grid_cap) {
    if (const char* e = getenv("GX_BAND_WAVES")) {
        const int w = atoi(e);
        for (int x : ws) if (x == w) return w;
    }
    int queued = ws[0];
    for (int x : ws) {
        if (x > 8) break;
        if (ceil_div(total_strips, x) <= grid_cap) return x;
        queued = x;
    }
    return queued;
}
// min_strips: the fewest strips of any pair in the launch.
int fill_band_waves(bool track, int total_strips, int grid_cap, int lay, int min_strips) {
    // layout 1 starts at 4-strip bands: fewer HBM hand-offs for the same one
    // compute wave per SIMD (the I/O wave shares a SIMD but mostly sleeps)
    static constexpr int kWidths1[] = {4, 6, 8, 11, 15};
    if (track) return pick_width(kFillWidthsTrack, total_strips, grid_cap);
    if (lay) return pick_width(kWidths1, total_strips, grid_cap);
    const int w = pick_width(kFillWidths, total_strips, grid_cap);
    // Deep queues of long pairs: 15-strip bands (four compute waves per SIMD)
    // once every pair spans >= 200 strips (25.6k rows) and the queue holds
    // >= 2.5 rounds of them: 64 x 30k 50.9 -> 49.1 ms, 45 Covid pairs 32.3 ->
    // 30.5; shallower queues (16 x 30k: 15.0 vs 22.5 ms, 12 x 64k) and shorter
    // pairs (128 x 16k, 1024 x 4k) stay faster with 8 (profiles/r01o_round_sweep.txt)
    if (w == 8 && !getenv("GX_BAND_WAVES") && min_strips >= 200 && 2 * ceil_div(total_strips, 15) >= 5 * grid_cap)
        return 15;
    return w;
}

// Compact score planes (layout 0, untracked: the batch path).  The
// fill stores per cell one signed byte each of x_I = I(i,j) - I(i,j-1),
// x_S = S(i,j) - I(i,j), x_D = D(i,j) - I(i,j) (gx_kernels.hip put_byte), 3 B
// instead of 12.  With g, h <= 0, a = h + g, smax/smin the larger/smaller of
// the match and mismatch scores and U = max(0, smax - a), every interior cell
// satisfies (DESIGN.md section 4.2 has the derivation from algo.rs:231-248)
//     a <= H(i,j) - H(i,j-1) <= U   (and the same down a column),
//     H(i,j-1) + a <= I(i,j) <= H(i,j-1),   H(i-1,j) + a <= D(i,j) <= H(i-1,j),
// so  x_I in [g, U - a],  x_S in [smin - U, smax - 2a],  x_D in [2a - U, U - 2a].
// The same holds in local mode (the 0 floor of I, D and H keeps every
// inequality; the row base is H(i, 0) + h = h).  Compact planes are used when
// those ranges fit a signed byte (the default scores give [-1, 13], [-9, 13],
// [-19, 19]); GX_PLANES32 forces int32 planes.
bool d8_planes_ok(const Scores32& sc, int is_local) {
    (void)is_local;
    if (sc.g > 0 || sc.h > 0 || getenv("GX_PLANES32")) return false;
    const long long g = sc.g, a = (long long)sc.h + sc.g;
    const long long smax = std::max(sc.sm, sc.smm), smin = std::min(sc.sm, sc.smm);
    const long long U = std::max(0LL, smax - a);
    // (the shifted fill, Scores32.shift, stores x_I - g: in [0, U - a - g])
    const long long lo = std::min({g, smin - U, 2 * a - U}), hi = std::max({U - a - g, smax - 2 * a, U - 2 * a});
    return lo >= -128 && hi <= 127;
}

// Twin plane codes (gx_fill_pk.hip w16_code: code = x_S + 32 x_D, of which
// the record keeps 12 bits, gx_device.h w12_pack; the format holds no x_I,
// which every decoder replays along the row): x_S in [smin - U, smax - 2a]
// must fit the low 5 bits (signed) and x_D in [2a - U, U - 2a] the other 7
// (w16_decode), the bounds of d8_planes_ok; the default scores give [-9, 13]
// and [-19, 19].  (Until round 5 an insert difference x_I - g in
// [0, U - a - g] had a 4-bit field too; tests/test_formats.py restates the
// codec.)  GX_PLANES_W16=0 keeps the byte format.
bool w16_ok(const Scores32& sc) {
    if (sc.g > 0 || sc.h > 0 || getenv("GX_PLANES32")) return false;
    if (const char* e = getenv("GX_PLANES_W16"); e && !strcmp(e, "0")) return false;
    const long long a = (long long)sc.h + sc.g;
    const long long smax = std::max(sc.sm, sc.smm), smin = std::min(sc.sm, sc.smm);
    const long long U = std::max(0LL, smax - a);
    return smin - U >= -16 && smax - 2 * a <= 15 && 2 * a - U >= -64 && U - 2 * a <= 63;
}

// The split column step (gx_cs2.hip) replaces layout 1's one-wave strips for
// untracked fills; GX_CS2=0 keeps the one-wave kernel.  Band width: the
// narrowest instantiated width whose bands fit the grid (W = 2: every compute
// wave of a CU on its own SIMD), else 7-strip bands queued for workgroups
// (GX_BAND_WAVES forces an instantiated width).
// The split column step (gx_cs2.hip) by default for local fills only: on a
// 30k global pair its two-wave strips in two-strip bands lose to layout 1's
// one-wave strips in four-strip bands (more band hand-offs through HBM,
// 5.33 vs 4.53 ms; BRCA2 local 1.76 vs 1.79 ms, profiles/r03a_bench.json).
// GX_CS2=1 / 0 forces it on / off.  Local fills need g <= 0: the split
// core applies the shifted 0 floor, -(i + j) g, after the delete chain's
// prefix max, which is the reference's per-row floor (algo.rs:238-243) only
// while the floor does not decrease down the rows; with g > 0 a floor reached
// at an upper row must carry down the chain, which the one-wave column step
// does (its per-lane chain offsets) and the split core does not.
bool cs2_enabled(int is_local, const Scores32& sc) {
    if (is_local && sc.g > 0) return false;
    const char* e = getenv("GX_CS2");
    if (e && *e) return strcmp(e, "0") != 0;
    return is_local != 0;
}
// Layout 3 (gx_skew.hip): 2-strip bands, each strip's core and side wave on
// SIMDs of their own; GX_BAND_WAVES picks another instantiated width (1-3;
// must match gx_skew.hip launch_fill_skew).
int skew_band_waves() {
    if (const char* e = getenv("GX_BAND_WAVES")) {
        const int w = atoi(e);
        if (w >= 1 && w <= 3) return w;
    }
    return 2;
}
int cs2_band_waves(int total_strips, int grid_cap) {
    static constexpr int kCs2Widths[] = {1, 2, 3, 4, 7};
    if (const char* e = getenv("GX_BAND_WAVES")) {
        const int w = atoi(e);
        for (int x : kCs2Widths) if (x == w) return w;
    }
    for (int x : {2, 3, 4})
        if (ceil_div(total_strips, x) <= grid_cap) return x;
    return 7;
}

// Fill layout (gx_internal.h): 0 = anti-diagonal 128-row strips, 1 = column
// step over 64-row strips (delete chain as a wave prefix max; a strip follows
// the one above a few columns behind instead of 64+ steps), 3 = anti-diagonal
// 64-row strips with one row per lane (gx_skew.hip, the latency fill).
// GX_LAYOUT forces one.  Layout 1 offsets the delete chain by up to 64
// (|g| + |h|) inside the scan, so it needs that much int32 headroom above the
// range guard's 2^28.
//
// Default: a latency layout while the job is latency-bound -- its 64-row
// strips fit about two per SIMD (one to three 30k pairs); layout 0 from four
// 30k pairs on, where the band-major queue keeps every CU busy and layout 0's
// 2-row lanes issue fewer instructions per cell (four 30k pairs 7.7 vs 8.4
// ms, eight 10.6 vs 15.9 ms; profiles/r01o_round_sweep.txt,
// profiles/r01d_layouts.txt).  The latency layout is 3 for untracked fills
// with h <= 0 (its recurrences fold the gap opening onto score_max, which is
// exact only then) when it is predicted faster than the column step, else
// the column step (below: a fitted cost model per layout).
// Covid 29,903 x 29,882 global: layout 3 (4.52 vs 4.62 ms); BRCA2 11,382 x
// 10,346 local: the split column step (1.74 vs 1.79); 64 x 30,000: layout 3
// (1.5 vs 3.4).
// Layout 3 needs h <= 0 (the folded gap opening), small penalties for the
// virtual columns of its global ramp-up (values drift from -2^30 by up to 64
// steps of |g| + |h| + |s''|, s'' = s - 2g the shifted substitution score),
// and fewer than 2^24 - 128 columns: its skeleton holds E + 64 in the 24 bits
// tb_chase_kernel decodes, and a strip's int32 plane (256 (m + 64) bytes)
// must stay inside one buffer descriptor's 32-bit range.
// Tracked fills (max_cell, matches_at_max) run on it too (round 6: the side
// wave carries the first maximum, the launch's leading workgroups the LCS
// as bit rows, gx_lcs.h; GX_TABLE_MATCHES exports rebuild *_matches from them).
bool skew_ok(const Scores32& sc, bool /*lcs_plane*/, size_t mmax) {
    const long long g = sc.g;
    const long long s2 = std::max(std::llabs((long long)sc.sm - 2 * g), std::llabs((long long)sc.smm - 2 * g));
    const long long drift = 64LL * (std::llabs(g) + std::llabs((long long)sc.h) + s2);
    return sc.h <= 0 && drift < (1LL << 28) && mmax + 128 < (1u << 24);
}
int fill_layout(const std::vector<PairHost>& ph, const Scores32& sc, int grid_cap, bool track, bool lcs_plane) {
    const long long span = 65LL * (std::llabs((long long)sc.g) + std::llabs((long long)sc.h));
    size_t mmax = 0;
    long long strips64 = 0;
    for (const PairHost& h : ph) {
        mmax = std::max(mmax, h.m);
        strips64 += ceil_div((int)h.n, kStripRows1);
    }
    const bool cs_ok = span < (1LL << 29) && mmax + 128 < (1u << 24);   // landing keys hold E + 64 in 24 bits
    // a pair's fill time ~ m x (a strip's pace per column) + S x (a strip's
    // start lag), fitted per layout on a lone 64-row strip and on the
    // BASELINE pairs: untracked (round 4, profiles/r04_layout_fit.json)
    // layout 3 50 ns + 6.46 us global, 57.5 ns + 6.66 us local; the column
    // step 113 ns + 2.66 us (global), split for local fills 110 ns + 3.37 us.
    // Tracked fills: the tracked column step 146 ns + 3.45 us (round 5,
    // profiles/r05_tracked_layouts.txt); layout 3 at its untracked pace since
    // round 6 (the side wave keeps only the first maximum, the LCS runs as
    // bit rows in workgroups of their own, gx_lcs.h; before, the side wave's
    // LCS chain set a 104 ns + 11.9 us pace)
    const bool local = sc.floor_ == 0;
    double est1 = 0, est3 = 0;   // the launch's slowest pair on each layout (ns)
    for (const PairHost& h : ph) {
        const double S = (double)ceil_div((int)h.n, kStripRows1), m = (double)h.m;
        if (track) {
            est1 = std::max(est1, m * 146.0 + S * 3450.0);
            est3 = std::max(est3, local ? m * 57.5 + S * 6660.0 : m * 50.0 + S * 6460.0);
        } else {
            est1 = std::max(est1, local ? m * 110.0 + S * 3370.0 : m * 113.0 + S * 2660.0);
            est3 = std::max(est3, local ? m * 57.5 + S * 6660.0 : m * 50.0 + S * 6460.0);
        }
    }
    const bool sk_ok = skew_ok(sc, lcs_plane, mmax);
    const int lat = sk_ok && (!cs_ok || est3 < est1) ? 3 : cs_ok ? 1 : 0;
    if (const char* e = getenv("GX_LAYOUT"); e && *e) {
        const int want = atoi(e);
        if (want == 3) return sk_ok ? 3 : cs_ok ? 1 : 0;
        return (want == 1 && cs_ok) ? 1 : 0;
    }
    return strips64 <= 6LL * grid_cap ? lat : 0;
}

// The twin fill (gx_fill_pk.hip): two pairs per band, one in each 16-bit
// half.  Its values are kept relative to bases that a band's
// strips inherit from its top row (see the file header); a value of strip k
// of a W-strip band lies within D (192 (k + 1) + 16) + 2 (|a| + |smax| + |smin|)
// of its base, D = max |V''(i,j) - V''(i',j')| over neighbours = max(|a - g|,
// |U - g|) (the range proof of d8_planes_ok).  Returns the widest admissible
// band width <= W_want from {3, 4, 7, 8, 15}, or 0 when the twin fill does not apply
// (shape, mode, scores, GX_TWIN=0; run_fill also skips it for short queues).
// The twins (twin_table) pair the batch's pairs by shape whatever their
// order; the sweep covers the larger n and m of a twin, the shorter pair's
// state stays at its last column (its values beyond lie in the row above's
// range, but the bound takes the column difference anyway); an odd last pair
// is twinned with itself.
// The admission bound of a W-strip twin band whose twins' column counts
// differ by up to dm: the largest |value - base| any state of the band can
// reach (see the comment above twin_table).
// Local twins (plain values, no shift) take D = max(|a|, U), the neighbour
// bound of d8_planes_ok itself (the 0 floor keeps it), and their score
// offsets carry + K (K = max(0, -s_min), run_fill) and the floor's -g term.
constexpr long long kTwinBoundLimit = 30000;   // < 2^15 with room for the derived offsets
static long long twin_step(const Scores32& sc, bool local) {
    const long long g = sc.g, a = (long long)sc.h + sc.g;
    const long long smax = std::max(sc.sm, sc.smm);
    const long long U = std::max(0LL, smax - a);
    return local ? std::max({std::llabs(a), U, 1LL}) : std::max({std::llabs(a - g), std::llabs(U - g), 1LL});
}
static long long twin_const(const Scores32& sc, bool local) {
    const long long g = sc.g, a = (long long)sc.h + sc.g;
    const long long smax = std::max(sc.sm, sc.smm), smin = std::min(sc.sm, sc.smm);
    return 2 * (std::llabs(a) + std::llabs(smax) + std::llabs(smin)) + 64 +
           (local ? std::max(0LL, -smin) + std::llabs(g) : 0);
}
long long twin_bound(const Scores32& sc, int W, long long dm, bool local) {
    return twin_step(sc, local) * (192LL * W + 16 + dm) + twin_const(sc, local);
}
// Largest column gap between twins that keeps band width W admissible under
// twin_width's bound (capped at 1,024): twin_table pairs no wider gaps, so one
// ill-matched twin never narrows the band width of a whole batch.
long long twin_gap_cap(const Scores32& sc, int W, bool local) {
    const long long rest = kTwinBoundLimit - 1 - twin_const(sc, local);
    return std::max(0LL, std::min(1024LL, rest / twin_step(sc, local) - 192LL * W - 16));
}
std::vector<std::pair<int, int>> twin_table(const std::vector<PairHost>& ph, long long gap_cap) {
    std::vector<int> idx(ph.size());
    for (size_t p = 0; p < ph.size(); ++p) idx[p] = (int)p;
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) {
        return ph[a].m != ph[b].m ? ph[a].m > ph[b].m : ph[a].n > ph[b].n;
    });
    // neighbours in that order, unless their column counts lie more than
    // gap_cap apart (the admission bound's column margin): such a pair is
    // twinned with itself
    std::vector<std::pair<int, int>> tw;
    for (size_t k = 0; k < idx.size();) {
        if (k + 1 < idx.size() && (long long)(ph[idx[k]].m - ph[idx[k + 1]].m) <= gap_cap) {
            tw.emplace_back(idx[k], idx[k + 1]);
            k += 2;
        } else {
            tw.emplace_back(idx[k], idx[k]);
            k += 1;
        }
    }
    return tw;
}
// long_ok: the launch will be the twin fill without landing columns (twin
// plane codes, no code words, no skeleton): no int16 column quantity is
// left, so the 31,920-column limit of the int16 landing columns is lifted.
// The local twin fill (gx_fill_pk.hip LOCAL) keeps plain values relative to
// the same per-block bases, under the same bound (twin_step's local D); its
// row maxima fold into int32 at each base change, and it tracks no columns,
// so neither the magnitude of its values nor the column count is limited.
// Only as the launch without code words or skeleton (twin plane codes, the
// sequential walk): long_ok.
int twin_width(const std::vector<PairHost>& ph, const std::vector<std::pair<int, int>>& tw, const Scores32& sc,
               int is_local, bool track, bool lcs, int lay, bool planes, bool d8, int W_want,
               bool long_ok) {
    if (const char* e = getenv("GX_TWIN"); e && !strcmp(e, "0")) return 0;
    if (lay != 0 || track || lcs || (planes && !d8) || sc.g > 0 || sc.h > 0) return 0;
    if (ph.empty()) return 0;
    if (is_local && (!planes || !long_ok)) return 0;
    long long dm = 0;
    for (const auto& t : tw) {
        const PairHost& x = ph[t.first];
        const PairHost& y = ph[t.second];
        if (!x.n || !x.m || !y.n || !y.m) return 0;
        if (std::max(x.m, y.m) + 80 > 32000 && !long_ok) return 0;
        dm = std::max(dm, std::llabs((long long)x.m - (long long)y.m));
    }
    for (int W : {15, 8, 7, 4, 3}) {
        if (W > W_want && W != 3) continue;
        if (twin_bound(sc, W, dm, is_local != 0) < kTwinBoundLimit) return W;
    }
    return 0;
}

// ---------------------------------------------------------------------------
// chunked batches: a batch whose device footprint exceeds the free HBM runs
// as contiguous chunks of pairs through the same (reused) device buffers

// Device bytes a fill + traceback of pair (n, m) holds: score planes
// (plane_bpc per cell), traceback codes (0.25 B/cell), skeleton and hand-off
// rows, traceback records.
double pair_device_bytes(size_t n, size_t m, double plane_bpc) {
    const double cells = (double)(n + 128) * (double)(m + 64);
    return cells * (plane_bpc + 0.25) + 64.0 * (double)(m + 64) * (double)(n / 64 + 2) / 8.0 + 65536.0;
}

// Budget for one chunk: GX_CHUNK_BYTES if set, else the free device memory
// plus the context's cached buffers, less 4 GiB of headroom.
double chunk_budget(gx_context* ctx) {
    if (const char* e = getenv("GX_CHUNK_BYTES"); e && *e) return atof(e);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 64e9;
    double cached = 0;
    for (const DevBuf& b : ctx->free_list) cached += (double)b.cap;
    return std::max(1e9, (double)fr + cached - 4.0 * (1ull << 30));
}

// Contiguous [begin, end) ranges of the pairs, each within the budget (a pair
// larger than the budget runs alone), balanced: the fewest chunks the budget
// allows, each near total / chunks (1024 x 16k: 4 x 256 pairs, not 3 x 330 +
// 34, whose short last chunk would lose the twin fill and leave CUs idle).
// (Twins are formed inside each chunk by twin_table, by shape, so a chunk's
// pair count need not be even.)
static std::vector<std::pair<size_t, size_t>> plan_chunks_within(const std::vector<PairHost>& ph, double plane_bpc,
                                                                 double budget) {
    std::vector<std::pair<size_t, size_t>> out;
    auto bytes = [&](size_t p) { return (ph[p].n && ph[p].m) ? pair_device_bytes(ph[p].n, ph[p].m, plane_bpc) : 0.0; };
    size_t b = 0;
    double acc = 0;
    for (size_t p = 0; p < ph.size(); ++p) {
        const double x = bytes(p);
        if (p > b && acc + x > budget) {
            out.emplace_back(b, p);
            b = p;
            acc = 0.0;
        }
        acc += x;
    }
    out.emplace_back(b, ph.size());
    return out;
}
std::vector<std::pair<size_t, size_t>> plan_chunks(gx_context* ctx, const std::vector<PairHost>& ph,
                                                   double plane_bpc) {
    const double budget = chunk_budget(ctx);
    auto out = plan_chunks_within(ph, plane_bpc, budget);
    if (const char* e = getenv("GX_LOG"); e && !strcmp(e, "debug")) {
        size_t fr = 0, tot = 0;
        (void)hipMemGetInfo(&fr, &tot);
        fprintf(stderr, "[gx DEBUG] chunk plan: %zu pairs, %.2f B/cell, budget %.3e B (free %zu of %zu, %zu cached) -> %zu chunks\n",
                ph.size(), plane_bpc, budget, fr, tot, ctx->free_list.size(), out.size());
    }
    if (out.size() > 1) {
        // the same number of chunks, pairs dealt out evenly two at a time (a
        // twin each): 1024 x 64k was 51 chunks of 20 and one of 4, whose lone
        // twins ran 4-wave bands; now 44 of 20 and 8 of 18 -- kept if every
        // chunk fits the budget
        {
            const size_t K = out.size(), P = ph.size(), twins = (P + 1) / 2;
            std::vector<std::pair<size_t, size_t>> even;
            size_t a = 0;
            bool fits = twins >= K;
            for (size_t c = 0; c < K && fits; ++c) {
                const size_t b = std::min(P, a + 2 * (twins / K + (c < twins % K ? 1 : 0)));
                double bytes = 0;
                for (size_t p = a; p < b; ++p)
                    bytes += (ph[p].n && ph[p].m) ? pair_device_bytes(ph[p].n, ph[p].m, plane_bpc) : 0.0;
                fits = b > a && bytes <= budget;
                even.emplace_back(a, b);
                a = b;
            }
            if (fits && a == P) return even;
        }
        double total = 0;
        for (size_t p = 0; p < ph.size(); ++p)
            total += (ph[p].n && ph[p].m) ? pair_device_bytes(ph[p].n, ph[p].m, plane_bpc) : 0.0;
        // the same number of chunks with a smaller target, if the greedy split allows it
        for (double f : {1.0, 1.02, 1.05, 1.1}) {
            const double target = std::min(budget, f * total / (double)out.size());
            auto bal = plan_chunks_within(ph, plane_bpc, target);
            if (bal.size() <= out.size()) return bal;
        }
    }
    return out;
}

extern "C" int gx_twin_admission(const gx_scores* scores, int band_waves, int64_t col_gap, int64_t* bound) {
    if (!scores || band_waves < 1 || col_gap < 0) return -1;
    HostScores hs;
    Scores32 sc;
    if (check_scores(scores, 1, 1, &hs, &sc, 0, nullptr) != GX_OK) return -1;
    const long long b = twin_bound(sc, band_waves, col_gap);
    if (bound) *bound = b;
    return (sc.g <= 0 && sc.h <= 0 && b < kTwinBoundLimit) ? 1 : 0;
}

extern "C" int gx_twin_admission_mode(const gx_scores* scores, int is_local, int band_waves, int64_t col_gap,
                                      int64_t* bound) {
    if (!scores || band_waves < 1 || col_gap < 0) return -1;
    HostScores hs;
    Scores32 sc;
    if (check_scores(scores, 1, 1, &hs, &sc, is_local, nullptr) != GX_OK) return -1;
    const long long b = twin_bound(sc, band_waves, col_gap, is_local != 0);
    if (bound) *bound = b;
    return (sc.g <= 0 && sc.h <= 0 && b < kTwinBoundLimit) ? 1 : 0;
}

extern "C" int gx_plan_layout(const gx_scores* scores, int is_local, const int64_t* n, const int64_t* m,
                              size_t npairs, int track, int grid_cap) {
    if (!scores || !n || !m || npairs == 0) return -1;
    int64_t nmax = 0, mmax = 0;
    for (size_t p = 0; p < npairs; ++p) {
        if (n[p] < 0 || m[p] < 0) return -1;
        nmax = std::max(nmax, n[p]); mmax = std::max(mmax, m[p]);
    }
    HostScores hs;
    Scores32 sc;
    if (check_scores(scores, (size_t)nmax, (size_t)mmax, &hs, &sc, is_local, nullptr) != GX_OK) return -1;
    std::vector<PairHost> ph(npairs);
    for (size_t p = 0; p < npairs; ++p) ph[p] = PairHost{nullptr, nullptr, (size_t)n[p], (size_t)m[p]};
    return fill_layout(ph, sc, grid_cap > 0 ? grid_cap : 256, track != 0, false);
}

extern "C" int gx_plane_bytes_per_cell(const gx_scores* scores, int is_local) {
    HostScores hs;
    Scores32 sc;
    if (check_scores(scores, 1, 1, &hs, &sc, is_local)) return -1;
    return d8_planes_ok(sc, is_local) ? 3 : 12;
}
