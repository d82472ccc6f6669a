// gx_skew.hip -- layout 3, the latency fill of a single pair (or a few):
// anti-diagonal skew over 64-row strips, ONE row per lane.
//
// The reference fills its table one cell at a time (src/alignment/algo.rs:
// 151-282).  Any schedule of that recurrence needs n + m dependent
// anti-diagonal steps, so a single pair's time is (n + m + strip lags) x the
// time of one step.  Layout 0 (gx_kernels.hip compute_wave) gives each lane
// two rows, so one of its steps is two dependent cells (~45 VALU); layout 1
// (the column step) takes m steps of a whole 64-row column but each is a
// 6-round DPP prefix scan (~270 cycles).  Here lane l of a strip's wave owns
// row 64 s + l + 1 and at step t computes column j = t - l + 1: one cell per
// lane per step, ~18 VALU, so a step is bound by one wave's VALU issue.
//   * the cell above (i-1, j) is lane l-1's previous step (DPP wave_shr:1;
//     lane 0 takes it from the LDS ring the strip above fills, or the band's
//     I/O wave at a band boundary, gx_io.h), the top-left (i-1, j-1) the one
//     before that (kept from the previous step's move);
//   * global fills keep V'' = V - (i + j) g and, with h <= 0,
//     fold both gap recurrences onto score_max:
//         I''(i,j)   = max(I''(i,j-1), H''(i,j-1) + h)        (algo.rs:231-236)
//         D''(i+1,j) = max(D''(i,j),   H''(i,j)   + h)        (algo.rs:238-243)
//         S''(i,j)   = H''(i-1,j-1) + s - 2g                  (algo.rs:245-248)
//     (H + h adds I + h <= I and D + h <= D, which never win); local fills
//     keep plain values with the 0 floor in each gap max (algo.rs:103);
//   * outputs in the step-indexed formats of layout 0 with one row per lane:
//     int32 planes plane[strip][t/4][lane][t%4] (1 KiB per wave and plane
//     every 4 steps, one dwordx4 per lane), code words codes[strip][t/16][lane]
//     (bit 31-k "delete beats insert and sub", bit 15-k "insert beats sub"),
//     and the landing-column skeleton of each strip's bottom row (stored
//     E + 64, as layout 1), so the traceback chases it and walks all strips
//     at once (gx_kernels.hip tb_chase_kernel / tb_strip_kernel, TbDev.skew).
// No MFMA: an integer max-plus recurrence.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>
#include "gx_internal.h"

#include "gx_device.h"
#include "gx_io.h"

namespace gx {

// State of a lane's row after its previous step, i.e. of cell (i, j-1).
struct SkState {
    int I;         // insert score
    int Hx;        // H + h (global) / H + h + g (local): the gap-open term of the next insert and delete
    int H;         // score_max
    int Dd;        // delete successor, D(i+1, j-1) (pushed / moved to the row below)
    int c2;        // column symbol of (i, j-1) (moved to the row below with the cell)
    int Hd, Ed;    // score_max and landing column + 64 of (i-1, j-1)
    int E;         // landing column + 64
    uint32_t cI, cD;
    int lbest, lstep, lE;   // LOCAL: the row's last max of score_max (algo.rs:310-322)
};

// One anti-diagonal step of a lane: cell (i, j), j = t - lane + 1.  r = the
// ring record of column t + 1 (lane 0's cell above).  act = false (ramp
// lanes outside columns 1..m) leaves the row unchanged.
template <bool LOCAL, bool MASKED, bool TBL>
__device__ __forceinline__ void sk_step(SkState& st, const Rec& r, const int t, const bool act, const int c1v,
                                        const Scores32& sc, int& oI, int& oD, int& oS) {
    const int Dn = shr1(r.dd, st.Dd);        // D(i, j): the delete successor of the cell above
    const int hu = shr1(r.sm, st.H);         // score_max(i-1, j)
    const int c2 = shr1(r.c2, st.c2);        // s2[j-1] (or its symbol code * 8, TBL)
    const int eu = shr1(t + 65, st.E);       // E(i-1, j) + 64; lane 0: the top boundary row, column j
    const bool mt = c2 == c1v;               // sequence.rs:113-114
    const int Sn = st.Hd + (TBL ? __builtin_amdgcn_sbfe(c1v, c2, 8) : (mt ? sc.sm : sc.smm));
    const int In = LOCAL ? max3i(st.I + sc.g, st.Hx, 0) : max(st.I, st.Hx);
    const int IS = max(In, Sn);
    const int Hn = max(IS, Dn);
    const int Hxn = Hn + (LOCAL ? sc.hg : sc.h);
    const int Ddn = LOCAL ? max3i(Dn + sc.g, Hxn, 0) : max(Dn, Hxn);
    // retrace priority S > I > D against the cell max (algo.rs:351-400): code
    // bits "I beats S" / "D beats both", and the landing column taken from the
    // predecessor the priority picks (I -> left, D -> up, else top-left)
    int En;
    {
        unsigned long long m1, m2, k1, k2;
        asm volatile(
            "v_cmp_gt_i32 %[m1], %[in], %[sn]\n\t"
            "v_cmp_gt_i32 %[m2], %[dn], %[is]\n\t"
            "v_cndmask_b32 %[en], %[etl], %[el], %[m1]\n\t"
            "v_addc_co_u32 %[ci], %[k1], %[ci], %[ci], %[m1]\n\t"
            "v_addc_co_u32 %[cd], %[k2], %[cd], %[cd], %[m2]\n\t"
            "v_cndmask_b32 %[en], %[en], %[eu], %[m2]"
            : [en] "=&v"(En), [ci] "+v"(st.cI), [cd] "+v"(st.cD), [m1] "=&s"(m1), [m2] "=&s"(m2), [k1] "=&s"(k1),
              [k2] "=&s"(k2)
            : [in] "v"(In), [sn] "v"(Sn), [dn] "v"(Dn), [is] "v"(IS), [etl] "v"(st.Ed), [el] "v"(st.E), [eu] "v"(eu));
    }
    if (LOCAL) {   // algo.rs:310-322: max_by keeps the LAST maximum
        const bool nl = act && Hn >= st.lbest;
        st.lbest = nl ? Hn : st.lbest; st.lstep = nl ? t : st.lstep; st.lE = nl ? En : st.lE;
    }
    if (MASKED) {
        st.I = act ? In : st.I; st.Hx = act ? Hxn : st.Hx; st.H = act ? Hn : st.H; st.Dd = act ? Ddn : st.Dd;
        st.E = act ? En : st.E; st.c2 = act ? c2 : st.c2;
    } else {
        st.I = In; st.Hx = Hxn; st.H = Hn; st.Dd = Ddn; st.E = En; st.c2 = c2;
    }
    st.Hd = hu;   // (ramp-up lanes receive the column-0 cells above: still the right top-left)
    st.Ed = eu;
    oI = In; oD = Dn; oS = Sn;
}

// Uniform per-strip values of a compute wave.
struct SkCtx {
    uint32_t* codes;
    const Rec* ring_in;
    lds_int* wcnt_in;
    lds_int* wcnt_out;
    int* status;
    __amdgpu_buffer_rsrc_t rI, rD, rS;    // the strip's planes (one descriptor each, group offset in soffset)
    __amdgpu_buffer_rsrc_t skel_rsrc;     // skeleton row of this strip (bottom-row E + 64)
    uint32_t skel_voff;                   // lane 63: 0; other lanes: out of range
    uint32_t scratch;                     // this lane's LDS scratch slot (full-group pushes)
    uint32_t cnt_addr;                    // lane 63 with a consumer: the ring counter; else scratch
    int m, lane, c1;
    unsigned tr_win;
};

// The previous group's cells, stored one plane per step during the next group.
struct SkPend {
    int4 I, D, S;
    int goff;        // its byte offset in the strip planes (soffset, uniform)
    uint32_t voff;   // this lane's offset in the group (lane * 16), or kNoStore: nothing pending
};

template <int PLANE>
__device__ __forceinline__ void sk_pend_store(const SkPend& pd, const SkCtx& w) {
#ifndef GX_DIAG_NO_PLANES
    const auto r = PLANE == 0 ? w.rI : PLANE == 1 ? w.rD : w.rS;
    const int4 v = PLANE == 0 ? pd.I : PLANE == 1 ? pd.D : pd.S;
    const v4i x = {v.x, v.y, v.z, v.w};
    // (the range check covers voffset, not soffset: kNoStore drops the store)
    __builtin_amdgcn_raw_buffer_store_b128(x, r, (int)pd.voff, __builtin_amdgcn_readfirstlane(pd.goff), GX_PLANE_AUX);
#endif
}

// One 4-step group.  `cur` holds validated ring records for these steps,
// `nxt` receives the next group's (the caller alternates the two, so no
// records are copied).  Ring protocol as gx_kernels.hip group4: observe the
// producer's counter, read the next group's records speculatively, compute,
// re-read after a wait if the counter did not cover them.
template <bool LOCAL, bool PLANES, bool TBL, bool MASKED, int G4>
__device__ __forceinline__ void sk_group4(SkState& st, const Rec (&cur)[4], Rec (&nxt)[4], SkCtx& w, const Scores32& sc,
                                          const int t0, const uint32_t out_base, const bool push_on, SkPend& pend) {
    const int t = t0 + 4 * G4;
    const int need = min(t + 8, w.m) + 1;                     // columns of the next group: t+5 .. t+8
    const int seen_v = *w.wcnt_in;
    asm volatile("" ::: "memory");
    read4(nxt, w.ring_in + ring_slot(t + 5));
    int oI[4], oD[4], oS[4], e[4];
    const int col0 = t - (kWave - 1);                          // lane 63's column before step 0 of the group
    const uint32_t pa = push_on && w.lane == kWave - 1 ? out_base : w.scratch;
#pragma unroll
    for (int U = 0; U < 4; ++U) {
        // lane 63 holds column t+U-63 before step U: push it to the strip below
        if (MASKED) {
            const unsigned long long mk = lane63_mask(push_on && col0 + U >= 0 && col0 + U <= w.m);
            if (U == 0) cs_push63<4 * G4 + 0, false>(out_base, mk, st.Dd, st.H, st.c2, 0);
            if (U == 1) cs_push63<4 * G4 + 1, false>(out_base, mk, st.Dd, st.H, st.c2, 0);
            if (U == 2) cs_push63<4 * G4 + 2, false>(out_base, mk, st.Dd, st.H, st.c2, 0);
            if (U == 3) {
                cs_push63<4 * G4 + 3, false>(out_base, mk, st.Dd, st.H, st.c2, 0);
                if (push_on && col0 + 3 >= 0 && col0 <= w.m) lds_store_lane0(w.wcnt_out, min(col0 + 3, w.m) + 1);
            }
        } else {
            if (U == 0) cs_push_all<4 * G4 + 0, false>(pa, st.Dd, st.H, st.c2, 0);
            if (U == 1) cs_push_all<4 * G4 + 1, false>(pa, st.Dd, st.H, st.c2, 0);
            if (U == 2) cs_push_all<4 * G4 + 2, false>(pa, st.Dd, st.H, st.c2, 0);
            if (U == 3) { cs_push_all<4 * G4 + 3, false>(pa, st.Dd, st.H, st.c2, 0); publish_all(w.cnt_addr, col0 + 4); }
        }
        const bool act = MASKED ? (unsigned)(t + U - w.lane) < (unsigned)w.m : true;
        sk_step<LOCAL, MASKED, TBL>(st, cur[U], t + U, act, w.c1, sc, oI[U], oD[U], oS[U]);
        e[U] = st.E;   // lane 63: E + 64 of its column t+U-62
        if (PLANES && !MASKED && U < 3) {
            if (U == 0) sk_pend_store<0>(pend, w);
            if (U == 1) sk_pend_store<1>(pend, w);
            if (U == 2) sk_pend_store<2>(pend, w);
        }
    }
    // lane 63's landing columns (+64) of its columns col0+1 .. col0+4: the skeleton
    if (!MASKED) {
        skel_store4(w.skel_rsrc, w.skel_voff + 4u * (uint32_t)(col0 + 1), e[0], e[1], e[2], e[3]);
    } else {
#pragma unroll
        for (int U = 0; U < 4; ++U) {
            const int c = col0 + 1 + U;
            skel_store(w.skel_rsrc, (c >= 1 && c <= w.m) ? w.skel_voff + 4u * (uint32_t)c : kSkelOff, e[U]);
        }
    }
    if (PLANES) {
        // (ramp groups: flush the pending group, store this one now)
        if (MASKED) { sk_pend_store<0>(pend, w); sk_pend_store<1>(pend, w); sk_pend_store<2>(pend, w); }
        pend.I = make_int4(oI[0], oI[1], oI[2], oI[3]);
        pend.D = make_int4(oD[0], oD[1], oD[2], oD[3]);
        pend.S = make_int4(oS[0], oS[1], oS[2], oS[3]);
        pend.goff = (t >> 2) * (kGroupInts1 * 4);
        pend.voff = (uint32_t)w.lane * 16u;
        if (MASKED) {
            sk_pend_store<0>(pend, w); sk_pend_store<1>(pend, w); sk_pend_store<2>(pend, w);
            pend.voff = kNoStore;
        }
    }
    if (__builtin_amdgcn_readfirstlane(seen_v) < need) {      // producer was behind: wait, re-read
        w.tr_win += wait_ge(w.wcnt_in, need, w.status);
        read4(nxt, w.ring_in + ring_slot(t + 5));
    }
    __builtin_amdgcn_sched_barrier(0);
}

template <bool LOCAL, bool PLANES, bool TBL>
__device__ void compute_wave_skew(const PairDev& P, const int s, const int lane, const Scores32& sc,
                                  const Rec* ring_in, Rec* ring_out, lds_int* wcnt_in, lds_int* rcnt_in,
                                  lds_int* wcnt_out, lds_int* rcnt_out, const bool has_consumer, StripRes* sres,
                                  PairRes* pres, int* status, const uint32_t scratch_base) {
    static_assert(kSub == 16, "16-step sub-blocks (code words, ring alignment)");
    const int n = P.n, m = P.m;
    const int i = s * kWave + lane + 1;          // this lane's row
    const bool ok = i <= n;
    SkCtx w;
    if (PLANES) {
        const size_t strip_planes = (size_t)s * P.t4 * kGroupInts1;
        const int pbytes = P.t4 * kGroupInts1 * 4;   // one strip's plane
        w.rI = rsrc_of(uniform_ptr(P.pI + strip_planes), pbytes);
        w.rD = rsrc_of(uniform_ptr(P.pD + strip_planes), pbytes);
        w.rS = rsrc_of(uniform_ptr(P.pS + strip_planes), pbytes);
    }
    w.codes = P.codes + (size_t)s * P.t16 * kWave;
    w.ring_in = ring_in; w.wcnt_in = wcnt_in; w.wcnt_out = wcnt_out; w.status = status;
    w.skel_rsrc = rsrc_of(uniform_ptr(P.skel + (size_t)s * P.skel_stride), has_consumer ? 4 * (m + 1) : 0);
    w.skel_voff = lane == kWave - 1 ? 0u : kSkelOff;
    w.scratch = scratch_base + 4u * (uint32_t)lane;
    w.cnt_addr = (has_consumer && lane == kWave - 1) ? lds_addr((const void*)wcnt_out) : w.scratch;
    w.m = m; w.lane = lane;
    w.c1 = ok ? (int)P.c1[i - 1] : 0x1FF;       // 0x1FF never equals a byte
    if (TBL) w.c1 = score_table(w.c1, sc);
    w.tr_win = 0;
    StripTrace* const trace = P.trace;

    // column 0 (algo.rs:204-211): I = S = neg_inf, D = h + i g, score_max
    // max(D, floor); global fills hold V - (i + 0) g
    SkState st;
    {
        const int D0 = sc.h + i * sc.g;
        const int H0 = LOCAL ? max(D0, 0) : D0 - i * sc.g;
        st.I = LOCAL ? kNeg : kNeg - i * sc.g;
        st.H = H0;
        st.Hx = H0 + (LOCAL ? sc.hg : sc.h);
        st.Dd = H0;                               // (column 0's successor is never read: column 0 is analytic)
        st.c2 = 0;
        st.E = 64 - (lane + 1);                   // column 0: the path reaches it at local row lane + 1
        st.cI = 0; st.cD = 0;
        st.lbest = ok ? INT_MIN : INT_MAX; st.lstep = 0; st.lE = 0;
    }
    if (has_consumer) {
        if (lane == kWave - 1) ring_out[ring_slot(0)] = Rec{st.Dd, st.H, 0, 0};
        lds_wait();
        if (lane == 0) *wcnt_out = 1;
    }
    const bool tracing = trace != nullptr;
    long long tr_start = 0, tr_first = 0, clk_first = 0;
    unsigned tr_wout = 0;
    long long tr_q[kTraceQ] = {};
    if (tracing) tr_start = __builtin_amdgcn_s_memrealtime();
    w.tr_win += wait_ge(wcnt_in, min(4, m) + 1, status);
    Rec ra[4], rb[4];   // records of the current / next group (alternating)
    {
        const Rec r0 = ring_in[ring_slot(0)];
        // column 1's top-left: lane 0 the row above the strip at column 0, the
        // others lane-1's column 0; its landing column: (64 s, 0) itself
        st.Hd = shr1(r0.sm, st.H);
        st.Ed = shr1(64, st.E);
        read4(ra, ring_in + ring_slot(1));
    }
    if (tracing) { tr_first = __builtin_amdgcn_s_memrealtime(); clk_first = __builtin_amdgcn_s_memtime(); }
    const int T = m + kWave;                      // lane 63 pushes column m at step m + 63
    SkPend pend;
    pend.goff = 0;
    pend.voff = kNoStore;   // nothing pending before the first group
    for (int t0 = 0; t0 < T; t0 += kSub) {
        const int last_col = min(t0 + kSub - 1 - (kWave - 1), m);   // last column pushed here
        if (has_consumer && last_col >= kRing) tr_wout += wait_ge(rcnt_out, last_col - kRing + 1, status);
        if (tracing) {
            const int q = (int)((long long)t0 * (kTraceQ + 1) / T) - 1;
            if (q >= 0 && q < kTraceQ && tr_q[q] == 0) tr_q[q] = __builtin_amdgcn_s_memrealtime();
        }
        const bool full = (t0 >= kWave) && (t0 + kSub - 1 <= m - 1);
        const uint32_t out_base = lds_addr(ring_out + ring_slot(t0 - (kWave - 1)));
        if (full) {
            sk_group4<LOCAL, PLANES, TBL, false, 0>(st, ra, rb, w, sc, t0, out_base, has_consumer, pend);
            sk_group4<LOCAL, PLANES, TBL, false, 1>(st, rb, ra, w, sc, t0, out_base, has_consumer, pend);
            sk_group4<LOCAL, PLANES, TBL, false, 2>(st, ra, rb, w, sc, t0, out_base, has_consumer, pend);
            sk_group4<LOCAL, PLANES, TBL, false, 3>(st, rb, ra, w, sc, t0, out_base, has_consumer, pend);
        } else {
            sk_group4<LOCAL, PLANES, TBL, true, 0>(st, ra, rb, w, sc, t0, out_base, has_consumer, pend);
            sk_group4<LOCAL, PLANES, TBL, true, 1>(st, rb, ra, w, sc, t0, out_base, has_consumer, pend);
            sk_group4<LOCAL, PLANES, TBL, true, 2>(st, ra, rb, w, sc, t0, out_base, has_consumer, pend);
            sk_group4<LOCAL, PLANES, TBL, true, 3>(st, rb, ra, w, sc, t0, out_base, has_consumer, pend);
        }
        // codes[strip][t/16][lane]
#ifndef GX_DIAG_NO_CODES
        gstore1(w.codes + (size_t)(t0 >> 4) * kWave + lane, (st.cD << 16) | (st.cI & 0xFFFFu));
#endif
        // every ring read up to column t0+20 (incl. the next group's) was issued before this store
        lds_store_lane0(rcnt_in, min(t0 + kSub + 5, m + 1));
    }
    if (PLANES) { sk_pend_store<0>(pend, w); sk_pend_store<1>(pend, w); sk_pend_store<2>(pend, w); }

    if (LOCAL) {   // the strip's last max: the highest lane (latest row) holding it
        const int lb = ok ? st.lbest : INT_MIN;
        int lmx = lb;
        for (int off = 32; off > 0; off >>= 1) lmx = max(lmx, __shfl_xor(lmx, off));
        const unsigned long long lmask = __ballot(ok && lb == lmx);
        const int ll = lmask ? (63 - __clzll((long long)lmask)) : 0;
        const int l_step = __shfl(st.lstep, ll), l_E = __shfl(st.lE, ll);
        if (lane == 0) {
            StripRes r{};
            r.best = INT_MIN;
            r.lbest = lmx; r.li = s * kWave + ll + 1; r.lj = l_step - ll + 1; r.lE = l_E - 64;
            sres[P.strip_base + s] = r;
        }
    }
    if (ok && i == n) { pres->end_SM = st.H; pres->end_E = st.E - 64; }   // cell (n, m) (algo.rs:308, 331)
    if (tracing && lane == 0) {
        StripTrace tr;
        tr.t_start = tr_start; tr.t_first = tr_first; tr.t_end = __builtin_amdgcn_s_memrealtime();
        tr.wait_in = (int)w.tr_win; tr.wait_out = (int)tr_wout;
        tr.clk = __builtin_amdgcn_s_memtime() - clk_first;
        for (int q = 0; q < kTraceQ; ++q) tr.t_q[q] = tr_q[q];
        trace[s] = tr;
    }
}

// Band hand-off of layout 3 in tagged 8-byte granules (MI355X_MICROARCH.md
// "handoff-1to1": a data-tagged granule is the cheapest cross-CU hand-off,
// no progress counter and no store drain before a flag).  The next band needs
// each bottom-row cell's delete successor dd and score_max sm (its column
// symbol it reads from the pair's chars itself); dd - sm lies in
// [h + g, max(g, 0)] (Ddn = max(Dn, H + h) with Dn <= H, local: the floor and
// + g), so one granule holds sm (low word) and (dd - sm) in 31 bits under a
// valid bit (bit 63).  The feed rows are zeroed before the launch, so a
// granule is valid exactly once it was written this launch.  Stores and
// loads are 8-byte agent-scope (sc1: write-through, L1 bypass).
template <bool TBL>
__device__ void io_wave_tag(const PairDev& P, const int lb, const int lane, const Scores32& sc, Rec* ring0,
                            const Rec* ringW, lds_int* wcnt0, lds_int* rcnt0, lds_int* wcntW, lds_int* rcntW,
                            const bool do_out, int* status) {
    const int m = P.m;
    int in_next = 0, out_next = 0;
    const gu64* feed_in = lb > 0 ? (const gu64*)(P.feed + (size_t)(lb - 1) * P.feed_stride) : nullptr;
    gu64* feed_out = do_out ? (gu64*)(P.feed + (size_t)lb * P.feed_stride) : nullptr;
    unsigned idle = 0;
    while (in_next <= m || (do_out && out_next <= m)) {
        bool moved = false;
        if (in_next <= m) {
            const int lim = min(m + 1, *rcnt0 + kRing);     // ring slots free below the strip's reads
            const int j = in_next + lane;
            Rec r{};
            bool valid = false;
            if (j < lim) {
                if (lb == 0) {
                    // row 0 (algo.rs:195-202, 213-220): I = h + j g, D = S = neg_inf
                    valid = true;
                    if (j > 0) {
                        const int I0 = sc.h + j * sc.g;
                        r.dd = max(I0 + sc.hg, sc.floor_);
                        r.sm = max(I0, sc.floor_);
                        if (sc.shift) { r.dd -= (1 + j) * sc.g; r.sm -= j * sc.g; }
                    }
                } else {
                    const unsigned long long gr = __hip_atomic_load(feed_in + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    valid = (gr >> 63) != 0;
                    r.sm = (int)(unsigned)gr;
                    r.dd = r.sm + ((int)((unsigned)(gr >> 32) << 1) >> 1);
                }
                r.c2 = j == 0 ? 0 : TBL ? sym_code(P.c2[j - 1], sc) * 8 : (int)P.c2[j - 1];
            }
            // the leading run of valid columns
            const unsigned long long vm = __ballot(valid);
            const int cnt = ~vm ? (int)__builtin_ctzll(~vm) : kWave;
            if (cnt > 0) {
                if (lane < cnt) ring0[ring_slot(j)] = r;
                lds_wait();
                if (lane == 0) *wcnt0 = in_next + cnt;
                in_next += cnt;
                moved = true;
            }
        }
        if (do_out && out_next <= m) {
            const int avail = *wcntW;
            const int chunk = min(avail - out_next, kWave);
            if (chunk > 0) {
                const int j = out_next + lane;
                Rec r{};
                if (lane < chunk) r = ringW[ring_slot(j)];
                lds_wait();
                if (lane == 0) *rcntW = out_next + chunk;   // ring slots free again
                if (lane < chunk) {
                    const unsigned long long gr = (unsigned long long)(unsigned)r.sm |
                                                  ((unsigned long long)(0x80000000u | ((unsigned)(r.dd - r.sm) & 0x7FFFFFFFu)) << 32);
                    __hip_atomic_store((gu64*)(feed_out + j), gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                out_next += chunk;
                moved = true;
            }
        }
        if (moved) idle = 0;
        else if (++idle > kSpinLimit ||
                 ((idle & 4095u) == 4095u &&
                  __hip_atomic_load((gint*)status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            __hip_atomic_store((gint*)status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        } else {
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

// One workgroup = one band of W strips (W compute waves, one per SIMD for W
// <= 4) + the I/O wave; persistent workgroups take bands from the host's
// band-major queue (gx_api.cpp run_fill), as fill_kernel does.
template <int W, bool LOCAL, bool PLANES, bool TBL>
__global__ __launch_bounds__((W + 1) * kWave, 1) void fill_skew_kernel(const PairDev* __restrict__ pairs,
                                                                       const int npairs, const int total_bands,
                                                                       int* band_counter, StripRes* sres,
                                                                       PairRes* pres, const Scores32 sc) {
    __shared__ Rec rings[W + 1][kRing];
    __shared__ uint32_t push_scratch[W][kPushScratch];
    __shared__ int wcnt[W + 1];
    __shared__ int rcnt[W + 1];
    __shared__ int band_sh;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int lane = threadIdx.x & (kWave - 1);
    for (;;) {
        if (threadIdx.x == 0) band_sh = atomicAdd(band_counter, 1);
        if (threadIdx.x < W + 1) { wcnt[threadIdx.x] = 0; rcnt[threadIdx.x] = 0; }
        __syncthreads();
        const int b = __builtin_amdgcn_readfirstlane(band_sh);
        if (b >= total_bands) return;
        const int2 ob = reinterpret_cast<const int2*>(pairs + npairs)[b];
        const int p = __builtin_amdgcn_readfirstlane(ob.x);
        const PairDev& P = pairs[p];
        const int lb = __builtin_amdgcn_readfirstlane(ob.y);
        const int s0 = lb * W;
        if (wave < W) {
            const int s = s0 + wave;
            if (s < P.strips) {
                const bool last_in_band = wave == W - 1;
                const bool has_consumer = last_in_band ? (lb + 1 < P.bands) : (s + 1 < P.strips);
                compute_wave_skew<LOCAL, PLANES, TBL>(P, s, lane, sc, rings[wave], rings[wave + 1],
                                                      (lds_int*)&wcnt[wave], (lds_int*)&rcnt[wave],
                                                      (lds_int*)&wcnt[wave + 1], (lds_int*)&rcnt[wave + 1],
                                                      has_consumer, sres, pres + p, band_counter + 1,
                                                      lds_addr(push_scratch[wave]));
            }
        } else {
            // a strip here consumes a column every few tens of ns: fixed
            // 16-column chunks with a store round trip each (gx_io.h) cannot
            // keep up; tagged granules move every column as soon as it exists
            io_wave_tag<TBL>(P, lb, lane, sc, rings[0], rings[W], (lds_int*)&wcnt[0], (lds_int*)&rcnt[0],
                             (lds_int*)&wcnt[W], (lds_int*)&rcnt[W], lb + 1 < P.bands, band_counter + 1);
        }
        __syncthreads();
    }
}

template <int W, bool LOCAL, bool PLANES, bool TBL>
static hipError_t launch_skew_t(const PairDev* d_pairs, int npairs, int total_bands, int* d_counter, StripRes* d_sres,
                                PairRes* d_pres, Scores32 sc, int grid, hipStream_t st) {
    hipLaunchKernelGGL((fill_skew_kernel<W, LOCAL, PLANES, TBL>), dim3(grid), dim3((W + 1) * kWave), 0, st, d_pairs,
                       npairs, total_bands, d_counter, d_sres, d_pres, sc);
    return hipGetLastError();
}

template <bool LO, bool PL, bool TB, int W0, int... Ws>
static hipError_t launch_skew_w(int W, const PairDev* d_pairs, int npairs, int total_bands, int* d_counter,
                                StripRes* d_sres, PairRes* d_pres, Scores32 sc, int grid, hipStream_t st) {
    if (W == W0) return launch_skew_t<W0, LO, PL, TB>(d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc, grid, st);
    if constexpr (sizeof...(Ws) > 0)
        return launch_skew_w<LO, PL, TB, Ws...>(W, d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc, grid, st);
    return hipErrorInvalidValue;
}

// Band widths of layout 3 (must match gx_api.cpp kSkewWidths).
hipError_t launch_fill_skew(int W, bool local, bool planes, bool tbl, const PairDev* d_pairs, int npairs,
                            int total_bands, int* d_counter, StripRes* d_sres, PairRes* d_pres, Scores32 sc, int grid,
                            hipStream_t st) {
#define GX_SKEW_CASE(LO, PL, TB)                                                                                   \
    if (local == LO && planes == PL && tbl == TB)                                                                  \
        return launch_skew_w<LO, PL, TB, 2, 3, 4, 8>(W, d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc, \
                                                     grid, st);
    GX_SKEW_CASE(false, false, false)
    GX_SKEW_CASE(false, false, true)
    GX_SKEW_CASE(false, true, false)
    GX_SKEW_CASE(false, true, true)
    GX_SKEW_CASE(true, false, false)
    GX_SKEW_CASE(true, false, true)
    GX_SKEW_CASE(true, true, false)
    GX_SKEW_CASE(true, true, true)
#undef GX_SKEW_CASE
    return hipErrorInvalidValue;
}

}  // namespace gx
