// gx_cs2.hip -- the split column-step fill: the latency path of a single pair
// or a few (BASELINE configs 2 and 3: one pair per align call, main.rs:143-150
// -> algo.rs:151-282).
//
// Same strips, data formats and hand-offs as the column-step layout of
// gx_kernels.hip (layout 1, gx_internal.h: 64-row strips, lane l = row
// 64 s + l + 1, step t = column t + 1 of every row, int32 planes
// plane[strip][t/4][lane][t%4], codes[strip][t/16][lane], the bottom-row
// landing-column skeleton), so the traceback, exports and checksums are
// shared.  What differs is who does the work.  A single 30k pair has ~470
// strips, fewer than half the chip's 1,024 SIMDs, and a strip's sweep of m
// columns is the whole critical path: time ~ m x (cycles per column) + the
// strip lags.  A lone wave issues at most one instruction per ~4.7 cycles
// whatever its kind, so the column-step wave of layout 1 (~60 VALU, SALU
// and LDS instructions per column) sweeps at ~270 cycles per column.  Here
// each strip has two waves:
//   * the CORE wave runs the recurrence only, on the shifted values
//     V'' = V - (i + j) g (local mode floors at -(i + j) g):
//         In''  = max(I'', max(S, D)'' + h [, fl])          (algo.rs:231-236)
//         S''   = SM''(i-1, j-1) + (s - 2g)                 (algo.rs:245-248)
//         D''(l)= max(D''(i0+1, j), max_{k<l} IS''(k) + h) [, fl]  (algo.rs:238-243)
//     the delete chain as a 64-lane prefix max (six DPP steps, no per-lane
//     offsets thanks to the shift); it pushes the strip's bottom row to the
//     strip below (LDS ring) and hands In, S, D of every cell to
//   * the SIDE wave through an LDS staging ring (kSB columns): the traceback
//     code bits (S > I > D, algo.rs:351-400), the landing column (its own
//     prefix max over lane keys, as layout 1), the int32 plane stores, the
//     skeleton, the end cell and (local mode) the last-max tracker
//     (algo.rs:310-322).
// Core and side sweep at the pace of their own dependent chains (~8 DPP
// steps per column each) instead of the sum of both instruction streams.
// A band of W strips = W core + W side + 1 I/O wave (gx_io.h); W = 2 puts
// every compute wave of a CU on its own SIMD.
#include <stdlib.h>
#include "gx_device.h"
#include "gx_io.h"

namespace gx {

#ifndef GX_CS2_ASM
#define GX_CS2_ASM 1   // 0: the core's cross-lane moves through update_dpp builtins (compiler-fused)
#endif

// core -> side staging: one group = In, S, D of 4 columns for every lane
// (a lane's 4 columns of one value are one ds_write_b128 / ds_read_b128)
struct SideGrp {
    int4 v[3][kWave];
};

// lane 63's record of column j for the strip below: {dd, sm, c2} (Rec), or
// the lane's scratch slot (full exec, no branch).  Plain LDS stores, not
// inline asm: the compiler may then schedule them into the dependent chain's
// DPP wait states (a volatile asm statement ends a scheduling region); the
// ring counter's publish (publish_all, a memory-clobbering asm) keeps them
// before it.
typedef __attribute__((address_space(3))) Rec lds_rec;
template <int U>
__device__ __forceinline__ void cs2_push(uint32_t vaddr, int dd, int sm, int c2) {
    lds_rec* r = (lds_rec*)(uintptr_t)vaddr + U;
    r->dd = dd; r->sm = sm; r->c2 = c2;
}

// One column of the core recurrence for the 64 rows of the strip.
// State (cell (i, j-1)): I = I'', SDh = max(S, D)'' + h, SM = score_max''.
// r = ring record of column j (dd = D''(i0 + 1, j), sm = SM''(i0, j), c2);
// psm = SM''(i0, j - 1).  fl = -(i + j) g (local floor, shifted).
template <bool LOCAL, bool TBL, bool ASM = GX_CS2_ASM>
__device__ __forceinline__ void cs2_core_step(int& I, int& SDh, int& SM, const int psm, const int fl, const Rec& r,
                                              const int c1v, const Scores32& sc, const int hv, int& oI, int& oS,
                                              int& oD, int& dd_out) {
    const int scv = TBL ? __builtin_amdgcn_sbfe(c1v, r.c2, 8) : (r.c2 == c1v ? sc.sm : sc.smm);
    const int In = LOCAL ? max3i(I, SDh, fl) : max(I, SDh);
    int Sn, IS, Y, Z;
    if constexpr (ASM) {
    // the two cross-lane moves fused with their adds (v_add_u32_dpp, lane 0
    // keeps the destination's value: the ring's input set beforehand), one
    // VALU op each on the column's dependent chain instead of a v_mov_dpp,
    // its old-value copy and the add; the s_nop covers the DPP read-after-
    // VALU-write hazard, which the compiler does not track into inline asm
    Sn = psm + scv;                                 // lane 0: SM''(i0, j-1) + s''
    asm("s_nop 1\n\tv_add_u32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf"
        : "+v"(Sn) : "v"(SM), "v"(scv));
    IS = max(In, Sn);
    Y = IS + sc.h;
    Z = r.dd;                                       // lane 0: D''(i0 + 1, j)
    asm("s_nop 1\n\tv_add_u32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf"
        : "+v"(Z) : "v"(IS), "v"(hv));            // lane l: IS''(l-1) + h
    } else {
    Sn = shr1(psm, SM) + scv;                       // lane 0: SM''(i0, j-1) from the ring
    IS = max(In, Sn);
    Y = IS + sc.h;
    Z = shr1(r.dd, Y);                              // lane 0: D''(i0 + 1, j); lane l: IS''(l-1) + h
    }
    Z = scan_max64(Z);
    const int Dn = LOCAL ? max(Z, fl) : Z;
    SM = max(IS, Dn);
    SDh = max(Sn, Dn) + sc.h;
    dd_out = max(Dn, Y);                            // D''(i + 1, j) (lane 63: the row below the strip)
    I = In;
    oI = In; oS = Sn; oD = Dn;
}

// One 4-column group of the core wave (columns t + 1 .. t + 4, t = t0 + 4 G):
// the same ring protocol as layout 1's cs_group4 -- observe the producer's
// counter, read the next group's records speculatively, compute, re-read
// after a wait if the counter did not cover them.
template <bool LOCAL, bool TBL, int KSB, bool TAIL, int G, int DIAG>
__device__ __forceinline__ void cs2_core_group(int& I, int& SDh, int& SM, int& psm, int& fl, Rec (&cur)[4],
                                               Rec (&nxt)[4], const int t0, const int m, const int c1v,
                                               const Scores32& sc, const Rec* ring_in, lds_int* wcnt_in,
                                               SideGrp* sb, const int lane, const uint32_t pa, const uint32_t scr,
                                               const uint32_t cnt_addr, const int hv, unsigned& twin,
                                               int* status) {
    constexpr int kSBG = KSB / 4;
    const int t = t0 + 4 * G;
    const int need = min(t + 8, m) + 1;             // (the next group may be past column m)
    const int seen = DIAG == 7 ? 0 : *wcnt_in;
    asm volatile("" ::: "memory");
    // the next group's 4 records: slots (t + 20 .. t + 23) mod kRing, one
    // aligned block of 4 (t is a multiple of 4)
    const Rec* const nb = ring_in + ring_slot(t + 5);
    if (DIAG < 4) { nxt[0] = nb[0]; nxt[1] = nb[1]; nxt[2] = nb[2]; nxt[3] = nb[3]; }
    int oI[4], oS[4], oD[4];
#pragma unroll
    for (int U = 0; U < 4; ++U) {
        int dd;
        if (DIAG == 2) {   // (timing only: no recurrence, the side alone sets the pace)
            oI[U] = I + cur[U].dd; oS[U] = SDh + cur[U].sm; oD[U] = SM; dd = oI[U]; SM = oS[U];
        } else
            cs2_core_step<LOCAL, TBL, DIAG == 6 ? false : bool(GX_CS2_ASM)>(I, SDh, SM, psm, fl, cur[U], c1v, sc, hv,
                                                                            oI[U], oS[U], oD[U], dd);
        psm = cur[U].sm;
        if (LOCAL) fl -= sc.g;
        // lane 63's record of column t + U + 1 (none past column m)
        const uint32_t a = (TAIL && t + U + 1 > m) ? scr : pa;
        if (DIAG == 8) { asm volatile("" :: "v"(dd), "v"(SM)); continue; }
        if (U == 0) cs2_push<4 * G + 0>(a, dd, SM, cur[U].c2);
        if (U == 1) cs2_push<4 * G + 1>(a, dd, SM, cur[U].c2);
        if (U == 2) cs2_push<4 * G + 2>(a, dd, SM, cur[U].c2);
        if (U == 3) cs2_push<4 * G + 3>(a, dd, SM, cur[U].c2);
    }
    SideGrp& g = sb[(t >> 2) & (kSBG - 1)];
    if (DIAG >= 3) {   // (timing only: nothing staged; keeps the values alive)
        asm volatile("" :: "v"(oI[0] ^ oI[1] ^ oI[2] ^ oI[3] ^ oS[0] ^ oS[1] ^ oS[2] ^ oS[3] ^ oD[0] ^ oD[1] ^ oD[2] ^ oD[3]));
    } else {
        g.v[0][lane] = make_int4(oI[0], oI[1], oI[2], oI[3]);
        g.v[1][lane] = make_int4(oS[0], oS[1], oS[2], oS[3]);
        g.v[2][lane] = make_int4(oD[0], oD[1], oD[2], oD[3]);
    }
    // the records and staging of columns .. t + 4 are written (one wave's DS
    // operations execute in order): publish to the strip below and the side
    if (DIAG != 7) publish_all(cnt_addr, TAIL ? min(t + 5, m + 1) : t + 5);
    if (DIAG < 4 && __builtin_amdgcn_readfirstlane(seen) < need) {
        twin += wait_ge(wcnt_in, need, status) + 1;
        nxt[0] = nb[0]; nxt[1] = nb[1]; nxt[2] = nb[2]; nxt[3] = nb[3];
    }
}

template <bool LOCAL, bool TBL, int KSB, int DIAG>
__device__ __forceinline__ void cs2_core(const PairDev& P, const int s, const int lane, const Scores32& sc, const Rec* ring_in,
                         Rec* ring_out, lds_int* wcnt_in, lds_int* rcnt_in, lds_int* wcnt_out, lds_int* rcnt_out,
                         lds_int* scnt, SideGrp* sb, const bool has_consumer, int* status, const uint32_t scratch) {
    const int n = P.n, m = P.m;
    const int i = s * kWave + lane + 1;
    const bool ok = i <= n;
    int c1v = ok ? (int)P.c1[i - 1] : 0x1FF;
    if (TBL) c1v = score_table(c1v, sc);
    // column 0 (algo.rs:204-211), shifted: D''(i, 0) = h, I = S = neg_inf
    const int D0 = sc.h + i * sc.g;
    int I = kNeg;
    int SDh = sc.h + sc.h;
    int SM = max(D0, sc.floor_) - i * sc.g;
    int fl = LOCAL ? -(i + 1) * sc.g : 0;           // floor'' of column 1
    const uint32_t cnt_addr = lds_addr((const void*)wcnt_out);
    {
        const int dd0 = max3i(kNeg + sc.hg, D0 + sc.g, sc.floor_) - (i + 1) * sc.g;
        if (has_consumer && lane == kWave - 1) ring_out[ring_slot(0)] = Rec{dd0, SM, 0, 0};
        lds_wait();
        if (lane == 0) *wcnt_out = 1;
    }
    StripTrace* const trace = P.trace;   // GX_TRACE_FILE diagnostics (tools/trace_summary.py)
    long long tr_start = 0, tr_first = 0, clk_first = 0;
    long long tr_q[kTraceQ] = {};
    if (trace) tr_start = stamp_rt();
    const unsigned tr_win0 = wait_ge(wcnt_in, min(4, m) + 1, status);
    if (trace) { tr_first = stamp_rt(); clk_first = stamp_clk(); }
    Rec ra[4], rb[4];
    int psm;
    {
        const Rec r0 = ring_in[ring_slot(0)];
        psm = r0.sm;
        ra[0] = ring_in[ring_slot(1)]; ra[1] = ring_in[ring_slot(2)];
        ra[2] = ring_in[ring_slot(3)]; ra[3] = ring_in[ring_slot(4)];
    }
    const uint32_t scr = scratch + 4u * (uint32_t)lane;
    unsigned tr_wait_in = 0, tr_wait_sb = 0;       // wait iterations (diagnostics)
    if (DIAG == 9) {   // (timing only: the recurrence alone in registers, m columns)
        int acc = 0;
        const int x0 = psm;
        for (int t0 = 0; t0 < m; t0 += kSub) {
#pragma unroll
            for (int u = 0; u < kSub; ++u) {
                Rec r{x0 + u, x0 - u, (u & 3) * 8, 0};
                int a0, a1, a2, dd;
                cs2_core_step<LOCAL, TBL>(I, SDh, SM, psm, fl, r, c1v, sc, sc.h, a0, a1, a2, dd);
                acc ^= dd ^ a0 ^ a1 ^ a2;
            }
        }
        if (acc == 0x7FFFFFFF) ring_out[0].dd = acc;
        return;
    }
    int hv = sc.h;                                  // (a VGPR: the DPP add's second operand)
    asm volatile("" : "+v"(hv));
    for (int t0 = 0; t0 < m; t0 += kSub) {
        const int last_col = min(t0 + kSub, m);
        if (trace) {
            const int q = (int)((long long)t0 * (kTraceQ + 1) / (m + 1)) - 1;
            if (q >= 0 && q < kTraceQ && tr_q[q] == 0) tr_q[q] = stamp_rt();
        }
        if (has_consumer && last_col >= kRing) wait_ge(rcnt_out, last_col - kRing + 1, status);
        // staging slots free: group g reuses the slot of group g - KSB/4, so the
        // sub-block's last group needs the side past column 4 (g - KSB/4) + 4
        if (DIAG < 5 && t0 + 12 >= KSB) tr_wait_sb += wait_ge(scnt, min(t0 + 17 - KSB, m + 1), status);
        const uint32_t out_base = lds_addr(ring_out + ring_slot(t0 + 1));
        const uint32_t pa = has_consumer && lane == kWave - 1 ? out_base : scr;
        if (t0 + kSub <= m) {
            cs2_core_group<LOCAL, TBL, KSB, false, 0, DIAG>(I, SDh, SM, psm, fl, ra, rb, t0, m, c1v, sc, ring_in, wcnt_in, sb, lane, pa, scr, cnt_addr, hv, tr_wait_in, status);
            cs2_core_group<LOCAL, TBL, KSB, false, 1, DIAG>(I, SDh, SM, psm, fl, rb, ra, t0, m, c1v, sc, ring_in, wcnt_in, sb, lane, pa, scr, cnt_addr, hv, tr_wait_in, status);
            cs2_core_group<LOCAL, TBL, KSB, false, 2, DIAG>(I, SDh, SM, psm, fl, ra, rb, t0, m, c1v, sc, ring_in, wcnt_in, sb, lane, pa, scr, cnt_addr, hv, tr_wait_in, status);
            cs2_core_group<LOCAL, TBL, KSB, false, 3, DIAG>(I, SDh, SM, psm, fl, rb, ra, t0, m, c1v, sc, ring_in, wcnt_in, sb, lane, pa, scr, cnt_addr, hv, tr_wait_in, status);
        } else {
            cs2_core_group<LOCAL, TBL, KSB, true, 0, DIAG>(I, SDh, SM, psm, fl, ra, rb, t0, m, c1v, sc, ring_in, wcnt_in, sb, lane, pa, scr, cnt_addr, hv, tr_wait_in, status);
            cs2_core_group<LOCAL, TBL, KSB, true, 1, DIAG>(I, SDh, SM, psm, fl, rb, ra, t0, m, c1v, sc, ring_in, wcnt_in, sb, lane, pa, scr, cnt_addr, hv, tr_wait_in, status);
            cs2_core_group<LOCAL, TBL, KSB, true, 2, DIAG>(I, SDh, SM, psm, fl, ra, rb, t0, m, c1v, sc, ring_in, wcnt_in, sb, lane, pa, scr, cnt_addr, hv, tr_wait_in, status);
            cs2_core_group<LOCAL, TBL, KSB, true, 3, DIAG>(I, SDh, SM, psm, fl, rb, ra, t0, m, c1v, sc, ring_in, wcnt_in, sb, lane, pa, scr, cnt_addr, hv, tr_wait_in, status);
        }
        lds_store_lane0(rcnt_in, min(t0 + kSub + 5, m + 1));
    }
    if (trace && lane == 0) {
        StripTrace tr;
        tr.t_start = tr_start; tr.t_first = tr_first; tr.t_end = stamp_rt();
        tr.wait_in = (int)(tr_win0 + tr_wait_in); tr.wait_out = (int)tr_wait_sb;
        tr.clk = stamp_clk() - clk_first;
        for (int q = 0; q < kTraceQ - 1; ++q) tr.t_q[q] = tr_q[q];
        // (t_q[kTraceQ - 1] belongs to the side wave: its own wait iterations)
        long long* d = &trace[s].t_start;
        d[0] = tr.t_start; d[1] = tr.t_first; d[2] = tr.t_end;
        trace[s].wait_in = tr.wait_in; trace[s].wait_out = tr.wait_out; trace[s].clk = tr.clk;
        for (int q = 0; q < kTraceQ - 1; ++q) trace[s].t_q[q] = tr.t_q[q];
    }
}

// The side wave's per-column work: retrace priority bits and the landing
// column (gx_internal.h; keys (lane + 1) << 24 | (E + 64), a delete cell
// takes the nearest non-delete lane above, or the top boundary column j).
// Ek = the scanned key of (i, j - 1) on entry, of (i, j) on return: E + 64 in
// its low 24 bits, the source lane above them (the skeleton and the results
// keep it; readers mask it off).  The lane field is replaced by one v_bfi_b32
// when the next key is built, so no mask sits on the chain.
__device__ __forceinline__ void cs2_side_bits(const int In, const int Sn, const int Dn, const int t, const int kl,
                                              const uint32_t low24, int& Ek, uint32_t& cI, uint32_t& cD) {
    const int IS = max(In, Sn);
    const bool m1 = In > Sn, m2 = Dn > IS;          // insert beats sub; delete beats both
    // the landing-column chain (depends on the previous column's Ek only
    // through etl and the select): builtins, so that the compiler fills its
    // DPP wait states with the independent compares and code bits
    const int etl = shr1(t + 64, Ek);               // lane 0: (i0, j - 1) on the boundary -> E = j - 1
    const int dkey = t + 65;                        // delete with no non-delete lane above: E = j
    int key = (int)((((uint32_t)(m1 ? Ek : etl)) & low24) | (uint32_t)kl);
    key = m2 ? dkey : key;
    cI = cI + cI + (m1 ? 1u : 0u);
    cD = cD + cD + (m2 ? 1u : 0u);
    Ek = scan_max64(key);
}

// Per-strip state of the side wave.
struct Cs2Side {
    int Ep;                 // scanned key of (i, j - 1): E + 64 in the low 24 bits (landing column, gx_internal.h)
    int e_last;             // the key of the column before the current group (skeleton)
    uint32_t cI, cD;        // code bit-planes of the current 16-column word
    int fl;                 // local: floor'' = -(i + j) g of the next column
    int lbest, lstep, lE;   // local: last max of the row (unshifted), its step and landing column
    int fin_sm, fin_E;      // score_max'' and E + 64 of cell (i, m)
};

// One 4-column group of the side wave (columns t + 1 .. t + 4).
template <bool LOCAL, bool PLANES, int KSB, bool TAIL, int DIAG>
__device__ __forceinline__ void cs2_side_group(Cs2Side& st, const int t, const int m, const int lane, const int kl,
                                               const Scores32& sc, lds_int* wcnt_core, const uint32_t scnt_addr,
                                               const SideGrp* sb, const __amdgpu_buffer_rsrc_t& rI,
                                               const __amdgpu_buffer_rsrc_t& rD, const __amdgpu_buffer_rsrc_t& rS,
                                               const __amdgpu_buffer_rsrc_t& skel_rsrc, const uint32_t skel_voff,
                                               unsigned& twait, int* status) {
    constexpr int kSBG = KSB / 4;
    twait += wait_ge(wcnt_core, TAIL ? min(t + 5, m + 1) : t + 5, status);
    const SideGrp& g = sb[(t >> 2) & (kSBG - 1)];
    const int4 vI = g.v[0][lane], vS = g.v[1][lane], vD = g.v[2][lane];
    publish_all(scnt_addr, TAIL ? min(t + 5, m + 1) : t + 5);   // (after the reads: in-order DS execution)
    if (DIAG == 1 || DIAG >= 3) return;   // (timing only: the side consumes, the core alone sets the pace)
    const int aI[4] = {vI.x, vI.y, vI.z, vI.w}, aS[4] = {vS.x, vS.y, vS.z, vS.w}, aD[4] = {vD.x, vD.y, vD.z, vD.w};
    int e[4];
#pragma unroll
    for (int U = 0; U < 4; ++U) {
        cs2_side_bits(aI[U], aS[U], aD[U], t + U, kl, 0xFFFFFFu, st.Ep, st.cI, st.cD);
        e[U] = st.Ep;
        if (LOCAL) {
            // H(i, j) = SM'' - fl'' (unshifted); the last max of the row wins ties
            const int H = max(max(aI[U], aS[U]), aD[U]) - st.fl;
            const bool nl = (!TAIL || t + U < m) && H >= st.lbest;
            st.lbest = nl ? H : st.lbest; st.lstep = nl ? t + U : st.lstep; st.lE = nl ? st.Ep : st.lE;
            st.fl -= sc.g;
        }
        if (TAIL && t + U == m - 1) { st.fin_sm = max(max(aI[U], aS[U]), aD[U]); st.fin_E = st.Ep; }
    }
    if (PLANES) {
        const uint32_t v = (uint32_t)lane * 16u + (uint32_t)(t >> 2) * (uint32_t)kGroupInts1 * 4u;
        bstore4(rI, v, vI);
        bstore4(rD, v, vD);
        bstore4(rS, v, vS);
    }
    // skeleton: lane 63's E + 64 of columns t .. t + 3 (16-B aligned)
    skel_store4(skel_rsrc, skel_voff + 4u * (uint32_t)t, st.e_last, e[0], e[1], e[2]);
    st.e_last = e[3];
}

template <bool LOCAL, bool PLANES, int KSB, int DIAG>
__device__ __forceinline__ void cs2_side(const PairDev& P, const int s, const int lane, const Scores32& sc,
                                         lds_int* wcnt_core, lds_int* scnt, const SideGrp* sb,
                                         const bool has_consumer, StripRes* sres, PairRes* pres, int* status) {
    const int n = P.n, m = P.m;
    const int i = s * kWave + lane + 1;
    const bool ok = i <= n;
    __amdgpu_buffer_rsrc_t rI, rD, rS;
    if (PLANES) {
        const size_t strip_planes = (size_t)s * P.t4 * kGroupInts1;
        const int pbytes = P.t4 * kGroupInts1 * 4;
        rI = rsrc_of(uniform_ptr(P.pI + strip_planes), pbytes);
        rD = rsrc_of(uniform_ptr(P.pD + strip_planes), pbytes);
        rS = rsrc_of(uniform_ptr(P.pS + strip_planes), pbytes);
    }
    uint32_t* const codes = P.codes + (size_t)s * P.t16 * kWave;
    const __amdgpu_buffer_rsrc_t skel_rsrc =
        rsrc_of(uniform_ptr(P.skel + (size_t)s * P.skel_stride), has_consumer ? 4 * (m + 1) : 0);
    const uint32_t skel_voff = lane == kWave - 1 ? 0u : kSkelOff;
    const uint32_t scnt_addr = lds_addr((const void*)scnt);
    const int kl = (lane + 1) << 24;
    Cs2Side st;
    st.Ep = 63 - lane;                              // column 0: E = -(lane + 1) (+ 64)
    st.e_last = st.Ep;
    st.cI = 0; st.cD = 0;
    st.fl = LOCAL ? -(i + 1) * sc.g : 0;
    st.lbest = ok ? INT_MIN : INT_MAX; st.lstep = 0; st.lE = 0;
    st.fin_sm = 0; st.fin_E = 0;
    unsigned twait = 0;
    for (int t0 = 0; t0 < m; t0 += kSub) {
        // the sub-block holding column m always runs as a tail (the end cell is taken there)
        if (t0 + kSub < m) {
#pragma unroll
            for (int G = 0; G < 4; ++G)
                cs2_side_group<LOCAL, PLANES, KSB, false, DIAG>(st, t0 + 4 * G, m, lane, kl, sc, wcnt_core, scnt_addr, sb,
                                                          rI, rD, rS, skel_rsrc, skel_voff, twait, status);
        } else {
#pragma unroll
            for (int G = 0; G < 4; ++G)
                cs2_side_group<LOCAL, PLANES, KSB, true, DIAG>(st, t0 + 4 * G, m, lane, kl, sc, wcnt_core, scnt_addr, sb,
                                                         rI, rD, rS, skel_rsrc, skel_voff, twait, status);
        }
        gstore1(codes + (size_t)(t0 >> 4) * kWave + lane, (st.cD << 16) | (st.cI & 0xFFFFu));
    }
    // the last group's fourth column (16 ceil(m / 16): stored only if it is m)
    skel_store(skel_rsrc, skel_voff + 4u * (uint32_t)((m + 15) & ~15), st.e_last);
    if (LOCAL) {
        const int lb = ok ? st.lbest : INT_MIN;
        int lmx = lb;
        for (int off = 32; off > 0; off >>= 1) lmx = max(lmx, __shfl_xor(lmx, off));
        const unsigned long long lmask = __ballot(ok && lb == lmx);
        const int ll = lmask ? (63 - __clzll((long long)lmask)) : 0;
        const int l_step = __shfl(st.lstep, ll), l_E = __shfl(st.lE, ll);
        if (lane == 0) {
            StripRes r;
            r.best = INT_MIN; r.bi = 0; r.bj = 0; r.bl = 0;
            r.lbest = lmx; r.li = s * kWave + ll + 1; r.lj = l_step + 1; r.lE = (l_E & 0xFFFFFF) - 64;
            sres[P.strip_base + s] = r;
        }
    }
    if (ok && i == n) { pres->end_SM = st.fin_sm; pres->end_E = (st.fin_E & 0xFFFFFF) - 64; }
    if (P.trace && lane == 0) P.trace[s].t_q[kTraceQ - 1] = (long long)twait;   // diagnostics
}

template <int W, bool LOCAL, bool PLANES, bool TBL, int DIAG = 0>
__global__ __launch_bounds__((2 * W + 1) * kWave) void fill_cs2_kernel(const PairDev* __restrict__ pairs,
                                                                       const int npairs, const int total_bands,
                                                                       int* band_counter, StripRes* sres,
                                                                       PairRes* pres, const Scores32 sc) {
    constexpr int KSB = W <= 4 ? 32 : 16;
    __shared__ Rec rings[W + 1][kRing];
    __shared__ SideGrp sbuf[W][KSB / 4];
    __shared__ uint32_t push_scratch[W][kPushScratch];   // lanes 0-62's pushes: 4 B per lane + the record offsets
    __shared__ int wcnt[W + 1];
    __shared__ int rcnt[W + 1];
    __shared__ int scnt[W];
    __shared__ int band_sh;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int lane = threadIdx.x & (kWave - 1);
    for (;;) {
        if (threadIdx.x == 0) band_sh = atomicAdd(band_counter, 1);
        if (threadIdx.x < W + 1) { wcnt[threadIdx.x] = 0; rcnt[threadIdx.x] = 0; }
        if (threadIdx.x < W) scnt[threadIdx.x] = 0;
        __syncthreads();
        const int b = __builtin_amdgcn_readfirstlane(band_sh);
        if (b >= total_bands) return;
        const int2 ob = reinterpret_cast<const int2*>(pairs + npairs)[b];
        const int p = __builtin_amdgcn_readfirstlane(ob.x);
        const PairDev& P = pairs[p];
        const int lb = __builtin_amdgcn_readfirstlane(ob.y);
        const int s0 = lb * W;
        if (DIAG >= 5 && wave >= W && wave < 2 * W) {
            // (timing only: the core waves and the I/O wave alone -- no side)
        } else if (wave < 2 * W) {
            const int k = wave < W ? wave : wave - W;
            const int s = s0 + k;
            if (s < P.strips) {
                const bool last_in_band = k == W - 1;
                const bool has_consumer = last_in_band ? (lb + 1 < P.bands) : (s + 1 < P.strips);
                if (wave < W)
                    cs2_core<LOCAL, TBL, KSB, DIAG>(P, s, lane, sc, rings[k], rings[k + 1], (lds_int*)&wcnt[k],
                                              (lds_int*)&rcnt[k], (lds_int*)&wcnt[k + 1], (lds_int*)&rcnt[k + 1],
                                              (lds_int*)&scnt[k], sbuf[k], has_consumer, band_counter + 1,
                                              lds_addr(push_scratch[k]));
                else
                    cs2_side<LOCAL, PLANES, KSB, DIAG>(P, s, lane, sc, (lds_int*)&wcnt[k + 1], (lds_int*)&scnt[k],
                                                 sbuf[k], has_consumer, sres, pres + p, band_counter + 1);
            }
        } else {
            io_wave<TBL, kIoChunk1, true, 8>(P, lb, lane, sc, rings[0], rings[W], (lds_int*)&wcnt[0],
                                             (lds_int*)&rcnt[0], (lds_int*)&wcnt[W], (lds_int*)&rcnt[W],
                                             lb + 1 < P.bands, band_counter + 1);
        }
        __syncthreads();
    }
}

template <int W, bool LOCAL, bool PLANES, bool TBL>
static hipError_t launch_cs2_t(const PairDev* d_pairs, int npairs, int total_bands, int* d_counter, StripRes* d_sres,
                               PairRes* d_pres, Scores32 sc, int grid, hipStream_t st) {
    // GX_CS2_DIAG (timing diagnostics, wrong results): 1 = the side only
    // consumes the staging, 2 = the core skips the recurrence, 3 = 1 and the
    // core stages nothing, 4 = 3 and the core reads no ring records, 5 = 4 with
    // the side waves idle (the core wave and the I/O wave alone on the CU); 6, 7, 8 = 5
    // with the builtin DPP moves, without the counters, without the pushes
    if constexpr (W == 2 && !LOCAL && PLANES && TBL) {
        if (const char* e = getenv("GX_CS2_DIAG"); e && atoi(e) >= 1 && atoi(e) <= 9) {
#define GX_CS2_DG(D) hipLaunchKernelGGL((fill_cs2_kernel<W, LOCAL, PLANES, TBL, D>), dim3(grid), \
                                        dim3((2 * W + 1) * kWave), 0, st, d_pairs, npairs, total_bands, d_counter, \
                                        d_sres, d_pres, sc)
            switch (atoi(e)) {
                case 1: GX_CS2_DG(1); break;
                case 2: GX_CS2_DG(2); break;
                case 3: GX_CS2_DG(3); break;
                case 4: GX_CS2_DG(4); break;
                case 5: GX_CS2_DG(5); break;
                case 6: GX_CS2_DG(6); break;
                case 7: GX_CS2_DG(7); break;
                case 8: GX_CS2_DG(8); break;
                default: GX_CS2_DG(9); break;
            }
#undef GX_CS2_DG
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((fill_cs2_kernel<W, LOCAL, PLANES, TBL>), dim3(grid), dim3((2 * W + 1) * kWave), 0, st, d_pairs,
                       npairs, total_bands, d_counter, d_sres, d_pres, sc);
    return hipGetLastError();
}

template <bool LOCAL, bool PLANES, bool TBL>
static hipError_t launch_cs2_w(int W, const PairDev* d_pairs, int npairs, int total_bands, int* d_counter,
                               StripRes* d_sres, PairRes* d_pres, Scores32 sc, int grid, hipStream_t st) {
    switch (W) {
        case 1: return launch_cs2_t<1, LOCAL, PLANES, TBL>(d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc, grid, st);
        case 2: return launch_cs2_t<2, LOCAL, PLANES, TBL>(d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc, grid, st);
        case 3: return launch_cs2_t<3, LOCAL, PLANES, TBL>(d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc, grid, st);
        case 4: return launch_cs2_t<4, LOCAL, PLANES, TBL>(d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc, grid, st);
        case 7: return launch_cs2_t<7, LOCAL, PLANES, TBL>(d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc, grid, st);
        default: return hipErrorInvalidValue;
    }
}

// Band widths instantiated (must match gx_api_plan.cpp kCs2Widths).
hipError_t launch_fill_cs2(int W, bool local, bool planes, bool tbl, const PairDev* d_pairs, int npairs,
                           int total_bands, int* d_counter, StripRes* d_sres, PairRes* d_pres, Scores32 sc, int grid,
                           hipStream_t st) {
#define GX_CS2_CASE(LO, PL, TB)                                                                                  \
    if (local == LO && planes == PL && tbl == TB)                                                               \
        return launch_cs2_w<LO, PL, TB>(W, d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc, grid, st);
    GX_CS2_CASE(false, false, false)
    GX_CS2_CASE(false, false, true)
    GX_CS2_CASE(false, true, false)
    GX_CS2_CASE(false, true, true)
    GX_CS2_CASE(true, false, false)
    GX_CS2_CASE(true, false, true)
    GX_CS2_CASE(true, true, false)
    GX_CS2_CASE(true, true, true)
#undef GX_CS2_CASE
    return hipErrorInvalidValue;
}

}  // namespace gx
