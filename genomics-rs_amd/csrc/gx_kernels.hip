// gx_kernels.hip -- CDNA4 (gfx950) kernels for the Gotoh-style affine-gap
// fill of nlaha/genomics-rs (src/alignment/algo.rs:151-282) and the
// per-cell-max traceback walk (algo.rs:339-422).
//
// Fill: one workgroup = one BAND of W 128-row strips (W compute waves) + 1 I/O
// wave; persistent workgroups (one per CU) take bands from an atomic queue.
//   * lane l of a compute wave owns rows 128*strip + 2l + 1 (A) and + 2 (B)
//     and sweeps the columns on the anti-diagonal skew (step t -> column
//     t - l + 1), row A then row B each step;
//   * the row above arrives through a 64-lane DPP wave_shr:1 (lane l reads
//     lane l-1's row B of the previous step); lane 0 takes it from an LDS ring
//     filled by the wave above (or by the I/O wave at a band boundary);
//   * lane 63's row-B cell is pushed into the LDS ring of the wave below;
//   * the three int32 score planes are written 16 B/lane/row every 4 steps
//     into the strip-major anti-diagonal layout (gx_internal.h) -- 1 KiB
//     contiguous per store -- plus the traceback codes and the landing-column
//     skeleton of the strip's bottom row;
//   * bands are taken in order, so the band a workgroup waits on is always
//     held by a running workgroup (no residency assumption); band-to-band
//     rows go through HBM with write-through (sc1) 8-byte agent atomics and a
//     per-boundary progress counter (cdna_hip_programming.md Guideline 16).
// No MFMA: the recurrence is an integer max-plus, not a contraction.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>
#include "gx_internal.h"

#include "gx_device.h"
#include "gx_io.h"
#include "gx_lcs.h"

namespace gx {



#ifndef GX_FILL_MIN_WAVES_TRACK
#define GX_FILL_MIN_WAVES_TRACK 2
#endif

// DP state of one row (the cell left of the one being computed, i.e. (i, j-1)
// in the reference's "top" naming, algo.rs:225).  A lane owns two rows of its
// strip: A = 128*strip + 2*lane + 1 and B = A + 1 (kRowsPerLane).
struct RowState {
    int I, SD, Dd, SM, SMtl;   // insert, max(sub, delete), delete-successor, score_max, SM(i-1, j-1)
    int L, Ltl;                // LCS field (TRACK only)
    int best, bstep, bl;       // first strict max of the row (TRACK only)
    int lbest, lstep, lE;      // last max of the row (LOCAL only) and its landing column
    uint32_t cI, cD;           // traceback code bit-planes (16 steps each)
    int E, Etl;                // landing column (gx_internal.h) of (i, j-1) and of (i-1, j-1)
};
struct LaneState {
    RowState a, b;
    int c2c;                   // s2[j-1] of the lane's current column
};

// Lane 63 pushes its row-B cell (the strip's bottom row) into the LDS ring of
// the wave below, under a lane-63 exec mask (no branch, no register tuple).
// Record = {dd, sm, c2, l}; without TRACK the l word is not written.  Compute
// waves run with all 64 lanes active, so exec is restored to -1, not saved.
// U = step within the 16-step sub-block (constant LDS offsets).  No global
// memory access in here: an SGPR address written by a VALU op (readfirstlane)
// needs wait states before a VMEM instruction reads it, which the compiler
// only inserts for the instructions it emits itself.
template <int U, bool TRACK>
__device__ __forceinline__ void push63(uint32_t base, const LaneState& st, unsigned long long m63) {
    if (TRACK)
        asm volatile(
            "s_mov_b64 exec, %0\n\t"
            "ds_write2_b32 %1, %2, %3 offset0:%6 offset1:%7\n\t"
            "ds_write2_b32 %1, %4, %5 offset0:%8 offset1:%9\n\t"
            "s_mov_b64 exec, -1"
            :
            : "s"(m63), "v"(base), "v"(st.b.Dd), "v"(st.b.SM), "v"(st.c2c), "v"(st.b.L), "i"(4 * U),
              "i"(4 * U + 1), "i"(4 * U + 2), "i"(4 * U + 3)
            : "memory");
    else
        asm volatile(
            "s_mov_b64 exec, %0\n\t"
            "ds_write2_b32 %1, %2, %3 offset0:%5 offset1:%6\n\t"
            "ds_write_b32 %1, %4 offset:%7\n\t"
            "s_mov_b64 exec, -1"
            :
            : "s"(m63), "v"(base), "v"(st.b.Dd), "v"(st.b.SM), "v"(st.c2c), "i"(4 * U), "i"(4 * U + 1),
              "i"(16 * U + 8)
            : "memory");
}

// The same push followed, in the same lane-63 window, by the store of the
// ring's write counter: LDS executes one wave's DS operations in order, so a
// consumer that sees the counter also sees every record pushed before it.
template <int U, bool TRACK>
__device__ __forceinline__ void push63_pub(uint32_t base, const LaneState& st, unsigned long long m63,
                                           uint32_t cnt_addr, int cnt) {
    if (TRACK)
        asm volatile(
            "s_mov_b64 exec, %0\n\t"
            "ds_write2_b32 %1, %2, %3 offset0:%8 offset1:%9\n\t"
            "ds_write2_b32 %1, %4, %5 offset0:%10 offset1:%11\n\t"
            "ds_write_b32 %6, %7\n\t"
            "s_mov_b64 exec, -1"
            :
            : "s"(m63), "v"(base), "v"(st.b.Dd), "v"(st.b.SM), "v"(st.c2c), "v"(st.b.L), "v"(cnt_addr), "v"(cnt),
              "i"(4 * U), "i"(4 * U + 1), "i"(4 * U + 2), "i"(4 * U + 3)
            : "memory");
    else
        asm volatile(
            "s_mov_b64 exec, %0\n\t"
            "ds_write2_b32 %1, %2, %3 offset0:%7 offset1:%8\n\t"
            "ds_write_b32 %1, %4 offset:%9\n\t"
            "ds_write_b32 %5, %6\n\t"
            "s_mov_b64 exec, -1"
            :
            : "s"(m63), "v"(base), "v"(st.b.Dd), "v"(st.b.SM), "v"(st.c2c), "v"(cnt_addr), "v"(cnt), "i"(4 * U),
              "i"(4 * U + 1), "i"(16 * U + 8)
            : "memory");
}

// Full-group pushes without an exec switch: every lane writes, lane 63 to
// the ring slot and the other lanes to their own scratch slots in LDS
// (per-lane address vaddr, chosen once per sub-block), so the wave never
// leaves full exec.  Same record layout as push63.
template <int U, bool TRACK>
__device__ __forceinline__ void push_all(uint32_t vaddr, const LaneState& st) {
    if (TRACK)
        asm volatile(
            "ds_write2_b32 %0, %1, %2 offset0:%5 offset1:%6\n\t"
            "ds_write2_b32 %0, %3, %4 offset0:%7 offset1:%8"
            :
            : "v"(vaddr), "v"(st.b.Dd), "v"(st.b.SM), "v"(st.c2c), "v"(st.b.L), "i"(4 * U), "i"(4 * U + 1),
              "i"(4 * U + 2), "i"(4 * U + 3)
            : "memory");
    else
        asm volatile(
            "ds_write2_b32 %0, %1, %2 offset0:%4 offset1:%5\n\t"
            "ds_write_b32 %0, %3 offset:%6"
            :
            : "v"(vaddr), "v"(st.b.Dd), "v"(st.b.SM), "v"(st.c2c), "i"(4 * U), "i"(4 * U + 1), "i"(16 * U + 8)
            : "memory");
}
// One cell of the Gotoh recurrence (algo.rs:222-268) for the row in `st`,
// given the cell above (dd_in = its delete-successor = D(i, j), sm_in =
// score_max(i-1, j), l_in = max_matches(i-1, j), e_up = its landing column)
// and s2[j-1].  act = false leaves the row unchanged (ramp lanes outside
// columns 1..m).
template <bool LOCAL, bool MASKED, bool CODES, bool TRACK, bool TBL>
__device__ __forceinline__ void cell(RowState& st, const int dd_in, const int sm_in, const int l_in, const int e_up,
                                     const int c2, const int c1v, const bool act, const int t, const Scores32& sc,
                                     int& oI, int& oD, int& oS, int& oL) {
    const int I_old = st.I;                // I(i, j-1): compact planes' x_I reference
    // algo.rs:231-236  insert_score = top.score_max(g, h+g, h+g)
    // untracked global (layout 0): every value is kept as V - (i + j) g
    // (Scores32.shift), so the insert and delete-successor recurrences lose
    // their "+ g" (one add each) and the sub score's -2g rides in sm / smm
    constexpr bool SHIFT = !LOCAL && !TRACK;
    const int In = LOCAL ? max3i(st.I + sc.g, st.SD + sc.hg, 0)
                         : SHIFT ? max(st.I, st.SD + sc.h) : max(st.I + sc.g, st.SD + sc.hg);
    static_assert(!(TBL && TRACK), "the LCS field needs the match bit");
    const bool mt = c2 == c1v;             // sequence.rs:113-114
    // algo.rs:245-248  sub_score = s_(mis)match + top_left.score_max(0,0,0);
    // TBL: c1v is the row's packed score table (one signed byte per symbol
    // code) and c2 the column's code * 8, so the score is one bit-field
    // extract instead of a compare and a select
    const int Sn = st.SMtl + (TBL ? __builtin_amdgcn_sbfe(c1v, c2, 8) : (mt ? sc.sm : sc.smm));
    const int Dn = dd_in;                  // algo.rs:238-243 (computed by the row above)
    const int IS = max(In, Sn);
    const int SMn = max(IS, Dn);           // cell.score_max(0,0,0); >= floor since In >= floor
    const int SDn = max(Sn, Dn);
    // delete-successor, i.e. D(i+1, j) = this.score_max(hg, g, hg) (algo.rs:238-243)
    const int Ddn = LOCAL ? max3i(IS + sc.hg, Dn + sc.g, 0) : SHIFT ? max(IS + sc.h, Dn) : max(IS + sc.hg, Dn + sc.g);
    int Ln = 0;
    if (TRACK) Ln = max3i(st.L, l_in, st.Ltl + (mt ? 1 : 0));   // algo.rs:250-255
    int En = 0;
    if (CODES) {
        // retrace priority S > I > D against the cell max (algo.rs:351-400):
        // code bit-planes "D beats both" / "I beats S" (decode D ? delete :
        // I ? insert : sub) and the landing column of the path through this
        // cell, taken from the predecessor the priority picks.  One asm block:
        // each compare feeds its select and its code bit at once (no SGPR-pair
        // masks kept alive, no chain sunk to the end of the sub-block).
        // the two compares write their own SGPR pairs, so the selects and the
        // code-bit shifts of the two compares overlap (no serial VCC chain)
        unsigned long long m1, m2, k1, k2;
        asm volatile(
            "v_cmp_gt_i32 %[m1], %[in], %[sn]\n\t"
            "v_cmp_gt_i32 %[m2], %[dn], %[is]\n\t"
            "v_cndmask_b32 %[en], %[etl], %[el], %[m1]\n\t"
            "v_addc_co_u32 %[ci], %[k1], %[ci], %[ci], %[m1]\n\t"
            "v_addc_co_u32 %[cd], %[k2], %[cd], %[cd], %[m2]\n\t"
            "v_cndmask_b32 %[en], %[en], %[eu], %[m2]"
            : [en] "=&v"(En), [ci] "+v"(st.cI), [cd] "+v"(st.cD), [m1] "=&s"(m1), [m2] "=&s"(m2),
              [k1] "=&s"(k1), [k2] "=&s"(k2)
            : [in] "v"(In), [sn] "v"(Sn), [dn] "v"(Dn), [is] "v"(IS), [etl] "v"(st.Etl), [el] "v"(st.E),
              [eu] "v"(e_up));
    }
    if (MASKED) {
        st.I = act ? In : st.I; st.SD = act ? SDn : st.SD; st.Dd = act ? Ddn : st.Dd; st.SM = act ? SMn : st.SM;
        if (TRACK) st.L = act ? Ln : st.L;
        if (CODES) st.E = act ? En : st.E;
    } else {
        st.I = In; st.SD = SDn; st.Dd = Ddn; st.SM = SMn;
        if (TRACK) st.L = Ln;
        if (CODES) st.E = En;
    }
    st.SMtl = sm_in;
    if (CODES) st.Etl = e_up;
    if (TRACK) {
        st.Ltl = l_in;
        // algo.rs:258-262: first strict maximum in row-major order
        const bool nb = act && SMn > st.best;
        st.best = nb ? SMn : st.best; st.bstep = nb ? t : st.bstep; st.bl = nb ? Ln : st.bl;
    }
    if (LOCAL) {
        // algo.rs:310-322: max_by keeps the LAST maximum
        const bool nl = act && SMn >= st.lbest;
        st.lbest = nl ? SMn : st.lbest; st.lstep = nl ? t : st.lstep; st.lE = nl ? En : st.lE;
    }
    oI = In; oD = Dn; oS = Sn; oL = TRACK ? Ln : I_old;   // untracked: oL carries I(i, j-1)
}

// One anti-diagonal step of a compute wave: both rows of every lane at
// column j = t - lane + 1.  Row A's cell above comes from row B of lane-1
// (wave_shr:1; lane 0 from the ring record r), row B's from row A.  Lane 0's
// row A is the strip's top row: its "landing column" from above is its own
// column j = t + 1 (a delete lands on (128s, j), a sub on (128s, j-1)).
template <bool LOCAL, bool MASKED, bool CODES, bool TRACK, bool TBL>
__device__ __forceinline__ void dp_step(LaneState& st, const Rec& r, const int t, const int lane, const int m,
                                        const int c1a, const int c1b, const Scores32& sc, int (&oI)[2],
                                        int (&oD)[2], int (&oS)[2], int (&oL)[2]) {
    const int dd_in = shr1(r.dd, st.b.Dd);
    const int sm_in = shr1(r.sm, st.b.SM);
    const int c2 = shr1(r.c2, st.c2c);
    const int l_in = TRACK ? shr1(r.l, st.b.L) : 0;
    const int e_in = CODES ? shr1(t + 1, st.b.E) : 0;
    const bool act = MASKED ? (unsigned)(t - lane) < (unsigned)m : true;
    cell<LOCAL, MASKED, CODES, TRACK, TBL>(st.a, dd_in, sm_in, l_in, e_in, c2, c1a, act, t, sc, oI[0], oD[0], oS[0],
                                      oL[0]);
    cell<LOCAL, MASKED, CODES, TRACK, TBL>(st.b, st.a.Dd, st.a.SM, st.a.L, st.a.E, c2, c1b, act, t, sc, oI[1], oD[1],
                                      oS[1], oL[1]);
    st.c2c = c2;
}

// Uniform per-strip values of a compute wave, hoisted out of the pair
// descriptor (which lives in global memory the plane stores could alias).
struct WaveCtx {
    int32_t* pI; int32_t* pD; int32_t* pS; int32_t* pL;   // plane bases of this strip
    uint32_t* codes;                                        // code words of this strip
    const Rec* ring_in;
    Rec* ring_out;
    lds_int* wcnt_in;
    lds_int* wcnt_out;
    int* status;
    __amdgpu_buffer_rsrc_t skel_rsrc;                       // skeleton row of this strip (bottom-row E)
    uint32_t skel_voff;                                     // lane 63: 0; other lanes: out of range
    uint32_t scratch;                                       // this lane's LDS scratch slot (full-group pushes)
    uint32_t cnt_addr;                                      // lane 63 with a consumer: the ring counter; else scratch
    int m, lane, c1a, c1b;
    unsigned tr_win;
    // layout 1: one descriptor per plane covering the strip's whole plane; the
    // group offset rides in the VGPR offset (no per-store descriptor SALU)
    __amdgpu_buffer_rsrc_t rI, rD, rS, rL;
};

// Plane stores of the previous 4-step group, issued one plane per step in
// the next group (six 1-KiB stores at the end of a group stall the wave's
// in-order issue; spread out they overlap the next group's arithmetic).
// bytes = 0 (nothing pending) empties the descriptor's range.
struct PendStore {
    int4 I0, I1, D0, D1, S0, S1, L0, L1;   // rows A/B of each plane
    size_t sb_off;                         // the group's sub-block (ints)
    int bytes;
};

template <bool LCSP, int PLANE, int G4P>
__device__ __forceinline__ void pend_store(const PendStore& pd, const WaveCtx& w) {
    constexpr int kSubBytes = kSub / 4 * kGroupInts * 4;
    (void)kSubBytes;
    const uint32_t v0 = (uint32_t)w.lane * 16u + G4P * kGroupInts * 4, v1 = v0 + kWave * 16;
    const int32_t* base = PLANE == 0 ? w.pI : PLANE == 1 ? w.pD : PLANE == 2 ? w.pS : w.pL;
    const auto r = rsrc_of(base + pd.sb_off, pd.bytes);
    bstore4(r, v0, PLANE == 0 ? pd.I0 : PLANE == 1 ? pd.D0 : PLANE == 2 ? pd.S0 : pd.L0);
    bstore4(r, v1, PLANE == 0 ? pd.I1 : PLANE == 1 ? pd.D1 : PLANE == 2 ? pd.S1 : pd.L1);
}

// One 4-step group of a sub-block.  `nxt` holds validated ring records for
// these steps.  The producer's counter is observed and the next group's
// records are read (in that LDS order) before computing, so the read latency
// hides behind the group; if the observed counter did not cover them, they
// are re-read after waiting.  MASKED (ramp-up / ramp-down sub-blocks, some
// lanes outside columns 1..m): state updates are masked per lane and each
// push per step (columns 0..m only: a push past m would land on the slot of
// column c - 256, which a lagging consumer may not have read yet).
template <bool LOCAL, int PLANES, bool CODES, bool TRACK, bool LCSP, bool TBL, bool MASKED, int G4>
__device__ __forceinline__ void group4(LaneState& st, Rec (&nxt)[4], WaveCtx& w, const Scores32& sc,
                                       const int t0, const uint32_t out_base, const bool push_on,
                                       const size_t sb_off, PendStore& pend) {
    constexpr int G4P = (G4 + 3) & 3;   // the pending group's index in its sub-block
    const int t = t0 + 4 * G4;
    Rec cur[4] = {nxt[0], nxt[1], nxt[2], nxt[3]};
    const int need = min(t + 8, w.m) + 1;                     // columns of the next group: t+5 .. t+8
    const int seen_v = *w.wcnt_in;                            // consumed only at the end of the group
    asm volatile("" ::: "memory");
    read4(nxt, w.ring_in + ring_slot(t + 5));
    int bI[4][2], bD[4][2], bS[4][2], bL[4][2];
    // lane 63 holds column t+U-63 before step U: push it (mask 0 when there is
    // no consumer); the last push of a full group also publishes the counter.
    // Skeleton: lane 63's landing column after step U (its column t+U-62).
    const int col0 = t - (kWave - 1);
    if (MASKED) {
        // per step: column in 0..m, else the push is masked off and the skeleton offset out of range
        auto sko = [&](int c) { return (c >= 0 && c <= w.m) ? w.skel_voff + 4u * (uint32_t)c : kSkelOff; };
        push63<4 * G4 + 0, TRACK>(out_base, st, lane63_mask(push_on && col0 >= 0 && col0 <= w.m));
        dp_step<LOCAL, true, CODES, TRACK, TBL>(st, cur[0], t + 0, w.lane, w.m, w.c1a, w.c1b, sc, bI[0], bD[0], bS[0], bL[0]);
        skel_store(w.skel_rsrc, sko(col0 + 1), st.b.E);   // lane 63's column after the step
        if (PLANES == 2) pend_store<LCSP, 0, G4P>(pend, w);
        push63<4 * G4 + 1, TRACK>(out_base, st, lane63_mask(push_on && col0 + 1 >= 0 && col0 + 1 <= w.m));
        dp_step<LOCAL, true, CODES, TRACK, TBL>(st, cur[1], t + 1, w.lane, w.m, w.c1a, w.c1b, sc, bI[1], bD[1], bS[1], bL[1]);
        skel_store(w.skel_rsrc, sko(col0 + 2), st.b.E);   // lane 63's column after the step
        if (PLANES == 2) pend_store<LCSP, 1, G4P>(pend, w);
        push63<4 * G4 + 2, TRACK>(out_base, st, lane63_mask(push_on && col0 + 2 >= 0 && col0 + 2 <= w.m));
        dp_step<LOCAL, true, CODES, TRACK, TBL>(st, cur[2], t + 2, w.lane, w.m, w.c1a, w.c1b, sc, bI[2], bD[2], bS[2], bL[2]);
        skel_store(w.skel_rsrc, sko(col0 + 3), st.b.E);   // lane 63's column after the step
        if (PLANES == 2) pend_store<LCSP, 2, G4P>(pend, w);
        if (PLANES == 2 && LCSP) pend_store<LCSP, 3, G4P>(pend, w);
        push63<4 * G4 + 3, TRACK>(out_base, st, lane63_mask(push_on && col0 + 3 >= 0 && col0 + 3 <= w.m));
        // publish the pushes (same wave, DS operations in order)
        if (push_on && col0 + 3 >= 0 && col0 <= w.m) lds_store_lane0(w.wcnt_out, min(col0 + 3, w.m) + 1);
        dp_step<LOCAL, true, CODES, TRACK, TBL>(st, cur[3], t + 3, w.lane, w.m, w.c1a, w.c1b, sc, bI[3], bD[3], bS[3], bL[3]);
        skel_store(w.skel_rsrc, sko(col0 + 4), st.b.E);   // lane 63's column after the step
    } else {
        // lane 63 (with a consumer) pushes to the ring, the other lanes to scratch
        const uint32_t pa = push_on && w.lane == kWave - 1 ? out_base : w.scratch;
        push_all<4 * G4 + 0, TRACK>(pa, st);
        dp_step<LOCAL, false, CODES, TRACK, TBL>(st, cur[0], t + 0, w.lane, w.m, w.c1a, w.c1b, sc, bI[0], bD[0], bS[0], bL[0]);
        if (PLANES == 2) pend_store<LCSP, 0, G4P>(pend, w);
        const int e0 = st.b.E;              // lane 63: column col0 + 1
        push_all<4 * G4 + 1, TRACK>(pa, st);
        dp_step<LOCAL, false, CODES, TRACK, TBL>(st, cur[1], t + 1, w.lane, w.m, w.c1a, w.c1b, sc, bI[1], bD[1], bS[1], bL[1]);
        if (PLANES == 2) pend_store<LCSP, 1, G4P>(pend, w);
        const int e1 = st.b.E;
        push_all<4 * G4 + 2, TRACK>(pa, st);
        dp_step<LOCAL, false, CODES, TRACK, TBL>(st, cur[2], t + 2, w.lane, w.m, w.c1a, w.c1b, sc, bI[2], bD[2], bS[2], bL[2]);
        if (PLANES == 2) pend_store<LCSP, 2, G4P>(pend, w);
        if (PLANES == 2 && LCSP) pend_store<LCSP, 3, G4P>(pend, w);
        const int e2 = st.b.E;
        push_all<4 * G4 + 3, TRACK>(pa, st);
        publish_all(w.cnt_addr, col0 + 3 + 1);   // after the records: LDS runs one wave's DS ops in order
        dp_step<LOCAL, false, CODES, TRACK, TBL>(st, cur[3], t + 3, w.lane, w.m, w.c1a, w.c1b, sc, bI[3], bD[3], bS[3], bL[3]);
        // lane 63's landing columns of columns col0+1 .. col0+4 (full groups: all in 1..m), one store
        skel_store4(w.skel_rsrc, w.skel_voff + 4u * (uint32_t)(col0 + 1), e0, e1, e2, st.b.E);
    }
    if (PLANES == 1) {
        // this group's cells, 16 B per lane per row and plane, stored now
        // (the widest bands have no VGPRs to keep them for the next group)
        constexpr int kSubBytes = kSub / 4 * kGroupInts * 4;      // one sub-block of one plane
        constexpr uint32_t kG = G4 * kGroupInts * 4;              // this group within it
        const uint32_t v0 = (uint32_t)w.lane * 16u + kG, v1 = v0 + kWave * 16;
        const auto rI = rsrc_of(w.pI + sb_off, kSubBytes), rD = rsrc_of(w.pD + sb_off, kSubBytes),
                   rS = rsrc_of(w.pS + sb_off, kSubBytes);
        bstore4(rI, v0, make_int4(bI[0][0], bI[1][0], bI[2][0], bI[3][0]));
        bstore4(rD, v0, make_int4(bD[0][0], bD[1][0], bD[2][0], bD[3][0]));
        bstore4(rS, v0, make_int4(bS[0][0], bS[1][0], bS[2][0], bS[3][0]));
        bstore4(rI, v1, make_int4(bI[0][1], bI[1][1], bI[2][1], bI[3][1]));
        bstore4(rD, v1, make_int4(bD[0][1], bD[1][1], bD[2][1], bD[3][1]));
        bstore4(rS, v1, make_int4(bS[0][1], bS[1][1], bS[2][1], bS[3][1]));
        if (LCSP) {
            const auto rL = rsrc_of(w.pL + sb_off, kSubBytes);
            bstore4(rL, v0, make_int4(bL[0][0], bL[1][0], bL[2][0], bL[3][0]));
            bstore4(rL, v1, make_int4(bL[0][1], bL[1][1], bL[2][1], bL[3][1]));
        }
    }
    if (PLANES == 3) {
        // compact planes: this group's 4 steps of a row are one dword per lane
        // and plane (x_I, x_S, x_D above put_byte), 256 B per wave, stored
        // at the group's end (storing them during the next group measured 2 %
        // slower, profiles/r01k_d8_pipe_ab.txt)
        uint32_t xI[2], xS[2], xD[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            put_byte<0>(xI[h], bI[0][h], bL[0][h]); put_byte<0>(xS[h], bS[0][h], bI[0][h]); put_byte<0>(xD[h], bD[0][h], bI[0][h]);
            put_byte<1>(xI[h], bI[1][h], bL[1][h]); put_byte<1>(xS[h], bS[1][h], bI[1][h]); put_byte<1>(xD[h], bD[1][h], bI[1][h]);
            put_byte<2>(xI[h], bI[2][h], bL[2][h]); put_byte<2>(xS[h], bS[2][h], bI[2][h]); put_byte<2>(xD[h], bD[2][h], bI[2][h]);
            put_byte<3>(xI[h], bI[3][h], bL[3][h]); put_byte<3>(xS[h], bS[3][h], bI[3][h]); put_byte<3>(xD[h], bD[3][h], bI[3][h]);
        }
        constexpr int kSubBytes = kSub / 4 * kGroupInts;              // one sub-block of one byte plane
        constexpr uint32_t kG = G4 * kGroupInts;
        const uint32_t v0 = (uint32_t)w.lane * 4u + kG, v1 = v0 + kWave * 4;
        const auto rI = rsrc_of((const uint8_t*)w.pI + sb_off, kSubBytes),
                   rD = rsrc_of((const uint8_t*)w.pD + sb_off, kSubBytes),
                   rS = rsrc_of((const uint8_t*)w.pS + sb_off, kSubBytes);
        bstore1(rI, v0, xI[0]); bstore1(rS, v0, xS[0]); bstore1(rD, v0, xD[0]);
        bstore1(rI, v1, xI[1]); bstore1(rS, v1, xS[1]); bstore1(rD, v1, xD[1]);
    }
    if (PLANES == 2) {
        // this group's cells: 16 B per lane per row and plane, stored during the next group
        pend.I0 = make_int4(bI[0][0], bI[1][0], bI[2][0], bI[3][0]);
        pend.I1 = make_int4(bI[0][1], bI[1][1], bI[2][1], bI[3][1]);
        pend.D0 = make_int4(bD[0][0], bD[1][0], bD[2][0], bD[3][0]);
        pend.D1 = make_int4(bD[0][1], bD[1][1], bD[2][1], bD[3][1]);
        pend.S0 = make_int4(bS[0][0], bS[1][0], bS[2][0], bS[3][0]);
        pend.S1 = make_int4(bS[0][1], bS[1][1], bS[2][1], bS[3][1]);
        if (LCSP) {
            pend.L0 = make_int4(bL[0][0], bL[1][0], bL[2][0], bL[3][0]);
            pend.L1 = make_int4(bL[0][1], bL[1][1], bL[2][1], bL[3][1]);
        }
        pend.sb_off = sb_off;
        pend.bytes = kSub / 4 * kGroupInts * 4;
    }
    if (__builtin_amdgcn_readfirstlane(seen_v) < need) {      // producer was behind: wait, re-read
        w.tr_win += wait_ge(w.wcnt_in, need, w.status);
        read4(nxt, w.ring_in + ring_slot(t + 5));
    }
    // keep groups apart: interleaving two groups' outputs overflows the VGPR budget
    __builtin_amdgcn_sched_barrier(0);
}

// One 16-step sub-block: four groups.  MASKED for the ramp-up (t0 < 64) and
// ramp-down (columns past m) sub-blocks.
template <bool LOCAL, int PLANES, bool CODES, bool TRACK, bool LCSP, bool TBL, bool MASKED>
__device__ __forceinline__ void sub_block(LaneState& st, Rec (&nxt)[4], WaveCtx& w, const Scores32& sc, const int t0,
                                          const uint32_t out_base, const bool push_on, const size_t sb_off,
                                          PendStore& pend) {
    group4<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, MASKED, 0>(st, nxt, w, sc, t0, out_base, push_on, sb_off, pend);
    group4<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, MASKED, 1>(st, nxt, w, sc, t0, out_base, push_on, sb_off, pend);
    group4<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, MASKED, 2>(st, nxt, w, sc, t0, out_base, push_on, sb_off, pend);
    group4<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, MASKED, 3>(st, nxt, w, sc, t0, out_base, push_on, sb_off, pend);
}

__device__ __forceinline__ void init_row(RowState& rs, const int i, const bool row_ok, const Scores32& sc,
                                         const bool d8 = false, const bool shift = false) {
    // cell (i, 0): algo.rs:204-211
    const int D0 = sc.h + i * sc.g;
    // compact planes: I(i, 0) = negative_inf is replaced by H(i, 0) + h
    // (H(i, 0) = max(D0, floor)), which gives column 1 the same insert score,
    // max(I + g, max(S, D) + h + g [, 0]) = max(H(i, 0) + h + g [, 0]); the
    // decoder's row base is the same H(i, 0) + h
    rs.I = d8 ? max(D0, sc.floor_) + sc.h : kNeg;
    rs.SD = D0;                                   // max(sub=neg_inf, delete)
    rs.SM = max(D0, sc.floor_);
    rs.Dd = max3i(kNeg + sc.hg, D0 + sc.g, sc.floor_);
    rs.L = 0; rs.Ltl = 0;
    rs.SMtl = 0;
    rs.best = row_ok ? INT_MIN : INT_MAX; rs.bstep = 0; rs.bl = 0;
    rs.lbest = row_ok ? INT_MIN : INT_MAX; rs.lstep = 0;
    rs.cI = 0; rs.cD = 0;
    if (shift) {   // V - (i + 0) g; the delete successor belongs to row i + 1
        rs.I -= i * sc.g; rs.SD -= i * sc.g; rs.SM -= i * sc.g; rs.Dd -= (i + 1) * sc.g;
    }
}

template <bool LOCAL, int PLANES, bool CODES, bool TRACK, bool LCSP, bool TBL>
__device__ void compute_wave(const PairDev& P, const int s, const int lane, const Scores32& sc, const Rec* ring_in,
                             Rec* ring_out, lds_int* wcnt_in, lds_int* rcnt_in, lds_int* wcnt_out, lds_int* rcnt_out,
                             const bool has_consumer, StripRes* sres, PairRes* pres, int* status,
                             const uint32_t scratch_base) {
    static_assert(kSub == 16, "16-step sub-blocks (code words, ring alignment)");
    static_assert(kRowsPerLane == 2, "two rows per lane");
    const int n = P.n, m = P.m;
    const int ia = s * kStripRows + kRowsPerLane * lane + 1;   // row A; row B = ia + 1
    const bool ok_a = ia <= n, ok_b = ia + 1 <= n;
    WaveCtx w;
    {
        const size_t strip_planes = (size_t)s * P.t4 * kGroupInts;   // ints per plane per strip
        // compact planes (mode 3): the same element offsets, in bytes
        auto at = [&](int32_t* b) { return PLANES >= 3 ? (int32_t*)((uint8_t*)b + strip_planes) : b + strip_planes; };
        w.pI = PLANES ? at(P.pI) : nullptr;
        w.pD = PLANES ? at(P.pD) : nullptr;
        w.pS = PLANES ? at(P.pS) : nullptr;
        w.pL = LCSP ? P.pL + strip_planes : nullptr;
        w.codes = CODES ? P.codes + (size_t)s * P.t16 * kWave * kRowsPerLane : nullptr;
    }
    w.ring_in = ring_in; w.ring_out = ring_out; w.wcnt_in = wcnt_in; w.wcnt_out = wcnt_out; w.status = status;
    // skeleton row (only stored when there is a strip below: otherwise an empty range)
    w.skel_rsrc = rsrc_of(uniform_ptr(P.skel + (size_t)s * P.skel_stride), has_consumer ? 4 * (m + 1) : 0);
    w.skel_voff = lane == kWave - 1 ? 0u : kSkelOff;
    // scratch: 4-B lane stride (conflict-free), room for a sub-block's 16 record offsets
    w.scratch = scratch_base + 4u * (uint32_t)lane;
    w.cnt_addr = (has_consumer && lane == kWave - 1) ? lds_addr((const void*)wcnt_out) : w.scratch;
    w.m = m; w.lane = lane;
    w.c1a = ok_a ? (int)P.c1[ia - 1] : 0x1FF;   // 0x1FF never equals a byte
    w.c1b = ok_b ? (int)P.c1[ia] : 0x1FF;
    if (TBL) { w.c1a = score_table(w.c1a, sc); w.c1b = score_table(w.c1b, sc); }
    w.tr_win = 0;
    StripTrace* const trace = P.trace;
    const int strip_base = P.strip_base;

    LaneState st;
    init_row(st.a, ia, ok_a, sc, PLANES >= 3, !LOCAL && !TRACK);
    init_row(st.b, ia + 1, ok_b, sc, PLANES >= 3, !LOCAL && !TRACK);
    st.c2c = 0;
    st.b.SMtl = st.a.SM;                          // (A, 0) is row B's top-left for column 1
    // landing columns of column 0: the path reaches column 0 at its own local row
    st.a.E = -(kRowsPerLane * lane + 1);
    st.b.E = -(kRowsPerLane * lane + 2);
    st.b.Etl = st.a.E;
    st.a.lE = 0; st.b.lE = 0;

    if (has_consumer) {
        if (lane == kWave - 1) ring_out[ring_slot(0)] = Rec{st.b.Dd, st.b.SM, 0, st.b.L};
        lds_wait();
        if (lane == 0) *wcnt_out = 1;
    }
    const bool tracing = trace != nullptr;
    long long tr_start = 0, tr_first = 0, clk_first = 0;
    unsigned tr_wout = 0;
    long long tr_q[kTraceQ] = {};
    if (tracing) tr_start = stamp_rt();
    // column 0 of the row above seeds row A's top-left of column 1; columns
    // 1..4 feed the first step group
    w.tr_win += wait_ge(wcnt_in, min(4, m) + 1, status);
    Rec nxt[4];
    {
        const Rec r0 = ring_in[ring_slot(0)];
        // lane 0: (row above the strip, 0); other lanes: row B of lane-1 at column 0
        st.a.SMtl = shr1(r0.sm, st.b.SM);
        st.a.Etl = shr1(0, st.b.E);               // lane 0: (128s, 0) itself
        st.a.Ltl = 0;
        read4(nxt, ring_in + ring_slot(1));
    }
    if (tracing) { tr_first = stamp_rt(); clk_first = stamp_clk(); }
    const int T = m + kWave;                          // lane 63 pushes column m at step m + 63
    const bool rolled_only = (sc.dbg & 1) != 0;
    PendStore pend;
    pend.sb_off = 0; pend.bytes = 0;   // nothing pending before the first group
    for (int t0 = 0; t0 < T; t0 += kSub) {
        const int last_col = min(t0 + kSub - 1 - (kWave - 1), m);   // last column pushed here
        if (has_consumer && last_col >= kRing) tr_wout += wait_ge(rcnt_out, last_col - kRing + 1, status);
        if (tracing) {   // progress stamps at k/(kTraceQ+1) of the sweep
            const int q = (int)((long long)t0 * (kTraceQ + 1) / T) - 1;
            if (q >= 0 && q < kTraceQ && tr_q[q] == 0) tr_q[q] = stamp_rt();
        }
        const size_t sb_off = (size_t)(t0 >> 2) * kGroupInts;         // this sub-block's plane offset (ints)
        const bool full = (t0 >= kWave) && (t0 + kSub - 1 <= m - 1) && !rolled_only;
        const uint32_t out_base = lds_addr(ring_out + ring_slot(t0 - (kWave - 1)));
        if (full)
            sub_block<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, false>(st, nxt, w, sc, t0, out_base, has_consumer, sb_off,
                                                                     pend);
        else
            sub_block<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, true>(st, nxt, w, sc, t0, out_base, has_consumer, sb_off,
                                                                    pend);
        if (CODES) {
            // codes[strip][t/16][lane][row-in-lane]: 8 B per lane
            typedef unsigned v2u __attribute__((ext_vector_type(2)));
            typedef __attribute__((address_space(1))) v2u gv2u;
            const v2u cw = {(st.a.cD << 16) | (st.a.cI & 0xFFFFu), (st.b.cD << 16) | (st.b.cI & 0xFFFFu)};
#ifndef GX_DIAG_NO_CODES
            *(gv2u*)(w.codes + ((size_t)(t0 >> 4) * kWave + lane) * kRowsPerLane) = cw;
#endif
        }
        // every ring read up to column t0+20 (incl. the next group's) was issued before this store
        lds_store_lane0(rcnt_in, min(t0 + kSub + 5, m + 1));
    }

    if (PLANES == 2) {   // the last group's planes (group 3 of the last sub-block)
        pend_store<LCSP, 0, 3>(pend, w);
        pend_store<LCSP, 1, 3>(pend, w);
        pend_store<LCSP, 2, 3>(pend, w);
        if (LCSP) pend_store<LCSP, 3, 3>(pend, w);
    }

    // ---- strip reduction of the max trackers ----
    if (TRACK || LOCAL) {
        // per lane: first max -> row A wins ties (earlier row); last max -> row B wins ties
        const int ba = (TRACK && ok_a) ? st.a.best : INT_MIN, bb = (TRACK && ok_b) ? st.b.best : INT_MIN;
        const bool fa = ba >= bb;
        const int best = fa ? ba : bb;
        const int bstep = fa ? st.a.bstep : st.b.bstep, bl = fa ? st.a.bl : st.b.bl, bh = fa ? 0 : 1;
        const int la = (LOCAL && ok_a) ? st.a.lbest : INT_MIN, lb2 = (LOCAL && ok_b) ? st.b.lbest : INT_MIN;
        const bool lbb = lb2 >= la && ok_b;
        const int lbest = lbb ? lb2 : la;
        const int lstep = lbb ? st.b.lstep : st.a.lstep, lh = lbb ? 1 : 0, lE = lbb ? st.b.lE : st.a.lE;
        const bool any_ok = ok_a;
        int mx = best, lmx = lbest;
        for (int off = 32; off > 0; off >>= 1) {
            mx = max(mx, __shfl_xor(mx, off));
            lmx = max(lmx, __shfl_xor(lmx, off));
        }
        const unsigned long long fmask = __ballot(any_ok && best == mx);
        const unsigned long long lmask = __ballot(any_ok && lbest == lmx);
        const int fl = fmask ? (__ffsll((long long)fmask) - 1) : 0;           // lowest lane
        const int ll = lmask ? (63 - __clzll((long long)lmask)) : 0;          // highest lane
        const int f_step = __shfl(bstep, fl), f_l = __shfl(bl, fl), f_h = __shfl(bh, fl);
        const int l_step = __shfl(lstep, ll), l_h = __shfl(lh, ll), l_E = __shfl(lE, ll);
        if (lane == 0) {
            StripRes r;
            r.best = mx; r.bi = s * kStripRows + kRowsPerLane * fl + f_h + 1; r.bj = f_step - fl + 1; r.bl = f_l;
            r.lbest = lmx; r.li = s * kStripRows + kRowsPerLane * ll + l_h + 1; r.lj = l_step - ll + 1; r.lE = l_E;
            sres[strip_base + s] = r;
        }
    }
    // cell (n, m) for the global-mode start (algo.rs:308, 331)
    if (ok_a && ia == n) { pres->end_SM = st.a.SM; pres->end_E = st.a.E; }
    if (ok_b && ia + 1 == n) { pres->end_SM = st.b.SM; pres->end_E = st.b.E; }
    if (tracing && lane == 0) {
        StripTrace tr;
        tr.t_start = tr_start; tr.t_first = tr_first; tr.t_end = stamp_rt();
        tr.wait_in = (int)w.tr_win; tr.wait_out = (int)tr_wout;
        tr.clk = stamp_clk() - clk_first;
        for (int q = 0; q < kTraceQ; ++q) tr.t_q[q] = tr_q[q];
        trace[s] = tr;
    }
}

// ===========================================================================
// Column-step fill (layout 1, gx_internal.h "colstep"): a strip is 64 rows,
// lane l owns row i = 64 s + l + 1, and step t computes column j = t + 1 of
// every row at once.  The insert (left) and sub (top-left) predecessors are
// the lane's own previous column and lane l-1's previous column (DPP
// wave_shr:1); the delete chain down the column,
//     D(i, j) = max(IS(i-1, j) + h + g, D(i-1, j) + g [, 0])   (algo.rs:238-243)
// is a max-plus linear recurrence along the lanes, solved as one inclusive
// prefix max over the wave (6 DPP steps):
//     D(l) = l*g + max_{k <= l} Z(k),  Z(0) = D(i0, j) (from the strip above),
//     Z(k) = IS(k-1) + h + g - k*g  [local: max(.., -k*g)]   (k >= 1).
// The landing column follows the same chain: a cell whose move is "delete"
// takes E from the nearest lane above it whose move is not, found by a prefix
// max over keys (lane << 25) | (E + 64).  No anti-diagonal skew: the strip
// below consumes column j as soon as this strip has produced it, so strips
// follow each other a few columns apart instead of 64 + steps.
// ===========================================================================

struct CsState {
    int I, SD, SM;             // insert, max(sub, delete), score_max of (i, j-1)
    int key;                   // landing-column key of (i, j-1), not yet scanned (see cs_step)
    int L;                     // LCS field of (i, j-1) (TRACK)
    int best, bstep, bl;       // first strict max of the row (TRACK)
    int lbest, lstep, lE;      // last max of the row and its landing column (LOCAL)
    uint32_t cI, cD;           // code bit-planes (16 steps)
    int fin_sm, fin_E;         // score_max and E at column m (cell (n, m) if this lane holds row n)
};
struct CsConst {
    int cY;      // h + g - (l+1) g
    int cZ;      // -(l+1) g (local zero floor of the delete chain)
    int lg;      // l g
    int kl;      // (lane + 1) << 24 (landing-column keys)
    int lg1;     // (l+1) g
    int c1;      // row char (or its packed score table, TBL)
};

// One column for all 64 rows, software-pipelined one column deep on the
// landing column: step t computes the scores of column j = t + 1 and scans
// the landing-column keys of column t (step t-1) in the same DPP sweep as the
// delete chain of column j, returning E(., t) in `e_prev`.
// r = ring record of column j (dd = D(i0, j), c2 = s2[j-1] or its code * 8,
// l = LCS of (i0-1, j)); psm / pl = score_max / LCS of (i0-1, j-1).
template <bool LOCAL, bool CODES, bool TRACK, bool TBL, bool TAIL>
__device__ __forceinline__ void cs_step(CsState& st, const CsConst& k, const Rec& r, const int psm, const int pl,
                                        const int t, const int m, const Scores32& sc, int& oI, int& oD, int& oS,
                                        int& pdd, int& psm_out, int& pl_out, int& e_prev) {
    const int smtl = shr1(psm, st.SM);                                  // SM(i-1, j-1)
    const int In = LOCAL ? max3i(st.I + sc.g, st.SD + sc.hg, 0) : max(st.I + sc.g, st.SD + sc.hg);
    const bool mt = r.c2 == k.c1;
    const int Sn = smtl + (TBL ? __builtin_amdgcn_sbfe(k.c1, r.c2, 8) : (mt ? sc.sm : sc.smm));
    const int IS = max(In, Sn);
    int Y = IS + k.cY;
    if (LOCAL) Y = max(Y, k.cZ);
    int Ln = 0, Dn, Ek = 0, Zs;
    if (TRACK) {
        int x[3] = {shr1(r.dd, Y), st.key, max(st.L, shr1(pl, st.L) + (mt ? 1 : 0))};   // algo.rs:250-255
        scan_max64_n(x);
        Zs = x[0]; Ek = x[1]; Ln = max(x[2], r.l);
    } else if (CODES) {
        int x[2] = {shr1(r.dd, Y), st.key};
        scan_max64_n(x);
        Zs = x[0]; Ek = x[1];
    } else {
        int x[1] = {shr1(r.dd, Y)};
        scan_max64_n(x);
        Zs = x[0];
    }
    Dn = Zs + k.lg;
    // E(i, t) + 64 (keys: ((lane+1) << 24) | (E + 64); a delete cell's key is
    // (t + 64) with lane field 0, so a lane with no non-delete move above it
    // reads the boundary column t -- the path leaves at (i0-1, t))
    const int Ep = Ek & 0xFFFFFF;
    e_prev = Ep;
    const int SMn = max(IS, Dn);
    const int SDn = max(Sn, Dn);
    if (CODES) {
        // D ? delete : I ? insert : sub (algo.rs:351-400).  One asm block: each
        // compare feeds its code bit (v_addc shift-in) and its select, so no
        // SGPR-pair mask stays alive (left to the compiler, a group's masks
        // are kept and spilled to VGPR lanes).  key = delete ? -1 :
        // (lane << 25) | (base + 64), base = E of the insert (own previous
        // column) or sub (top-left) predecessor.
        const int etl = shr1(t + 64, Ep);                               // lane 0: (i0-1, j-1) on the boundary
        const int dkey = t + 65;                                        // delete: boundary column j + 64 (a VGPR:
                                                                        // VOP3 may read one SGPR, the mask)
        unsigned long long m1, m2, k1, k2;
        asm volatile(
            "v_cmp_gt_i32 %[m1], %[in], %[sn]\n\t"
            "v_cmp_gt_i32 %[m2], %[dn], %[is]\n\t"
            "v_cndmask_b32 %[key], %[etl], %[el], %[m1]\n\t"
            "v_addc_co_u32 %[ci], %[k1], %[ci], %[ci], %[m1]\n\t"
            "v_or_b32 %[key], %[key], %[kl]\n\t"
            "v_addc_co_u32 %[cd], %[k2], %[cd], %[cd], %[m2]\n\t"
            "v_cndmask_b32 %[key], %[key], %[dk], %[m2]"
            : [key] "=&v"(st.key), [ci] "+v"(st.cI), [cd] "+v"(st.cD), [m1] "=&s"(m1), [m2] "=&s"(m2),
              [k1] "=&s"(k1), [k2] "=&s"(k2)
            : [in] "v"(In), [sn] "v"(Sn), [dn] "v"(Dn), [is] "v"(IS), [etl] "v"(etl), [el] "v"(Ep),
              [kl] "v"(k.kl), [dk] "v"(dkey));
    }
    if (TRACK) {
        const bool act = TAIL ? t < m : true;
        const bool nb = act && SMn > st.best;
        st.best = nb ? SMn : st.best; st.bstep = nb ? t : st.bstep; st.bl = nb ? Ln : st.bl;
    }
    if (LOCAL) {
        // the last max of step t-1 (its landing column is known now)
        const bool act = t >= 1 && (TAIL ? t <= m : true);
        const bool nl = act && st.SM >= st.lbest;
        st.lbest = nl ? st.SM : st.lbest; st.lstep = nl ? t - 1 : st.lstep; st.lE = nl ? Ep : st.lE;
    }
    if (TAIL && t == m - 1) st.fin_sm = SMn;
    if (TAIL && t == m) st.fin_E = Ep;
    // D(i+1, j) = max(D + g, IS + h + g [, 0]) = (l+1) g + max(Zscan, Y): one step
    // further down the same chain (lane 63's value is the record pushed below)
    pdd = LOCAL ? max3i(IS + sc.hg, Dn + sc.g, 0) : max(Zs, Y) + k.lg1;
    psm_out = SMn;
    pl_out = Ln;
    st.I = In; st.SD = SDn; st.SM = SMn;
    if (TRACK) st.L = Ln;
    oI = In; oD = Dn; oS = Sn;
}

struct CsPend {
    int4 I, D, S, L;   // the previous group's cells (one row per lane)
    uint32_t voff;     // this lane's byte offset in the strip plane; kNoStore: nothing pending
};

template <bool LCSP>
__device__ __forceinline__ void cs_pend_store(const CsPend& pd, const WaveCtx& w, int plane) {
    const auto rr = plane == 0 ? w.rI : plane == 1 ? w.rD : plane == 2 ? w.rS : w.rL;
    bstore4(rr, pd.voff, plane == 0 ? pd.I : plane == 1 ? pd.D : plane == 2 ? pd.S : pd.L);
}

// One 4-column group (columns t+1 .. t+4).  Same ring protocol as group4:
// observe the producer's counter, speculatively read the next group's
// records, compute, re-read after a wait if the counter did not cover them.
template <bool LOCAL, int PLANES, bool CODES, bool TRACK, bool LCSP, bool TBL, bool TAIL, int G4>
__device__ __forceinline__ void cs_group4(CsState& st, const CsConst& kc, Rec (&cur)[4], Rec (&nxt)[4], int& psm,
                                          int& pl, WaveCtx& w, const Scores32& sc, const int t0,
                                          const uint32_t out_base, const bool push_on, CsPend& pend) {
    // cur: this group's validated records; nxt: filled with the next group's
    // (the caller alternates the two buffers, so no records are copied)
    const int t = t0 + 4 * G4;
    const int need = min(t + 8, w.m) + 1;
    const int seen_v = *w.wcnt_in;
    asm volatile("" ::: "memory");
    read4(nxt, w.ring_in + ring_slot(t + 5));
    int oI[4], oD[4], oS[4], oL[4], e[4];
    const uint32_t pa = push_on && w.lane == kWave - 1 ? out_base : w.scratch;
#pragma unroll
    for (int U = 0; U < 4; ++U) {
        int dd, sm, l;
        cs_step<LOCAL, CODES, TRACK, TBL, TAIL>(st, kc, cur[U], psm, pl, t + U, w.m, sc, oI[U], oD[U], oS[U], dd, sm, l,
                                                e[U]);
        oL[U] = l;
        psm = cur[U].sm;
        pl = cur[U].l;
        // lane 63's record of column t+U+1 for the strip below
        if (!TAIL) {
            if (U == 0) cs_push_all<4 * G4 + 0, TRACK>(pa, dd, sm, cur[U].c2, l);
            if (U == 1) cs_push_all<4 * G4 + 1, TRACK>(pa, dd, sm, cur[U].c2, l);
            if (U == 2) cs_push_all<4 * G4 + 2, TRACK>(pa, dd, sm, cur[U].c2, l);
            if (U == 3) { cs_push_all<4 * G4 + 3, TRACK>(pa, dd, sm, cur[U].c2, l); publish_all(w.cnt_addr, t + 5); }
        } else {
            const unsigned long long mk = lane63_mask(push_on && t + U + 1 <= w.m);
            if (U == 0) cs_push63<4 * G4 + 0, TRACK>(out_base, mk, dd, sm, cur[U].c2, l);
            if (U == 1) cs_push63<4 * G4 + 1, TRACK>(out_base, mk, dd, sm, cur[U].c2, l);
            if (U == 2) cs_push63<4 * G4 + 2, TRACK>(out_base, mk, dd, sm, cur[U].c2, l);
            if (U == 3) cs_push63<4 * G4 + 3, TRACK>(out_base, mk, dd, sm, cur[U].c2, l);
            if (U == 3 && push_on && t + 1 <= w.m) lds_store_lane0(w.wcnt_out, min(t + 4, w.m) + 1);
        }
        if (PLANES == 2 && !TAIL && (U < 3 || LCSP)) cs_pend_store<LCSP>(pend, w, U);   // the previous group's plane U
    }
    // lane 63's landing columns of columns t .. t+3 (the strip's bottom row: skeleton)
    if (!TAIL) {
        skel_store4(w.skel_rsrc, w.skel_voff + 4u * (uint32_t)t, e[0], e[1], e[2], e[3]);
    } else {
#pragma unroll
        for (int U = 0; U < 4; ++U)
            skel_store(w.skel_rsrc, t + U <= w.m ? w.skel_voff + 4u * (uint32_t)(t + U) : kSkelOff, e[U]);
    }
    const size_t g_off = (size_t)(t >> 2) * kGroupInts1;
    if (PLANES == 1 || (PLANES == 2 && TAIL)) {
        if (PLANES == 2) {   // flush the pending group first
            cs_pend_store<LCSP>(pend, w, 0); cs_pend_store<LCSP>(pend, w, 1); cs_pend_store<LCSP>(pend, w, 2);
            if (LCSP) cs_pend_store<LCSP>(pend, w, 3);
            pend.voff = kNoStore;
        }
        const uint32_t v = (uint32_t)w.lane * 16u + (uint32_t)g_off * 4u;
        bstore4(w.rI, v, make_int4(oI[0], oI[1], oI[2], oI[3]));
        bstore4(w.rD, v, make_int4(oD[0], oD[1], oD[2], oD[3]));
        bstore4(w.rS, v, make_int4(oS[0], oS[1], oS[2], oS[3]));
        if (LCSP) bstore4(w.rL, v, make_int4(oL[0], oL[1], oL[2], oL[3]));
    } else if (PLANES == 2) {
        pend.I = make_int4(oI[0], oI[1], oI[2], oI[3]);
        pend.D = make_int4(oD[0], oD[1], oD[2], oD[3]);
        pend.S = make_int4(oS[0], oS[1], oS[2], oS[3]);
        if (LCSP) pend.L = make_int4(oL[0], oL[1], oL[2], oL[3]);
        pend.voff = (uint32_t)w.lane * 16u + (uint32_t)g_off * 4u;
    }
    if (__builtin_amdgcn_readfirstlane(seen_v) < need) {
        w.tr_win += wait_ge(w.wcnt_in, need, w.status);
        read4(nxt, w.ring_in + ring_slot(t + 5));
    }
    __builtin_amdgcn_sched_barrier(0);
}

template <bool LOCAL, int PLANES, bool CODES, bool TRACK, bool LCSP, bool TBL>
__device__ void compute_wave_cs(const PairDev& P, const int s, const int lane, const Scores32& sc, const Rec* ring_in,
                                Rec* ring_out, lds_int* wcnt_in, lds_int* rcnt_in, lds_int* wcnt_out,
                                lds_int* rcnt_out, const bool has_consumer, StripRes* sres, PairRes* pres,
                                int* status, const uint32_t scratch_base) {
    static_assert(kSub == 16, "16-step sub-blocks (code words, ring alignment)");
    const int n = P.n, m = P.m;
    const int i = s * kWave + lane + 1;          // this lane's row
    const bool ok = i <= n;
    WaveCtx w;
    {
        const size_t strip_planes = (size_t)s * P.t4 * kGroupInts1;
        w.pI = PLANES ? P.pI + strip_planes : nullptr;
        w.pD = PLANES ? P.pD + strip_planes : nullptr;
        w.pS = PLANES ? P.pS + strip_planes : nullptr;
        w.pL = LCSP ? P.pL + strip_planes : nullptr;
        w.codes = CODES ? P.codes + (size_t)s * P.t16 * kWave : nullptr;
        const int pbytes = P.t4 * kGroupInts1 * 4;   // one strip's plane
        if (PLANES) {
            w.rI = rsrc_of(uniform_ptr(w.pI), pbytes);
            w.rD = rsrc_of(uniform_ptr(w.pD), pbytes);
            w.rS = rsrc_of(uniform_ptr(w.pS), pbytes);
        }
        if (LCSP) w.rL = rsrc_of(uniform_ptr(w.pL), pbytes);
    }
    w.ring_in = ring_in; w.ring_out = ring_out; w.wcnt_in = wcnt_in; w.wcnt_out = wcnt_out; w.status = status;
    w.skel_rsrc = rsrc_of(uniform_ptr(P.skel + (size_t)s * P.skel_stride), has_consumer ? 4 * (m + 1) : 0);
    w.skel_voff = lane == kWave - 1 ? 0u : kSkelOff;
    w.scratch = scratch_base + 4u * (uint32_t)lane;
    w.cnt_addr = (has_consumer && lane == kWave - 1) ? lds_addr((const void*)wcnt_out) : w.scratch;
    w.m = m; w.lane = lane;
    w.tr_win = 0;
    CsConst kc;
    kc.cY = sc.hg - (lane + 1) * sc.g;
    kc.cZ = -(lane + 1) * sc.g;
    kc.lg = lane * sc.g;
    kc.lg1 = (lane + 1) * sc.g;
    kc.kl = (lane + 1) << 24;
    kc.c1 = ok ? (int)P.c1[i - 1] : 0x1FF;
    if (TBL) kc.c1 = score_table(kc.c1, sc);
    StripTrace* const trace = P.trace;
    const int strip_base = P.strip_base;

    // column 0 (algo.rs:204-211): I = S = neg_inf, D = h + i g
    CsState st;
    {
        RowState rs;
        init_row(rs, i, ok, sc);
        st.I = rs.I; st.SD = rs.SD; st.SM = rs.SM; st.L = 0;
        st.best = rs.best; st.bstep = 0; st.bl = 0;
        st.lbest = rs.lbest; st.lstep = 0; st.lE = 0;
        st.cI = 0; st.cD = 0;
        st.key = kc.kl | (63 - lane);             // column 0: E = -(lane + 1) (+ 64), no delete moves
        st.fin_sm = 0; st.fin_E = 0;
        if (has_consumer) {
            if (lane == kWave - 1) ring_out[ring_slot(0)] = Rec{rs.Dd, rs.SM, 0, 0};
            lds_wait();
            if (lane == 0) *wcnt_out = 1;
        }
    }
    const bool tracing = trace != nullptr;
    long long tr_start = 0, tr_first = 0, clk_first = 0;
    unsigned tr_wout = 0;
    long long tr_q[kTraceQ] = {};
    if (tracing) tr_start = stamp_rt();
    w.tr_win += wait_ge(wcnt_in, min(4, m) + 1, status);
    Rec ra[4], rb[4];   // records of the current / next group (alternating)
    int psm, pl;
    {
        const Rec r0 = ring_in[ring_slot(0)];
        psm = r0.sm;
        pl = 0;
        read4(ra, ring_in + ring_slot(1));
    }
    if (tracing) { tr_first = stamp_rt(); clk_first = stamp_clk(); }
    CsPend pend;
    pend.voff = kNoStore;   // nothing pending before the first group
    // steps 0 .. m: step t computes column t + 1 and finishes E of column t,
    // so one step past the last column completes its landing columns
    for (int t0 = 0; t0 <= m; t0 += kSub) {
        const int last_col = min(t0 + kSub, m);   // last column pushed in this sub-block
        if (has_consumer && last_col >= kRing) tr_wout += wait_ge(rcnt_out, last_col - kRing + 1, status);
        if (tracing) {
            const int q = (int)((long long)t0 * (kTraceQ + 1) / (m + 1)) - 1;
            if (q >= 0 && q < kTraceQ && tr_q[q] == 0) tr_q[q] = stamp_rt();
        }
        const uint32_t out_base = lds_addr(ring_out + ring_slot(t0 + 1));
        if (t0 + kSub < m) {   // step m - 1 (cell (., m)) and step m always run in a tail sub-block
            cs_group4<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, false, 0>(st, kc, ra, rb, psm, pl, w, sc, t0, out_base, has_consumer, pend);
            cs_group4<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, false, 1>(st, kc, rb, ra, psm, pl, w, sc, t0, out_base, has_consumer, pend);
            cs_group4<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, false, 2>(st, kc, ra, rb, psm, pl, w, sc, t0, out_base, has_consumer, pend);
            cs_group4<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, false, 3>(st, kc, rb, ra, psm, pl, w, sc, t0, out_base, has_consumer, pend);
        } else {
            cs_group4<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, true, 0>(st, kc, ra, rb, psm, pl, w, sc, t0, out_base, has_consumer, pend);
            cs_group4<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, true, 1>(st, kc, rb, ra, psm, pl, w, sc, t0, out_base, has_consumer, pend);
            cs_group4<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, true, 2>(st, kc, ra, rb, psm, pl, w, sc, t0, out_base, has_consumer, pend);
            cs_group4<LOCAL, PLANES, CODES, TRACK, LCSP, TBL, true, 3>(st, kc, rb, ra, psm, pl, w, sc, t0, out_base, has_consumer, pend);
        }
        if (CODES) {
            // codes[strip][t/16][lane]
#ifndef GX_DIAG_NO_CODES
            gstore1(w.codes + (size_t)(t0 >> 4) * kWave + lane, (st.cD << 16) | (st.cI & 0xFFFFu));
#endif
        }
        lds_store_lane0(rcnt_in, min(t0 + kSub + 5, m + 1));
    }
    if (PLANES == 2 && pend.voff != kNoStore) {
        cs_pend_store<LCSP>(pend, w, 0); cs_pend_store<LCSP>(pend, w, 1); cs_pend_store<LCSP>(pend, w, 2);
        if (LCSP) cs_pend_store<LCSP>(pend, w, 3);
    }
    if (TRACK || LOCAL) {
        const int best = (TRACK && ok) ? st.best : INT_MIN;
        const int lbest = (LOCAL && ok) ? st.lbest : INT_MIN;
        int mx = best, lmx = lbest;
        for (int off = 32; off > 0; off >>= 1) {
            mx = max(mx, __shfl_xor(mx, off));
            lmx = max(lmx, __shfl_xor(lmx, off));
        }
        const unsigned long long fmask = __ballot(ok && best == mx);
        const unsigned long long lmask = __ballot(ok && lbest == lmx);
        const int fl = fmask ? (__ffsll((long long)fmask) - 1) : 0;
        const int ll = lmask ? (63 - __clzll((long long)lmask)) : 0;
        const int f_step = __shfl(st.bstep, fl), f_l = __shfl(st.bl, fl);
        const int l_step = __shfl(st.lstep, ll), l_E = __shfl(st.lE, ll);
        if (lane == 0) {
            StripRes r;
            r.best = mx; r.bi = s * kWave + fl + 1; r.bj = f_step + 1; r.bl = f_l;
            r.lbest = lmx; r.li = s * kWave + ll + 1; r.lj = l_step + 1; r.lE = l_E - 64;
            sres[strip_base + s] = r;
        }
    }
    if (ok && i == n) { pres->end_SM = st.fin_sm; pres->end_E = st.fin_E - 64; }
    if (tracing && lane == 0) {
        StripTrace tr;
        tr.t_start = tr_start; tr.t_first = tr_first; tr.t_end = stamp_rt();
        tr.wait_in = (int)w.tr_win; tr.wait_out = (int)tr_wout;
        tr.clk = stamp_clk() - clk_first;
        for (int q = 0; q < kTraceQ; ++q) tr.t_q[q] = tr_q[q];
        trace[s] = tr;
    }
}

// PLANES: 0 none, 1 int32 planes, 2 compact byte planes (layout 0 only).  compute_wave
// plane modes: 0 none, 1/2 int32 stored now / during the next group, 3/4 compact
// (byte) stored now / during the next group
template <int W, bool LOCAL, int PLANES, bool CODES, bool TRACK, bool LCSP, bool TBL, int LAY>
__global__ __launch_bounds__((W + 1) * kWave, (LOCAL || TRACK) ? GX_FILL_MIN_WAVES_TRACK : (W + 1 + 3) / 4) void fill_kernel(
    const PairDev* __restrict__ pairs, const int npairs, const int total_bands, int* band_counter, StripRes* sres,
    PairRes* pres, const Scores32 sc) {
    __shared__ Rec rings[W + 1][kRing];
    __shared__ uint32_t push_scratch[W][kPushScratch];   // lanes 0-62's writes of the full-group pushes
    __shared__ int wcnt[W + 1];
    __shared__ int rcnt[W + 1];
    __shared__ int band_sh;
    // readfirstlane: tell the compiler these are wave-uniform, so the pair
    // descriptor, plane bases and exec masks live in SGPRs
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int lane = threadIdx.x & (kWave - 1);
    for (;;) {
        if (threadIdx.x == 0) band_sh = atomicAdd(band_counter, 1);
        if (threadIdx.x < W + 1) { wcnt[threadIdx.x] = 0; rcnt[threadIdx.x] = 0; }
        __syncthreads();
        const int b = __builtin_amdgcn_readfirstlane(band_sh);
        if (b >= total_bands) return;
        // queue entry b -> (pair, band in pair): the host's order table after the descriptors
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
                // plane stores pipelined one group late, except in 16-wave
                // workgroups (128 VGPRs: no room for a group of pending cells)
                if constexpr (LAY == 0)
                    compute_wave<LOCAL, PLANES == 2 ? 3 : PLANES ? ((W + 1) <= 12 ? 2 : 1) : 0, CODES, TRACK, LCSP, TBL>(
                        P, s, lane, sc, rings[wave], rings[wave + 1], (lds_int*)&wcnt[wave], (lds_int*)&rcnt[wave],
                        (lds_int*)&wcnt[wave + 1], (lds_int*)&rcnt[wave + 1], has_consumer, sres, pres + p,
                        band_counter + 1, lds_addr(push_scratch[wave]));
                else
                    compute_wave_cs<LOCAL, PLANES ? ((W + 1) <= 12 ? 2 : 1) : 0, CODES, TRACK, LCSP, TBL>(
                        P, s, lane, sc, rings[wave], rings[wave + 1], (lds_int*)&wcnt[wave], (lds_int*)&rcnt[wave],
                        (lds_int*)&wcnt[wave + 1], (lds_int*)&rcnt[wave + 1], has_consumer, sres, pres + p,
                        band_counter + 1, lds_addr(push_scratch[wave]));
            }
        } else {
            // layout 1 strips run a few columns apart: hand band rows over in
            // smaller chunks, so the next band does not wait for 16 columns
            // layout 1's I/O waves poll less often: their polls of the band
            // progress counters slowed every strip of a single pair by ~3 %
            io_wave<TBL, LAY ? kIoChunk1 : kIoChunk, LAY == 1, LAY ? 8 : GX_IO_SLEEP>(P, lb, lane, sc, rings[0], rings[W], (lds_int*)&wcnt[0], (lds_int*)&rcnt[0], (lds_int*)&wcnt[W],
                    (lds_int*)&rcnt[W], lb + 1 < P.bands, band_counter + 1);
        }
        __syncthreads();
    }
}

// Per-pair reduction of the strip results (first max: lowest strip wins ties;
// last max: highest strip wins ties).
// One wave per pair: each lane scans strips lane, lane+64, ... in order, then
// the wave combines (first max: lowest strip wins ties, i.e. the lowest lane
// holding the max after the per-lane scans, whose strips are increasing; last
// max: the highest strip holding it).
__global__ void finalize_kernel(const PairDev* __restrict__ pairs, const StripRes* __restrict__ sres,
                                PairRes* pres) {
    const int p = blockIdx.x;
    const PairDev& P = pairs[p];
    const int lane = threadIdx.x;
    int best = INT_MIN, bs = INT_MAX, lbest = INT_MIN, ls = -1;
    for (int s = lane; s < P.strips; s += kWave) {
        const StripRes r = sres[P.strip_base + s];
        if (r.best > best) { best = r.best; bs = s; }
        if (r.lbest >= lbest) { lbest = r.lbest; ls = s; }
    }
    int mx = best, lmx = lbest;
    for (int off = 32; off > 0; off >>= 1) {
        mx = max(mx, __shfl_xor(mx, off));
        lmx = max(lmx, __shfl_xor(lmx, off));
    }
    int fs = best == mx ? bs : INT_MAX, lsel = lbest == lmx ? ls : -1;
    for (int off = 32; off > 0; off >>= 1) {
        fs = min(fs, __shfl_xor(fs, off));
        lsel = max(lsel, __shfl_xor(lsel, off));
    }
    // matches_at_max = max_matches(max_cell) (algo.rs:279): from the fill's
    // LCS field, or from the LCS bit rows of a layout-3 launch (gx_lcs.h):
    // LM(i, j) = j - popcount(V_i & (2^j - 1))
    int mam = 0;
    if (fs != INT_MAX) {
        const StripRes r = sres[P.strip_base + fs];
        mam = r.bl;
        if (P.lwords > 0 && P.lbits && r.bj > 0)   // (bj = 0: layout 3 finds the column later, skew_max_col_kernel)
            mam = lcs_matches(P, r.bi, r.bj, lane);
    }
    if (lane == 0) {
        PairRes& o = pres[p];
        o.max_val = mx; o.lmax_val = lmx; o.nstrips = P.strips;
        if (fs != INT_MAX) {
            const StripRes r = sres[P.strip_base + fs];
            o.max_i = r.bi; o.max_j = r.bj > 0 ? r.bj : INT_MAX; o.mam = mam;
        } else {
            o.max_i = 0; o.max_j = 0; o.mam = 0;
        }
        if (lsel >= 0) {
            const StripRes r = sres[P.strip_base + lsel];
            o.lmax_i = r.li; o.lmax_j = r.lj; o.lmax_E = r.lE;
        } else {
            o.lmax_i = 0; o.lmax_j = 0; o.lmax_E = 0;
        }
    }
}

// Traceback (algo.rs:339-422), interior cells only; the host finishes the
// boundary part and labels the moves.
//
// 1. Skeleton chase (tb_chase_kernel, one lane per pair): the fill stored,
//    for every strip's bottom row, the landing column E of the traceback path
//    through each cell on the strip's top boundary (gx_internal.h).  Starting
//    from E of the start cell, a chain of lookups gives the column at which
//    the path enters every strip above -- about n/128 dependent loads.
// 2. Strip walks (tb_strip_kernel, one wave per strip on the path, all in
//    parallel): each walks its strip from its entry cell to its top boundary.
//    Row view: on row i the path is a run of insert moves (j-1) ending at the
//    nearest cell to the left whose code is not "insert", followed by one sub
//    (i-1, j-1) or delete (i-1, j) move; the cells of a row are consecutive
//    steps of its code words, so a row is a bit-scan of the "not insert" mask
//    D | ~I.  One record per row, (run << 2) | kind (0 sub, 2 delete, 1 = the
//    run reached column 0).  The 64 rows of a block are solved as a
//    lane-parallel fixed point: lane k guesses its row's entry column (the
//    diagonal from the block's entry), all lanes scan at once, and each lane's
//    next guess is the exit column of the lane above (DPP wave_shl:1); the top
//    lane's entry is known, so the iteration ends at the sequential walk.  A
//    block's code window (kTbWin words per row) is read from LDS (LDS-DMA,
//    the next block prefetched) with a per-lane "nearest non-insert below
//    this word" table, so a round is two LDS reads and no loop.
constexpr int kTbWin = 32;
constexpr int kTbRows = 64;   // rows per walked block (half a fill strip); lane = row

__device__ __forceinline__ int tb_q0(int t) {
    return __builtin_amdgcn_readfirstlane(max((t >> 4) - (kTbWin - 1), 0));
}

typedef __attribute__((address_space(1))) const void gcvoid;
typedef __attribute__((address_space(3))) void lvoid;
typedef __attribute__((address_space(3))) const uint32_t lu32;
typedef __attribute__((address_space(3))) int lint;
typedef __attribute__((address_space(1))) const uint32_t gcu32;
typedef __attribute__((address_space(1))) const int gcint;

// Code word of row-in-strip rho, word q of strip s (codes[strip][q][rho]).
__device__ __forceinline__ size_t tb_word(const TbDev& J, int s, int q, int rho) {
    return ((size_t)s * J.t16 + q) * J.srows + rho;
}
// Walked blocks are 64 rows: two per 128-row strip (layout 0), one per 64-row
// strip (layout 1).  Row-in-strip of lane `lane` of block vb, and the step at
// which that row computes column 1 (layout 0: the anti-diagonal skew rho/2;
// layout 1: none).
__device__ __forceinline__ int tb_rho(const TbDev& J, int vb, int lane) {
    return J.srows == kStripRows ? ((vb & 1) << 6) + lane : lane;
}
__device__ __forceinline__ int tb_lot(const TbDev& J, int rho) {
    return J.srows == kStripRows ? rho >> 1 : J.skew ? rho : 0;   // layout 3: one row per lane, skewed
}
__device__ __forceinline__ int tb_strip_of(const TbDev& J, int vb) { return J.srows == kStripRows ? vb >> 1 : vb; }

// async: words q0 .. q0+kTbWin-1 of block vb (rows 64*vb .. +63), lane = row -> buf[k][lane]
__device__ __forceinline__ void tb_prefetch(uint32_t* buf, const TbDev& J, int vb, int q0, int lane) {
    const int s = tb_strip_of(J, vb), rho = tb_rho(J, vb, lane);
#pragma unroll
    for (int k = 0; k < kTbWin; ++k)
        __builtin_amdgcn_global_load_lds((gcvoid*)(J.codes + tb_word(J, s, min(q0 + k, J.t16 - 1), rho)),
                                         (lvoid*)(buf + k * kWave), 4, 0, 0);
}

__global__ void tb_chase_kernel(const TbDev* __restrict__ jobs) {
    const TbDev J = jobs[blockIdx.x];
    if (threadIdx.x != 0) return;
    int i = J.start_i, j = J.start_j;
    int first = -1;
    if (i >= 1 && j >= 1) {
        const int SR = J.srows;
        int s = (i - 1) / SR;
        first = s;
        J.seg[4 * s + 0] = i; J.seg[4 * s + 1] = j; J.seg[4 * s + 3] = 1;
        int E = J.start_E_dev ? *J.start_E_dev : J.start_E;
        for (;;) {
            // a landing column outside the strip's range (a fill that did not
            // complete): report (-1, -1), the host returns GX_EHIP
            if (E < -SR || E > J.m) { i = -1; j = -1; first = -1; break; }
            if (E < 0) { i = s * SR - E; j = 0; break; }          // reaches (i, 0) at local row -E
            if (s == 0 || E == 0) { i = s * SR; j = E; break; }   // lands on row 0 / column 0
            s -= 1;                                               // enters strip s at its bottom row
            J.seg[4 * s + 0] = (s + 1) * SR; J.seg[4 * s + 1] = E; J.seg[4 * s + 3] = 1;
            E = ((gcint*)J.skel)[(size_t)s * J.skel_stride + E];
            if (J.skel_half >= 0) E = (int)(short)((unsigned)E >> (16 * J.skel_half));   // twin fill (gx_fill_pk.hip)
            if (SR == kStripRows1) E = (E & 0xFFFFFF) - 64;        // layouts 1 and 3 store E + 64 (the split column
                                                                   // step keeps the key's lane field above it)
        }
    }
    J.end_ij[0] = i; J.end_ij[1] = j; J.end_ij[2] = first;
}

// Code words of the strips on the path from the twin plane codes (DESIGN.md
// 4.4), for a twin fill that stored no code words.  A cell's plane code holds
// x_S = S - I and x_D = D - I, and the retrace priority S > I > D
// (algo.rs:351-400) is "insert beats sub" = x_S < 0 and "delete beats both" =
// x_D > max(0, x_S).  The path crosses strip s between its entry column
// (seg[s], the bottom row) and the entry column of the strip above (or where
// it leaves the interior), so only the words holding those columns of each
// row are rebuilt; the walk (tb_strip_kernel) never uses a word outside them
// once its rows have converged (every path cell lies in that range).  One
// block of 128 threads per strip, one thread per row.
// A twin plane code (gx_fill_pk.hip w16_code: x_S + 32 x_D, of which the
// record keeps the low 12 bits, gx_device.h w12_pack; this pair's half of a
// step's dword) -> x_S = S - I (5-bit signed), x_D = D - I (7-bit signed).
__device__ __forceinline__ void w16_decode(uint32_t code, int& xS, int& xD) {
    xS = (int)(code << 27) >> 27;
    xD = (int)((code - (uint32_t)xS) << 20) >> 25;
}
// The format stores no x_I: I(i, j) from I(i, j-1) and the previous cell's
// max(x_S, x_D) -- the fill's insert recurrence, algo.rs:231-236 --
// I + g + max(0, m + h), local max(that, 0).  A row starts at I(i, 0) =
// H(i, 0) + h with m = -h (global) or 0 (local), as the fill seeds it.
__device__ __forceinline__ int w16_next_I(int I, int mprev, int h, int g, bool local) {
    const int v = I + g + max(0, mprev + h);
    return local ? max(v, 0) : v;
}

// The code word (cD << 16 | cI, first step in bit 15) of 16 steps of one row
// from its four 4-step groups of twin plane codes (this pair's half `sh`).
__device__ __forceinline__ uint32_t w16_word_of(const uint4 (&w4)[4], const int sh) {
    uint32_t cI = 0, cD = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const uint32_t wk[4] = {w4[g].x, w4[g].y, w4[g].z, w4[g].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            int xS, xD;
            w16_decode((wk[k] >> sh) & 0xFFFFu, xS, xD);
            cI = (cI << 1) | (uint32_t)(xS < 0);
            cD = (cD << 1) | (uint32_t)(xD > max(0, xS));
        }
    }
    return (cD << 16) | cI;
}
// Row rho's 4-step group G of strip s in the twin code plane: the four
// steps' dwords (gx_device.h w12_load).
__device__ __forceinline__ uint4 w16_group(const TbDev& J, int s, int G, int rho) {
    return w12_load(J.w16 + w12_rec_off(s, J.t4, G, rho));
}
// Code word q of row rho of strip s, derived from the twin plane codes.
__device__ __forceinline__ uint32_t w16_word(const TbDev& J, int s, int q, int rho) {
    uint4 w4[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) w4[g] = w16_group(J, s, 4 * q + g, rho);
    return w16_word_of(w4, 16 * J.w16_half);
}

__global__ __launch_bounds__(128) void tb_w16_codes_kernel(const TbDev* __restrict__ jobs) {
    const TbDev J = jobs[blockIdx.y];
    const int s = blockIdx.x;
    if (!J.w16 || s >= J.strips) return;
    const int* seg = J.seg;
    if (!((gcint*)seg)[4 * s + 3]) return;                     // not on the path
    const int j_hi = ((gcint*)seg)[4 * s + 1];
    int j_lo = (s > 0 && ((gcint*)seg)[4 * (s - 1) + 3]) ? ((gcint*)seg)[4 * (s - 1) + 1] : ((gcint*)J.end_ij)[1];
    j_lo = max(j_lo, 1);
    const int rho = threadIdx.x, lane = rho >> 1, hh = rho & 1;
    const int q_lo = (j_lo - 1 + lane) >> 4, q_hi = min((j_hi - 1 + lane) >> 4, J.t16 - 1);
    (void)hh;
    const uint8_t* base = J.w16 + w12_rec_off(s, J.t4, 0, rho);
    const int sh = 16 * J.w16_half;
    guint* const out = (guint*)(J.codes + (size_t)s * J.t16 * kStripRows + rho);
    for (int q = q_lo; q <= q_hi; ++q) {
        uint4 w4[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) w4[g] = w12_load(base + (size_t)(4 * q + g) * kTwinGroupBytes);
        out[(size_t)q * kStripRows] = w16_word_of(w4, sh);
    }
}

// One 64-row block of a strip's walk (tb_strip_kernel, tb_seq_kernel).  The
// path enters the block at lane R (row-in-block), column ce; win holds words
// q0 .. q0 + WIN - 1 of every lane's row.  Writes the records of the rows it
// covers (from the entry row upwards) at recs[nrec ..], advances nrec, and
// returns the lane where the walk leaves the strip or the interior (-1: it
// goes on in the block above, entered at its lane 63 at column nj of lane 0).
// Per lane: nj = the column after its row's last move, run_end = the row's
// insert run reached column 0.  W16: words outside the window are derived
// from the twin plane codes (no code words in HBM).
template <int WIN, bool W16>
__device__ __forceinline__ int tb_walk_block(const TbDev& J, const int ss, const int vb, const int vb_top, const int R,
                                             const int ce, const int q0, const lu32* win, lint* ltbl, const int lane,
                                             guint* recs, int& nrec, int& nj, bool& run_end) {
    gcu32* const codes = (gcu32*)J.codes;
    const int rho = tb_rho(J, vb, lane);
    const int lo_t = tb_lot(J, rho);  // step of column 1 on this row
    {   // per lane: nearest non-insert step strictly below each window word (branch-free)
        int run = -1;
#pragma unroll 8
        for (int x = 0; x < WIN; ++x) {
            ltbl[x * kWave + lane] = run;
            const uint32_t w = win[x * kWave + lane];
            const uint32_t m = ((w >> 16) | ~w) & 0xFFFFu;
            const int k = 15 - (int)__builtin_ctz(m | 0x10000u);
            const int cand = ((16 * (q0 + x) + k) << 1) | (int)((w >> ((31 - k) & 31)) & 1u);
            run = m ? cand : run;
        }
    }
    const bool act = lane <= R;
    const bool top_row = vb == vb_top && lane == 0;   // its move leaves the strip
    int g = ce - (R - lane);          // diagonal guess of this row's entry column
    int rec = 0;
    bool end = true;
    nj = 0; run_end = false;
    for (;;) {
        const bool valid = act && g >= 1;
        const int t_in = g - 1 + lo_t;
        const int x = (t_in >> 4) - q0;
        const int xc = min(max(x, 0), WIN - 1);
        const uint32_t w = win[xc * kWave + lane];
        const int tb = ltbl[xc * kWave + lane];
        const uint32_t nonI = ((w >> 16) | ~w) & ((0xFFFFu << (15 - (t_in & 15))) & 0xFFFFu);
        const int kw = 15 - (int)__builtin_ctz(nonI | 0x10000u);
        int tf = nonI ? (t_in & ~15) + kw : (tb >> 1);
        int del = nonI ? (int)((w >> ((31 - kw) & 31)) & 1u) : (tb & 1);
        const bool need_scan = valid && (x < 0 || (!nonI && tb < 0 && 16 * q0 > lo_t));
        if (__builtin_amdgcn_ballot_w64(need_scan)) {
            if (need_scan) {          // below the window (rare): scan the HBM words
                int t = x < 0 ? t_in : 16 * q0 - 1;
                tf = -1; del = 0;
                while (t >= lo_t) {
                    const uint32_t wg = W16 ? w16_word(J, ss, t >> 4, rho) : codes[tb_word(J, ss, t >> 4, rho)];
                    const uint32_t ng = ((wg >> 16) | ~wg) & ((0xFFFFu << (15 - (t & 15))) & 0xFFFFu);
                    if (ng) {
                        tf = (t & ~15) + (15 - __builtin_ctz(ng));
                        del = (wg >> (31 - (tf & 15))) & 1u;
                        break;
                    }
                    t = (t & ~15) - 1;
                }
            }
        }
        run_end = valid && tf < lo_t;     // (i, g..1) all insert: the walk leaves at (i, 0)
        nj = tf - lo_t + del;             // del ? tf-lo_t+1 : tf-lo_t
        end = !valid || run_end || nj < 1 || top_row;
        rec = run_end ? ((g << 2) | 1) : (((t_in - tf) << 2) | (del << 1));
        // next guess: the exit column of the lane above; the top lane's entry is fixed
        const int prop = end ? 0 : nj;
        int gn = __builtin_amdgcn_update_dpp(0, prop, 0x130 /* wave_shl:1 */, 0xF, 0xF, false);
        gn = lane == R ? ce : gn;
        if (__builtin_amdgcn_ballot_w64(act && gn != g) == 0) break;
        g = gn;
    }
    // the path covers lanes R down to the first lane (from the top) where it ends
    const unsigned long long em = __builtin_amdgcn_ballot_w64(act && end);
    const int E = em ? 63 - __builtin_clzll(em) : -1;
    const int lo = E >= 0 ? E : 0;
    if (act && lane >= lo) recs[nrec + (R - lane)] = (uint32_t)rec;
    nrec += R - lo + 1;
    return E;
}

__global__ __launch_bounds__(64) void tb_strip_kernel(const TbDev* __restrict__ jobs) {
    __shared__ uint32_t tbuf[2][kTbWin * kWave];
    __shared__ int tbl[kTbWin * kWave];   // nearest non-insert step below each word, (step << 1) | del
    const TbDev J = jobs[blockIdx.y];
    const int ss = blockIdx.x;            // strip
    if (ss >= J.strips) return;
    const int active = __builtin_amdgcn_readfirstlane(((gcint*)J.seg)[4 * ss + 3]);
    if (!active) return;
    const int lane = threadIdx.x;
    const int i0 = __builtin_amdgcn_readfirstlane(((gcint*)J.seg)[4 * ss + 0]);
    const int j0 = __builtin_amdgcn_readfirstlane(((gcint*)J.seg)[4 * ss + 1]);
    guint* const recs = (guint*)(J.recs + (size_t)ss * J.srows);
    lint* const ltbl = (lint*)(uintptr_t)lds_addr(tbl);
    const int vb_top = J.srows == kStripRows ? 2 * ss : ss;   // the strip's top block
    int vb = (i0 - 1) / kTbRows;          // current block
    int R = (i0 - 1) % kTbRows;           // the path's top lane in it
    int ce = j0;                          // its entry column
    int nrec = 0;
    int cb = 0;
    int q_c = tb_q0(ce - 1 + tb_lot(J, tb_rho(J, vb, R)));
    tb_prefetch(tbuf[cb], J, vb, q_c, lane);
    for (;;) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");         // this block's window has landed
        // the block above (if in this strip) is entered at its lane 63, no further right than ce
        const int q_n = vb > vb_top ? tb_q0(ce - 1 + tb_lot(J, tb_rho(J, vb - 1, kTbRows - 1))) : 0;
        if (vb > vb_top) tb_prefetch(tbuf[cb ^ 1], J, vb - 1, q_n, lane);
        const lu32* win = (const lu32*)(uintptr_t)lds_addr(tbuf[cb]);
        int nj;
        bool run_end;
        const int E = tb_walk_block<kTbWin, false>(J, ss, vb, vb_top, R, ce, q_c, win, ltbl, lane, recs, nrec, nj, run_end);
        if (E >= 0) break;                // the walk leaves the strip (or the interior) here
        ce = __builtin_amdgcn_readlane(nj, 0);
        vb -= 1;
        R = kTbRows - 1;
        cb ^= 1;
        q_c = q_n;
    }
    if (lane == 0) ((gint*)J.seg)[4 * ss + 2] = nrec;
}

// The walk of a twin fill that kept no landing columns (gx_fill_pk.hip,
// PLANES 16: no skeleton) and no code words: the strips are walked in
// sequence from the start cell, each entered where the one below left it
// (what tb_chase_kernel's hops through the skeleton give the parallel strip
// walks), the code words of each 64-row block's window derived from the
// plane codes.  One workgroup per pair: wave 0 walks block k (the
// tb_strip_kernel block walk, its window in LDS) while kSqHelp helper waves
// derive block k + 1's window (kSqWin words a row ending at block k's entry
// column: the path only moves left) into the other LDS buffer, so a block
// costs about the larger of the walk and one window's loads + derivation
// instead of their sum.  Writes the same seg / recs / end_ij as
// tb_chase_kernel + tb_strip_kernel, so the host's labelling is unchanged.
// The walk, not the windows, sets the pace: ~22k cycles a block (on gapped
// paths the fixed point needs about one ~340-cycle round per row).  Walkers
// doing the rows one by one on wave-uniform values were slower still: ~650
// cycles a row with the window in LDS read a row ahead, ~565 with a
// per-row "nearest non-insert" table in LDS, ~475 with the window transposed
// into registers (row r's words in the lanes of Wr[r], two v_readlane a row)
// -- a lone wave's instruction latency, not the memory, sets a row's cost.
// Layout 0 only.
constexpr int kSqWin = 12;
constexpr int kSqHelp = 4;
struct SqCtl {
    int s, vb, R, ce, q0, done, end_i, end_j;
};
// words q0 .. q0 + kSqWin - 1 of block vb's rows (strip vb / 2), derived by
// the kSqHelp helper waves: helper h takes words h, h + kSqHelp, ... (all its
// loads in flight at once)
static_assert(kSqWin % kSqHelp == 0, "helper word split");
__device__ __forceinline__ void tb_seq_window(const TbDev& J, const int vb, const int q0, uint32_t* buf, const int hw,
                                              const int lane) {
    typedef __attribute__((address_space(3))) uint32_t lu32w;
    lu32w* const lw = (lu32w*)(uintptr_t)lds_addr(buf);
    const int s = vb >> 1, rho = tb_rho(J, vb, lane), sh = 16 * J.w16_half;
    constexpr int kPer = kSqWin / kSqHelp;
    uint4 w4[kPer][4];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        const int q = min(q0 + hw + u * kSqHelp, J.t16 - 1);
#pragma unroll
        for (int g = 0; g < 4; ++g) w4[u][g] = w16_group(J, s, 4 * q + g, rho);
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) lw[(hw + u * kSqHelp) * kWave + lane] = w16_word_of(w4[u], sh);
}
__global__ __launch_bounds__((1 + kSqHelp) * kWave) void tb_seq_kernel(const TbDev* __restrict__ jobs) {
    __shared__ uint32_t wbuf[2][kSqWin * kWave];
    __shared__ int tbl[kSqWin * kWave];
    __shared__ SqCtl ctl;
    const TbDev J = jobs[blockIdx.x];
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave);
    const int lane = threadIdx.x & (kWave - 1);
    // (local fills in the overlapped pipeline: the last max, from the fill's results on the device)
    const int i = J.start_ij_dev ? ((gcint*)J.start_ij_dev)[0] : J.start_i;
    const int j = J.start_ij_dev ? ((gcint*)J.start_ij_dev)[1] : J.start_j;
    if (i < 1 || j < 1) {
        if (threadIdx.x == 0) { J.end_ij[0] = i; J.end_ij[1] = j; J.end_ij[2] = -1; }
        return;
    }
    const int first = (i - 1) / J.srows;
    // the walker wave issues ahead of its helpers and of a fill sharing the
    // CU (the walk runs beside the next pass's fill): 1024 x 1k 0.84 -> 0.83
    // ms a pass with the walk on its own stream, 0.94 -> 0.90 without
    // (tools/walk_prio_ab.sh)
#ifndef GX_TB_NOPRIO
    if (wave == 0) __builtin_amdgcn_s_setprio(3);
#endif
    // block 0 of the walk: its window from every wave
    int vb = (i - 1) / kTbRows, R = (i - 1) % kTbRows, ce = j;
    int q0 = max(((ce - 1 + tb_lot(J, tb_rho(J, vb, R))) >> 4) - (kSqWin - 1), 0);
    if (wave > 0) tb_seq_window(J, vb, q0, wbuf[0], wave - 1, lane);
    if (threadIdx.x == 0) { J.seg[4 * first + 0] = i; J.seg[4 * first + 1] = j; J.seg[4 * first + 3] = 1; }
    lint* const ltbl = (lint*)(uintptr_t)lds_addr(tbl);
    int s = first, nrec = 0, cb = 0;
    int end_i = -1, end_j = -1;
    long long clk0 = stamp_clk(), walk_clk = 0;   // (diagnostics: end_ij[3])
    int nblk = 0;
    __syncthreads();
    for (int guard = 0; guard <= 2 * J.strips + 2; ++guard) {
        // the next block in the walk is always vb - 1 (the strip above once vb
        // is its strip's top block); its window ends at this block's entry
        const int qn = vb > 0 ? max(((ce - 1 + tb_lot(J, tb_rho(J, vb - 1, kTbRows - 1))) >> 4) - (kSqWin - 1), 0) : 0;
        if (wave > 0) {
            if (vb > 0) tb_seq_window(J, vb - 1, qn, wbuf[cb ^ 1], wave - 1, lane);
        } else {
            const int vb_top = 2 * s;
            guint* const recs = (guint*)(J.recs + (size_t)s * J.srows);
            int nj;
            bool run_end;
            const long long w0 = stamp_clk();
            const int E = tb_walk_block<kSqWin, true>(J, s, vb, vb_top, R, ce, q0, (const lu32*)(uintptr_t)lds_addr(wbuf[cb]),
                                                      ltbl, lane, recs, nrec, nj, run_end);
            walk_clk += stamp_clk() - w0;
            ++nblk;
            int done = 0;
            if (E < 0) {                  // on into the block above, in this strip
                ce = __builtin_amdgcn_readlane(nj, 0);
            } else {
                if (lane == 0) J.seg[4 * s + 2] = nrec;
                const int iE = vb * kTbRows + E + 1;   // the row where this strip's walk ends
                const int njE = __builtin_amdgcn_readlane(nj, E);
                if (__builtin_amdgcn_readlane((int)run_end, E)) { end_i = iE; end_j = 0; done = 1; }   // inserts to (iE, 0)
                else if (E == 0 && vb == vb_top && njE >= 1 && s >= 1) {
                    // the top row's move enters strip s - 1 at its bottom row
                    s -= 1; ce = njE; nrec = 0;
                    if (lane == 0) { J.seg[4 * s + 0] = iE - 1; J.seg[4 * s + 1] = njE; J.seg[4 * s + 3] = 1; }
                } else { end_i = iE - 1; end_j = njE; done = 1; }   // row 0 or column 0
            }
            if (lane == 0) { ctl.s = s; ctl.ce = ce; ctl.done = done; ctl.end_i = end_i; ctl.end_j = end_j; }
        }
        __syncthreads();
        if (ctl.done) break;
        s = ctl.s; ce = ctl.ce;
        vb -= 1; R = kTbRows - 1; q0 = qn; cb ^= 1;
        __syncthreads();   // (ctl read by every wave before wave 0 writes it again)
    }
    if (threadIdx.x == 0) {
        end_i = ctl.done ? ctl.end_i : -1;
        end_j = ctl.done ? ctl.end_j : -1;
        J.end_ij[0] = end_i; J.end_ij[1] = end_j; J.end_ij[2] = end_i < 0 ? -1 : first;
        // cycles per block: all (high 16 bits) and the walk's (low 16)
        const long long all = (stamp_clk() - clk0) / max(nblk, 1), wk = walk_clk / max(nblk, 1);
        J.end_ij[3] = (int)((min(all, 65535LL) << 16) | min(wk, 65535LL));
    }
}

// Plane checksums of every pair of a fill launch, decoded from the planes as
// the exports decode them: for each of the I, D, S planes the sum over the
// interior cells of value * (1 + i * 0x9E3779B1 + j * 0x85EBCA77) mod 2^64
// (the oracle's plane_sums, oracle/gx_oracle.c oracle_align_lean).  One
// thread per row, walking its row in step order (t = j - 1 + l on layout 0,
// j - 1 on layout 1) so that a wave reads one contiguous group at a time;
// the compact format keeps a running insert value along the row.  Wave sums
// go to out[pair][3] with 64-bit atomic adds (order-independent mod 2^64).
// mode: 1 = int32 planes, 2 = compact byte planes.
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

__global__ __launch_bounds__(64) void plane_sums_kernel(const PairDev* __restrict__ pairs, int lay, int mode, int h,
                                                       int g, int floor_, int gshift,
                                                       unsigned long long* __restrict__ out) {
    const PairDev d = pairs[blockIdx.y];
    const int lane = threadIdx.x;
    const int SR = lay ? kStripRows1 : kStripRows;
    const int s = blockIdx.x / (SR / kWave);            // strip (layout 0: two blocks of 64 rows per strip)
    const int hh = lay ? 0 : (int)(blockIdx.x & 1);     // layout 0: row-in-lane of this block
    if (s >= d.strips || !d.pI) return;
    const int i = lay ? s * SR + lane + 1 : s * SR + 2 * lane + hh + 1;
    const int l = lay == 1 ? 0 : lane;                  // step of column 1 on this row (layouts 0 and 3: the skew)
    const bool row_ok = i <= d.n;
    unsigned long long sI = 0, sD = 0, sS = 0;
    const unsigned long long wi = 1ull + (unsigned long long)i * 0x9E3779B1ull;
    const size_t gints = lay ? kGroupInts1 : kGroupInts;
    const size_t row0 = (size_t)s * d.t4 * gints + (lay ? (size_t)lane * 4 : (size_t)hh * kWave * 4 + (size_t)lane * 4);
    if (mode == 3) {   // twin plane codes (gx_fill_pk.hip w16_code): this pair's half of each dword
        const int half = d.twin_half;      // the twin's two pairs share its code plane
        const uint8_t* base = (const uint8_t*)d.pI + w12_rec_off(s, d.t4, 0, 2 * lane + hh);
        const bool local = floor_ == 0;
        int I = max(h + i * g, floor_) + h;             // H(i, 0) + h, as the fill seeds it
        int mp = local ? 0 : -h;                        // (its max(S, D) - I)
        for (int q = 0; q < d.t4; ++q) {
            uint4 w4 = make_uint4(0u, 0u, 0u, 0u);
            if (row_ok) w4 = w12_load(base + (size_t)q * kTwinGroupBytes);
            const uint32_t wk[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = 4 * q + k - l + 1;
                if (!row_ok || j < 1 || j > d.m) continue;
                int xS, xD;
                w16_decode((wk[k] >> (16 * half)) & 0xFFFFu, xS, xD);
                I = w16_next_I(I, mp, h, g, local);
                mp = max(xS, xD);
                const long long vI = I, vD = I + xD, vS = I + xS;
                const unsigned long long w = wi + (unsigned long long)j * 0x85EBCA77ull;
                sI += (unsigned long long)vI * w;
                sD += (unsigned long long)vD * w;
                sS += (unsigned long long)vS * w;
            }
        }
    } else if (mode == 2) {
        const uint8_t* pI = (const uint8_t*)d.pI;
        const uint8_t* pD = (const uint8_t*)d.pD;
        const uint8_t* pS = (const uint8_t*)d.pS;
        int I = max(h + i * g, floor_) + h;             // H(i, 0) + h, as the fill seeds it
        for (int q = 0; q < d.t4; ++q) {
            const size_t off = row0 + (size_t)q * gints;
            const uint32_t wI = row_ok ? *(const uint32_t*)(pI + off) : 0u;
            const uint32_t wD = row_ok ? *(const uint32_t*)(pD + off) : 0u;
            const uint32_t wS = row_ok ? *(const uint32_t*)(pS + off) : 0u;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = 4 * q + k - l + 1;
                if (!row_ok || j < 1 || j > d.m) continue;
                I += (int)(int8_t)(wI >> (8 * k)) + gshift;   // shifted fills store x_I - g
                const long long vI = I, vD = I + (int)(int8_t)(wD >> (8 * k)), vS = I + (int)(int8_t)(wS >> (8 * k));
                const unsigned long long w = wi + (unsigned long long)j * 0x85EBCA77ull;
                sI += (unsigned long long)vI * w;
                sD += (unsigned long long)vD * w;
                sS += (unsigned long long)vS * w;
            }
        }
    } else {
        for (int q = 0; q < d.t4; ++q) {
            const size_t off = row0 + (size_t)q * gints;
            int4 a = make_int4(0, 0, 0, 0), b = a, c = a;
            if (row_ok) {
                a = *(const int4*)(d.pI + off);
                b = *(const int4*)(d.pD + off);
                c = *(const int4*)(d.pS + off);
            }
            const int va[4] = {a.x, a.y, a.z, a.w}, vb[4] = {b.x, b.y, b.z, b.w}, vc[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = 4 * q + k - l + 1;
                if (!row_ok || j < 1 || j > d.m) continue;
                const long long sh = (long long)(i + j) * gshift;   // shifted fills: V - (i + j) g
                const unsigned long long w = wi + (unsigned long long)j * 0x85EBCA77ull;
                sI += (unsigned long long)(va[k] + sh) * w;
                sD += (unsigned long long)(vb[k] + sh) * w;
                sS += (unsigned long long)(vc[k] + sh) * w;
            }
        }
    }
    sI = wave_sum_u64(sI);
    sD = wave_sum_u64(sD);
    sS = wave_sum_u64(sS);
    if (lane == 0) {
        atomicAdd(&out[3 * blockIdx.y + 0], sI);
        atomicAdd(&out[3 * blockIdx.y + 1], sD);
        atomicAdd(&out[3 * blockIdx.y + 2], sS);
    }
}

// Export: strip-major anti-diagonal planes -> row-major int32 rows
// row0 .. row0 + rows - 1 of the (n+1) x (m+1) table (interior only; the host
// fills the boundary in int64).
__global__ void export_kernel(const int32_t* __restrict__ plane, int32_t* __restrict__ out, int n, int m, int t4,
                              int lay, int gshift, int row0, int rows) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)rows * m;
    if (idx >= total) return;
    const int i = (int)(idx / m) + row0;
    const int j = (int)(idx % m) + 1;
    if (i < 1 || i > n) return;
    size_t o;
    if (lay == 0) {
        const int s = (i - 1) / kStripRows, rho = (i - 1) % kStripRows;
        const int l = rho >> 1, h = rho & 1, t = j - 1 + l;
        o = ((size_t)s * t4 + (t >> 2)) * kGroupInts + h * kWave * 4 + l * 4 + (t & 3);
    } else {
        // layout 1: step t = j - 1; layout 3: the skew, t = j - 1 + l
        const int s = (i - 1) / kStripRows1, l = (i - 1) % kStripRows1, t = j - 1 + (lay == 3 ? l : 0);
        o = ((size_t)s * t4 + (t >> 2)) * kGroupInts1 + l * 4 + (t & 3);
    }
    out[(size_t)(i - row0) * (m + 1) + j] = plane[o] + (i + j) * gshift;   // shifted fills: V - (i + j) g
}

// Export of a compact (mode 3) plane: one thread per row rebuilds
// I(i, j) = (D0 + h) + sum_{j' <= j} x_I(i, j') and, for the delete or sub
// plane, adds that plane's x (gx_kernels.hip put_byte).  Rows row0 ..
// row0 + rows - 1 (each at least 1).
__global__ void export_d8_kernel(const uint8_t* __restrict__ pI, const uint8_t* __restrict__ px,
                                 int32_t* __restrict__ out, int n, int m, int t4, int h, int g, int floor_,
                                 int gshift, int row0, int rows) {
    const int r = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int i = r + row0;
    if (r >= rows || i < 1 || i > n) return;
    const int s = (i - 1) / kStripRows, rho = (i - 1) % kStripRows;
    const int l = rho >> 1, hh = rho & 1;
    const size_t rowoff = (size_t)s * t4 * kGroupInts + hh * kWave * 4 + l * 4;
    int I = max(h + i * g, floor_) + h;   // H(i, 0) + h, as the fill seeds it
    int32_t* o = out + (size_t)r * (m + 1);
    for (int j = 1; j <= m; ++j) {
        const int t = j - 1 + l;
        const size_t off = rowoff + (size_t)(t >> 2) * kGroupInts + (t & 3);
        I += (int8_t)pI[off] + gshift;   // shifted fills store x_I - g
        o[j] = px ? I + (int8_t)px[off] : I;
    }
}

// Export of the twin fill's plane codes (gx_fill_pk.hip w16_code, DESIGN.md
// 4.4): one thread per row decodes this pair's 16-bit half of each dword,
// replays I(i, j) along the row (w16_next_I) and adds the plane's x_D or x_S
// -- the decode of plane_sums_kernel mode 3.  `half` = the pair's half
// (PairDev.twin_half), the code plane layout [strip][t/4][row-in-lane][lane][t%4]
// dwords.  Rows row0 .. row0 + rows - 1 (each at least 1).
__global__ void export_w16_kernel(const uint8_t* __restrict__ codes, int half, int which, int32_t* __restrict__ out,
                                  int n, int m, int t4, int h, int g, int floor_, int gshift, int row0, int rows) {
    const int r = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int i = r + row0;
    if (r >= rows || i < 1 || i > n) return;
    const int s = (i - 1) / kStripRows, rho = (i - 1) % kStripRows;
    const int l = rho >> 1, hh = rho & 1;
    (void)hh;
    const uint8_t* base = codes + w12_rec_off(s, t4, 0, rho);
    const bool local = floor_ == 0;
    (void)gshift;
    int I = max(h + i * g, floor_) + h;   // H(i, 0) + h, as the fill seeds it
    int mp = local ? 0 : -h;              // (its max(S, D) - I)
    int32_t* o = out + (size_t)r * (m + 1);
    uint4 rec = make_uint4(0u, 0u, 0u, 0u);
    for (int j = 1; j <= m; ++j) {
        const int t = j - 1 + l;
        if (j == 1 || (t & 3) == 0) rec = w12_load(base + (size_t)(t >> 2) * kTwinGroupBytes);
        const uint32_t wd = (t & 3) == 0 ? rec.x : (t & 3) == 1 ? rec.y : (t & 3) == 2 ? rec.z : rec.w;
        int xS, xD;
        w16_decode((wd >> (16 * half)) & 0xFFFFu, xS, xD);
        I = w16_next_I(I, mp, h, g, local);
        mp = max(xS, xD);
        o[j] = which == 0 ? I : which == 1 ? I + xD : I + xS;
    }
}

}  // namespace gx

// ---- explicit launch wrappers (C++ linkage, used by gx_api_fill.cpp and the table exports) ----
namespace gx {

template <int W, bool LOCAL, int PLANES, bool TRACK, bool LCSP, bool TBL>
static hipError_t launch_fill_t(int lay, const PairDev* d_pairs, int npairs, int total_bands, int* d_counter,
                                StripRes* d_sres, PairRes* d_pres, Scores32 sc, int grid, hipStream_t st) {
    if (lay == 0) {
        hipLaunchKernelGGL((fill_kernel<W, LOCAL, PLANES, true, TRACK, LCSP, TBL, 0>), dim3(grid), dim3((W + 1) * kWave),
                           0, st, d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc);
    } else {
        if constexpr (PLANES == 2) return hipErrorInvalidValue;   // compact planes: layout 0 only
        else
            hipLaunchKernelGGL((fill_kernel<W, LOCAL, PLANES, true, TRACK, LCSP, TBL, 1>), dim3(grid),
                               dim3((W + 1) * kWave), 0, st, d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc);
    }
    return hipGetLastError();
}

// Launch with the band width W from the variant's width list (gx_internal.h).
template <bool LO, int PL, bool TR, bool LC, bool TB, int W0, int... Ws>
static hipError_t launch_fill_w(int W, int lay, const PairDev* d_pairs, int npairs, int total_bands, int* d_counter,
                                StripRes* d_sres, PairRes* d_pres, Scores32 sc, int grid, hipStream_t st) {
    if (W == W0)
        return launch_fill_t<W0, LO, PL, TR, LC, TB>(lay, d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc,
                                                      grid, st);
    if constexpr (sizeof...(Ws) > 0)
        return launch_fill_w<LO, PL, TR, LC, TB, Ws...>(W, lay, d_pairs, npairs, total_bands, d_counter, d_sres, d_pres,
                                                        sc, grid, st);
    return hipErrorInvalidValue;
}

// Variants: mode (global/local) x planes x {no max tracking, first max + LCS
// field, first max + LCS plane}.  Traceback codes are always produced.  The
// untracked global variants (the batch path) come in every width of kFillWidths
// and with the small-alphabet score table (tbl) or the byte compare,
// the tracked and local ones (256-VGPR builds) in kFillWidthsTrack.
hipError_t launch_fill(int W, int lay, bool local, int planes, bool track, bool lcs, bool tbl, const PairDev* d_pairs,
                       int npairs, int total_bands, int* d_counter, StripRes* d_sres, PairRes* d_pres, Scores32 sc,
                       int grid, hipStream_t st) {
#define GX_FILL_CASE(LO, PL, TR, LC, TB, ...)                                                                \
    if (local == LO && planes == PL && track == TR && lcs == LC && tbl == TB)                                \
        return launch_fill_w<LO, PL, TR, LC, TB, __VA_ARGS__>(W, lay, d_pairs, npairs, total_bands, d_counter, d_sres, \
                                                              d_pres, sc, grid, st);
#define GX_W_ALL 3, 4, 6, 8, 11, 15
#define GX_W_TRACK 3, 7
    GX_FILL_CASE(false, 0, false, false, false, GX_W_ALL)
    GX_FILL_CASE(false, 0, false, false, true, GX_W_ALL)
    GX_FILL_CASE(false, 0, true, false, false, GX_W_TRACK)
    GX_FILL_CASE(false, 1, false, false, false, GX_W_ALL)
    GX_FILL_CASE(false, 1, false, false, true, GX_W_ALL)
    GX_FILL_CASE(false, 2, false, false, false, GX_W_ALL)   // compact planes (layout 0)
    GX_FILL_CASE(false, 2, false, false, true, GX_W_ALL)
    GX_FILL_CASE(false, 1, true, false, false, GX_W_TRACK)
    GX_FILL_CASE(false, 1, true, true, false, GX_W_TRACK)
    GX_FILL_CASE(true, 0, false, false, false, GX_W_TRACK)
    GX_FILL_CASE(true, 0, false, false, true, GX_W_TRACK)
    GX_FILL_CASE(true, 0, true, false, false, GX_W_TRACK)
    GX_FILL_CASE(true, 1, false, false, false, GX_W_TRACK)
    GX_FILL_CASE(true, 1, false, false, true, GX_W_TRACK)
    GX_FILL_CASE(true, 2, false, false, false, GX_W_TRACK)   // compact planes, local (layout 0)
    GX_FILL_CASE(true, 2, false, false, true, GX_W_TRACK)
    GX_FILL_CASE(true, 1, true, false, false, GX_W_TRACK)
    GX_FILL_CASE(true, 1, true, true, false, GX_W_TRACK)
#undef GX_FILL_CASE
    return hipErrorInvalidValue;
}

hipError_t launch_finalize(const PairDev* d_pairs, int npairs, const StripRes* d_sres, PairRes* d_pres,
                           hipStream_t st) {
    hipLaunchKernelGGL(finalize_kernel, dim3(npairs), dim3(64), 0, st, d_pairs, d_sres, d_pres);
    return hipGetLastError();
}

hipError_t launch_traceback(const TbDev* d_jobs, int njobs, int max_strips, bool w16, bool seq, hipStream_t st) {
    if (seq) {   // no skeleton: the strips walked in sequence (twin plane codes only)
        hipLaunchKernelGGL(tb_seq_kernel, dim3(njobs), dim3((1 + kSqHelp) * kWave), 0, st, d_jobs);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(tb_chase_kernel, dim3(njobs), dim3(64), 0, st, d_jobs);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (w16) {   // code words of the path's strips from the twin plane codes
        hipLaunchKernelGGL(tb_w16_codes_kernel, dim3(max_strips, njobs), dim3(kStripRows), 0, st, d_jobs);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(tb_strip_kernel, dim3(max_strips, njobs), dim3(64), 0, st, d_jobs);
    return hipGetLastError();
}

hipError_t launch_export_d8(const uint8_t* pI, const uint8_t* px, int32_t* out, int n, int m, int t4, int h, int g,
                            int floor_, int gshift, int row0, int rows, hipStream_t st) {
    if (n == 0 || m == 0 || rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(export_d8_kernel, dim3((unsigned)((rows + 63) / 64)), dim3(64), 0, st, pI, px, out, n, m, t4, h,
                       g, floor_, gshift, row0, rows);
    return hipGetLastError();
}

hipError_t launch_export_w16(const uint8_t* codes, int half, int which, int32_t* out, int n, int m, int t4, int h,
                             int g, int floor_, int gshift, int row0, int rows, hipStream_t st) {
    if (n == 0 || m == 0 || rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(export_w16_kernel, dim3((unsigned)((rows + 63) / 64)), dim3(64), 0, st, codes, half, which, out,
                       n, m, t4, h, g, floor_, gshift, row0, rows);
    return hipGetLastError();
}

hipError_t launch_export(const int32_t* plane, int32_t* out, int n, int m, int t4, int lay, int gshift, int row0,
                         int rows, hipStream_t st) {
    const size_t total = (size_t)rows * m;
    if (total == 0 || rows <= 0) return hipSuccess;
    const int blk = 256;
    hipLaunchKernelGGL(export_kernel, dim3((unsigned)((total + blk - 1) / blk)), dim3(blk), 0, st, plane, out, n, m,
                       t4, lay, gshift, row0, rows);
    return hipGetLastError();
}

// Plane checksums of the npairs pairs of a launch (descriptors on the device)
// into out[npairs][3] (zeroed here); max_strips = the most strips of any pair.
// The local twin fill (gx_fill_pk.hip LOCAL) keeps each row's largest
// score_max only; finalize_kernel has picked the last row holding the pair's
// maximum (PairRes.lmax_i, lmax_val).  This finds that row's LAST column
// holding it (the reference's row-major max_by, algo.rs:310-322) from the twin
// plane codes: I(i, j) = max(I(i, j-1) + d_j, 0) with d_j = g + max(0,
// m(i, j-1) + h), m = max(x_S, x_D) of the previous cell (w16_next_I; I(i, 0)
// = H(i, 0) + h = h, m = 0), score_max = I + max(0, x_S, x_D).
// One wave per pair: each lane takes a chunk of the row; the maps x -> max(x
// + A, B) that the chunks apply to I compose (max(max(x + A1, B1) + A2, B2)
// = max(x + A1 + A2, max(B1 + A2, B2))), so an exclusive scan of them gives
// every lane its starting I, and the highest matching column wins.
__global__ __launch_bounds__(64) void local_col_kernel(const PairDev* __restrict__ pairs, PairRes* __restrict__ pres,
                                                      const int h, const int g) {
    const PairDev d = pairs[blockIdx.x];
    PairRes* const r = pres + blockIdx.x;
    const int lane = threadIdx.x;
    const int i = __builtin_amdgcn_readfirstlane(r->lmax_i), target = __builtin_amdgcn_readfirstlane(r->lmax_val);
    if (i < 1 || i > d.n || d.m < 1 || !d.pI) return;
    const int s = (i - 1) / kStripRows, rr = (i - 1) % kStripRows, l = rr >> 1, hh = rr & 1;
    (void)hh;
    const uint8_t* base = (const uint8_t*)d.pI + w12_rec_off(s, d.t4, 0, rr);
    const int sh = 16 * d.twin_half;
    const int C = (d.m + kWave - 1) / kWave, j0 = lane * C + 1, j1 = min(d.m, j0 + C - 1);
    auto code_at = [&](int j, int& xS, int& xD) {
        const int t = j + l - 1;   // the step at which this row computes column j (anti-diagonal skew)
        const uint4 rec = w12_load(base + (size_t)(t >> 2) * kTwinGroupBytes);
        const uint32_t w = (t & 3) == 0 ? rec.x : (t & 3) == 1 ? rec.y : (t & 3) == 2 ? rec.z : rec.w;
        w16_decode((w >> sh) & 0xFFFFu, xS, xD);
    };
    constexpr int kLow = INT_MIN / 4;   // "no floor yet" (far below every value, no overflow when shifted)
    int mp0 = 0;                        // m of the cell before the chunk (column 0: 0)
    if (j0 >= 2 && j0 <= j1) { int a, b; code_at(j0 - 1, a, b); mp0 = max(a, b); }
    int A = 0, B = kLow, mp = mp0;      // the chunk's map x -> max(x + A, B)
    for (int j = j0; j <= j1; ++j) {
        int a, b;
        code_at(j, a, b);
        const int dj = g + max(0, mp + h);
        A += dj; B = max(B + dj, 0);
        mp = max(a, b);
    }
    // exclusive scan of the maps over the lanes (earlier chunks first)
    int SA = A, SB = B;                 // inclusive: this chunk after all earlier ones
    for (int o = 1; o < kWave; o <<= 1) {
        const int pa = __shfl_up(SA, o), pb = __shfl_up(SB, o);
        if (lane >= o) { SB = max(pb + SA, SB); SA = pa + SA; }
    }
    int EA = __shfl_up(SA, 1), EB = __shfl_up(SB, 1);   // exclusive
    if (lane == 0) { EA = 0; EB = kLow; }
    int I = max(h + EA, EB), last = 0;
    mp = mp0;
    for (int j = j0; j <= j1; ++j) {
        int a, b;
        code_at(j, a, b);
        I = w16_next_I(I, mp, h, g, true);
        mp = max(a, b);
        if (I + max(0, max(a, b)) == target) last = j;
    }
    for (int o = 32; o > 0; o >>= 1) last = max(last, __shfl_xor(last, o));
    if (lane == 0) r->lmax_j = last;
}
hipError_t launch_local_col(const PairDev* d_pairs, int npairs, PairRes* d_pres, int h, int g, hipStream_t st) {
    if (npairs <= 0) return hipSuccess;
    hipLaunchKernelGGL(local_col_kernel, dim3((unsigned)npairs), dim3(64), 0, st, d_pairs, d_pres, h, g);
    return hipGetLastError();
}

hipError_t launch_plane_sums(const PairDev* d_pairs, int npairs, int max_strips, int lay, int mode, int h, int g,
                             int floor_, int gshift, unsigned long long* out, hipStream_t st) {
    if (npairs <= 0 || max_strips <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(out, 0, (size_t)npairs * 3 * sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    const int blocks = max_strips * (lay ? 1 : kStripRows / kWave);
    hipLaunchKernelGGL(plane_sums_kernel, dim3((unsigned)blocks, (unsigned)npairs), dim3(64), 0, st, d_pairs, lay,
                       mode, h, g, floor_, gshift, out);
    return hipGetLastError();
}

}  // namespace gx
