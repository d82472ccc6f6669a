// gx_skew.hip -- layout 3, the latency fill of a single pair (or a few):
// anti-diagonal skew over 64-row strips, ONE row per lane, each strip on two
// waves.
//
// The reference fills its table one cell at a time (src/alignment/algo.rs:
// 151-282).  Any schedule of that recurrence needs n + m dependent
// anti-diagonal steps, so a single pair's time is (n + m + strip lags) x the
// time of one step.  Layout 0 (gx_kernels.hip compute_wave) gives each lane
// two rows, so one of its steps is two dependent cells; layout 1 (the column
// step) takes m steps of a whole 64-row column but each is a 6-round DPP
// prefix scan.  Here lane l of a strip owns row 64 s + l + 1 and at step t
// computes column j = t - l + 1: one cell per lane per step.
//
// A lone wave issues about one instruction per 4-5 cycles whatever its kind
// (VALU, SALU, LDS, VMEM), so a step costs its instruction count.  One wave
// doing everything took ~30 instructions (~200 cycles) a step; the strip is
// therefore split over two waves on different SIMDs:
//   * the CORE wave runs the recurrence only (10 VALU a step) and hands each
//     4-step group's cells (S, D per lane) to the side wave through an LDS
//     ring, 2 ds_write_b128 a group;
//   * the SIDE wave re-derives I from the row's previous cell, then the
//     retrace bits and the landing column of every cell (algo.rs:351-400 priority S > I > D), stores the three int32 score
//     planes straight from the registers it read, the code words and the
//     skeleton, and tracks the local last maximum.
// The cell above (i-1, j) is lane l-1's previous step (DPP wave_shr:1 with
// bound_ctrl, folded into one v_add_u32_dpp with a register that holds lane
// 0's ring value and 0 elsewhere: lane 0 takes the cell from the ring the
// strip above's core wave fills, or the band's I/O wave at a band boundary),
// the top-left (i-1, j-1) the one before (kept from the previous step's move).
// Global fills start every lane at step 0 on virtual columns <= 0 whose
// "minus infinity" state yields column 0 exactly (no per-lane masks in the
// ramp-up); local fills mask the ramp-up with selects.  Measured costs and
// the floor of this design: DESIGN.md 4.5.  Global fills keep V'' = V - (i + j) g (DESIGN.md
// 4.3) and, with h <= 0, fold both gap recurrences onto score_max:
//         I''(i,j)   = max(I''(i,j-1), H''(i,j-1) + h)        (algo.rs:231-236)
//         D''(i+1,j) = max(D''(i,j),   H''(i,j)   + h)        (algo.rs:238-243)
//         S''(i,j)   = H''(i-1,j-1) + s - 2g                  (algo.rs:245-248)
// (H + h adds I + h <= I and D + h <= D, which never win); local fills keep
// plain values with the 0 floor in each gap max (algo.rs:103).
// Outputs in the step-indexed formats of layout 0 with one row per lane:
// int32 planes plane[strip][t/4][lane][t%4], code words
// codes[strip][t/16][lane] (bit 31-k "delete beats insert and sub", bit 15-k
// "insert beats sub"), and each strip's bottom-row landing columns + 64 as the
// skeleton, so the traceback chases it and walks all strips at once
// (gx_kernels.hip tb_chase_kernel / tb_strip_kernel, TbDev.skew).
// Strip-to-strip rings hold 4-column groups in SoA form (dd[4], sm[4] of
// columns 4G-3 .. 4G, column c in group (c + 3) / 4): the core wave of the
// strip above pushes a group as two ds_write_b128 from lane 63 and the core
// below reads it as two ds_read_b128.  Each lane reads its own column symbols
// (one dwordx4 per group, prefetched four groups ahead) from an int32 copy of
// s2 (skew_codes_kernel), so no symbol moves between lanes.
// No MFMA: an integer max-plus recurrence.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>
#include "gx_internal.h"

#include "gx_device.h"
#include "gx_lcs.h"

namespace gx {

typedef __attribute__((address_space(3))) v4i lds_v4i;
constexpr int kSkRingG = 64;     // ring groups per strip boundary (256 columns)
constexpr int kSkHo = 8;         // core -> side hand-off ring depth (4-step groups)

struct SkRing {                  // one strip boundary (see the file header)
    int dd[kSkRingG][4];
    int sm[kSkRingG][4];
};
struct SkHo {                    // one strip's core -> side ring: [group][S, D][lane] int4 (the side
    int4 v[kSkHo][2][kWave];     // wave derives I from them: side_group)
};
__device__ __forceinline__ int sk_grp(int c) { return ((c + 3) >> 2) & (kSkRingG - 1); }
__device__ __forceinline__ int sk_pos(int c) { return (c + 3) & 3; }

// ---------------------------------------------------------------------------
// core wave

struct CoreState {               // cell (i, j-1) of the lane's row
    int I;                       // insert score
    int Hx;                      // H + h (global) / H + h + g (local): the next insert's and delete's gap term
    int H;                       // score_max
    int Dd;                      // delete successor D(i+1, j-1)
    int Hd;                      // score_max(i-1, j-1)
};

// One anti-diagonal step: cell (i, j), j = t - lane + 1.  (rdd, rsm) = lane
// 0's cell above from the ring (0 in the other lanes); c2 = s2[j-1] (its symbol code * 8 with score
// tables).  MASKED (ramp-down): act = false keeps the row at its last column.
template <bool LOCAL, bool TBL, bool MASKED>
__device__ __forceinline__ void core_step(CoreState& st, const int rdd, const int rsm, const int c2, const bool act,
                                          const int c1v, const Scores32& sc, int& oI, int& oS, int& oD) {
    const int Dn = shz(st.Dd) + rdd;         // D(i, j): the delete successor of the cell above
    const int hu = shz(st.H) + rsm;          // score_max(i-1, j)  (rdd, rsm: 0 but in lane 0)
    const bool mt = c2 == c1v;               // sequence.rs:113-114
    const int Sn = st.Hd + (TBL ? c2 : (mt ? sc.sm : sc.smm));   // (TBL: c2 is the score of this row's symbol against s2[j-1])
    const int In = LOCAL ? max3i(st.I + sc.g, st.Hx, 0) : max(st.I, st.Hx);
    const int IS = max(In, Sn);
    const int Hn = max(IS, Dn);
    const int Hxn = Hn + (LOCAL ? sc.hg : sc.h);
    const int Ddn = LOCAL ? max3i(Dn + sc.g, Hxn, 0) : max(Dn, Hxn);
    if (MASKED) {
        st.I = act ? In : st.I; st.Hx = act ? Hxn : st.Hx; st.H = act ? Hn : st.H; st.Dd = act ? Ddn : st.Dd;
    } else {
        st.I = In; st.Hx = Hxn; st.H = Hn; st.Dd = Ddn;
    }
    st.Hd = hu;
    oI = In; oS = Sn; oD = Dn;
}

struct CoreCtx {
    __amdgpu_buffer_rsrc_t crs;  // the pair's int32 column symbols (PairDev.ccodes)
    uint32_t cvoff;              // 4 (64 - lane): this lane's column of step 0, less one
    uint32_t push_base;          // LDS address; lane 63: the ring below's dd[0]; other lanes (or no consumer): their sink slot
    uint32_t push_m16;           // lane 63: 16 (a ring group's bytes); other lanes: 0
    lds_int* pcnt;               // wcnt_out (no consumer: a sink)
    uint32_t rd_base;            // LDS address; lane 0: the ring above's dd[0]; other lanes: a zero block
    uint32_t rd_m16;             // lane 0: 16; other lanes: 0
    const SkRing* rin;
    SkRing* rout;
    lds_int* wcnt_in;            // columns the strip above published
    lds_int* rcnt_in;            // ... of which this strip has read (its flow control)
    lds_int* wcnt_out;
    lds_int* rcnt_out;
    SkHo* ho;
    lds_int* hcnt;               // hand-off groups written (core) / read (side), per sub-block
    lds_int* bcnt;
    v4i* hv_sub;                 // this lane's slot of the sub-block's first group (ho->v[(t0/4) % kSkHo][0][lane])
    int* status;
    int m, lane, c1;
    int space_out, space_ho;     // rcnt_out / bcnt as read at the previous sub-block (lower bounds, core_sub)
    bool push_on;
    unsigned tr_win, tr_ho;      // (diagnostics: spins waiting for the strip above / for hand-off space)
    long long* tl;               // (diagnostics: the strip's dense timeline, StripTrace.tl)
};

// Lane 0 reads ring group G (dd, then sm 1 KB on), the other lanes a zero block.
__device__ __forceinline__ void read_grp(v4i (&r)[2], const CoreCtx& w, int G) {
    const lds_v4i* p = (const lds_v4i*)(uintptr_t)(w.rd_base + __umul24((uint32_t)G, w.rd_m16));
    r[0] = p[0];
    r[1] = p[kSkRingG];
}
// This lane's column symbols of steps t .. t+3 (columns t-lane+1 ..).
__device__ __forceinline__ int4 load_codes(const CoreCtx& w, int t) {
    const v4i x = __builtin_amdgcn_raw_buffer_load_b128(w.crs, (int)w.cvoff, __builtin_amdgcn_readfirstlane(4 * t), 0);
    return make_int4(x[0], x[1], x[2], x[3]);
}

// One 4-step group of the core wave.  MODE 0: every lane steps; 2: per-lane
// selects (ramp-down of the strip holding row n: lanes past column m keep
// their state; local ramp-up: lanes not started keep their column-0 state;
// selects measured 72 ns a step against 100 for a branch per step); 3: the
// ramp-down of every other global strip: every lane steps on into virtual
// columns past m (nothing reads a lane's state after its column m: the pushes
// stop at column m, the side wave masks its own state), pushes as in MODE 2.
// The ramp-down is on the chain's critical path (a strip's last columns wait
// for the strip above's), so it runs at the steady pace (30k pair 4.36 -> 4.05 ms).
// A group's LDS store data (hand-off I, S, D; push dd, sm) stays allocated
// through the next group (pinned there), so the next group's results never
// reuse registers an LDS store may still be reading (which would cost a wait
// for that store: LDS reads store data after issue).
struct CorePend {
    v4i v[4];                    // hand-off S, D; push dd, sm
};
__device__ __forceinline__ void pin(const CorePend& p) {
    asm volatile("" ::"v"(p.v[0]), "v"(p.v[1]), "v"(p.v[2]), "v"(p.v[3]));
}

template <bool LOCAL, bool TBL, int MODE, int Q>
__device__ __forceinline__ void core_group(CoreState& st, const v4i (&cur)[2], v4i (&nxt)[2], int4& cc, CoreCtx& w,
                                           const Scores32& sc, const int t, CorePend& mine, const CorePend& prev) {
    const int need = min(t + 8, w.m) + 1;                      // columns of the next group: t+5 .. t+8
    const int seen_v = lds_peek(w.wcnt_in);
    asm volatile("" ::: "memory");
    read_grp(nxt, w, sk_grp(t + 5));
    const int pdd = st.Dd, psm = st.H;                         // lane 63: column t - 63 (the push below)
    int oI[4] = {}, oS[4] = {}, oD[4] = {}, qdd[3], qsm[3];
    const int cd[4] = {cur[0][0], cur[0][1], cur[0][2], cur[0][3]};
    const int cs[4] = {cur[1][0], cur[1][1], cur[1][2], cur[1][3]};
    const int c2[4] = {cc.x, cc.y, cc.z, cc.w};
#pragma unroll
    for (int U = 0; U < 4; ++U) {
        // MODE 2: selects per lane (global fills run the virtual columns <= 0
        // too: only columns > m stop; local fills also hold lanes not started)
        const int c = t + U - w.lane;   // column - 1
        const bool act = MODE == 2 ? (LOCAL ? (unsigned)c < (unsigned)w.m : c < w.m) : true;
        core_step<LOCAL, TBL, MODE == 2>(st, cd[U], cs[U], c2[U], act, w.c1, sc, oI[U], oS[U], oD[U]);
        if (U < 3) { qdd[U] = st.Dd; qsm[U] = st.H; }
    }
    // the symbols of this group's steps four groups on, into the registers
    // just consumed (loaded after the steps, so that the loop carries them
    // in place)
    cc = load_codes(w, t + 16);
    // hand the group's cells to the side wave (slot t/4 mod kSkHo; the side
    // wave has read the slot's previous group: checked per sub-block)
    {
        v4i* hv = w.hv_sub + Q * 2 * kWave;
        mine.v[0] = v4i{oS[0], oS[1], oS[2], oS[3]};
        mine.v[1] = v4i{oD[0], oD[1], oD[2], oD[3]};
        hv[0] = mine.v[0];
        hv[kWave] = mine.v[1];
        asm volatile("" ::: "memory");                         // (the data stores stay before the count)
        if (Q == 3) lds_post(w.hcnt, (t >> 2) + 1);            // (per sub-block; every lane, one value; LDS keeps the order)
    }
    // lane 63 pushes ring group (t - 60) / 4: its columns t-63 .. t-60 (before
    // this group's step 0, after steps 0, 1, 2), then the count (same wave,
    // LDS in order).  Every lane writes (lanes 0..62 into a sink), so the
    // compiler sees and counts the stores: no exec change, no branch.
    mine.v[2] = v4i{pdd, qdd[0], qdd[1], qdd[2]};
    mine.v[3] = v4i{psm, qsm[0], qsm[1], qsm[2]};
    if (MODE == 0 || (t >= 64 && t - 63 <= w.m)) {            // (full groups: always inside; no consumer: all into the sink)
        lds_v4i* a = (lds_v4i*)(uintptr_t)(w.push_base + __umul24((uint32_t)sk_grp(t - 63), w.push_m16));
        const int cnt = (MODE == 0 ? t - 60 : min(t - 60, w.m)) + 1;   // (MODE 0: t - 60 < m; 2, 3: the ramp-down)
        a[0] = mine.v[2];
        a[kSkRingG] = mine.v[3];
        asm volatile("" ::: "memory");
        lds_post(w.pcnt, cnt);
    }
    if (__builtin_amdgcn_readfirstlane(seen_v) < need) {       // the strip above was behind: wait, re-read
        w.tr_win += wait_ge_tight(w.wcnt_in, need, w.status);
        // re-read into the same registers and wait for it here (one asm: no
        // copies on the fast path, nothing pending after the join)
        const uint32_t a = w.rd_base + __umul24((uint32_t)sk_grp(t + 5), w.rd_m16);
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:%3\n\ts_waitcnt lgkmcnt(0)"
                     : "+v"(nxt[0]), "+v"(nxt[1])
                     : "v"(a), "i"(kSkRingG * 16)
                     : "memory");
    }
    pin(prev);
    __builtin_amdgcn_sched_barrier(0);
}

struct CoreLoop {                 // the core wave's loop-carried state besides CoreState
    v4i ra[2], rb[2];            // ring groups (current / next), alternating
    int4 cc[4];                  // column symbols of the next four groups
    CorePend pa, pb;             // pinned store data, alternating
    long long tr_q[kTraceQ];     // (diagnostics: timeline stamps)
};

// One 16-step sub-block: flow control, then four groups.
template <bool LOCAL, bool TBL, int MODE, bool TRACE>
__device__ __forceinline__ void core_sub(CoreState& st, CoreLoop& L, CoreCtx& w, const Scores32& sc, const int t0,
                                         const int T, const bool trace) {
    // ring space below: the strip below has read what these pushes
    // overwrite (the last group pushes columns up to t0 + 12 - 60); hand-off
    // space: the side wave has read this sub-block's slots' previous groups.
    // Both checked against counts read one sub-block ago, so that no LDS
    // round trip is waited for unless those fall short (the ring holds 256
    // columns, the strip below reads ~72 behind; the side keeps up).
    const int last_col = min(t0 - 48, w.m);
    if (w.push_on && last_col >= kSkRingG * 4 - 4) {
        const int v = last_col - (kSkRingG * 4 - 4) + 1;
        if (w.space_out < v) wait_ge(w.rcnt_out, v, w.status);
    }
    if (t0 >= 4 * kSkHo) {
        const int v = (t0 >> 2) + 4 - kSkHo;
        if (w.space_ho < v) w.tr_ho += wait_ge(w.bcnt, v, w.status);
    }
    if (w.push_on) w.space_out = lds_peek(w.rcnt_out);
    w.space_ho = lds_peek(w.bcnt);
    w.hv_sub = (v4i*)&w.ho->v[(t0 >> 2) & (kSkHo - 1)][0][w.lane];
    if (TRACE && trace) {
        const int q = (int)((long long)t0 * (kTraceQ + 1) / T) - 1;
        const long long now = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int k = 0; k < kTraceQ; ++k)   // (constant indices: the stamps stay in registers)
            if (k >= 1 && k == q && L.tr_q[k] == 0) L.tr_q[k] = now;
        if (t0 == kWave) L.tr_q[0] = now;                  // (the end of the ramp-up)
        if ((t0 & 1023) == 0 && (t0 >> 10) < kTraceTL && w.lane == 0) {
            w.tl[t0 >> 10] = now;
            w.tl[kTraceTL + (t0 >> 10)] = __builtin_amdgcn_s_memtime();   // (StripTrace.tc follows tl)
        }
    }
    core_group<LOCAL, TBL, MODE, 0>(st, L.ra, L.rb, L.cc[0], w, sc, t0, L.pa, L.pb);
    core_group<LOCAL, TBL, MODE, 1>(st, L.rb, L.ra, L.cc[1], w, sc, t0 + 4, L.pb, L.pa);
    core_group<LOCAL, TBL, MODE, 2>(st, L.ra, L.rb, L.cc[2], w, sc, t0 + 8, L.pa, L.pb);
    core_group<LOCAL, TBL, MODE, 3>(st, L.rb, L.ra, L.cc[3], w, sc, t0 + 12, L.pb, L.pa);
    // every ring read up to column t0+20 (incl. the next group's) was issued before this store
    asm volatile("" ::: "memory");
    lds_post(w.rcnt_in, min(t0 + kSub + 5, w.m + 1));
}

// TRACE: a diagnostics build (GX_TRACE_FILE).  Its stamps are scalar-memory
// instructions, which count on lgkmcnt out of order: any that may be in
// flight make the compiler wait for lgkmcnt(0) at every LDS use (30k pair
// 4.0 -> 3.8 ms without them), so the stamps live in their own instantiation.
template <bool LOCAL, bool TBL, bool TRACE>
__device__ void core_wave(const PairDev& P, const int s, const int lane, const Scores32& sc, CoreCtx& w,
                          PairRes* pres) {
    const int n = P.n, m = P.m;
    const int i = s * kWave + lane + 1;          // this lane's row
    const bool ok = i <= n;
    StripTrace* const trace = TRACE ? P.trace : nullptr;
    w.m = m; w.lane = lane; w.tr_win = 0; w.tr_ho = 0;
    w.space_out = w.space_ho = 0;
    w.tl = trace ? trace[s].tl : nullptr;
    w.c1 = ok ? (int)P.c1[i - 1] : 0x1FF;        // 0x1FF never equals a byte
    // column 0 (algo.rs:204-211): I = S = neg_inf, D = h + i g, score_max
    // max(D, floor); global fills hold V - (i + 0) g
    // Global fills: lane l >= 1 starts at step 0 on virtual columns 1 - l .. 0
    // (no per-lane masks in the ramp-up).  Its state starts at "minus
    // infinity", so virtual columns < 0 stay there and column 0 comes out of
    // the recurrence exactly: I = S = -inf, D''(i, 0) = max(D''(i-1, 0),
    // H''(i-1, 0) + h) = h from lane l-1, score_max = D (algo.rs:204-211).
    // Local fills keep the masked ramp-up (their 0 floor lifts virtual cells).
    CoreState st;
    int H0;                                       // score_max(i, 0) (shifted for global fills)
    {
        const int D0 = sc.h + i * sc.g;
        H0 = LOCAL ? max(D0, 0) : D0 - i * sc.g;
        const bool virt = !LOCAL && lane > 0;
        st.I = LOCAL ? kNeg : kNeg - i * sc.g;
        st.H = virt ? kNeg : H0;
        st.Hx = virt ? kNeg : H0 + (LOCAL ? sc.hg : sc.h);
        st.Dd = virt ? kNeg : H0;                 // (lane 0: the successor D''(i+1, 0) = max(h, 2h) = h)
    }
    {   // this lane's column inputs (skew_codes_kernel): with score tables
        // (<= 4 symbols) the scores of its row's symbol against every column
        // -- one of four int32 rows, so a step adds the loaded value -- else
        // the column symbols themselves
        const uint32_t row = 4u * (uint32_t)(m + 192);
        const uint32_t k = TBL ? (uint32_t)sym_code(w.c1, sc) : 0u;   // (rows past n: symbol 0, never stored)
        w.crs = rsrc_of(uniform_ptr(P.ccodes), (int)((TBL ? 4 : 1) * row));
        w.cvoff = 4u * (uint32_t)(64 - lane) + k * row;
    }
    if (w.push_on) {                              // column 0 of the bottom row: the next strip's first top-left
        if (lane == kWave - 1) {
            w.rout->dd[0][3] = H0;                // (the delete successor of column 0: H0, see above)
            w.rout->sm[0][3] = H0;
            asm volatile("" ::: "memory");
            *w.wcnt_out = 1;
        }
    }
    long long tr_start = 0, tr_first = 0, clk_first = 0;
    if (trace) tr_start = __builtin_amdgcn_s_memrealtime();
    w.tr_win += wait_ge(w.wcnt_in, min(4, m) + 1, w.status);
    CoreLoop L = {};
#pragma unroll
    for (int q = 0; q < 4; ++q) L.cc[q] = load_codes(w, 4 * q);
    st.Hd = shr1(w.rin->sm[0][3], st.H);          // column 1's top-left: (64 s, 0) for lane 0, lane-1's column 0
    if (!LOCAL && lane > 0) st.Hd = kNeg;         // (virtual columns)
    read_grp(L.ra, w, sk_grp(1));
    if (trace) { tr_first = __builtin_amdgcn_s_memrealtime(); clk_first = __builtin_amdgcn_s_memtime(); }
    const int T = m + kWave;                      // lane 63 computes column m at step m + 62; pushes run to t = m + 63
    // ramp-up (global: every lane steps, on virtual columns until its column
    // 1 at step l; local: per-lane selects) while no lane passes column m;
    // then every lane inside columns 1..m; then masked per lane.  One loop per
    // phase, so that the loop-carried registers (ring groups, prefetched
    // symbols, pinned store data) keep their places across the back-edge
    // (a merge of differently allocated phases costs copies that wait for
    // the symbol loads in flight).
    int t0 = 0;
    if (!LOCAL)   // (virtual columns: every lane runs from step 0, see the column-0 state above)
        for (; t0 < T && t0 + kSub <= kWave && t0 + kSub - 1 <= m - 1; t0 += kSub)
            core_sub<LOCAL, TBL, 0, TRACE>(st, L, w, sc, t0, T, trace != nullptr);
    for (; t0 < T && t0 + kSub <= kWave && t0 + kSub - 1 <= m - 1; t0 += kSub)
        core_sub<LOCAL, TBL, 2, TRACE>(st, L, w, sc, t0, T, trace != nullptr);
    for (; t0 < T && t0 >= kWave && t0 + kSub - 1 <= m - 1; t0 += kSub)
        core_sub<LOCAL, TBL, 0, TRACE>(st, L, w, sc, t0, T, trace != nullptr);
    if (!LOCAL && s + 1 < P.strips)               // (row n is in the last strip: its lane keeps column m's state)
        for (; t0 < T; t0 += kSub)
            core_sub<LOCAL, TBL, 3, TRACE>(st, L, w, sc, t0, T, trace != nullptr);
    for (; t0 < T; t0 += kSub)
        core_sub<LOCAL, TBL, 2, TRACE>(st, L, w, sc, t0, T, trace != nullptr);
    if (ok && i == n) pres->end_SM = st.H;        // score_max(n, m) (algo.rs:308, 331)
    if (trace && lane == 0) {
        StripTrace tr;
        tr.t_start = tr_start; tr.t_first = tr_first; tr.t_end = __builtin_amdgcn_s_memrealtime();
        tr.wait_in = (int)w.tr_win;
        tr.clk = __builtin_amdgcn_s_memtime() - clk_first;
        for (int q = 0; q < kTraceQ; ++q) tr.t_q[q] = L.tr_q[q];
        tr.t_q[kTraceQ - 2] = w.tr_ho;            // (layout 3: hand-off space waits; the side wave writes wait_out
        trace[s].t_start = tr.t_start;            // and the last stamp, its own waits and end)
        trace[s].t_first = tr.t_first;
        trace[s].t_end = tr.t_end;
        trace[s].wait_in = tr.wait_in;
        trace[s].clk = tr.clk;
        for (int q = 0; q < kTraceQ - 1; ++q) trace[s].t_q[q] = tr.t_q[q];
    }
}

// ---------------------------------------------------------------------------
// side wave

struct SideState {
    int I, H;                    // insert score and score_max of (i, j-1) (I of (i, j) follows from them)
    int E, Ed;                   // landing column + 64 of (i, j-1) and of (i-1, j-1)
    uint32_t cI, cD;
    int lbest, lstep, lE;        // LOCAL: the row's last max of score_max (algo.rs:310-322)
    // TRACK: the row's FIRST maximum of score_max (algo.rs:258-262: strict <),
    // held as thr = best - (i + j) g at the current column j for shifted
    // (global) fills, so that a step compares its shifted value directly
    // (max_matches is not carried here: the bit-parallel LCS rows of the
    // launch's leading workgroups, gx_lcs.h)
    int thr, bstep;
};

// Retrace bits and landing column of cell (i, j) from its I, S, D.
template <bool LOCAL, bool MASKED>
__device__ __forceinline__ void side_step(SideState& st, const int I, const int S, const int D, const int t,
                                          const bool act) {
    const int eu = shr1(t + 65, st.E);        // E(i-1, j) + 64; lane 0: the top boundary row, column j
    const int IS = max(I, S);
    int En;
    {   // I beats S -> insert (E from the left), D beats both -> delete (E from above), else sub (top-left)
        unsigned long long m1, m2;
        asm volatile(
            "v_cmp_gt_i32 %[m1], %[in], %[sn]\n\t"
            "v_cmp_gt_i32 %[m2], %[dn], %[is]\n\t"
            "v_cndmask_b32 %[en], %[etl], %[el], %[m1]\n\t"
            "v_addc_co_u32 %[ci], vcc, %[ci], %[ci], %[m1]\n\t"
            "v_addc_co_u32 %[cd], vcc, %[cd], %[cd], %[m2]\n\t"
            "v_cndmask_b32 %[en], %[en], %[eu], %[m2]"
            : [en] "=&v"(En), [ci] "+v"(st.cI), [cd] "+v"(st.cD), [m1] "=&s"(m1), [m2] "=&s"(m2)
            : [in] "v"(I), [sn] "v"(S), [dn] "v"(D), [is] "v"(IS), [etl] "v"(st.Ed), [el] "v"(st.E), [eu] "v"(eu)
            : "vcc");
    }
    if (LOCAL) {   // algo.rs:310-322: max_by keeps the LAST maximum
        const int H = max(IS, D);
        const bool nl = act && H >= st.lbest;
        st.lbest = nl ? H : st.lbest; st.lstep = nl ? t : st.lstep; st.lE = nl ? En : st.lE;
    }
    st.E = MASKED ? (act ? En : st.E) : En;
    st.Ed = eu;
}

struct SideCtx {
    SkHo* ho;
    lds_int* hcnt;
    lds_int* bcnt;
    int* status;
    uint32_t* codes;
    __amdgpu_buffer_rsrc_t rI, rD, rS;   // the strip's planes (offset in the VGPR; see gx_device.h bstore4)
    __amdgpu_buffer_rsrc_t skel_rsrc;    // skeleton row of this strip (bottom-row E + 64)
    uint32_t skel_voff;                  // lane 63: 0; other lanes: out of range
    int m, lane;
    int h, g, hg;                        // gap open / extend (global fills: shifted, g folded: g = 0)
    unsigned tr_wait;                    // (diagnostics: spins waiting for the core wave)
    long long* ts;                       // (diagnostics: the side's dense timeline, StripTrace.ts)
    int gs;                              // TRACK: the shift per column of the tracked values (global: g; local: 0)
};

// I(i, j) from the row's previous cell, as the core computes it (the core
// hands over only S and D, one ds_write_b128 fewer per group on its path):
// global (shifted, h <= 0) max(I, H + h); local max(I + g, H + h + g, 0).
template <bool LOCAL, bool MASKED>
__device__ __forceinline__ int side_insert(SideState& st, const SideCtx& w, const int S, const int D, const bool act) {
    const int In = LOCAL ? max3i(st.I + w.g, st.H + w.hg, 0) : max(st.I, st.H + w.h);
    const int Hn = max3i(In, S, D);
    st.I = MASKED ? (act ? In : st.I) : In;
    st.H = MASKED ? (act ? Hn : st.H) : Hn;
    return In;
}

// TRACK: the row's first maximum of score_max (algo.rs:258-262), H that of
// cell (i, j) at step t.  COL: with its column (a compare and two selects);
// without (fills that keep their planes), the row's largest value only --
// thr = max(thr - g, H), two instructions a cell (local: one) -- and
// skew_max_col_kernel finds the first column holding it in the one row that
// finalize_kernel picks, from the planes (the side wave sets a tracked
// fill's pace: 30k pair 4.87 ms with the column against 4.25 untracked).
template <bool MASKED, bool LOCAL, bool COL>
__device__ __forceinline__ void track_step(SideState& st, const SideCtx& w, const int H, const int t, const bool act) {
#ifdef GX_DIAG_NO_TRACK_STEP
    return;   // (timing only: the tracked fill without its per-cell tracking)
#endif
    const int thr = LOCAL ? st.thr : st.thr - w.gs;   // best - (i + j) g at this column
    if (!COL) {
        st.thr = MASKED ? (act ? max(thr, H) : st.thr) : max(thr, H);
        return;
    }
    const bool nb = act && H > thr;
    st.thr = nb ? H : (MASKED ? (act ? thr : st.thr) : thr);
    st.bstep = nb ? t : st.bstep;
}

template <bool LOCAL, bool PLANES, int MODE, bool TRACK>
__device__ __forceinline__ void side_group(SideState& st, SideCtx& w, const int t, const int4 (&hv)[2]) {
    const int g = t >> 2;
    const int4 vS = hv[0], vD = hv[1];
    const int aS[4] = {vS.x, vS.y, vS.z, vS.w}, aD[4] = {vD.x, vD.y, vD.z, vD.w};
    int aI[4] = {0, 0, 0, 0};
    int e[4];
#pragma unroll
    for (int U = 0; U < 4; ++U) {
        if (MODE == 1) {
            if (w.lane <= t + U) {
                aI[U] = side_insert<LOCAL, false>(st, w, aS[U], aD[U], true);
                if (TRACK) track_step<false, LOCAL, !PLANES>(st, w, max3i(aI[U], aS[U], aD[U]), t + U, true);
                side_step<LOCAL, false>(st, aI[U], aS[U], aD[U], t + U, true);
            }
        } else {
            const bool act = MODE == 2 ? (unsigned)(t + U - w.lane) < (unsigned)w.m : true;
            aI[U] = side_insert<LOCAL, MODE == 2>(st, w, aS[U], aD[U], act);
            if (TRACK) track_step<MODE == 2, LOCAL, !PLANES>(st, w, max3i(aI[U], aS[U], aD[U]), t + U, act);
            side_step<LOCAL, MODE == 2>(st, aI[U], aS[U], aD[U], t + U, act);
        }
        e[U] = st.E;   // lane 63: E + 64 of its column t+U-62
    }
    if (PLANES) {   // the group's cells, one dwordx4 per lane and plane
        const uint32_t vo = (uint32_t)w.lane * 16u + (uint32_t)g * (kGroupInts1 * 4);
        bstore4(w.rI, vo, make_int4(aI[0], aI[1], aI[2], aI[3]));
        bstore4(w.rS, vo, vS);
        bstore4(w.rD, vo, vD);
    }
    // lane 63's landing columns (+64) of its columns t-62 .. t-59: the skeleton
    const int c0 = t - (kWave - 2);
    if (MODE == 0) {
        skel_store4(w.skel_rsrc, w.skel_voff + 4u * (uint32_t)c0, e[0], e[1], e[2], e[3]);
    } else {
#pragma unroll
        for (int U = 0; U < 4; ++U) {
            const int c = c0 + U;
            skel_store(w.skel_rsrc, (c >= 1 && c <= w.m) ? w.skel_voff + 4u * (uint32_t)c : kSkelOff, e[U]);
        }
    }
}

template <bool LOCAL, bool PLANES, bool TRACE, bool TRACK>
__device__ void side_wave(const PairDev& P, const int s, const int lane, SideCtx& w, const bool has_consumer,
                          StripRes* sres, PairRes* pres) {
    const int n = P.n, m = P.m;
    const int i = s * kWave + lane + 1;
    const bool ok = i <= n;
    w.m = m; w.lane = lane; w.tr_wait = 0;
    w.ts = TRACE && P.trace ? P.trace[s].ts : nullptr;
    if (PLANES) {
        const size_t strip_planes = (size_t)s * P.t4 * kGroupInts1;
        const int pbytes = P.t4 * kGroupInts1 * 4;   // one strip's plane
        w.rI = rsrc_of(uniform_ptr(P.pI + strip_planes), pbytes);
        w.rD = rsrc_of(uniform_ptr(P.pD + strip_planes), pbytes);
        w.rS = rsrc_of(uniform_ptr(P.pS + strip_planes), pbytes);
    }
    w.codes = P.codes + (size_t)s * P.t16 * kWave;
    w.skel_rsrc = rsrc_of(uniform_ptr(P.skel + (size_t)s * P.skel_stride), has_consumer ? 4 * (m + 1) : 0);
    w.skel_voff = lane == kWave - 1 ? 0u : kSkelOff;
    SideState st;
    {   // column 0 (algo.rs:204-211), as the core starts it (core_wave)
        const int D0 = w.h + i * w.g;
        st.H = LOCAL ? max(D0, 0) : w.h;          // (global: shifted, D0 - i g = h)
        st.I = LOCAL ? kNeg : kNeg - i * w.g;
    }
    st.E = 64 - (lane + 1);                       // column 0: the path reaches it at local row lane + 1
    st.Ed = shr1(64, st.E);                       // column 1's top-left: (64 s, 0) for lane 0
    st.cI = 0; st.cD = 0;
    st.lbest = ok ? INT_MIN : INT_MAX; st.lstep = 0; st.lE = 0;
    // TRACK: no maximum yet (INT_MIN + 2^29: the thresholds drift by
    // (n + m) |g| < 2^28 and stay below every value)
    st.thr = INT_MIN + (1 << 29); st.bstep = 0;
    const int T = m + kWave;
    for (int t0 = 0; t0 < T; t0 += kSub) {
        if (TRACE && w.ts && (t0 & 1023) == 0 && (t0 >> 10) < kTraceTL && lane == 0)
            w.ts[t0 >> 10] = __builtin_amdgcn_s_memrealtime();
        // the core publishes whole sub-blocks: read all four groups at once
        w.tr_wait += wait_ge(w.hcnt, (t0 >> 2) + 4, w.status);
        int4 sub[4][2];
        {
            const int4* hv = &w.ho->v[(t0 >> 2) & (kSkHo - 1)][0][lane];
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int k = 0; k < 2; ++k) sub[q][k] = hv[(2 * q + k) * kWave];
        }
        asm volatile("" ::: "memory");
        lds_post(w.bcnt, (t0 >> 2) + 4);          // (reads issued first: LDS keeps the order)
        if (t0 + kSub <= kWave && t0 + kSub - 1 <= m - 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) side_group<LOCAL, PLANES, 1, TRACK>(st, w, t0 + 4 * q, sub[q]);
        } else if (t0 >= kWave && t0 + kSub - 1 <= m - 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) side_group<LOCAL, PLANES, 0, TRACK>(st, w, t0 + 4 * q, sub[q]);
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) side_group<LOCAL, PLANES, 2, TRACK>(st, w, t0 + 4 * q, sub[q]);
        }
        // codes[strip][t/16][lane]
        gstore1(w.codes + (size_t)(t0 >> 4) * kWave + lane, (st.cD << 16) | (st.cI & 0xFFFFu));
    }
    int fbest = INT_MIN, fi = 0, fj = 0, fl = 0;   // (fl: max_matches there, from the LCS rows: finalize_kernel)
    if (TRACK) {   // the strip's first max in row-major order: the lowest lane (earliest row) holding the largest
        const int best = ok ? st.thr + (LOCAL ? 0 : (i + m) * w.gs) : INT_MIN;   // (the threshold at column m, unshifted)
        int mx = best;
        for (int off = 32; off > 0; off >>= 1) mx = max(mx, __shfl_xor(mx, off));
        const unsigned long long fmask = __ballot(ok && best == mx);
        const int fl_ = fmask ? (int)__builtin_ctzll(fmask) : 0;
        fbest = mx; fi = s * kWave + fl_ + 1;
        fj = PLANES ? 0 : __shfl(st.bstep, fl_) - fl_ + 1;   // (0: the column is found later, skew_max_col_kernel)
    }
    if (TRACK && !LOCAL && lane == 0) {
        StripRes r{};
        r.best = fbest; r.bi = fi; r.bj = fj; r.bl = fl;
        r.lbest = INT_MIN;
        sres[P.strip_base + s] = r;
    }
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
            if (TRACK) { r.best = fbest; r.bi = fi; r.bj = fj; r.bl = fl; }
            r.lbest = lmx; r.li = s * kWave + ll + 1; r.lj = l_step - ll + 1; r.lE = l_E - 64;
            sres[P.strip_base + s] = r;
        }
    }
    if (ok && i == n) pres->end_E = st.E - 64;   // landing column of cell (n, m)
    if (TRACE && P.trace && lane == 0) {
        P.trace[s].wait_out = (int)w.tr_wait;
        P.trace[s].t_q[kTraceQ - 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// ---------------------------------------------------------------------------
// band hand-off (I/O wave)

// Band rows move between workgroups in tagged 8-byte granules
// (MI355X_MICROARCH.md "handoff-1to1": a data-tagged granule is the cheapest
// cross-CU hand-off, no progress counter and no store drain before a flag).
// The next band needs each bottom-row cell's delete successor dd and
// score_max sm (every lane reads its column symbols from PairDev.ccodes);
// dd - sm lies in [h + g, max(g, 0)] (Ddn = max(Dn, H + h) with Dn <= H; local:
// the floor and + g), so one granule holds sm (low word) and (dd - sm) in 31
// bits under a valid bit (bit 63).  The feed rows are zeroed before the launch
// (gx_api_fill.cpp run_fill), so a granule is valid exactly once it was written by
// this launch.  Stores and loads are 8-byte agent-scope (sc1: write-through,
// L1 bypass).
template <bool TBL>
__device__ void io_wave_tag(const PairDev& P, const int lb, const int lane, const Scores32& sc, SkRing* ring0,
                            const SkRing* ringW, lds_int* wcnt0, lds_int* rcnt0, lds_int* wcntW, lds_int* rcntW,
                            const bool do_out, int* status) {
    const int m = P.m;
    int in_next = 0, out_next = 0;
    const gu64* feed_in = lb > 0 ? (const gu64*)(P.feed + (size_t)(lb - 1) * P.feed_stride) : nullptr;
    gu64* feed_out = do_out ? (gu64*)(P.feed + (size_t)lb * P.feed_stride) : nullptr;
    unsigned idle = 0;
    while (in_next <= m || (do_out && out_next <= m)) {
        bool moved = false;
        if (in_next <= m) {
            const int lim = min(m + 1, *rcnt0 + kSkRingG * 4 - 4);   // ring slots the strip has read
            const int j = in_next + lane;
            int dd = 0, sm = 0;
            bool valid = false;
            if (j < lim) {
                if (lb == 0) {
                    // row 0 (algo.rs:195-202, 213-220): I = h + j g, D = S = neg_inf
                    valid = true;
                    if (j > 0) {
                        const int I0 = sc.h + j * sc.g;
                        dd = max(I0 + sc.hg, sc.floor_);
                        sm = max(I0, sc.floor_);
                        if (sc.shift) { dd -= (1 + j) * sc.g; sm -= j * sc.g; }
                    }
                } else {
                    const unsigned long long gr = __hip_atomic_load(feed_in + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    valid = (gr >> 63) != 0;
                    sm = (int)(unsigned)gr;
                    dd = sm + ((int)((unsigned)(gr >> 32) << 1) >> 1);
                }
            }
            const unsigned long long vm = __ballot(valid);
            const int cnt = ~vm ? (int)__builtin_ctzll(~vm) : kWave;   // the leading run of valid columns
            if (cnt > 0) {
                if (lane < cnt) {
                    const int G = sk_grp(j), u = sk_pos(j);
                    ring0->dd[G][u] = dd;
                    ring0->sm[G][u] = sm;
                }
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
                int dd = 0, sm = 0;
                if (lane < chunk) { dd = ringW->dd[sk_grp(j)][sk_pos(j)]; sm = ringW->sm[sk_grp(j)][sk_pos(j)]; }
                lds_wait();
                if (lane == 0) *rcntW = out_next + chunk;   // ring slots free again
                if (lane < chunk) {
                    const unsigned long long gr = (unsigned long long)(unsigned)sm |
                                                  ((unsigned long long)(0x80000000u | ((unsigned)(dd - sm) & 0x7FFFFFFFu)) << 32);
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
            __builtin_amdgcn_s_sleep(4);   // (a poll costs its SIMD's issue slots: keep it rare)
        }
    }
}

// ---------------------------------------------------------------------------

// One workgroup = one band of W strips: wave 0 the I/O wave, waves 1..W the
// strips' core waves, W+1..2W their side waves.  Waves go to the CU's SIMDs
// round-robin, so at W = 2 the two core waves have SIMDs of their own (the
// I/O wave, which polls, shares one with a side wave); at W = 3 two core
// waves share a SIMD with other waves.  Persistent workgroups take bands from the
// host's band-major queue (gx_api_fill.cpp run_fill), as fill_kernel does.
// TRACK: the first lcs_blocks workgroups (one per pair) compute the pairs'
// LCS rows instead (gx_lcs.h); they come first so that they are dispatched
// with the fill and run beside it, and nothing waits for them but the
// kernels after the launch.
template <int W, bool LOCAL, bool PLANES, bool TBL, bool TRACE, bool TRACK>
__global__ __launch_bounds__((2 * W + 1) * kWave, 1) void fill_skew_kernel(const PairDev* __restrict__ pairs,
                                                                           const int npairs, const int total_bands,
                                                                           int* band_counter, StripRes* sres,
                                                                           PairRes* pres, const Scores32 sc,
                                                                           const int lcs_blocks) {
    __shared__ SkRing rings[W + 1];
    __shared__ SkHo ho[W];
    __shared__ int wcnt[W + 1], rcnt[W + 1], hcnt[W], bcnt[W];
    __shared__ int band_sh;
    __shared__ int4 push_sink[2 * kWave];          // the core waves' lanes 0..62 push here (core_group)
    __shared__ int push_sink_cnt;
    __shared__ int4 zero_blk[kSkRingG + 1];        // ... and their lanes 1..63 read [0] and [64] (read_grp)
    if (threadIdx.x <= kSkRingG) zero_blk[threadIdx.x] = make_int4(0, 0, 0, 0);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int lane = threadIdx.x & (kWave - 1);
    if (TRACK && (int)blockIdx.x < lcs_blocks) {   // an LCS workgroup (gx_lcs.h)
        const int blk = (int)blockIdx.x;
        int p = 0;
        while (p + 1 < npairs && pairs[p + 1].lcs_base <= blk) ++p;
        p = __builtin_amdgcn_readfirstlane(p);
        const PairDev& P = pairs[p];
        lcs_workgroup(P, blk - P.lcs_base, (P.lcs_waves >> 8) & 0xFF, wave, 2 * W + 1, lane, (char*)ho, sizeof(ho), band_counter + 1);
        return;
    }
    for (;;) {
        if (threadIdx.x == 0) band_sh = atomicAdd(band_counter, 1);
        if (threadIdx.x < W + 1) { wcnt[threadIdx.x] = 0; rcnt[threadIdx.x] = 0; }
        if (threadIdx.x < W) { hcnt[threadIdx.x] = 0; bcnt[threadIdx.x] = 0; }
        __syncthreads();
        const int b = __builtin_amdgcn_readfirstlane(band_sh);
        if (b >= total_bands) return;
        const int2 ob = reinterpret_cast<const int2*>(pairs + npairs)[b];
        const int p = __builtin_amdgcn_readfirstlane(ob.x);
        const PairDev& P = pairs[p];
        const int lb = __builtin_amdgcn_readfirstlane(ob.y);
        const int k = wave <= W ? wave - 1 : wave - 1 - W;   // the strip (in the band) of a compute wave
        const int s = lb * W + k;
        const bool has_consumer = k == W - 1 ? (lb + 1 < P.bands) : (s + 1 < P.strips);
        if (wave == 0) {
            io_wave_tag<TBL>(P, lb, lane, sc, &rings[0], &rings[W], (lds_int*)&wcnt[0], (lds_int*)&rcnt[0],
                             (lds_int*)&wcnt[W], (lds_int*)&rcnt[W], lb + 1 < P.bands, band_counter + 1);
        } else if (wave <= W) {
            if (s < P.strips) {
                CoreCtx w;
                w.rin = &rings[k]; w.rout = &rings[k + 1];
                w.wcnt_in = (lds_int*)&wcnt[k]; w.rcnt_in = (lds_int*)&rcnt[k];
                w.wcnt_out = (lds_int*)&wcnt[k + 1]; w.rcnt_out = (lds_int*)&rcnt[k + 1];
                w.ho = &ho[k]; w.hcnt = (lds_int*)&hcnt[k]; w.bcnt = (lds_int*)&bcnt[k];
                w.status = band_counter + 1;
                w.push_on = has_consumer;
                const bool pl = has_consumer && lane == kWave - 1;
                w.push_base = lds_addr(pl ? (const void*)rings[k + 1].dd[0] : (const void*)&push_sink[lane]);
                w.push_m16 = pl ? 16 : 0;
                w.pcnt = has_consumer ? w.wcnt_out : (lds_int*)&push_sink_cnt;
                w.rd_base = lds_addr(lane == 0 ? (const void*)rings[k].dd[0] : (const void*)zero_blk);
                w.rd_m16 = lane == 0 ? 16 : 0;
                core_wave<LOCAL, TBL, TRACE>(P, s, lane, sc, w, pres + p);
            }
        } else {
            if (s < P.strips) {
                SideCtx w;
                w.ho = &ho[k]; w.hcnt = (lds_int*)&hcnt[k]; w.bcnt = (lds_int*)&bcnt[k];
                w.status = band_counter + 1;
                w.h = sc.h; w.g = sc.g; w.hg = sc.hg;
                w.gs = LOCAL ? 0 : sc.g;   // TRACK: global fills hold V - (i + j) g
                side_wave<LOCAL, PLANES, TRACE, TRACK>(P, s, lane, w, has_consumer, sres, pres + p);
            }
        }
        __syncthreads();
    }
}

// Tracked layout-3 fills that keep their planes track each row's largest
// score_max only (track_step): finalize_kernel picks the first row holding
// the maximum (max_i, max_val) and leaves max_j = INT_MAX; this finds the
// first column of that row with score_max == max_val (algo.rs:258-262: the
// first maximum in row-major order) from the row's I, D, S planes (shifted
// for global fills: score_max = max(I, D, S) + (i + j) g), one thread per
// column, atomicMin.  Then skew_mam_kernel: matches_at_max = max_matches
// there from the LCS rows (algo.rs:279; gx_lcs.h).
__global__ void skew_max_col_kernel(const PairDev* __restrict__ pairs, PairRes* pres, const int gshift) {
    const PairDev& P = pairs[blockIdx.y];
    PairRes* const r = pres + blockIdx.y;
    const int i = r->max_i, j = (int)(blockIdx.x * blockDim.x + threadIdx.x) + 1;
    if (i < 1 || i > P.n || j > P.m || !P.pI) return;
    const int s = (i - 1) / kWave, lane = (i - 1) % kWave, t = j - 1 + lane;
    const size_t o = (size_t)s * P.t4 * kGroupInts1 + (size_t)(t >> 2) * kGroupInts1 + (size_t)lane * 4 + (t & 3);
    const int H = max3i(P.pI[o], P.pD[o], P.pS[o]) + (i + j) * gshift;
    if (H == r->max_val) atomicMin(&r->max_j, j);
}
__global__ void skew_mam_kernel(const PairDev* __restrict__ pairs, PairRes* pres) {
    const PairDev& P = pairs[blockIdx.x];
    PairRes* const r = pres + blockIdx.x;
    const int lane = threadIdx.x;
    const int i = r->max_i, j = r->max_j;
    if (i < 1 || i > P.n || j < 1 || j > P.m) return;
    const int mam = lcs_matches(P, i, j, lane);   // LM(i, j) (gx_lcs.h)
    if (lane == 0) r->mam = mam;
}
hipError_t launch_skew_max_col(const PairDev* d_pairs, int npairs, int mmax, PairRes* d_pres, int gshift, hipStream_t st) {
    if (npairs <= 0 || mmax <= 0) return hipSuccess;
    hipLaunchKernelGGL(skew_max_col_kernel, dim3((unsigned)((mmax + 255) / 256), (unsigned)npairs), dim3(256), 0, st,
                       d_pairs, d_pres, gshift);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(skew_mam_kernel, dim3((unsigned)npairs), dim3(kWave), 0, st, d_pairs, d_pres);
    return hipGetLastError();
}

// The column inputs of every pair as int32 rows of m + 192, 64 zeros before
// and 128 after (the steps where a lane is outside columns 1..m read them):
// index j - 1 + 64 holds s2[j-1], or with score tables (<= 4 symbols) four
// such rows, row k the score of symbol k (Scores32.sym) against s2[j-1]
// (sequence.rs:113-114; the launch's s - 2g for shifted fills).
__global__ void skew_codes_kernel(const PairDev* __restrict__ pairs, const Scores32 sc, const int tbl) {
    const PairDev& P = pairs[blockIdx.y];
    const int k = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int row = P.m + 192;
    if (k >= row) return;
    const int j = k - 64;
    const bool in = j >= 0 && j < P.m;
    if (!tbl) {
        ((int*)P.ccodes)[k] = in ? (int)P.c2[j] : 0;
        return;
    }
    const int c = in ? sym_code(P.c2[j], sc) : -1;
#pragma unroll
    for (int r = 0; r < 4; ++r) ((int*)P.ccodes)[(size_t)r * row + k] = in ? (c == r ? sc.sm : sc.smm) : 0;
}
hipError_t launch_skew_codes(const PairDev* d_pairs, int npairs, int mmax, Scores32 sc, bool tbl, hipStream_t st) {
    if (npairs <= 0) return hipSuccess;
    hipLaunchKernelGGL(skew_codes_kernel, dim3((unsigned)((mmax + 192 + 255) / 256), (unsigned)npairs), dim3(256), 0, st,
                       d_pairs, sc, (int)tbl);
    return hipGetLastError();
}

template <int W, bool LOCAL, bool PLANES, bool TBL, bool TRACE, bool TRACK>
static hipError_t launch_skew_t(const PairDev* d_pairs, int npairs, int total_bands, int* d_counter, StripRes* d_sres,
                                PairRes* d_pres, Scores32 sc, int grid, int lcs_blocks, hipStream_t st) {
    hipLaunchKernelGGL((fill_skew_kernel<W, LOCAL, PLANES, TBL, TRACE, TRACK>), dim3(grid + (TRACK ? lcs_blocks : 0)),
                       dim3((2 * W + 1) * kWave), 0, st, d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc,
                       TRACK ? lcs_blocks : 0);
    return hipGetLastError();
}

template <bool LO, bool PL, bool TB, bool TR, bool TK, int W0, int... Ws>
static hipError_t launch_skew_w(int W, const PairDev* d_pairs, int npairs, int total_bands, int* d_counter,
                                StripRes* d_sres, PairRes* d_pres, Scores32 sc, int grid, int lcs_blocks,
                                hipStream_t st) {
    if (W == W0)
        return launch_skew_t<W0, LO, PL, TB, TR, TK>(d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc, grid,
                                                     lcs_blocks, st);
    if constexpr (sizeof...(Ws) > 0)
        return launch_skew_w<LO, PL, TB, TR, TK, Ws...>(W, d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, sc,
                                                        grid, lcs_blocks, st);
    return hipErrorInvalidValue;
}

// LCS workgroups of a tracked launch (gx_lcs.h): four sweeping waves a
// workgroup, one a SIMD (at five, two share a SIMD and every strip's pace
// drops: Covid's sweep alone 4.56 ms with 5 x 2 workgroups, 3.92 with 4 x 3,
// 3.77 with 2 x 5 -- but then more strips cross workgroups through HBM --
// tools/lcs_trace.py, gpurun_out/r06t_waves.log), within what the LDS of the
// fill's core -> side rings holds rings for; and enough workgroups that
// about T / 64 + 1 strips are swept at once -- a strip starts ~80 steps after
// the one above, so that many keep up with the dependence chain -- and no
// more than the strips.
int skew_lcs_sweep(int W) { return std::min(std::min(4, 2 * W + 1), lcs_max_sweep((size_t)W * sizeof(SkHo))); }
int skew_lcs_blocks(int W, int n, int m) {
    const int T = lcs_steps(ceil_div(m, kLcsBits)), S = ceil_div(n, kWave);
    const int waves = std::min(S, ceil_div(T, 64) + 1);
    return std::max(1, std::min(8, ceil_div(waves, std::max(1, skew_lcs_sweep(W)))));
}

// Band widths of layout 3 (must match gx_api_plan.cpp skew_band_waves).  trace:
// the diagnostics instantiation (PairDev.trace set; untracked fills with
// planes only, the others run untraced).
// track: the first maximum (alignment_table's max_cell, algo.rs:258-262)
// in the side waves, and max_matches as LCS rows in lcs_blocks leading
// workgroups (gx_lcs.h; matches_at_max, algo.rs:279, by finalize_kernel).
bool skew_traced(bool planes, bool trace, bool track) { return trace && planes && !track; }
hipError_t launch_fill_skew(int W, bool local, bool planes, bool tbl, bool trace, bool track, const PairDev* d_pairs,
                            int npairs, int total_bands, int* d_counter, StripRes* d_sres, PairRes* d_pres, Scores32 sc,
                            int grid, int lcs_blocks, hipStream_t st) {
#define GX_SKEW_CASE(LO, PL, TB, TR, TK)                                                                           \
    if (local == LO && planes == PL && tbl == TB && skew_traced(planes, trace, track) == TR && track == TK)         \
        return launch_skew_w<LO, PL, TB, TR, TK, 1, 2, 3>(W, d_pairs, npairs, total_bands, d_counter, d_sres, d_pres, \
                                                             sc, grid, lcs_blocks, st);
    GX_SKEW_CASE(false, false, false, false, false)
    GX_SKEW_CASE(false, false, true, false, false)
    GX_SKEW_CASE(false, true, false, false, false)
    GX_SKEW_CASE(false, true, true, false, false)
    GX_SKEW_CASE(true, false, false, false, false)
    GX_SKEW_CASE(true, false, true, false, false)
    GX_SKEW_CASE(true, true, false, false, false)
    GX_SKEW_CASE(true, true, true, false, false)
    GX_SKEW_CASE(false, true, false, true, false)
    GX_SKEW_CASE(false, true, true, true, false)
    GX_SKEW_CASE(true, true, false, true, false)
    GX_SKEW_CASE(true, true, true, true, false)
    GX_SKEW_CASE(false, false, false, false, true)
    GX_SKEW_CASE(false, true, false, false, true)
    GX_SKEW_CASE(true, false, false, false, true)
    GX_SKEW_CASE(true, true, false, false, true)
    GX_SKEW_CASE(false, false, true, false, true)
    GX_SKEW_CASE(false, true, true, false, true)
    GX_SKEW_CASE(true, false, true, false, true)
    GX_SKEW_CASE(true, true, true, false, true)
#undef GX_SKEW_CASE
    return hipErrorInvalidValue;
}

}  // namespace gx
