// gx_fill_pk.hip -- the twin fill: two independent pairs (laid out for the
// larger n and m of the two) swept by one band of waves, one pair in each 16-bit half of every
// register (VOP3P packed arithmetic: one v_pk_max_i16 / v_pk_add_u16 /
// v_pk_mad_u16 computes the same cell of both pairs).  Specialised to the
// batch path's untracked global fill on the anti-diagonal layout (layout 0,
// gx_internal.h) with compact score planes (or none): the same strips, bands,
// rings, band hand-offs, codes and compact planes as gx_kernels.hip's
// fill_kernel, the same recurrence on the shifted values V - (i + j) g
// (DESIGN.md 4.3), so the traceback and the exports are unchanged.
//
// 16-bit values.  A strip's values span a few thousand around a moving
// reference, far less than 2^15, but not their absolute magnitude (V'' reaches
// ~4e4 at the end of a 30k pair).  Every value is therefore kept relative to a
// per-pair base B (int32, a wave-uniform SGPR pair), exact modulo 2^16:
//   * the I/O wave of a band picks the base of each 16-column block of the
//     band's top row (the first column's score_max) and of column 0;
//   * a strip adopts, at each 16-step sub-block, the base of the block it
//     consumes (its producer wrote it beside the records), shifting its state
//     by the difference (ten v_pk_sub per sub-block), so ring records never
//     need converting; the blocks it pushes carry that same base;
//   * the I/O wave converts the band's bottom row back to int32 for HBM.
// The host admits a launch only when the worst-case spread of a band's values
// around the inherited bases stays below 2^15 (gx_api_plan.cpp twin_width).
// Comparisons and max are exact on values within 2^15 of each other, so the
// codes, landing columns, planes and results equal the int32 fill's.
#include "gx_device.h"

namespace gx {

typedef short s2 __attribute__((ext_vector_type(2)));
typedef unsigned short u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s2 as_s2(uint32_t x) { return __builtin_bit_cast(s2, x); }
__device__ __forceinline__ uint32_t as_u(s2 x) { return __builtin_bit_cast(uint32_t, x); }
// VOP3P arithmetic on the two halves.  The sign masks pass through an empty
// asm so that the compiler keeps them as bit masks (v_bfi_b32, v_and_or_b32):
// seen as sign splats, the bit-selects are lowered to per-half compares and
// selects.  (Non-empty inline asm here costs an s_nop after each statement.)
__device__ __forceinline__ uint32_t pmax(uint32_t a, uint32_t b) {
    return as_u(__builtin_elementwise_max(as_s2(a), as_s2(b)));
}
// Values are held in offset binary (each half + 0x8000, "biased"): the
// admission bound keeps every value within 30,000 of its base, so a biased
// half lies in [2768, 62768] and adding a small non-negative constant (a
// score-table byte) or subtracting one (|h|) never carries or borrows across
// the halves -- those adds run as one 32-bit v_add_u32 / v_sub_u32, a
// dual-rate VOP2 form (~2.4 cycles per wave64 at two waves per SIMD against
// ~4.6 for a VOP3P v_pk_add, profiles/valu_probe_r02k.json).  Comparisons
// of biased halves are unsigned (v_pk_max_u16); differences are unbiased.
constexpr uint32_t kBias2 = 0x80008000u;
typedef unsigned short us2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pmaxu(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(us2, a), __builtin_bit_cast(us2, b)));
}
// The same as an opaque v_pk_max_u16, for running maxima: LLVM reassociates
// a chain of umax across the unrolled sub-block and holds every step's
// operand until a tree at its end (the local row maximum, 4 groups x 2 rows:
// 149 VGPRs against 123 this way -- and 3.5 % faster, so the local fill keeps
// the reassociable form; GX_PK_LB_OPAQUE builds this one)
__device__ __forceinline__ uint32_t pmaxu_acc(uint32_t a, uint32_t b) {
    uint32_t d;
    asm("v_pk_max_u16 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
__device__ __forceinline__ uint32_t padd(uint32_t a, uint32_t b) { return as_u(as_s2(a) + as_s2(b)); }
__device__ __forceinline__ uint32_t padds(uint32_t a, uint32_t b) { return padd(a, b); }
__device__ __forceinline__ uint32_t psub(uint32_t a, uint32_t b) { return as_u(as_s2(a) - as_s2(b)); }
__device__ __forceinline__ uint32_t psubs(uint32_t a, uint32_t b) { return psub(a, b); }
// 0xFFFF in each half whose value is negative, else 0
__device__ __forceinline__ uint32_t psign(uint32_t a) {
    uint32_t m = as_u(as_s2(a) >> (s2){15, 15});
    asm("" : "+v"(m));
    return m;
}
// (m & a) | (~m & b)
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t d;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(d) : "v"(m), "v"(a), "v"(b));
    return d;
}
// Code bit-planes, kept negated: with N = -C (mod 2^16 per half) and the
// sign mask m = -bit, C' = 2C + bit becomes N' = 2N + m -- one v_pk_mad_u16
// (a shift and a masked or on C).  The code words are negated back once per
// 16 steps, when they are stored.
__device__ __forceinline__ uint32_t pcode(uint32_t n, uint32_t m) {
    uint32_t d;
    asm("v_pk_mad_u16 %0, %1, 2, %2 op_sel_hi:[1,0,1]" : "=v"(d) : "v"(n), "v"(m));
    return d;
}
// 0 where the two bytes match, 1 elsewhere (per half)
__device__ __forceinline__ uint32_t pmis(uint32_t c1, uint32_t c2) {
    uint32_t d;
    asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(d) : "v"(c1 ^ c2));
    return d;
}
// a * b + c per half (mod 2^16)
__device__ __forceinline__ uint32_t pmad(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b), "v"(c));
    return d;
}
__device__ __forceinline__ uint32_t pk2(int lo, int hi) { return ((uint32_t)lo & 0xFFFFu) | ((uint32_t)hi << 16); }
__device__ __forceinline__ int lo16(uint32_t x) { return (int)(short)(x & 0xFFFFu); }
__device__ __forceinline__ int hi16(uint32_t x) { return (int)(short)(x >> 16); }

// (a - b) of half H into byte K of acc (SDWA; byte 0 clears the rest)
template <int K, int H>
__device__ __forceinline__ void put_byte_h(uint32_t& acc, uint32_t a, uint32_t b) {
#define GX_PBH(DST, UNUSED, SEL)                                                                         \
    asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:" DST " dst_unused:" UNUSED " src0_sel:" SEL " src1_sel:" SEL \
        : "+v"(acc) : "v"(a), "v"(b))
#define GX_PBH0(SEL)                                                                                          \
    asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:" SEL " src1_sel:" SEL        \
        : "=v"(acc) : "v"(a), "v"(b))
    if constexpr (K == 0 && H == 0) GX_PBH0("WORD_0");
    if constexpr (K == 1 && H == 0) GX_PBH("BYTE_1", "UNUSED_PRESERVE", "WORD_0");
    if constexpr (K == 2 && H == 0) GX_PBH("BYTE_2", "UNUSED_PRESERVE", "WORD_0");
    if constexpr (K == 3 && H == 0) GX_PBH("BYTE_3", "UNUSED_PRESERVE", "WORD_0");
    if constexpr (K == 0 && H == 1) GX_PBH0("WORD_1");
    if constexpr (K == 1 && H == 1) GX_PBH("BYTE_1", "UNUSED_PRESERVE", "WORD_1");
    if constexpr (K == 2 && H == 1) GX_PBH("BYTE_2", "UNUSED_PRESERVE", "WORD_1");
    if constexpr (K == 3 && H == 1) GX_PBH("BYTE_3", "UNUSED_PRESERVE", "WORD_1");
#undef GX_PBH
#undef GX_PBH0
}

// The compact plane bytes of step U (both pairs, both rows), as soon as the
// step's cells exist (keeping a group's cells for the end costs 32 VGPRs).
template <int U>
__device__ __forceinline__ void bytes_step(uint32_t (&xI)[2][2], uint32_t (&xS)[2][2], uint32_t (&xD)[2][2],
                                           const uint32_t (&oI)[2], const uint32_t (&oD)[2], const uint32_t (&oS)[2],
                                           const uint32_t (&oL)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        put_byte_h<U, 0>(xI[0][h], oI[h], oL[h]); put_byte_h<U, 0>(xS[0][h], oS[h], oI[h]);
        put_byte_h<U, 0>(xD[0][h], oD[h], oI[h]);
        put_byte_h<U, 1>(xI[1][h], oI[h], oL[h]); put_byte_h<U, 1>(xS[1][h], oS[h], oI[h]);
        put_byte_h<U, 1>(xD[1][h], oD[h], oI[h]);
    }
}

// Packed scores (both halves equal): h, sm'' = s_match - 2g, dsm = (s_mismatch - 2g) - sm''
struct PkScores {
    uint32_t nh, smp, dsm;   // -h (>= 0) in both halves, the score_max offset, the mismatch - match delta
    uint32_t ng, na, Z;      // local (unshifted values): -g, -(h + g) (>= 0), and the biased zero of the floor
};

// Twin plane code (PLANES == 2, 2 B per cell): a cell's two differences in
// one 16-bit word, code = x_S + 32 x_D (mod 2^16), x_S = S - I in [-16, 15],
// x_D = D - I in [-64, 63] (gx_api_plan.cpp w16_ok checks the ranges); both
// pairs' codes of a cell in one dword, as the halves already hold them.  I
// itself is not stored: it follows from the row's previous cell, I(i, j) =
// I(i, j-1) + g + max(0, max(x_S, x_D)(i, j-1) + h) (local: then max(., 0)),
// the insert recurrence of algo.rs:231-236 (cell_pk), which every decoder
// replays along the row (round 5; the x_I field of the earlier format cost a
// third v_pk_mad_u16 per two cells).
// Small-alphabet twins (TBL, the launch's <= 4 symbols in Scores32.sym): a
// row's score table (byte k: the shifted match score if c1 is symbol k, else
// the shifted mismatch score, both in [0, 255]) and a column's selector for
// v_perm_b32.
__device__ __forceinline__ uint32_t score_table_pk(int c1, const Scores32& sc) {
    uint32_t t = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) t |= ((uint32_t)(c1 == sc.sym[k] ? sc.sm : sc.smm) & 0xFFu) << (8 * k);
    return t;
}
__device__ __forceinline__ uint32_t perm_selector(int code0, int code1) {
    return (uint32_t)code0 | 0x0C00u | ((uint32_t)(4 + code1) << 16) | 0x0C000000u;
}

// code = S + 32 D - 33 I (mod 2^16): two v_pk_mad_u16 on the cell's values
// directly; the offset-binary bias cancels (1 + 32 - 33 = 0).  Decoders:
// gx_kernels.hip w16_word_of, plane_sums_kernel, export_w16_kernel,
// local_col_kernel.  (Iold: unused since the format dropped x_I.)
__device__ __forceinline__ uint32_t w16_code(uint32_t I, uint32_t D, uint32_t S, uint32_t Iold) {
    (void)Iold;
    return pmad(I, 0xFFDFFFDFu, pmad(D, 0x00200020u, S));
}

// One row of a lane, both pairs: the cell left of the one being computed.
struct RowPk {
    uint32_t I, Hx, Dd, SMp, SMtl;   // insert, score_max + h (local + g), delete successor, score_max + sm'', SMp(i-1, j-1)
    uint32_t cI, cD;                 // code bit-planes, negated (16 steps, one per half; pcode)
    uint32_t E, Etl;                 // landing columns (int16 per half)
    uint32_t lb;                     // local: the largest score_max along the row (biased)
};
struct LanePk {
    RowPk a, b;
    uint32_t c2c;                    // s2[j-1] of both pairs (bytes in the halves)
};

// algo.rs:222-268 on the shifted values, both pairs at once; MASKED keeps
// the lanes outside columns 1..m unchanged, per pair (a twin's two pairs may
// differ in length: the shorter one's state stays at its last column).
//
// LOCAL (Smith-Waterman, algo.rs:231-248 with is_local): plain (unshifted)
// values, relative to per-block bases like the global twin's (neighbouring
// local values differ by at most max(|h + g|, U) as global ones do, the 0
// floor keeps every inequality: gx_api_plan.cpp twin_bound), so the 0 floor of
// score_max is one v_pk_max_u16 against k.Z, the biased relative zero of the
// current bases (-B per half, clamped to -2^15: a base above 2^15 lies more
// than the admission bound above every value of the band, whose floor then
// never binds), in each gap recurrence, and the row keeps its largest
// score_max since the last base change (one v_pk_max_u16; folded into an
// absolute int32 maximum when the bases move, fold_lb; the last column
// holding it, algo.rs:310-322, is recovered from the chosen row's plane codes
// by local_col_kernel, so the fill tracks no columns).  Plane codes store
// x_I - g as the shifted fill does (Iold - |g| is the insert recurrence's own
// term).
template <bool MASKED, bool TBL, bool CODES, bool NOE = false, bool LOCAL = false>
__device__ __forceinline__ void cell_pk(RowPk& st, const uint32_t dd_in, const uint32_t sm_in, const uint32_t e_up,
                                        const uint32_t c2, const uint32_t c1, const uint32_t c1h, const uint32_t act,
                                        const PkScores& k,
                                        uint32_t& oI, uint32_t& oD, uint32_t& oS, uint32_t& oIold) {
    const uint32_t Ig = LOCAL ? st.I - k.ng : st.I;                // (biased halves: no borrow across them)
    // the gap terms fold onto score_max H = max(I, S, D) (h <= 0: I + h never
    // wins against I, nor D + h against D): I' = max(I, H + h) and D(i+1) =
    // max(D, H + h) share Hx = H + h, one subtraction and one max fewer per
    // cell pair than max(S, D) + h and max(I, S) + h (round 5; local: + g and
    // the 0 floor, algo.rs:231-243)
    const uint32_t In = LOCAL ? pmaxu(pmaxu(Ig, st.Hx), k.Z)         // max(I + g, H + h + g, 0)
                              : pmaxu(st.I, st.Hx);                 // max(I, H + h)   (algo.rs:231-236)
    // SM(i-1,j-1) + s''  (algo.rs:245-248).  TBL: c1/c1h are the row's score
    // tables of the two pairs (byte k: s_match'' if the row's char is symbol
    // k, else s_mismatch''; SM is then kept without the s_match'' offset) and
    // c2 the column's selector (pair 0's symbol in byte 0, 4 + pair 1's in
    // byte 2, zero bytes between): one v_perm_b32 reads both scores (xor +
    // min + mad, and the offset's add, without the table)
    const uint32_t Sn = TBL ? st.SMtl + __builtin_amdgcn_perm(c1h, c1, c2) : pmad(pmis(c1, c2), k.dsm, st.SMtl);
    const uint32_t Dn = dd_in;                                     // (algo.rs:238-243, from the row above)
    const uint32_t IS = pmaxu(In, Sn);
    const uint32_t SMn = pmaxu(IS, Dn);
    const uint32_t Hxn = LOCAL ? SMn - k.na : SMn - k.nh;          // (biased halves: no borrow across them)
    const uint32_t Ddn = LOCAL ? pmaxu(pmaxu(Hxn, Dn - k.ng), k.Z)   // D(i+1, j), local
                               : pmaxu(Hxn, Dn);                   // D(i+1, j)
    // retrace priority S > I > D (algo.rs:351-400): m1 = I beats S, m2 = D beats both
    // (NOE: no landing columns -- the twin fill without a skeleton, whose
    // traceback walks the strips in sequence, tb_seq_kernel; with no code
    // words either, neither mask is needed)
    const uint32_t m1 = (CODES || !NOE) ? psign(psub(Sn, In)) : 0u, m2 = (CODES || !NOE) ? psign(psub(IS, Dn)) : 0u;
    const uint32_t E1 = NOE ? 0u : bfi(m1, st.E, st.Etl);
    const uint32_t En = NOE ? 0u : bfi(m2, e_up, E1);
    const uint32_t cIn = CODES ? pcode(st.cI, m1) : 0u;   // (no code words: the traceback derives
    const uint32_t cDn = CODES ? pcode(st.cD, m2) : 0u;   // them from the plane codes, tb_w16_codes_kernel)
    const uint32_t SMpn = (TBL && !LOCAL) ? SMn : padds(SMn, k.smp);   // TBL: no offset (the tables hold s''; local: - K)
    oI = In; oD = Dn; oS = Sn; oIold = Ig;
    if (LOCAL) {    // the row's largest score_max (its last column: local_col_kernel, from the plane codes)
#ifndef GX_PK_LB_OPAQUE
        st.lb = pmaxu(st.lb, MASKED ? bfi(act, SMn, k.Z) : SMn);
#else   // (123 VGPRs instead of 149, but 3.5 % slower at 8-wave bands: DESIGN.md 10, item 3)
        st.lb = pmaxu_acc(st.lb, MASKED ? bfi(act, SMn, k.Z) : SMn);
#endif
    }
    if (MASKED) {   // act: 0xFFFF in each half whose pair has this column
        st.I = bfi(act, In, st.I); st.Hx = bfi(act, Hxn, st.Hx); st.Dd = bfi(act, Ddn, st.Dd);
        st.SMp = bfi(act, SMpn, st.SMp);
        if (!NOE) st.E = bfi(act, En, st.E);
    } else {
        st.I = In; st.Hx = Hxn; st.Dd = Ddn; st.SMp = SMpn;
        if (!NOE) st.E = En;
    }
    if (CODES) { st.cI = cIn; st.cD = cDn; }
    st.SMtl = sm_in;
    if (!NOE) st.Etl = e_up;
}

template <bool MASKED, bool TBL, bool CODES, bool NOE = false, bool LOCAL = false>
__device__ __forceinline__ void dp_step_pk(LanePk& st, const Rec& r, const int t, const int lane, const int m0,
                                           const int m1, const uint32_t c1a, const uint32_t c1b, const uint32_t c1ah,
                                           const uint32_t c1bh, const PkScores& k,
                                           uint32_t (&oI)[2], uint32_t (&oD)[2], uint32_t (&oS)[2],
                                           uint32_t (&oL)[2]) {
    const uint32_t dd_in = (uint32_t)shr1(r.dd, (int)st.b.Dd);
    const uint32_t sm_in = (uint32_t)shr1(r.sm, (int)st.b.SMp);
    const uint32_t c2 = (uint32_t)shr1(r.c2, (int)st.c2c);
    const uint32_t e_in = NOE ? 0u : (uint32_t)shr1((int)pk2(t + 1, t + 1), (int)st.b.E);   // lane 0: its own column
    const uint32_t act = MASKED ? ((unsigned)(t - lane) < (unsigned)m0 ? 0xFFFFu : 0u) |
                                      ((unsigned)(t - lane) < (unsigned)m1 ? 0xFFFF0000u : 0u)
                                : ~0u;
    cell_pk<MASKED, TBL, CODES, NOE, LOCAL>(st.a, dd_in, sm_in, e_in, c2, c1a, c1ah, act, k, oI[0], oD[0], oS[0], oL[0]);
    cell_pk<MASKED, TBL, CODES, NOE, LOCAL>(st.b, st.a.Dd, st.a.SMp, st.a.E, c2, c1b, c1bh, act, k, oI[1], oD[1], oS[1], oL[1]);
    st.c2c = c2;
}

template <int U>
__device__ __forceinline__ void push63_pk(uint32_t base, const LanePk& st, unsigned long long m63) {
    asm volatile(
        "s_mov_b64 exec, %0\n\t"
        "ds_write2_b32 %1, %2, %3 offset0:%5 offset1:%6\n\t"
        "ds_write_b32 %1, %4 offset:%7\n\t"
        "s_mov_b64 exec, -1"
        :
        : "s"(m63), "v"(base), "v"(st.b.Dd), "v"(st.b.SMp), "v"(st.c2c), "i"(4 * U), "i"(4 * U + 1), "i"(16 * U + 8)
        : "memory");
}
template <int U>
__device__ __forceinline__ void push_all_pk(uint32_t vaddr, const LanePk& st) {
    asm volatile(
        "ds_write2_b32 %0, %1, %2 offset0:%4 offset1:%5\n\t"
        "ds_write_b32 %0, %3 offset:%6"
        :
        : "v"(vaddr), "v"(st.b.Dd), "v"(st.b.SMp), "v"(st.c2c), "i"(4 * U), "i"(4 * U + 1), "i"(16 * U + 8)
        : "memory");
}

// The fields load one by one (ds_read_b32, kept apart by empty asm): each
// lands in a register of its own that the step's DPP move then writes in
// place (lane 0 keeps the record), where a merged ds_read_b96 tuple cost a
// v_mov per field to free the tuple for the next group's loads.
__device__ __forceinline__ void read4_pk(Rec (&r)[4], const Rec* rin) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        r[u].dd = rin[u].dd;
        asm volatile("" ::: "memory");
        r[u].sm = rin[u].sm;
        asm volatile("" ::: "memory");
        r[u].c2 = rin[u].c2;
        asm volatile("" ::: "memory");
    }
}

// Bases of a ring: slot 0 = column 0; slot 1 + (b mod kBaseSlots) = block b
// (columns 16b+1 .. 16b+16); two ints (the two pairs) each.
constexpr int kBaseSlots = 32;
// (as lds_int pairs: slot k = ints 2k, 2k + 1)

struct WavePk {
    uint8_t* pI[2]; uint8_t* pD[2]; uint8_t* pS[2];   // this strip's compact planes, per pair
    uint32_t* codes[2];
    const Rec* ring_in;
    lds_int* wcnt_in;
    lds_int* wcnt_out;
    lds_int* base_in;
    lds_int* base_out;
    int* status;
    __amdgpu_buffer_rsrc_t skel_rsrc;
    uint32_t skel_voff;
    uint32_t scratch;
    uint32_t cnt_addr;
    int m, lane;                                      // m: the twin's columns (the longer pair's)
    int m0, m1;                                       // each pair's own columns
    uint32_t c1a, c1b;                                // rows A, B: both pairs' chars (TBL: pair 0's penalty tables)
    uint32_t c1ah, c1bh;                              // TBL: pair 1's penalty tables
    int B0, B1;                                       // current bases (wave-uniform)
};

template <int PLANES, bool MASKED, int G4>
__device__ __forceinline__ void group4_pk(LanePk& st, Rec (&nxt)[4], WavePk& w, const PkScores& k, const int t0,
                                          const uint32_t out_base, const bool push_on, const size_t sb_off) {
    const int t = t0 + 4 * G4;
    Rec cur[4] = {nxt[0], nxt[1], nxt[2], nxt[3]};
    const int need = min(t + 8, w.m) + 1;
    const int seen_v = *w.wcnt_in;
    asm volatile("" ::: "memory");
    read4_pk(nxt, w.ring_in + ring_slot(t + 5));
    uint32_t bI[4][2], bD[4][2], bS[4][2], bL[4][2];
    uint32_t xI[2][2], xS[2][2], xD[2][2];   // compact plane dwords [pair][row], filled step by step (PLANES 1)
    uint32_t wc[2][4];                        // twin plane codes [row][step] (PLANES 2)
    const int col0 = t - (kWave - 1);
    if (MASKED) {
        auto sko = [&](int c) { return (c >= 0 && c <= w.m) ? w.skel_voff + 4u * (uint32_t)c : kSkelOff; };
        push63_pk<4 * G4 + 0>(out_base, st, lane63_mask(push_on && col0 >= 0 && col0 <= w.m));
        dp_step_pk<true, (PLANES & 4) != 0, (PLANES & 8) == 0, (PLANES & 16) != 0, (PLANES & 32) != 0>(st, cur[0], t + 0, w.lane, w.m0, w.m1, w.c1a, w.c1b, w.c1ah, w.c1bh, k, bI[0], bD[0], bS[0], bL[0]);
        if ((PLANES & 3) == 1) bytes_step<0>(xI, xS, xD, bI[0], bD[0], bS[0], bL[0]);
        if ((PLANES & 3) == 2) { wc[0][0] = w16_code(bI[0][0], bD[0][0], bS[0][0], bL[0][0]);
                           wc[1][0] = w16_code(bI[0][1], bD[0][1], bS[0][1], bL[0][1]); }
        if ((PLANES & 16) == 0) skel_store(w.skel_rsrc, sko(col0 + 1), (int)st.b.E);
        push63_pk<4 * G4 + 1>(out_base, st, lane63_mask(push_on && col0 + 1 >= 0 && col0 + 1 <= w.m));
        dp_step_pk<true, (PLANES & 4) != 0, (PLANES & 8) == 0, (PLANES & 16) != 0, (PLANES & 32) != 0>(st, cur[1], t + 1, w.lane, w.m0, w.m1, w.c1a, w.c1b, w.c1ah, w.c1bh, k, bI[1], bD[1], bS[1], bL[1]);
        if ((PLANES & 3) == 1) bytes_step<1>(xI, xS, xD, bI[1], bD[1], bS[1], bL[1]);
        if ((PLANES & 3) == 2) { wc[0][1] = w16_code(bI[1][0], bD[1][0], bS[1][0], bL[1][0]);
                           wc[1][1] = w16_code(bI[1][1], bD[1][1], bS[1][1], bL[1][1]); }
        if ((PLANES & 16) == 0) skel_store(w.skel_rsrc, sko(col0 + 2), (int)st.b.E);
        push63_pk<4 * G4 + 2>(out_base, st, lane63_mask(push_on && col0 + 2 >= 0 && col0 + 2 <= w.m));
        dp_step_pk<true, (PLANES & 4) != 0, (PLANES & 8) == 0, (PLANES & 16) != 0, (PLANES & 32) != 0>(st, cur[2], t + 2, w.lane, w.m0, w.m1, w.c1a, w.c1b, w.c1ah, w.c1bh, k, bI[2], bD[2], bS[2], bL[2]);
        if ((PLANES & 3) == 1) bytes_step<2>(xI, xS, xD, bI[2], bD[2], bS[2], bL[2]);
        if ((PLANES & 3) == 2) { wc[0][2] = w16_code(bI[2][0], bD[2][0], bS[2][0], bL[2][0]);
                           wc[1][2] = w16_code(bI[2][1], bD[2][1], bS[2][1], bL[2][1]); }
        if ((PLANES & 16) == 0) skel_store(w.skel_rsrc, sko(col0 + 3), (int)st.b.E);
        push63_pk<4 * G4 + 3>(out_base, st, lane63_mask(push_on && col0 + 3 >= 0 && col0 + 3 <= w.m));
        if (push_on && col0 + 3 >= 0 && col0 <= w.m) lds_store_lane0(w.wcnt_out, min(col0 + 3, w.m) + 1);
        dp_step_pk<true, (PLANES & 4) != 0, (PLANES & 8) == 0, (PLANES & 16) != 0, (PLANES & 32) != 0>(st, cur[3], t + 3, w.lane, w.m0, w.m1, w.c1a, w.c1b, w.c1ah, w.c1bh, k, bI[3], bD[3], bS[3], bL[3]);
        if ((PLANES & 3) == 1) bytes_step<3>(xI, xS, xD, bI[3], bD[3], bS[3], bL[3]);
        if ((PLANES & 3) == 2) { wc[0][3] = w16_code(bI[3][0], bD[3][0], bS[3][0], bL[3][0]);
                           wc[1][3] = w16_code(bI[3][1], bD[3][1], bS[3][1], bL[3][1]); }
        if ((PLANES & 16) == 0) skel_store(w.skel_rsrc, sko(col0 + 4), (int)st.b.E);
    } else {
        const uint32_t pa = push_on && w.lane == kWave - 1 ? out_base : w.scratch;
        push_all_pk<4 * G4 + 0>(pa, st);
        dp_step_pk<false, (PLANES & 4) != 0, (PLANES & 8) == 0, (PLANES & 16) != 0, (PLANES & 32) != 0>(st, cur[0], t + 0, w.lane, w.m0, w.m1, w.c1a, w.c1b, w.c1ah, w.c1bh, k, bI[0], bD[0], bS[0], bL[0]);
        if ((PLANES & 3) == 1) bytes_step<0>(xI, xS, xD, bI[0], bD[0], bS[0], bL[0]);
        if ((PLANES & 3) == 2) { wc[0][0] = w16_code(bI[0][0], bD[0][0], bS[0][0], bL[0][0]);
                           wc[1][0] = w16_code(bI[0][1], bD[0][1], bS[0][1], bL[0][1]); }
        const uint32_t e0 = st.b.E;
        push_all_pk<4 * G4 + 1>(pa, st);
        dp_step_pk<false, (PLANES & 4) != 0, (PLANES & 8) == 0, (PLANES & 16) != 0, (PLANES & 32) != 0>(st, cur[1], t + 1, w.lane, w.m0, w.m1, w.c1a, w.c1b, w.c1ah, w.c1bh, k, bI[1], bD[1], bS[1], bL[1]);
        if ((PLANES & 3) == 1) bytes_step<1>(xI, xS, xD, bI[1], bD[1], bS[1], bL[1]);
        if ((PLANES & 3) == 2) { wc[0][1] = w16_code(bI[1][0], bD[1][0], bS[1][0], bL[1][0]);
                           wc[1][1] = w16_code(bI[1][1], bD[1][1], bS[1][1], bL[1][1]); }
        const uint32_t e1 = st.b.E;
        push_all_pk<4 * G4 + 2>(pa, st);
        dp_step_pk<false, (PLANES & 4) != 0, (PLANES & 8) == 0, (PLANES & 16) != 0, (PLANES & 32) != 0>(st, cur[2], t + 2, w.lane, w.m0, w.m1, w.c1a, w.c1b, w.c1ah, w.c1bh, k, bI[2], bD[2], bS[2], bL[2]);
        if ((PLANES & 3) == 1) bytes_step<2>(xI, xS, xD, bI[2], bD[2], bS[2], bL[2]);
        if ((PLANES & 3) == 2) { wc[0][2] = w16_code(bI[2][0], bD[2][0], bS[2][0], bL[2][0]);
                           wc[1][2] = w16_code(bI[2][1], bD[2][1], bS[2][1], bL[2][1]); }
        const uint32_t e2 = st.b.E;
        push_all_pk<4 * G4 + 3>(pa, st);
        publish_all(w.cnt_addr, col0 + 3 + 1);
        dp_step_pk<false, (PLANES & 4) != 0, (PLANES & 8) == 0, (PLANES & 16) != 0, (PLANES & 32) != 0>(st, cur[3], t + 3, w.lane, w.m0, w.m1, w.c1a, w.c1b, w.c1ah, w.c1bh, k, bI[3], bD[3], bS[3], bL[3]);
        if ((PLANES & 3) == 1) bytes_step<3>(xI, xS, xD, bI[3], bD[3], bS[3], bL[3]);
        if ((PLANES & 3) == 2) { wc[0][3] = w16_code(bI[3][0], bD[3][0], bS[3][0], bL[3][0]);
                           wc[1][3] = w16_code(bI[3][1], bD[3][1], bS[3][1], bL[3][1]); }
        if ((PLANES & 16) == 0)
            skel_store4(w.skel_rsrc, w.skel_voff + 4u * (uint32_t)(col0 + 1), (int)e0, (int)e1, (int)e2, (int)st.b.E);
    }
    if ((PLANES & 3) == 2) {
        // twin plane codes: per strip [group][row][lane] 12-B records (1.5 KB a
        // group; gx_device.h w12_pack), one dwordx3 per row and lane
        const auto r = rsrc_of(w.pI[0] + sb_off * (kTwinGroupBytes / kGroupInts), 4 * kTwinGroupBytes);
        const uint32_t v = (uint32_t)G4 * kTwinGroupBytes + (uint32_t)w.lane * kTwinRec;
        typedef int v3i __attribute__((ext_vector_type(3)));
#pragma unroll
        for (int row = 0; row < 2; ++row) {
            uint32_t w0, w1, w2;
#ifdef GX_DIAG_NO_PACK   // (timing only: the codes computed, neither packed nor stored)
            asm volatile("" ::"v"(wc[row][0]), "v"(wc[row][1]), "v"(wc[row][2]), "v"(wc[row][3]));
            continue;
#endif
            w12_pack(wc[row][0], wc[row][1], wc[row][2], wc[row][3], w0, w1, w2);
#ifndef GX_DIAG_NO_PLANES
            __builtin_amdgcn_raw_buffer_store_b96(v3i{(int)w0, (int)w1, (int)w2}, r,
                                                  (int)(v + (uint32_t)row * (kTwinGroupBytes / 2)), 0, GX_PLANE_AUX);
#else
            asm volatile("" ::"v"(w0), "v"(w1), "v"(w2));
#endif
        }
    }
    if ((PLANES & 3) == 1) {
        // compact planes of both pairs (bytes_step): x_I = I - I(j-1) (shifted:
        // x_I - g), x_S = S - I, x_D = D - I, one byte per cell
        constexpr int kSubBytes = kSub / 4 * kGroupInts;
        constexpr uint32_t kG = G4 * kGroupInts;
        const uint32_t v0 = (uint32_t)w.lane * 4u + kG, v1 = v0 + kWave * 4;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const auto rI = rsrc_of(w.pI[p] + sb_off, kSubBytes), rD = rsrc_of(w.pD[p] + sb_off, kSubBytes),
                       rS = rsrc_of(w.pS[p] + sb_off, kSubBytes);
            bstore1(rI, v0, xI[p][0]); bstore1(rS, v0, xS[p][0]); bstore1(rD, v0, xD[p][0]);
            bstore1(rI, v1, xI[p][1]); bstore1(rS, v1, xS[p][1]); bstore1(rD, v1, xD[p][1]);
        }
    }
    if (__builtin_amdgcn_readfirstlane(seen_v) < need) {
        wait_ge(w.wcnt_in, need, w.status);
        read4_pk(nxt, w.ring_in + ring_slot(t + 5));
    }
    __builtin_amdgcn_sched_barrier(0);
}

// The bases of block `blk` of ring `in` (slot 1 + blk mod kBaseSlots).
__device__ __forceinline__ int2 base_of(lds_int* b, int blk) {
    const int k = 1 + (blk & (kBaseSlots - 1));
    return make_int2(__builtin_amdgcn_readfirstlane(b[2 * k]), __builtin_amdgcn_readfirstlane(b[2 * k + 1]));
}

// The local floor (true 0) relative to bases (B0, B1), biased; clamped to the
// lowest biased value when a base exceeds 2^15 (no value of the band then
// lies within 2^15 of 0, so the floor never binds: cell_pk LOCAL).
__device__ __forceinline__ uint32_t local_floor(int B0, int B1) {
    return pk2(max(-B0, -32768), max(-B1, -32768)) ^ kBias2;
}
// A row's local maximum since the last base change into its absolute int32
// maxima (both pairs); the 16-bit tracker restarts at the lowest value.
__device__ __forceinline__ void fold_lb(RowPk& r, int (&mx)[2], int B0, int B1) {
    const uint32_t v = r.lb ^ kBias2;
    mx[0] = max(mx[0], lo16(v) + B0);
    mx[1] = max(mx[1], hi16(v) + B1);
    r.lb = 0;
}

// Shift every value of the lane state to new bases (delta = new - old).
__device__ __forceinline__ void rebase_row(RowPk& r, uint32_t dpk) {
    r.I = psubs(r.I, dpk); r.Hx = psubs(r.Hx, dpk); r.Dd = psubs(r.Dd, dpk);
    r.SMp = psubs(r.SMp, dpk); r.SMtl = psubs(r.SMtl, dpk);
}
__device__ __forceinline__ void rebase(LanePk& st, uint32_t dpk) {
    rebase_row(st.a, dpk);
    rebase_row(st.b, dpk);
}

template <int PLANES, bool MASKED>
__device__ __forceinline__ void sub_block_pk(LanePk& st, Rec (&nxt)[4], WavePk& w, const PkScores& k, const int t0,
                                             const uint32_t out_base, const bool push_on, const size_t sb_off) {
    group4_pk<PLANES, MASKED, 0>(st, nxt, w, k, t0, out_base, push_on, sb_off);
    group4_pk<PLANES, MASKED, 1>(st, nxt, w, k, t0, out_base, push_on, sb_off);
    group4_pk<PLANES, MASKED, 2>(st, nxt, w, k, t0, out_base, push_on, sb_off);
    group4_pk<PLANES, MASKED, 3>(st, nxt, w, k, t0, out_base, push_on, sb_off);
}

// Initial state of row i (column 0, algo.rs:204-211) in shifted values:
// H(i, 0) = h + i g -> h; I = H + h (compact planes' seed) -> 2h;
// delete successor (row i+1) -> h; relative to the bases (B0, B1).
// LOCAL (plain values): H(i, 0) = score_max = 0, I = H + h = h; the max(S, D)
// seed only needs max(S, D) + h + g <= 0 (the floor decides I(i, 1)); the
// row maximum tracker starts at the lowest value (fold_lb).
template <bool LOCAL = false>
__device__ __forceinline__ void init_row_pk(RowPk& rs, const Scores32& sc, int B0, int B1, const PkScores& k) {
    rs.lb = 0;
    if (LOCAL) {
        rs.I = pk2(sc.h - B0, sc.h - B1) ^ kBias2;
        rs.Hx = pk2(sc.hg - B0, sc.hg - B1) ^ kBias2;   // H(i, 0) + h + g = h + g
        rs.Dd = pk2(-B0, -B1) ^ kBias2;
        rs.SMp = padds(pk2(-B0, -B1) ^ kBias2, k.smp);
        rs.SMtl = 0;
        rs.cI = 0; rs.cD = 0;
        return;
    }
    rs.I = pk2(2 * sc.h - B0, 2 * sc.h - B1) ^ kBias2;
    rs.Hx = pk2(2 * sc.h - B0, 2 * sc.h - B1) ^ kBias2;   // H''(i, 0) + h = 2h
    rs.Dd = pk2(sc.h - B0, sc.h - B1) ^ kBias2;
    rs.SMp = padds(pk2(sc.h - B0, sc.h - B1) ^ kBias2, k.smp);
    rs.SMtl = 0;
    rs.cI = 0; rs.cD = 0;
}

template <int PLANES>
__device__ void compute_wave_pk(const PairDev& P0, const PairDev& P1, const int s, const int lane, const Scores32& sc,
                                const PkScores& k, const Rec* ring_in, Rec* ring_out, lds_int* wcnt_in,
                                lds_int* rcnt_in, lds_int* wcnt_out, lds_int* rcnt_out, lds_int* base_in,
                                lds_int* base_out, const bool has_consumer, PairRes* pres0, PairRes* pres1,
                                int* status, const uint32_t scratch_base, StripRes* sres) {
    constexpr bool LOCAL = (PLANES & 32) != 0;
    // a twin's pairs may differ in shape: the sweep covers the longer's rows
    // and columns (the host lays both out for that shape); each pair keeps
    // its own characters, column masks and end cell
    const int m = max(P0.m, P1.m), mmin = min(P0.m, P1.m);
    const int ia = s * kStripRows + kRowsPerLane * lane + 1;
    WavePk w;
    {
        // bytes per compact plane per strip (PLANES 2: the twin's one code plane, 1.5 KB a group)
        const size_t strip_planes = (size_t)s * P0.t4 * ((PLANES & 3) == 2 ? kTwinGroupBytes : kGroupInts);
        w.pI[0] = (PLANES & 3) ? (uint8_t*)P0.pI + strip_planes : nullptr;
        w.pD[0] = (PLANES & 3) == 1 ? (uint8_t*)P0.pD + strip_planes : nullptr;
        w.pS[0] = (PLANES & 3) == 1 ? (uint8_t*)P0.pS + strip_planes : nullptr;
        w.pI[1] = (PLANES & 3) == 1 ? (uint8_t*)P1.pI + strip_planes : nullptr;
        w.pD[1] = (PLANES & 3) == 1 ? (uint8_t*)P1.pD + strip_planes : nullptr;
        w.pS[1] = (PLANES & 3) == 1 ? (uint8_t*)P1.pS + strip_planes : nullptr;
        w.codes[0] = P0.codes + (size_t)s * P0.t16 * kWave * kRowsPerLane;
        w.codes[1] = P1.codes + (size_t)s * P0.t16 * kWave * kRowsPerLane;
    }
    w.ring_in = ring_in; w.wcnt_in = wcnt_in; w.wcnt_out = wcnt_out; w.status = status;
    w.base_in = base_in; w.base_out = base_out;
    // the twin's packed skeleton (P0.skel): int16 landing columns of both pairs per column
    w.skel_rsrc = rsrc_of(uniform_ptr(P0.skel + (size_t)s * P0.skel_stride), has_consumer ? 4 * (m + 1) : 0);
    w.skel_voff = lane == kWave - 1 ? 0u : kSkelOff;
    w.scratch = scratch_base + 4u * (uint32_t)lane;
    w.cnt_addr = (has_consumer && lane == kWave - 1) ? lds_addr((const void*)wcnt_out) : w.scratch;
    w.m = m; w.lane = lane; w.m0 = P0.m; w.m1 = P1.m;
    if constexpr ((PLANES & 4) != 0) {   // TBL: score tables of rows A, B per pair
        w.c1a = score_table_pk(ia <= P0.n ? (int)P0.c1[ia - 1] : 0x100, sc);
        w.c1ah = score_table_pk(ia <= P1.n ? (int)P1.c1[ia - 1] : 0x100, sc);
        w.c1b = score_table_pk(ia + 1 <= P0.n ? (int)P0.c1[ia] : 0x100, sc);
        w.c1bh = score_table_pk(ia + 1 <= P1.n ? (int)P1.c1[ia] : 0x100, sc);
    } else {
        w.c1a = pk2(ia <= P0.n ? (int)P0.c1[ia - 1] : 0x100, ia <= P1.n ? (int)P1.c1[ia - 1] : 0x100);
        w.c1b = pk2(ia + 1 <= P0.n ? (int)P0.c1[ia] : 0x100, ia + 1 <= P1.n ? (int)P1.c1[ia] : 0x100);
        w.c1ah = w.c1bh = 0;
    }

    // column 0 of the row above: its bases and record (published with the ring's first counter)
    wait_ge(wcnt_in, min(4, m) + 1, status);
    w.B0 = __builtin_amdgcn_readfirstlane(base_in[0]);   // slot 0: column 0
    w.B1 = __builtin_amdgcn_readfirstlane(base_in[1]);
    PkScores kl = k;                                      // (LOCAL: the floor follows the bases)
    int lmx[2][2] = {{0, 0}, {0, 0}};                     // LOCAL: rows A, B: absolute row maxima, both pairs
    if (LOCAL) kl.Z = local_floor(w.B0, w.B1);
    LanePk st;
    init_row_pk<LOCAL>(st.a, sc, w.B0, w.B1, kl);
    init_row_pk<LOCAL>(st.b, sc, w.B0, w.B1, kl);
    st.c2c = 0;
    st.b.SMtl = st.a.SMp;                                   // (A, 0) is row B's top-left for column 1
    st.a.E = pk2(-(kRowsPerLane * lane + 1), -(kRowsPerLane * lane + 1));
    st.b.E = pk2(-(kRowsPerLane * lane + 2), -(kRowsPerLane * lane + 2));
    st.b.Etl = st.a.E;
    if (has_consumer) {
        if (lane == kWave - 1) ring_out[ring_slot(0)] = Rec{(int)st.b.Dd, (int)st.b.SMp, 0, 0};
        if (lane == 0) { base_out[0] = w.B0; base_out[1] = w.B1; }
        lds_wait();
        if (lane == 0) *wcnt_out = 1;
    }
    Rec nxt[4];
    {
        const Rec r0 = ring_in[ring_slot(0)];
        st.a.SMtl = (uint32_t)shr1(r0.sm, (int)st.b.SMp);
        st.a.Etl = (uint32_t)shr1(0, (int)st.b.E);
        read4_pk(nxt, ring_in + ring_slot(1));
    }
    const int T = m + kWave;
    for (int t0 = 0; t0 < T; t0 += kSub) {
        const int last_col = min(t0 + kSub - 1 - (kWave - 1), m);
        if (has_consumer && last_col >= kRing) wait_ge(rcnt_out, last_col - kRing + 1, status);
        // adopt the bases of the block consumed now (columns t0+1 .. t0+16); the
        // block pushed now (columns t0-62 .. t0-47, block t0/16 - 4) carries them
        const int blk = t0 >> 4;
        if (t0 < m) {
            const int2 nb = base_of(base_in, blk);
            if (nb.x != w.B0 || nb.y != w.B1) {
                if (LOCAL) { fold_lb(st.a, lmx[0], w.B0, w.B1); fold_lb(st.b, lmx[1], w.B0, w.B1); }
                rebase(st, pk2(nb.x - w.B0, nb.y - w.B1));
                w.B0 = nb.x; w.B1 = nb.y;
                if (LOCAL) kl.Z = local_floor(w.B0, w.B1);
            }
        }
        // (sub-block 3 pushes column 0 again, now in the current bases: slot 0
        // follows it; the consumer reads both only once the counter passes 4)
        if (has_consumer && blk >= 3 && lane == 0) {
            const int kk = blk == 3 ? 0 : 1 + ((blk - 4) & (kBaseSlots - 1));
            base_out[2 * kk] = w.B0;
            base_out[2 * kk + 1] = w.B1;
        }
        const size_t sb_off = (size_t)(t0 >> 2) * kGroupInts;
        const bool full = (t0 >= kWave) && (t0 + kSub - 1 <= mmin - 1);
        const uint32_t out_base = lds_addr(ring_out + ring_slot(t0 - (kWave - 1)));
        if (full) sub_block_pk<PLANES, false>(st, nxt, w, kl, t0, out_base, has_consumer, sb_off);
        else sub_block_pk<PLANES, true>(st, nxt, w, kl, t0, out_base, has_consumer, sb_off);
        if constexpr ((PLANES & 8) == 0) {   // code words of both pairs: codes[strip][t/16][lane][row-in-lane]
            typedef unsigned v2u __attribute__((ext_vector_type(2)));
            typedef __attribute__((address_space(1))) v2u gv2u;
            const uint32_t aI = psub(0, st.a.cI), aD = psub(0, st.a.cD), bI = psub(0, st.b.cI), bD = psub(0, st.b.cD);
            const v2u c0 = {(aD << 16) | (aI & 0xFFFFu), (bD << 16) | (bI & 0xFFFFu)};
            const v2u c1 = {(aD & 0xFFFF0000u) | (aI >> 16), (bD & 0xFFFF0000u) | (bI >> 16)};
            const size_t wo = ((size_t)(t0 >> 4) * kWave + lane) * kRowsPerLane;
            *(gv2u*)(w.codes[0] + wo) = c0;
            *(gv2u*)(w.codes[1] + wo) = c1;
        }
        lds_store_lane0(rcnt_in, min(t0 + kSub + 5, m + 1));
    }
    if constexpr (LOCAL) {
        // each pair's last max row of the strip (row-major: the later row wins
        // ties) -> StripRes, which finalize_kernel reduces over the strips;
        // local_col_kernel then finds the row's last column holding it
        // (algo.rs:310-322)
        fold_lb(st.a, lmx[0], w.B0, w.B1);
        fold_lb(st.b, lmx[1], w.B0, w.B1);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const PairDev& P = h ? P1 : P0;
            const bool oka = ia <= P.n, okb = ia + 1 <= P.n;
            const int va = oka ? lmx[0][h] : INT_MIN;
            const int vb = okb ? lmx[1][h] : INT_MIN;
            const bool tb = okb && vb >= va;
            const int v = tb ? vb : va;
            int mx = v;
            for (int off = 32; off > 0; off >>= 1) mx = max(mx, __shfl_xor(mx, off));
            const unsigned long long lm = __ballot(oka && v == mx);
            const int ll = lm ? 63 - __clzll((long long)lm) : 0;
            const int lh = __shfl((int)tb, ll);
            if (lane == 0 && (h == 0 || &P1 != &P0)) {
                StripRes r;
                r.best = INT_MIN; r.bi = 0; r.bj = 0; r.bl = 0;
                r.lbest = mx; r.li = s * kStripRows + kRowsPerLane * ll + lh + 1; r.lj = 0; r.lE = 0;
                sres[P.strip_base + s] = r;
            }
        }
    }
    // cell (n, m) of each pair: score_max (shifted, absolute) and landing
    // column (a shorter pair's lanes stopped at its own last column)
    if (ia == P0.n || ia + 1 == P0.n) {
        const bool fa = ia == P0.n;
        const uint32_t sm = psubs(fa ? st.a.SMp : st.b.SMp, k.smp), e = fa ? st.a.E : st.b.E;
        pres0->end_SM = lo16(sm ^ kBias2) + w.B0; pres0->end_E = (PLANES & 16) ? 0 : lo16(e);
    }
    if (ia == P1.n || ia + 1 == P1.n) {
        const bool fa = ia == P1.n;
        const uint32_t sm = psubs(fa ? st.a.SMp : st.b.SMp, k.smp), e = fa ? st.a.E : st.b.E;
        pres1->end_SM = hi16(sm ^ kBias2) + w.B1; pres1->end_E = (PLANES & 16) ? 0 : hi16(e);
    }
}

// Record of the band hand-off rows (HBM): both pairs, absolute (int32).
struct __attribute__((aligned(16))) RecW {
    int dd0, dd1, sm0, sm1;   // delete successor, score_max + sm'' (shifted values)
    int c2, pad0, pad1, pad2; // s2[j-1] of both pairs (packed bytes)
};

// I/O wave of a twin band: ring 0 from row 0 (analytic) or the previous
// band's bottom row (absolute -> relative to the bases it picks per block);
// ring W to HBM (relative -> absolute with the last strip's bases).
template <bool TBL, bool LOCAL>
__device__ void io_wave_pk(const PairDev& P0, const PairDev& P1, const int lb, const int lane, const Scores32& sc,
                           const PkScores& k, Rec* ring0, const Rec* ringW, lds_int* wcnt0, lds_int* rcnt0,
                           lds_int* wcntW, lds_int* rcntW, lds_int* base0, lds_int* baseW, const bool do_out,
                           int* status) {
    const int m = max(P0.m, P1.m);   // the twin's columns; a shorter pair's columns beyond its own never match
    constexpr int CH = 16;
    int in_next = 0, out_next = 0;
    RecW* feed = reinterpret_cast<RecW*>(P0.feed);
    const RecW* feed_in = lb > 0 ? feed + (size_t)(lb - 1) * P0.feed_stride : nullptr;
    RecW* feed_out = do_out ? feed + (size_t)lb * P0.feed_stride : nullptr;
    const int* prog_in = lb > 0 ? P0.progress + (size_t)(lb - 1) * kProgStride : nullptr;
    int* prog_out = do_out ? P0.progress + (size_t)lb * kProgStride : nullptr;
    // sm'' (the launch's scores carry the shift's -2g, Scores32.shift); TBL: no
    // offset.  LOCAL: plain values, the score_max offset of k.smp.
    const int smp = LOCAL ? lo16(k.smp) : TBL ? 0 : sc.sm;
    unsigned idle = 0;
    int bprev0 = 0, bprev1 = 0;         // bases of the block before the current chunk's first column
    while (in_next <= m || (do_out && out_next <= m)) {
        bool moved = false;
        if (in_next <= m) {
            const int chunk = min(CH, m + 1 - in_next);
            bool ok = in_next + chunk - 1 < *rcnt0 + kRing;
            if (ok && lb > 0) ok = ld_agent(prog_in) > in_next + chunk - 1;
            if (ok) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const int j = in_next + lane;
                int dd0 = 0, dd1 = 0, sm0 = 0, sm1 = 0, c2 = 0;
                if (lane < chunk) {
                    if (lb == 0) {   // row 0 (algo.rs:195-202, 213-220), shifted: D' = 2h, SM = h
                        if (j == 0) { dd0 = dd1 = 0; sm0 = sm1 = smp; c2 = 0; }   // (local: every row-0 SM and
                        else {                                                    // D(1, j) is the 0 floor)
                            dd0 = dd1 = LOCAL ? 0 : 2 * sc.h;
                            sm0 = sm1 = (LOCAL ? 0 : sc.h) + smp;
                            if (TBL)   // the column's v_perm_b32 selector (cell_pk)
                                c2 = (int)perm_selector(j <= P0.m ? sym_code(P0.c2[j - 1], sc) : 0,
                                                        j <= P1.m ? sym_code(P1.c2[j - 1], sc) : 0);
                            else
                                c2 = (int)pk2(j <= P0.m ? (int)P0.c2[j - 1] : 0x200, j <= P1.m ? (int)P1.c2[j - 1] : 0x200);
                        }
                    } else {
                        const gu64* q = (const gu64*)(feed_in + j);
                        const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const unsigned long long c = __hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        dd0 = (int)(a & 0xffffffffu); dd1 = (int)(a >> 32);
                        sm0 = (int)(b & 0xffffffffu); sm1 = (int)(b >> 32);
                        c2 = (int)(c & 0xffffffffu);
                    }
                }
                // bases: column 0 -> slot 0; block c (columns 16c+1 ..) from its first column
                const int c0 = in_next >> 4;                     // chunk = columns 16c0 .. 16c0+15
                if (in_next == 0) {
                    bprev0 = __builtin_amdgcn_readlane(sm0, 0);
                    bprev1 = __builtin_amdgcn_readlane(sm1, 0);
                    if (lane == 0) { base0[0] = bprev0; base0[1] = bprev1; }
                }
                int nb0 = bprev0, nb1 = bprev1;
                if (chunk > 1) {
                    nb0 = __builtin_amdgcn_readlane(sm0, 1);
                    nb1 = __builtin_amdgcn_readlane(sm1, 1);
                    if (lane == 0) {
                        const int kk = 1 + (c0 & (kBaseSlots - 1));
                        base0[2 * kk] = nb0;
                        base0[2 * kk + 1] = nb1;
                    }
                }
                if (lane < chunk) {
                    // lane 0 (column 16 c0) belongs to the previous block (or column 0)
                    const int u0 = lane == 0 ? bprev0 : nb0, u1 = lane == 0 ? bprev1 : nb1;
                    Rec r;
                    r.dd = (int)(pk2(dd0 - u0, dd1 - u1) ^ kBias2);   // (biased halves)
                    r.sm = (int)(pk2(sm0 - u0, sm1 - u1) ^ kBias2);
                    r.c2 = c2;
                    r.l = 0;
                    ring0[ring_slot(j)] = r;
                }
                bprev0 = nb0; bprev1 = nb1;
                lds_wait();
                if (lane == 0) *wcnt0 = in_next + chunk;
                in_next += chunk;
                moved = true;
            }
        }
        if (do_out && out_next <= m) {
            const int avail = *wcntW;
            const int chunk = min(CH, avail - out_next);
            if (chunk == CH || (avail == m + 1 && chunk > 0)) {
                const int j = out_next + lane;
                if (lane < chunk) {
                    const Rec r = ringW[ring_slot(j)];
                    const int kk = j == 0 ? 0 : 1 + (((j - 1) >> 4) & (kBaseSlots - 1));
                    const int2 b = make_int2(baseW[2 * kk], baseW[2 * kk + 1]);
                    const unsigned long long a =
                        (unsigned long long)(unsigned)(lo16((uint32_t)r.dd ^ kBias2) + b.x) |
                        ((unsigned long long)(unsigned)(hi16((uint32_t)r.dd ^ kBias2) + b.y) << 32);
                    const unsigned long long bb =
                        (unsigned long long)(unsigned)(lo16((uint32_t)r.sm ^ kBias2) + b.x) |
                        ((unsigned long long)(unsigned)(hi16((uint32_t)r.sm ^ kBias2) + b.y) << 32);
                    gu64* q = (gu64*)(feed_out + j);
                    __hip_atomic_store(q, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(q + 1, bb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(q + 2, (unsigned long long)(unsigned)r.c2, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
                vm_wait();
                lds_wait();
                if (lane == 0) {
                    *rcntW = out_next + chunk;
                    st_agent(prog_out, out_next + chunk);
                }
                out_next += chunk;
                moved = true;
            }
        }
        if (moved) idle = 0;
        else if (++idle > kSpinLimit) {
            __hip_atomic_store((gint*)status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        } else {
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

// Twin fill: the two pairs of twin q share every band.  After the npairs
// descriptors: the band queue (total_bands entries (twin q, band lb)), then
// the twin table (ntwins entries (pair a, pair b); b == a twins a pair with
// itself, both halves writing the same bytes).
template <int W, int PLANES>
__global__ __launch_bounds__((W + 1) * kWave, (W + 1 + 3) / 4) void fill_pk_kernel(
    const PairDev* __restrict__ pairs, const int npairs, const int ntwins, const int total_bands, int* band_counter,
    PairRes* pres, StripRes* sres, const Scores32 sc) {
    __shared__ Rec rings[W + 1][kRing];
    __shared__ uint32_t push_scratch[W][kPushScratch];
    __shared__ int bases[W + 1][2 * (1 + kBaseSlots)];
    __shared__ int wcnt[W + 1];
    __shared__ int rcnt[W + 1];
    __shared__ int band_sh;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int lane = threadIdx.x & (kWave - 1);
    const int smp = sc.sm, smmp = sc.smm;   // s - 2g: the launch's scores carry the shift (Scores32.shift)
    // score_max is kept as SM + sm'' (TBL: as SM; its tables add the score).
    // LOCAL: the scores carry + K (sc.koff, so the tables' bytes are >= 0):
    // SM + s - K, i.e. SM - K with the tables
    const int off = (PLANES & 32) ? ((PLANES & 4) ? -sc.koff : smp - sc.koff) : (PLANES & 4) ? 0 : smp;
    const PkScores k{pk2(-sc.h, -sc.h), pk2(off, off), pk2(smmp - smp, smmp - smp),
                     pk2(-sc.g, -sc.g), pk2(-sc.hg, -sc.hg), kBias2};
    for (;;) {
        if (threadIdx.x == 0) band_sh = atomicAdd(band_counter, 1);
        if (threadIdx.x < W + 1) { wcnt[threadIdx.x] = 0; rcnt[threadIdx.x] = 0; }
        __syncthreads();
        const int b = __builtin_amdgcn_readfirstlane(band_sh);
        if (b >= total_bands) return;
        const int2* queue = reinterpret_cast<const int2*>(pairs + npairs);
        const int2 ob = queue[b];
        const int q = __builtin_amdgcn_readfirstlane(ob.x);
        const int2 tw = queue[total_bands + q];
        const int pa = __builtin_amdgcn_readfirstlane(tw.x), pb = __builtin_amdgcn_readfirstlane(tw.y);
        const PairDev& P0 = pairs[pa];
        const PairDev& P1 = pairs[pb];
        const int lb = __builtin_amdgcn_readfirstlane(ob.y);
        const int s0 = lb * W;
        if (wave < W) {
            const int s = s0 + wave;
            if (s < P0.strips) {
                const bool last_in_band = wave == W - 1;
                const bool has_consumer = last_in_band ? (lb + 1 < P0.bands) : (s + 1 < P0.strips);
                compute_wave_pk<PLANES>(P0, P1, s, lane, sc, k, rings[wave], rings[wave + 1], (lds_int*)&wcnt[wave],
                                        (lds_int*)&rcnt[wave], (lds_int*)&wcnt[wave + 1], (lds_int*)&rcnt[wave + 1],
                                        (lds_int*)bases[wave], (lds_int*)bases[wave + 1], has_consumer,
                                        pres + pa, pres + pb, band_counter + 1,
                                        lds_addr(push_scratch[wave]), sres);
            }
        } else {
            io_wave_pk<(PLANES & 4) != 0, (PLANES & 32) != 0>(P0, P1, lb, lane, sc, k, rings[0], rings[W], (lds_int*)&wcnt[0], (lds_int*)&rcnt[0],
                       (lds_int*)&wcnt[W], (lds_int*)&rcnt[W], (lds_int*)bases[0], (lds_int*)bases[W],
                       lb + 1 < P0.bands, band_counter + 1);
        }
        __syncthreads();
    }
}

template <int W0, int... Ws>
static hipError_t launch_pk_w(int W, int planes, const PairDev* d_pairs, int npairs, int ntwins, int total_bands,
                              int* d_counter, PairRes* d_pres, StripRes* d_sres, Scores32 sc, int grid,
                              hipStream_t st) {
    if (W == W0) {
#define GX_PK(PL) hipLaunchKernelGGL((fill_pk_kernel<W0, PL>), dim3(grid), dim3((W0 + 1) * kWave), 0, st, d_pairs, \
                                     npairs, ntwins, total_bands, d_counter, d_pres, d_sres, sc)
        switch (planes) {
#ifndef GX_PK_ONLY_LOCAL   // (register-allocation experiments: the local instantiation alone compiles in seconds)
            case 0: GX_PK(0); break;
            case 1: GX_PK(1); break;
            case 2: GX_PK(2); break;
            case 4: GX_PK(4); break;
            case 6: GX_PK(6); break;
            case 10: GX_PK(10); break;   // twin codes, no code words
            case 14: GX_PK(14); break;
            case 26: GX_PK(26); break;   // twin codes, no code words, no skeleton (tb_seq_kernel)
            case 30: GX_PK(30); break;
            case 58: GX_PK(58); break;   // local (Smith-Waterman): twin codes, no code words, no skeleton
#endif
            case 62: GX_PK(62); break;
            default: return hipErrorInvalidValue;
        }
#undef GX_PK
        return hipGetLastError();
    }
    if constexpr (sizeof...(Ws) > 0) return launch_pk_w<Ws...>(W, planes, d_pairs, npairs, ntwins, total_bands,
                                                               d_counter, d_pres, d_sres, sc, grid, st);
    return hipErrorInvalidValue;
}

// Twin launch: W from {3, 4, 7, 8, 15}; planes: 0 none, 1 compact bytes per
// pair (3 B/cell), 2 twin codes (2 B/cell); + 4: small-alphabet score tables
// (with none or twin codes: the batch launches); + 8 (with twin codes): no
// code words (the traceback derives them from the plane codes); + 16: no
// skeleton; + 32 (with 2 + 8 + 16): local mode, each strip's last max of each
// pair into d_sres (finalize_kernel reduces them).
hipError_t launch_fill_pk(int W, int planes, const PairDev* d_pairs, int npairs, int ntwins, int total_bands,
                          int* d_counter, PairRes* d_pres, StripRes* d_sres, Scores32 sc, int grid, hipStream_t st) {
#ifndef GX_PK_ONLY_LOCAL
    return launch_pk_w<3, 4, 7, 8, 15>(W, planes, d_pairs, npairs, ntwins, total_bands, d_counter, d_pres, d_sres, sc,
                                       grid, st);
#else
    return launch_pk_w<7>(W, planes, d_pairs, npairs, ntwins, total_bands, d_counter, d_pres, d_sres, sc, grid, st);
#endif
}

}  // namespace gx
