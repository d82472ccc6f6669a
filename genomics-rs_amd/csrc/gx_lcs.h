// gx_lcs.h -- max_matches of alignment_table (algo.rs:113-121, 250-256, 279)
// as a bit-parallel LCS computed beside the fill.
//
// The reference carries *_matches in every cell: insert_matches =
// max_matches(i, j-1), delete_matches = max_matches(i-1, j), sub_matches =
// max_matches(i-1, j-1) + is_match, and max_matches = the largest of the
// three (and 0).  So LM(i, j) = max_matches(cell(i, j)) obeys
//     LM(i, j) = max(LM(i, j-1), LM(i-1, j), LM(i-1, j-1) + is_match(i-1, j-1))
// with LM = 0 on row 0 and column 0: the plain LCS length of s1[..i] and
// s2[..j] under is_match (sequence.rs:102-115, on the processed bytes, None
// == None included).  It does not depend on the scores, so it need not ride
// in the fill: the row-by-row bit-vector recurrence of Allison-Dix / Hyyro
//     U = V & M[s1[i-1]],   V' = (V + U) | (V & ~M[s1[i-1]]),   V_0 = ~0
// gives LM(i, j) = j - popcount(V_i & (2^j - 1)) (bit k of V_i: column k + 1).
//
// Layout: the bit rows are swept like the DP fill itself -- 64-row STRIPS
// on the anti-diagonal skew, one row per lane, 64 columns a word.  At step t
// lane l (row i = 64 s + l + 1) advances word w = t - l of its row: the word
// of the row above comes from lane l - 1's previous step (DPP wave_shr:1;
// lane 0 from the strip above's lane 63, 63 steps later in that strip), the
// carry from the row's word w - 1 stays in the lane (VCC inside a 4-step
// block, lcs_block4), and the match mask is one buffer load (masks[byte][64 +
// w], zero-padded 64 words on either side so that ramp-up and ramp-down steps
// read 0).  A step is 8 VALU with a one-deep dependence, so the sweep is
// bound by its dependence chain -- about n + m / 64 steps, a strip passing
// its bottom row down 64 steps after its top row -- not by throughput: it
// takes a few CUs beside the fill.  The strips go to LCS workgroups in blocks
// of nsweep (wave k of a workgroup takes strip b nsweep + k of its blocks b =
// wg, wg + nwg, ...); within a block a wave hands its bottom row to the next
// wave through an LDS ring (256 steps + 8 mirrored, flow-controlled by two
// counters), from block to block (workgroup to workgroup) through HBM feed
// rows (tagged words, zeroed before the launch, a slot per step: no flow
// control), read a group ahead so that their latency is paid once per block.
// Output: bits[strip][t][lane] (PairDev.lbits), word w of row i at
// ((s T + w + l) 64 + l), T = lcs_steps(lwords); finalize_kernel /
// skew_mam_kernel read row max_i for matches_at_max, the table export
// rebuilds the *_matches fields from the rows (gx_api_table.cpp).  No MFMA:
// 32-bit adds with carry and bit logic.
#pragma once
#include "gx_device.h"

namespace gx {

template <typename T>
__device__ __forceinline__ T* uni_ptr(T* p) {   // a pointer the compiler is told is wave-uniform
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (T*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

// Four steps of one lane: step k takes the word of the row above from lane
// l - 1's previous step (lane 0: top[k]; the DPP leaves the old value in lane
// 0) and the mask mk[k], and leaves the row's word in o[k]; c (0 / 1) is the
// row's carry into the next word, held in VCC inside the block.
//     u = v & mk,  s = v + u + carry,  o = s | (v & ~mk)      (bitop3 0xF4)
// The s_nops keep the DPP reads two wait states after the VALU writes of the
// words they read (the assembler inserts no hazard waits in inline asm).
__device__ __forceinline__ void lcs_block4(uint32_t (&tl)[4], uint32_t (&th)[4], const uint32_t (&ml)[4],
                                           const uint32_t (&mh)[4], uint32_t (&ol)[4], uint32_t (&oh)[4], uint32_t vl,
                                           uint32_t vh, uint32_t& c) {
    uint32_t ul, uh;
#define GX_LCS_STEP(K, VL, VH)                                                              \
    "v_mov_b32_dpp %[tl" #K "], " VL " wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"         \
    "v_mov_b32_dpp %[th" #K "], " VH " wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"         \
    "v_and_b32_e32 %[ul], %[tl" #K "], %[ml" #K "]\n\t"                                    \
    "v_and_b32_e32 %[uh], %[th" #K "], %[mh" #K "]\n\t"                                    \
    "v_addc_co_u32_e32 %[ul], vcc, %[tl" #K "], %[ul], vcc\n\t"                            \
    "v_addc_co_u32_e32 %[uh], vcc, %[th" #K "], %[uh], vcc\n\t"                            \
    "v_bitop3_b32 %[ol" #K "], %[ul], %[tl" #K "], %[ml" #K "] bitop3:0xf4\n\t"            \
    "v_bitop3_b32 %[oh" #K "], %[uh], %[th" #K "], %[mh" #K "] bitop3:0xf4\n\t"            \
    "s_nop 0\n\t"
    asm volatile(
        "s_nop 1\n\t"
        "v_cmp_ne_u32_e32 vcc, 0, %[c]\n\t"
        GX_LCS_STEP(0, "%[vl]", "%[vh]")
        GX_LCS_STEP(1, "%[ol0]", "%[oh0]")
        GX_LCS_STEP(2, "%[ol1]", "%[oh1]")
        GX_LCS_STEP(3, "%[ol2]", "%[oh2]")
        "v_cndmask_b32_e64 %[c], 0, 1, vcc\n\t"
        : [tl0] "+v"(tl[0]), [tl1] "+v"(tl[1]), [tl2] "+v"(tl[2]), [tl3] "+v"(tl[3]),
          [th0] "+v"(th[0]), [th1] "+v"(th[1]), [th2] "+v"(th[2]), [th3] "+v"(th[3]),
          [ol0] "=&v"(ol[0]), [ol1] "=&v"(ol[1]), [ol2] "=&v"(ol[2]), [ol3] "=&v"(ol[3]),
          [oh0] "=&v"(oh[0]), [oh1] "=&v"(oh[1]), [oh2] "=&v"(oh[2]), [oh3] "=&v"(oh[3]),
          [ul] "=&v"(ul), [uh] "=&v"(uh), [c] "+v"(c)
        : [ml0] "v"(ml[0]), [ml1] "v"(ml[1]), [ml2] "v"(ml[2]), [ml3] "v"(ml[3]),
          [mh0] "v"(mh[0]), [mh1] "v"(mh[1]), [mh2] "v"(mh[2]), [mh3] "v"(mh[3]),
          [vl] "v"(vl), [vh] "v"(vh)
        : "vcc");
#undef GX_LCS_STEP
}

// LDS of an LCS workgroup (carved from the fill's own arrays, gx_skew.hip):
// the published / consumed step counters of every sweeping wave, then a ring
// per wave of its bottom row's words, slot t mod 256 for step t (8 slots
// mirrored past the end, so that a read of 8 consecutive steps never wraps).
constexpr int kLcsRing = 256;
constexpr int kLcsMaxSweep = 8;
constexpr int kLcsLdsHead = 2 * kLcsMaxSweep * 4;
__host__ __device__ constexpr int lcs_max_sweep(size_t lds_bytes) {
    return lds_bytes < (size_t)kLcsLdsHead + (kLcsRing + 8) * 8
               ? 0
               : ((lds_bytes - kLcsLdsHead) / ((kLcsRing + 8) * 8) < (size_t)kLcsMaxSweep
                      ? (int)((lds_bytes - kLcsLdsHead) / ((kLcsRing + 8) * 8))
                      : kLcsMaxSweep);
}

// Wave `wave` (of nwave) of LCS workgroup `wg` (of nwg) of pair P; lds /
// lds_bytes: LDS the workgroup may use (at least one ring); status: the
// launch's timeout word.  Every workgroup builds the whole mask table itself
// (the same values: each then reads only its own writes).
__device__ __forceinline__ void lcs_workgroup(const PairDev& P, const int wg, const int nwg, const int wave,
                                              const int nwave, const int lane, char* lds, const size_t lds_bytes,
                                              int* status) {
    const int n = __builtin_amdgcn_readfirstlane(P.n), m = __builtin_amdgcn_readfirstlane(P.m);
    const int wd = __builtin_amdgcn_readfirstlane(P.lwords);
    if (n <= 0 || m <= 0 || wd <= 0) return;   // (uniform for the workgroup: no barrier reached)
    const int ws = wd + 2 * kLcsMaskPad;       // mask row stride (words)
    const int T = lcs_steps(wd);
    const int S = (n + kWave - 1) / kWave;
    unsigned long long* const masks = uni_ptr(P.lmask);
    unsigned long long* const bits = uni_ptr(P.lbits);
    unsigned long long* const feed = uni_ptr(P.llink);
    const uint8_t* const c1 = uni_ptr(P.c1);
    const uint8_t* const c2 = uni_ptr(P.c2);
    const int lw = __builtin_amdgcn_readfirstlane(P.lcs_waves) & 0xFF;
    const bool full = (__builtin_amdgcn_readfirstlane(P.lcs_waves) >> 16) & 1;   // every row, or the strips' last only
    int ns = lw > 0 && lw < nwave ? lw : nwave;
    ns = min(ns, lcs_max_sweep(lds_bytes));
    int* const pub = (int*)lds;                  // [wave] steps of its strips published (q T + t)
    int* const con = pub + kLcsMaxSweep;         // [wave] steps of its strips its consumer is done with
    unsigned long long* const ring0 = (unsigned long long*)(lds + kLcsLdsHead);
    if ((int)threadIdx.x < 2 * kLcsMaxSweep) pub[threadIdx.x] = 0;
    // 1. match masks masks[b][64 + w] (bit k: s2[64 w + k] == b), words shared out over the workgroup's waves
    for (int w0 = wave * 8; w0 < wd; w0 += nwave * 8) {
        int cb[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int col = (w0 + q) * kLcsBits + lane;
            cb[q] = (w0 + q < wd && col < m) ? (int)c2[col] : 0x100;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            unsigned long long rem = __ballot(cb[q] < 0x100);
            while (rem) {
                const int b = __builtin_amdgcn_readlane(cb[q], (int)__builtin_ctzll(rem));
                const unsigned long long mk = __ballot(cb[q] == b);
                if (lane == 0) *(gu64*)(masks + (size_t)b * ws + kLcsMaskPad + w0 + q) = mk;
                rem &= ~mk;
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (wave >= ns) return;
    // 2. the strips
    const __amdgpu_buffer_rsrc_t mrs = rsrc_of(masks, __builtin_amdgcn_readfirstlane(256 * ws * 8));
    typedef int v2i __attribute__((ext_vector_type(2)));
    unsigned long long* const rin = ring0 + (size_t)(wave > 0 ? wave - 1 : 0) * (kLcsRing + 8);
    unsigned long long* const rout = ring0 + (size_t)wave * (kLcsRing + 8);
    int q = 0;   // this wave's strip count (its producer's and consumer's are the same)
    for (int blk = wg; blk * ns < S; blk += nwg, ++q) {
        const int s = blk * ns + wave;
        if (s >= S) break;
        const int i = s * kWave + lane + 1;
        const int b = i <= n ? (int)c1[i - 1] : 0;
        // this lane's mask word of step t: masks[b][64 + t - lane]
        const uint32_t vb = (uint32_t)(b * ws + kLcsMaskPad - lane) * 8u;
        bool has_in = s > 0, has_out = s + 1 < S;
#ifndef GX_DIAG_LCS_NOFEED   // (timing only: wrong rows)
        const bool hbm_in = has_in && wave == 0, hbm_out = has_out && wave == ns - 1;
#else
        const bool hbm_in = false, hbm_out = false;
        has_in = has_in && wave > 0;
        has_out = has_out && wave < ns - 1;
#endif
        const int qT = q * T;
        const __amdgpu_buffer_rsrc_t brs =
            full ? rsrc_of(uni_ptr(bits + (size_t)s * T * kWave), __builtin_amdgcn_readfirstlane(T * kWave * 8))
                 : rsrc_of(uni_ptr(bits + (size_t)s * T), __builtin_amdgcn_readfirstlane(T * 8));
        const gu64* const fin = (const gu64*)(feed + (size_t)(s > 0 ? s - 1 : 0) * T * 2);
        gu64* const fout = (gu64*)(feed + (size_t)s * T * 2);
        uint32_t c = 0, vl = ~0u, vh = ~0u;   // the carry; this lane's word of the previous step
#ifndef GX_DIAG_LCS_NOMASK   // (timing only: wrong rows)
        auto mask_at = [&](int t) -> v2i { return __builtin_amdgcn_raw_buffer_load_b64(mrs, (int)vb, t * 8, 0); };
#else
        auto mask_at = [&](int t) -> v2i { return v2i{(int)vb ^ t, t}; };
#endif
        // a group's 8 mask words of this lane -- consecutive words of its row,
        // as four 16-B loads (against eight 8-B ones: the sweep's pace 101 ->
        // 87.5 ns a step, Covid's sweep alone 3.93 -> 3.43 ms; the per-lane
        // loads gather from up to four rows at once and are what bounds it,
        // tools/lcs_step_probe.hip)
        auto mask_group = [&](int t, v2i (&m)[8]) {
#ifndef GX_DIAG_LCS_NOMASK
            typedef int v4i __attribute__((ext_vector_type(4)));
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const v4i x = __builtin_amdgcn_raw_buffer_load_b128(mrs, (int)vb, (t + 2 * k) * 8, 0);
                m[2 * k] = v2i{x[0], x[1]};
                m[2 * k + 1] = v2i{x[2], x[3]};
            }
#else
#pragma unroll
            for (int k = 0; k < 8; ++k) m[k] = mask_at(t + k);
#endif
        };
        // the feed words of the strip above's steps t0 + 63 .. t0 + 70 (clamped
        // to its last step): lane k < 16 loads half k & 1 of step t0 + 63 + k / 2
        auto feed_at = [&](int t0) -> unsigned long long {
            return lane < 16 ? __hip_atomic_load(fin + 2 * min(t0 + 63 + (lane >> 1), T - 1) + (lane & 1), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : 0ull;
        };
        unsigned conc = 0;   // (LDS output: the consumer's counter as last read)
        unsigned have = 0;   // (LDS input: the producer's counter as last read)
        // One group of 8 steps from t0: first the loads of group t0 + 24 into
        // the set the previous group used (masks; feed words for wave 0), then
        // the steps with this group's set -- four sets in rotation, so a load
        // has three groups to land and no register is copied (a copy would wait
        // on its load).
        auto group = [&](const int t0, v2i (&mc)[8], const unsigned long long fc, v2i (&mn)[8],
                         unsigned long long& fn) __attribute__((always_inline)) {
            mask_group(t0 + 24, mn);
            if (hbm_in) fn = feed_at(t0 + 24);
            // lane 0's words of the row above (words t0 .. t0 + 7: the strip
            // above's steps t0 + 63 .. t0 + 70), or row 0 (all ones)
            uint32_t tl[8], th[8];
            const int need = min(t0 + 71, T);   // (steps past the strip above's last: don't care)
            if (hbm_in) {
                // (the check reads the prefetched words where they landed; only
                // a miss enters the reload loop -- a loop around the registers
                // themselves would wait on every load in flight)
                const auto valid = [&](unsigned long long f) {
                    return __ballot(!(lane >= 16 || t0 + 63 + (lane >> 1) >= need || (f >> 32) != 0)) == 0;
                };
                unsigned long long f = fc;
                if (!valid(f)) {
                    unsigned it = 0;
                    do {
                        if (++it > kSpinLimit) { __hip_atomic_store((gint*)status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
                        if ((it & 4095u) == 4095u && __hip_atomic_load((gint*)status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
                        __builtin_amdgcn_s_sleep(1);
                        f = feed_at(t0);
                    } while (!valid(f));
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    tl[k] = __builtin_amdgcn_readlane((uint32_t)f, 2 * k);
                    th[k] = __builtin_amdgcn_readlane((uint32_t)f, 2 * k + 1);
                }
            } else if (has_in) {
                if (have < (unsigned)(qT + need)) {
                    unsigned it = 0;
                    for (;;) {
                        have = (unsigned)__hip_atomic_load(pub + wave - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (have >= (unsigned)(qT + need)) break;
                        if (++it > kSpinLimit) { __hip_atomic_store((gint*)status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
                        if ((it & 4095u) == 4095u && __hip_atomic_load((gint*)status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                __atomic_signal_fence(__ATOMIC_SEQ_CST);   // (LDS executes a wave's ops in order: the ring after the counter)
                const int r0 = (qT + t0 + 63) & (kLcsRing - 1);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const unsigned long long x = rin[r0 + k];
                    tl[k] = (uint32_t)x; th[k] = (uint32_t)(x >> 32);
                }
                // (the counter moves after the reads, in LDS order; no release
                // fence -- at workgroup scope it would wait for every load and
                // store in flight, the mask prefetch included)
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                if (lane == 0) __hip_atomic_store(con + wave - 1, qT + need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) { tl[k] = ~0u; th[k] = ~0u; }
            }
            uint32_t ol[8], oh[8];
            {
                uint32_t a[4], bh[4], mlo[4], mhi[4], o1[4], o2[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) { a[k] = tl[k]; bh[k] = th[k]; mlo[k] = (uint32_t)mc[k][0]; mhi[k] = (uint32_t)mc[k][1]; }
                lcs_block4(a, bh, mlo, mhi, o1, o2, vl, vh, c);
#pragma unroll
                for (int k = 0; k < 4; ++k) { ol[k] = o1[k]; oh[k] = o2[k]; }
#pragma unroll
                for (int k = 0; k < 4; ++k) { a[k] = tl[4 + k]; bh[k] = th[4 + k]; mlo[k] = (uint32_t)mc[4 + k][0]; mhi[k] = (uint32_t)mc[4 + k][1]; }
                lcs_block4(a, bh, mlo, mhi, o1, o2, ol[3], oh[3], c);
#pragma unroll
                for (int k = 0; k < 4; ++k) { ol[4 + k] = o1[k]; oh[4 + k] = o2[k]; }
                vl = ol[7]; vh = oh[7];
            }
#ifndef GX_DIAG_LCS_NOSTORE   // (timing only: no bit rows)
            if (full) {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    __builtin_amdgcn_raw_buffer_store_b64(v2i{(int)ol[k], (int)oh[k]}, brs, (int)(lane * 8), (t0 + k) * kWave * 8, 0);
            } else if (lane == kWave - 1) {   // (the strip's bottom row: lcs_matches restarts from it)
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    __builtin_amdgcn_raw_buffer_store_b64(v2i{(int)ol[k], (int)oh[k]}, brs, 0, (t0 + k) * 8, 0);
            }
#endif
            // lane 63 passes its words of steps t0 .. t0 + 7 down
            if (hbm_out) {
                if (lane == kWave - 1) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        __hip_atomic_store(fout + 2 * (t0 + k), (unsigned long long)ol[k] | (1ull << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(fout + 2 * (t0 + k) + 1, (unsigned long long)oh[k] | (1ull << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            } else if (has_out) {
                // the consumer must be done with the slots' previous steps (qT + t0 - 256 ..)
                const int G = qT + t0;
                if ((int)conc < G + 8 - kLcsRing) {
                    unsigned it = 0;
                    for (;;) {
                        conc = (unsigned)__hip_atomic_load(con + wave, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if ((int)conc >= G + 8 - kLcsRing) break;
                        if (++it > kSpinLimit) { __hip_atomic_store((gint*)status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
                        if ((it & 4095u) == 4095u && __hip_atomic_load((gint*)status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                if (lane == kWave - 1) {
                    const int r0 = G & (kLcsRing - 1);
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const unsigned long long x = ((unsigned long long)oh[k] << 32) | ol[k];
                        rout[r0 + k] = x;
                        if (r0 == 0) rout[kLcsRing + k] = x;
                    }
                    // (the ring words land before the counter: LDS order, and the
                    // compiler may not sink them past it)
                    __atomic_signal_fence(__ATOMIC_SEQ_CST);
                    __hip_atomic_store(pub + wave, G + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        };
        unsigned long long* const ltr = P.ltrace;   // (diagnostics: strip start, first group done, end)
        if (ltr && lane == 0) ltr[(size_t)s * 4] = __builtin_amdgcn_s_memrealtime();
        v2i mA[8], mB[8], mC[8], mD[8];
        unsigned long long fA = 0, fB = 0, fC = 0, fD = 0;
        mask_group(0, mA); mask_group(8, mB); mask_group(16, mC);
        if (hbm_in) { fA = feed_at(0); fB = feed_at(8); fC = feed_at(16); }
        for (int t0 = 0; t0 < T; t0 += 32) {   // (T: a multiple of 32)
            group(t0, mA, fA, mD, fD);
            if (ltr && t0 == 0 && lane == 0) ltr[(size_t)s * 4 + 1] = __builtin_amdgcn_s_memrealtime();
            group(t0 + 8, mB, fB, mA, fA);
            group(t0 + 16, mC, fC, mB, fB);
            group(t0 + 24, mD, fD, mC, fC);
        }
        if (ltr && lane == 0) {
            ltr[(size_t)s * 4 + 2] = __builtin_amdgcn_s_memrealtime();
            ltr[(size_t)s * 4 + 3] = (unsigned long long)(wg * 64 + wave);
        }
    }
}

// LM(i, j) = max_matches of cell (i, j) (algo.rs:279 matches_at_max), one
// wave (all 64 lanes, wave-uniform i, j): from the stored row when the sweep
// kept every row, otherwise by sweeping strip (i - 1) / 64 again from the
// bottom row of the strip above (which the sweep keeps: bits[strip][step],
// word w at step w + 63) up to row i's word (j - 1) / 64 -- a few hundred
// steps of one wave, against the 64x traffic of keeping every row.
__device__ __forceinline__ int lcs_matches(const PairDev& P, const int i, const int j, const int lane) {
    const int wd = __builtin_amdgcn_readfirstlane(P.lwords);
    // (a cell outside the table -- e.g. strip results a diagnostics launch
    // never wrote, GX_LCS_ALONE -- reads nothing)
    if (wd <= 0 || !P.lbits || i < 1 || i > P.n || j < 1 || j > P.m) return 0;
    const unsigned long long* const bits = uni_ptr(P.lbits);
    const int T = lcs_steps(wd);
    const int wj = (j + kLcsBits - 1) / kLcsBits;   // words of row i that count
    int ones = 0;
    if ((__builtin_amdgcn_readfirstlane(P.lcs_waves) >> 16) & 1) {
        for (int w = lane; w < wj; w += kWave) {
            unsigned long long x = bits[lcs_word_index(i, w, wd)];
            const int rem = j - w * kLcsBits;
            if (rem < kLcsBits) x &= (1ull << rem) - 1ull;
            ones += __popcll(x);
        }
    } else {
        const int s = (i - 1) / kWave, li = (i - 1) % kWave;
        const int ws = wd + 2 * kLcsMaskPad;
        const int r = s * kWave + lane + 1;
        const int b = r <= P.n ? (int)P.c1[r - 1] : 0;
        const uint32_t vb = (uint32_t)(b * ws + kLcsMaskPad - lane) * 8u;
        const __amdgpu_buffer_rsrc_t mrs = rsrc_of(uni_ptr(P.lmask), __builtin_amdgcn_readfirstlane(256 * ws * 8));
        typedef int v2i __attribute__((ext_vector_type(2)));
        const unsigned long long* const above = bits + (size_t)(s > 0 ? s - 1 : 0) * T;
        const int tend = li + wj;   // steps: lane li finishes word wj - 1 at step tend - 1
        auto top_at = [&](int t0) -> unsigned long long {   // lane k < 8: the row above's word t0 + k
            return s > 0 && lane < 8 ? above[min(t0 + lane + 63, T - 1)] : ~0ull;
        };
        uint32_t c = 0, vl = ~0u, vh = ~0u;
        // (groups of 8 steps; the loads of group t0 + 24 go out before group
        // t0 runs, into four register sets in rotation, as in lcs_workgroup)
        auto grp = [&](const int t0, const v2i (&mc)[8], const unsigned long long tc, v2i (&mn)[8],
                       unsigned long long& tn) __attribute__((always_inline)) {
#pragma unroll
            for (int k = 0; k < 8; ++k) mn[k] = __builtin_amdgcn_raw_buffer_load_b64(mrs, (int)vb, (t0 + 24 + k) * 8, 0);
            tn = top_at(t0 + 24);
            uint32_t ol[8], oh[8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint32_t a[4], bh[4], ml[4], mh[4], o1[4], o2[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    a[k] = __builtin_amdgcn_readlane((uint32_t)tc, 4 * h + k);
                    bh[k] = __builtin_amdgcn_readlane((uint32_t)(tc >> 32), 4 * h + k);
                    ml[k] = (uint32_t)mc[4 * h + k][0]; mh[k] = (uint32_t)mc[4 * h + k][1];
                }
                lcs_block4(a, bh, ml, mh, o1, o2, vl, vh, c);
#pragma unroll
                for (int k = 0; k < 4; ++k) { ol[4 * h + k] = o1[k]; oh[4 * h + k] = o2[k]; }
                vl = o1[3]; vh = o2[3];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int w = t0 + k - lane;   // this lane's word of step t0 + k
                if (lane == li && w >= 0 && w < wj) {
                    unsigned long long x = ((unsigned long long)oh[k] << 32) | ol[k];
                    const int rem = j - w * kLcsBits;
                    if (rem < kLcsBits) x &= (1ull << rem) - 1ull;
                    ones += __popcll(x);
                }
            }
        };
        v2i mA[8], mB[8], mC[8], mD[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            mA[k] = __builtin_amdgcn_raw_buffer_load_b64(mrs, (int)vb, k * 8, 0);
            mB[k] = __builtin_amdgcn_raw_buffer_load_b64(mrs, (int)vb, (8 + k) * 8, 0);
            mC[k] = __builtin_amdgcn_raw_buffer_load_b64(mrs, (int)vb, (16 + k) * 8, 0);
        }
        unsigned long long tA = top_at(0), tB = top_at(8), tC = top_at(16), tD = 0;
        for (int t0 = 0; t0 < tend; t0 += 32) {   // (steps past tend: harmless, nothing counted)
            grp(t0, mA, tA, mD, tD);
            grp(t0 + 8, mB, tB, mA, tA);
            grp(t0 + 16, mC, tC, mB, tB);
            grp(t0 + 24, mD, tD, mC, tC);
        }
    }
    for (int off = 32; off > 0; off >>= 1) ones += __shfl_xor(ones, off);
    return j - ones;
}

}  // namespace gx
