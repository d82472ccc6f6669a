// gx_wide.hip -- the wide (int64) fill: alignment_table (algo.rs:151-282) in
// the reference's own integer type, for jobs outside the exact-int32 range of
// the main fill (gx_api_plan.cpp check_scores: score magnitudes above 2^24, |score|
// bounds above 2^28, the g < 0 < h configurations whose boundary arithmetic
// wraps, sequences longer than 2^26).  Every add wraps modulo 2^64 exactly as
// the reference's release build does (i64 overflow is not checked there), and
// the max / compare semantics are those of score_max (algo.rs:98-107).
//
// Layout: one wave per pair, 64-row strips (lane = row) swept one after the
// other, each on the anti-diagonal skew (step t: lane l computes column
// j = t - l + 1).  The cell above arrives from lane l - 1 through a DPP /
// ds_bpermute shuffle; lane 0 takes it from the previous strip's bottom row
// (a per-strip row in HBM, prefetched 64 columns at a time).  Outputs are in
// the formats the column-step layout (layout 1) uses, so the traceback
// kernels and the host walk are shared: codes[strip][q][lane] (two bit-planes,
// gx_internal.h) and skel[strip][column] = landing column + 64 of the strip's
// bottom row; score planes are int64 row-major (n x m interior cells), and
// the LCS plane int32.  A rare path: correctness, not throughput.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gx_internal.h"

namespace gx {

__device__ __forceinline__ long long wadd64(long long a, long long b) {
    return (long long)((unsigned long long)a + (unsigned long long)b);
}
// score_max(cell, im, sm, dm, local) (algo.rs:98-107) with wrapping adds
__device__ __forceinline__ long long smax64(long long I, long long S, long long D, long long im, long long sm,
                                            long long dm, long long floor_) {
    long long r = wadd64(I, im);
    r = max(r, wadd64(S, sm));
    r = max(r, wadd64(D, dm));
    return max(r, floor_);
}
__device__ __forceinline__ long long shfl_up64(long long v) {
    const int lo = __shfl_up((int)(unsigned long long)v, 1, kWave);
    const int hi = __shfl_up((int)((unsigned long long)v >> 32), 1, kWave);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ long long readlane64(long long v, int l) {
    const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned long long)v, l);
    const unsigned hi = __builtin_amdgcn_readlane((int)((unsigned long long)v >> 32), l);
    return (long long)(((unsigned long long)hi << 32) | lo);
}

__global__ __launch_bounds__(64) void fill_wide_kernel(const WideDev* __restrict__ pairs, WideScores sc,
                                                       WideRes* __restrict__ res, int local, int track) {
    const WideDev P = pairs[blockIdx.x];
    const int lane = threadIdx.x;
    const int n = P.n, m = P.m;
    const long long g = sc.g, h = sc.h, hg = wadd64(sc.h, sc.g), ninf = sc.neg_inf;
    const long long floor_ = local ? 0 : LLONG_MIN;
    // first strict max (TRACK, algo.rs:258-262) and last max (local, algo.rs:310-322) over the pair
    long long best = LLONG_MIN, lbest = LLONG_MIN;
    int bi = 0, bj = 0, li = 0, lj = 0, lE = 0;
    unsigned bl = 0;
    for (int s = 0; s < P.strips; ++s) {
        const int i = s * kWave + lane + 1;                  // this lane's row
        const bool row_ok = i <= n;
        // the cell left of the current one: (i, 0) (algo.rs:204-211)
        long long I = ninf, D = wadd64(h, (long long)((unsigned long long)i * (unsigned long long)g)), S = ninf;
        unsigned Lc = 0;                                     // max_matches of the left cell
        int E = -(lane + 1);                                 // reaches column 0 at its own local row
        // top-left (i-1, 0): boundary of column 0 (row 0 for strip 0's lane 0)
        long long smtl;
        if (i - 1 == 0) smtl = smax64(0, 0, 0, 0, 0, 0, floor_);
        else smtl = smax64(ninf, ninf, wadd64(h, (long long)((unsigned long long)(i - 1) * (unsigned long long)g)), 0,
                           0, 0, floor_);
        unsigned ltl = 0;
        int etl = lane == 0 ? 0 : -lane;
        // lane l's outputs for lane l + 1: delete successor, score_max, max_matches, landing column
        long long o_dd = 0, o_sm = 0;
        unsigned o_lm = 0;
        int o_E = 0;
        long long rb_dd = 0, rb_sm = 0;                      // prefetched row above (lane k: column base + k)
        unsigned rb_lm = 0;
        int rb_base = -1000000;
        uint32_t cI = 0, cD = 0;
        const WideRow* above = s > 0 ? P.rows + (size_t)(s - 1) * (m + 1) : nullptr;
        WideRow* below = P.rows + (size_t)s * (m + 1);
        if (lane == 0) P.skel[(size_t)s * P.skel_stride] = 0;   // column 0: E = -64 (+64)
        const int T = m + kWave - 1;
        for (int t = 0; t < T; ++t) {
            // the cell above (i-1, j) from lane l-1's previous step
            long long up_dd = shfl_up64(o_dd), up_sm = shfl_up64(o_sm);
            unsigned up_lm = (unsigned)__shfl_up((int)o_lm, 1, kWave);
            int up_E = __shfl_up(o_E, 1, kWave);
            const int j0 = t + 1;                            // lane 0's column this step
            if (above && (j0 - rb_base >= kWave || j0 < rb_base) && j0 <= m) {
                rb_base = j0;                                // prefetch columns j0 .. j0+63 of the row above
                const int c = j0 + lane;
                if (c <= m) {
                    const WideRow r = above[c];
                    rb_dd = r.dd; rb_sm = r.sm; rb_lm = r.lm;
                }
            }
            if (lane == 0) {
                if (above) {
                    const int k = j0 - rb_base;
                    up_dd = readlane64(rb_dd, k); up_sm = readlane64(rb_sm, k);
                    up_lm = (unsigned)__builtin_amdgcn_readlane((int)rb_lm, k);
                } else {   // row 0: cell (0, j) (algo.rs:213-220)
                    const long long I0 = wadd64(h, (long long)((unsigned long long)j0 * (unsigned long long)g));
                    up_dd = smax64(I0, ninf, ninf, hg, hg, g, floor_);
                    up_sm = smax64(I0, ninf, ninf, 0, 0, 0, floor_);
                    up_lm = 0;
                }
                up_E = j0;                                   // the path leaves through the strip's top row
            }
            const int j = t - lane + 1;
            const bool act = row_ok && j >= 1 && j <= m;
            if (act) {
                const bool mt = P.c1[i - 1] == P.c2[j - 1];  // sequence.rs:113-114 (processed chars)
                const long long In = smax64(I, S, D, g, hg, hg, floor_);        // algo.rs:231-236
                const long long Dn = up_dd;                                     // algo.rs:238-243
                const long long Sn = wadd64(mt ? sc.sm : sc.smm, smtl);         // algo.rs:245-248
                const unsigned Im = Lc, Dm = up_lm, Sm = ltl + (mt ? 1u : 0u);  // algo.rs:250-255
                const long long IS = max(In, Sn);
                const long long SMn = max(max(IS, Dn), floor_);
                const bool m1 = In > Sn, m2 = Dn > IS;        // retrace priority S > I > D (algo.rs:351-400)
                const int En = m2 ? up_E : (m1 ? E : etl);
                const unsigned Ln = max(max(Im, Sm), Dm);
                const int k = (j - 1) & 15;
                cI |= (m1 ? 1u : 0u) << (15 - k);
                cD |= (m2 ? 1u : 0u) << (31 - k);
                if (k == 15 || j == m) {
                    P.codes[((size_t)s * P.t16 + (j - 1) / 16) * kWave + lane] = cI | cD;
                    cI = 0; cD = 0;
                }
                if (P.pI) {
                    const size_t o = (size_t)(i - 1) * m + (j - 1);
                    P.pI[o] = In; P.pD[o] = Dn; P.pS[o] = Sn;
                    if (P.pL) P.pL[o] = Ln;
                }
                if (track && SMn > best) { best = SMn; bi = i; bj = j; bl = Ln; }
                if (local && SMn >= lbest && !(SMn == lbest && i < li)) { lbest = SMn; li = i; lj = j; lE = En; }
                if (i == n && j == m) { res[blockIdx.x].end_SM = SMn; res[blockIdx.x].end_E = En; }
                // outputs for the row below
                o_dd = smax64(In, Sn, Dn, hg, hg, g, floor_);
                o_sm = SMn; o_lm = Ln; o_E = En;
                if (lane == kWave - 1) {
                    below[j] = WideRow{o_dd, o_sm, o_lm, 0};
                    P.skel[(size_t)s * P.skel_stride + j] = En + 64;
                }
                // state for column j + 1: left = this cell, top-left = the cell above
                I = In; D = Dn; S = Sn; Lc = Ln; E = En;
                smtl = up_sm; ltl = up_lm; etl = up_E;
            }
        }
        // the rest of the strip's code words (columns past m), zeroed
        for (int q = (m + 15) / 16; q < P.t16; ++q) P.codes[((size_t)s * P.t16 + q) * kWave + lane] = 0;
        __threadfence();   // the bottom row is read by the next strip (other lanes)
        __builtin_amdgcn_s_waitcnt(0);
    }
    // pair reductions: first max -> the smallest row (then its own first column);
    // last max -> the largest row (then its own last column)
    for (int off = 32; off > 0; off >>= 1) {
        const long long ob = __shfl_xor(best, off), ol = __shfl_xor(lbest, off);
        const int obi = __shfl_xor(bi, off), obj = __shfl_xor(bj, off), oli = __shfl_xor(li, off),
                  olj = __shfl_xor(lj, off), olE = __shfl_xor(lE, off);
        const unsigned obl = (unsigned)__shfl_xor((int)bl, off);
        if (ob > best || (ob == best && obi != 0 && (bi == 0 || obi < bi))) { best = ob; bi = obi; bj = obj; bl = obl; }
        if (ol > lbest || (ol == lbest && oli > li)) { lbest = ol; li = oli; lj = olj; lE = olE; }
    }
    if (lane == 0) {
        WideRes& r = res[blockIdx.x];
        r.max_val = best; r.max_i = bi; r.max_j = bj; r.mam = bl;
        r.lmax_val = lbest; r.lmax_i = li; r.lmax_j = lj; r.lmax_E = lE;
    }
}

// Plane checksums of a wide table (as plane_sums_kernel): one thread per row.
__global__ void wide_plane_sums_kernel(const int64_t* __restrict__ pI, const int64_t* __restrict__ pD,
                                       const int64_t* __restrict__ pS, int n, int m,
                                       unsigned long long* __restrict__ out) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x) + 1;
    unsigned long long a = 0, b = 0, c = 0;
    if (i <= n) {
        const unsigned long long wi = 1ull + (unsigned long long)i * 0x9E3779B1ull;
        const size_t row = (size_t)(i - 1) * m;
        for (int j = 1; j <= m; ++j) {
            const unsigned long long w = wi + (unsigned long long)j * 0x85EBCA77ull;
            a += (unsigned long long)pI[row + j - 1] * w;
            b += (unsigned long long)pD[row + j - 1] * w;
            c += (unsigned long long)pS[row + j - 1] * w;
        }
    }
    for (int o = 32; o >= 1; o >>= 1) {
        a += __shfl_xor(a, o, kWave);
        b += __shfl_xor(b, o, kWave);
        c += __shfl_xor(c, o, kWave);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&out[0], a);
        atomicAdd(&out[1], b);
        atomicAdd(&out[2], c);
    }
}

hipError_t launch_fill_wide(const WideDev* d_pairs, int npairs, WideScores sc, WideRes* d_res, int local, int track,
                            hipStream_t st) {
    if (npairs <= 0) return hipSuccess;
    hipLaunchKernelGGL(fill_wide_kernel, dim3(npairs), dim3(kWave), 0, st, d_pairs, sc, d_res, local, track);
    return hipGetLastError();
}

hipError_t launch_wide_plane_sums(const int64_t* pI, const int64_t* pD, const int64_t* pS, int n, int m,
                                  unsigned long long* out, hipStream_t st) {
    hipError_t e = hipMemsetAsync(out, 0, 3 * sizeof(unsigned long long), st);
    if (e != hipSuccess || n <= 0 || m <= 0) return e;
    hipLaunchKernelGGL(wide_plane_sums_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, pI, pD, pS, n, m, out);
    return hipGetLastError();
}

}  // namespace gx
