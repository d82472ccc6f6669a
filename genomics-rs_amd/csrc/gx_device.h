// gx_device.h -- device helpers shared by the fill kernels (gx_kernels.hip,
// gx_fill_pk.hip): address-space views, bounded LDS waits, agent-scope record
// loads/stores, ring slots, buffer-descriptor stores, compact-plane byte
// inserts, skeleton stores, lane-63 pushes and the small-alphabet score table.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>
#include "gx_internal.h"

namespace gx {

// Explicit address spaces.  Generic (flat) accesses count on both vmcnt and
// lgkmcnt, so a flat LDS poll would also wait for every outstanding HBM
// store; LDS counters are therefore AS3 and global words AS1.
typedef __attribute__((address_space(1))) int gint;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(3))) volatile int lds_int;

#define DPP_WAVE_SHR1 0x138

__device__ __forceinline__ int shr1(int old, int src) {
    // lane l <- src[l-1]; lane 0 keeps `old` (bound_ctrl off)
    return __builtin_amdgcn_update_dpp(old, src, DPP_WAVE_SHR1, 0xF, 0xF, false);
}
__device__ __forceinline__ int shz(int src) {
    // lane l <- src[l-1]; lane 0 reads 0 (bound_ctrl): shz(x) + y folds into one v_add_u32_dpp
    return __builtin_amdgcn_update_dpp(0, src, DPP_WAVE_SHR1, 0xF, 0xF, true);
}
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }

// Counter reads and writes on a wave's hot path: relaxed workgroup-scope
// atomics rather than volatile accesses, for which the compiler's memory
// legalizer waits (s_waitcnt lgkmcnt(0)) right behind the access -- a
// counter read at a group's start then exposed a full LDS round trip each
// group (layout 3's core wave, ~10 % of a step).  Ordering against the data
// is the writer's: an asm memory barrier between data and counter stores
// (LDS executes one wave's operations in order).
typedef __attribute__((address_space(3))) int lds_plain;
__device__ __forceinline__ int lds_peek(lds_int* p) {
    return __hip_atomic_load((lds_plain*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_post(lds_int* p, int v) {
    __hip_atomic_store((lds_plain*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Trace stamps (GX_TRACE_FILE diagnostics): scalar-memory reads of the clocks.
// They count on lgkmcnt out of order, so a stamp whose result is still in
// flight when an LDS wait comes forces that wait to lgkmcnt(0) -- and the
// compiler carries such an outstanding stamp through the whole strip loop.
// Each stamp is therefore consumed on the spot (the asm use makes the
// compiler wait for it there, on the traced path only).
__device__ __forceinline__ long long stamp_rt() {
    const long long v = __builtin_amdgcn_s_memrealtime();
    asm volatile("" ::"s"(v));
    return v;
}
__device__ __forceinline__ long long stamp_clk() {
    const long long v = __builtin_amdgcn_s_memtime();
    asm volatile("" ::"s"(v));
    return v;
}

__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Every spin is bounded (~2^25 sleeps, seconds): on expiry the wave records a
// timeout in *status and carries on, so the grid always drains; the host
// turns a non-zero status into GX_EHIP.
constexpr unsigned kSpinLimit = 1u << 25;

// A wave that has spun 2^12 times also checks the status word: once any
// wave of the launch has timed out, every other waiting wave gives up at once
// and the grid drains in about one spin limit instead of one per wait.
__device__ __forceinline__ unsigned wait_ge(lds_int* p, int v, int* status) {
    unsigned it = 0;
    for (; *p < v; ++it) {
        if (it > kSpinLimit) { __hip_atomic_store((gint*)status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
        if ((it & 4095u) == 4095u && __hip_atomic_load((gint*)status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
        __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
    return it;
}

// The same without the sleep between polls, for a wave alone on its SIMD
// whose wait is on the critical path (layout 3's strip input): a poll is an
// LDS round trip already, and s_sleep 1 adds 64 cycles to each.
__device__ __forceinline__ unsigned wait_ge_tight(lds_int* p, int v, int* status) {
    unsigned it = 0;
    for (; *p < v; ++it) {
        if (it > 4 * kSpinLimit) { __hip_atomic_store((gint*)status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
        if ((it & 16383u) == 16383u && __hip_atomic_load((gint*)status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    }
    asm volatile("" ::: "memory");
    return it;
}

__device__ __forceinline__ int ld_agent(const int* p) {
    return __hip_atomic_load((gint*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(int* p, int v) {
    __hip_atomic_store((gint*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ Rec ld_rec_agent(const Rec* p) {
    const gu64* q = (const gu64*)p;
    unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    Rec r;
    r.dd = (int)(a & 0xffffffffu); r.sm = (int)(a >> 32);
    r.l = (int)(b & 0xffffffffu);  r.c2 = (int)(b >> 32);
    return r;
}
__device__ __forceinline__ void st_rec_agent(Rec* p, Rec r) {
    gu64* q = (gu64*)p;
    __hip_atomic_store(q, (unsigned long long)(unsigned)r.dd | ((unsigned long long)(unsigned)r.sm << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, (unsigned long long)(unsigned)r.l | ((unsigned long long)(unsigned)r.c2 << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Ring slot of column c.  The producer pushes column c at step c + 63 and the
// consumer reads it at step c - 1, so with 16-step sub-blocks both touch 16
// consecutive, 16-aligned slots per sub-block (constant LDS offsets).
__device__ __forceinline__ int ring_slot(int c) { return (c + 15) & (kRing - 1); }

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)p;   // low 32 bits of a generic LDS address = LDS offset
}

// Global-address-space views: stores through them compile to global_store
// (counted on vmcnt only).  Through a generic pointer they become flat_store,
// which also counts on lgkmcnt and makes every LDS wait wait for HBM stores.
typedef int v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4i gv4i;
typedef __attribute__((address_space(1))) uint32_t guint;
__device__ __forceinline__ void gstore4(int32_t* p, int4 v) {
    v4i x = {v.x, v.y, v.z, v.w};
    *(gv4i*)p = x;
}
__device__ __forceinline__ void gstore1(uint32_t* p, uint32_t v) { *(guint*)p = v; }
#ifndef GX_PLANE_AUX
#define GX_PLANE_AUX 2   // nt: the planes are written once and never read back here
#endif
// Plane stores: one 16-B store per lane through a buffer descriptor of the
// sub-block (uniform base, per-lane offset + immediate; the compiler places
// the wait states for the SGPR operands).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
__device__ __forceinline__ void bstore4(__amdgpu_buffer_rsrc_t r, uint32_t voff, int4 v) {
#ifndef GX_DIAG_NO_PLANES
    v4i x = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(x, r, (int)voff, 0, GX_PLANE_AUX);
#endif
}

// Compact planes (plane mode 3, layout 0, global untracked launches whose
// scores pass the host's range proof, gx_api_plan.cpp d8_planes_ok): per cell one
// signed byte each of
//     x_I = I(i,j) - I(i,j-1),  x_S = S(i,j) - I(i,j),  x_D = D(i,j) - I(i,j)
// in the int32 plane layout with bytes for ints (4 steps of a row = one dword
// per lane).  The decoder (export_d8_kernel) rebuilds a row with one running
// sum.  put_byte<K> writes (a - b) into byte K of acc in one VALU op (SDWA,
// other bytes preserved; byte 0 clears the rest).
template <int K>
__device__ __forceinline__ void put_byte(uint32_t& acc, int a, int b) {
    if constexpr (K == 0)
        asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD"
            : "=v"(acc) : "v"(a), "v"(b));
    else if constexpr (K == 1)
        asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
            : "+v"(acc) : "v"(a), "v"(b));
    else if constexpr (K == 2)
        asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
            : "+v"(acc) : "v"(a), "v"(b));
    else
        asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
            : "+v"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void bstore1(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t v) {
#if defined(GX_DIAG_SINK_PLANES)
    asm volatile("" ::"v"(v));   // (timing only) the bytes are computed, not stored
#elif !defined(GX_DIAG_NO_PLANES)
    __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)voff, 0, GX_PLANE_AUX);
#endif
}

// Occupancy floor (waves per SIMD), which sets the fill kernel's VGPR cap
// (512 / floor, at most 256): one workgroup per CU, so the floor is the
// workgroup's waves per SIMD.  The variants that also track the maxima
// (first max + LCS, local mode) carry more state per row and get 256 VGPRs
// (8-wave workgroups at most).

// Skeleton stores of lane 63's landing columns through a buffer descriptor:
// every lane issues them, the other lanes' offsets lie past the descriptor's
// range (kSkelOff) and are dropped by the range check -- no exec switch.
// Full groups store their four columns at once; ramp groups one per step.
constexpr uint32_t kSkelOff = 0x40000000u;
// (GX_DIAG_* builds drop a kind of store, for timing only: tools/strip_pace.py)
__device__ __forceinline__ void skel_store(__amdgpu_buffer_rsrc_t r, uint32_t voff, int E) {
#ifndef GX_DIAG_NO_SKEL
    __builtin_amdgcn_raw_buffer_store_b32(E, r, (int)voff, 0, 0);
#endif
}
__device__ __forceinline__ void skel_store4(__amdgpu_buffer_rsrc_t r, uint32_t voff, int e0, int e1, int e2, int e3) {
#ifndef GX_DIAG_NO_SKEL
    v4i x = {e0, e1, e2, e3};
    __builtin_amdgcn_raw_buffer_store_b128(x, r, (int)voff, 0, 0);
#endif
}

constexpr int kPushScratch = 128;   // uint32 per wave: 64 lanes x 4 B + a sub-block's record offsets (252 B)

// ... and the ring's write counter (lane 63: the counter; others: scratch)
__device__ __forceinline__ void publish_all(uint32_t caddr, int cnt) {
    asm volatile("ds_write_b32 %0, %1" : : "v"(caddr), "v"(cnt) : "memory");
}

// A wave-uniform pointer forced into an SGPR pair (for "s" asm operands).
__device__ __forceinline__ const int* uniform_ptr(const int* p) {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (const int*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

// exec mask selecting lane 63 (or no lane), forced into an SGPR pair: the
// "s" asm operand of the pushes must not be given a VGPR.
__device__ __forceinline__ unsigned long long lane63_mask(bool on) {
    return (unsigned long long)__builtin_amdgcn_readfirstlane(on ? 0x80000000u : 0u) << 32;
}

// One lane stores an LDS counter (exec = lane 0 only, no branch).
__device__ __forceinline__ void lds_store_lane0(lds_int* p, int v) {
    asm volatile(
        "s_mov_b64 exec, 1\n\t"
        "ds_write_b32 %0, %1\n\t"
        "s_mov_b64 exec, -1"
        :
        : "v"((uint32_t)(uintptr_t)p), "v"(v)
        : "memory");
}

// in-place inclusive prefix max over the 64 lanes (lanes without a DPP source
// keep their value: old = INT_MIN is the identity of max)
template <int CTRL, int RM, int BM>
__device__ __forceinline__ int dpp_max(int x) {
    return max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, CTRL, RM, BM, false));
}
__device__ __forceinline__ int scan_max64(int x) {
    x = dpp_max<0x111, 0xF, 0xF>(x);   // row_shr:1
    x = dpp_max<0x112, 0xF, 0xF>(x);   // row_shr:2
    x = dpp_max<0x114, 0xF, 0xF>(x);   // row_shr:4
    x = dpp_max<0x118, 0xF, 0xF>(x);   // row_shr:8
    x = dpp_max<0x142, 0xA, 0xF>(x);   // row_bcast:15 -> rows 1, 3
    x = dpp_max<0x143, 0xC, 0xF>(x);   // row_bcast:31 -> rows 2, 3
    return x;
}

// Interleaved scans: independent chains side by side, so each DPP step's
// latency (~14 cycles on a dependent chain, tools/dpp_probe.hip) is covered
// by the other chain's step instead of wait states.
template <int CTRL, int RM, int BM, int N>
__device__ __forceinline__ void dpp_max_n(int (&x)[N]) {
#pragma unroll
    for (int q = 0; q < N; ++q) x[q] = dpp_max<CTRL, RM, BM>(x[q]);
}
template <int N>
__device__ __forceinline__ void scan_max64_n(int (&x)[N]) {
    dpp_max_n<0x111, 0xF, 0xF>(x);
    dpp_max_n<0x112, 0xF, 0xF>(x);
    dpp_max_n<0x114, 0xF, 0xF>(x);
    dpp_max_n<0x118, 0xF, 0xF>(x);
    dpp_max_n<0x142, 0xA, 0xF>(x);
    dpp_max_n<0x143, 0xC, 0xF>(x);
}

// Small-alphabet scoring (TBL): the host maps the job's <= 4 distinct
// processed bytes to codes 0..3 (Scores32.sym); a row's table holds
// score(c1, sym[k]) as signed byte k.
__device__ __forceinline__ int sym_code(int c, const Scores32& sc) {
    return c == sc.sym[1] ? 1 : c == sc.sym[2] ? 2 : c == sc.sym[3] ? 3 : 0;
}
__device__ __forceinline__ int score_table(int c1, const Scores32& sc) {
    int t = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) t |= ((c1 == sc.sym[k] ? sc.sm : sc.smm) & 0xFF) << (8 * k);
    return t;
}

// The ring pointers are deliberately NOT __restrict__: another wave writes the
// ring, and with noalias the compiler may fold the re-read after a wait into
// the earlier speculative read of the same slots (stale records).
__device__ __forceinline__ void read4(Rec (&r)[4], const Rec* rin) {
    r[0] = rin[0]; r[1] = rin[1]; r[2] = rin[2]; r[3] = rin[3];
}

// record pushes with explicit values (all lanes write: lane 63 to the ring,
// the others to scratch; or exec-masked to lane 63 in the tail)
template <int U, bool TRACK>
__device__ __forceinline__ void cs_push_all(uint32_t vaddr, int dd, int sm, int c2, int l) {
    if (TRACK)
        asm volatile(
            "ds_write2_b32 %0, %1, %2 offset0:%5 offset1:%6\n\t"
            "ds_write2_b32 %0, %3, %4 offset0:%7 offset1:%8"
            :
            : "v"(vaddr), "v"(dd), "v"(sm), "v"(c2), "v"(l), "i"(4 * U), "i"(4 * U + 1), "i"(4 * U + 2),
              "i"(4 * U + 3)
            : "memory");
    else
        asm volatile(
            "ds_write2_b32 %0, %1, %2 offset0:%4 offset1:%5\n\t"
            "ds_write_b32 %0, %3 offset:%6"
            :
            : "v"(vaddr), "v"(dd), "v"(sm), "v"(c2), "i"(4 * U), "i"(4 * U + 1), "i"(16 * U + 8)
            : "memory");
}
template <int U, bool TRACK>
__device__ __forceinline__ void cs_push63(uint32_t base, unsigned long long m63, int dd, int sm, int c2, int l) {
    if (TRACK)
        asm volatile(
            "s_mov_b64 exec, %0\n\t"
            "ds_write2_b32 %1, %2, %3 offset0:%6 offset1:%7\n\t"
            "ds_write2_b32 %1, %4, %5 offset0:%8 offset1:%9\n\t"
            "s_mov_b64 exec, -1"
            :
            : "s"(m63), "v"(base), "v"(dd), "v"(sm), "v"(c2), "v"(l), "i"(4 * U), "i"(4 * U + 1), "i"(4 * U + 2),
              "i"(4 * U + 3)
            : "memory");
    else
        asm volatile(
            "s_mov_b64 exec, %0\n\t"
            "ds_write2_b32 %1, %2, %3 offset0:%5 offset1:%6\n\t"
            "ds_write_b32 %1, %4 offset:%7\n\t"
            "s_mov_b64 exec, -1"
            :
            : "s"(m63), "v"(base), "v"(dd), "v"(sm), "v"(c2), "i"(4 * U), "i"(4 * U + 1), "i"(16 * U + 8)
            : "memory");
}

constexpr uint32_t kNoStore = 0xFFFFFFF0u;   // past every strip plane's range: the store is dropped

// Twin plane codes, 12 bits a cell.  The fill computes each
// step's dword d_k = code_A | code_B << 16 (the twin's two pairs; a code is
// x_S + 32 x_D mod 2^16, of which the low 12 bits decode exactly while x_D
// fits 7 signed bits).  A lane's four steps of one row pack into 12 B:
//   w0 = the codes' low bytes of steps 0, 1 [A0, B0, A1, B1]
//   w1 = those of steps 2, 3                [A2, B2, A3, B3]
//   w2 = the high nibbles: byte k = nibble of w0's byte k | nibble of w1's byte k << 4
// four v_perm_b32, a shift and a v_bfi_b32 (1.5 B a cell instead of 2: the
// plane stores were a third of the headline fill's time).
__device__ __forceinline__ void w12_pack(const uint32_t d0, const uint32_t d1, const uint32_t d2, const uint32_t d3,
                                         uint32_t& w0, uint32_t& w1, uint32_t& w2) {
    w0 = __builtin_amdgcn_perm(d1, d0, 0x06040200u);
    w1 = __builtin_amdgcn_perm(d3, d2, 0x06040200u);
    const uint32_t n01 = __builtin_amdgcn_perm(d1, d0, 0x07050301u), n23 = __builtin_amdgcn_perm(d3, d2, 0x07050301u);
    w2 = (n01 & 0x0F0F0F0Fu) | ((n23 << 4) & 0xF0F0F0F0u);
}
// The four steps' dwords (code_A | code_B << 16, 12 bits each) of a record.
__device__ __forceinline__ uint4 w12_unpack(const uint32_t w0, const uint32_t w1, const uint32_t w2) {
    const uint32_t n = (w2 >> 4) & 0x0F0F0F0Fu;
    uint4 d;
    d.x = __builtin_amdgcn_perm(w2, w0, 0x05010400u) & 0x0FFF0FFFu;
    d.y = __builtin_amdgcn_perm(w2, w0, 0x07030602u) & 0x0FFF0FFFu;
    d.z = __builtin_amdgcn_perm(n, w1, 0x05010400u);
    d.w = __builtin_amdgcn_perm(n, w1, 0x07030602u);
    return d;
}
// A record at `rec` (4-byte aligned, global memory).
__device__ __forceinline__ uint4 w12_load(const uint8_t* rec) {
    const __attribute__((address_space(1))) uint32_t* p = (const __attribute__((address_space(1))) uint32_t*)rec;
    return w12_unpack(p[0], p[1], p[2]);   // (one global_load_dwordx3)
}
// Byte offset of the record of row-in-strip rho (lane rho / 2, row-in-lane
// rho % 2) in 4-step group G of strip s, for strips of t4 groups.
__device__ __forceinline__ size_t w12_rec_off(const int s, const int t4, const int G, const int rho) {
    return ((size_t)s * t4 + G) * kTwinGroupBytes + (size_t)(rho & 1) * (kTwinGroupBytes / 2) + (size_t)(rho >> 1) * kTwinRec;
}

}  // namespace gx
