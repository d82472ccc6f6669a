// valu_probe.hip -- VALU issue rate of one MI355X SIMD at 1, 2, 4 and 8 waves
// per SIMD, for the integer instruction forms the DP fill issues (v_add_u32,
// v_max_i32, v_max3_i32, DPP row_shr, SDWA byte insert, v_cndmask_b32).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_probe tools/valu_probe.hip
//   tools/valu_probe > profiles/valu_probe_r02.json
//
// Each wave runs 8 independent chains (no dependent-issue stalls) of one
// instruction form, ITERS x 16 x 8 instructions, bracketed by s_memtime
// (shader clock) and s_memrealtime (100 MHz).  A 256-thread workgroup puts one
// wave on each of a CU's 4 SIMDs; a grid of k x (CUs) workgroups puts k waves
// on every SIMD.  cycles per wave64 instruction per SIMD = (median wave
// cycles) / (instructions per wave x k) -- if a SIMD issued one wave64 op per
// 2 cycles (32 lanes per cycle) this would fall to 2 from k = 2 on.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int kIters = 256;
constexpr int kUnroll = 16;
constexpr int kChains = 8;

enum Op { ADD, MAX, MAX3, DPP, SDWA, CNDMASK, SUB, ADDC, BFE, PK_MAX, PK_ADD, PK_SUB, BFI, MOV_DPP, ADD3, MIX_ADD_MAX,
          CMP, MOV, NOPS };
static const char* kNames[] = {"v_add_u32", "v_max_i32", "v_max3_i32", "v_max_i32_dpp row_shr:1",
                               "v_sub_u32_sdwa dst_sel:BYTE_1", "v_cndmask_b32", "v_sub_u32", "v_addc_co_u32",
                               "v_bfe_i32", "v_pk_max_i16", "v_pk_add_u16", "v_pk_sub_i16", "v_bfi_b32",
                               "v_mov_b32_dpp wave_shr:1", "v_add3_u32", "v_add_u32 + v_max_i32 alternating",
                               "v_cmp_gt_i32 (SGPR-pair dst)", "v_mov_b32"};

template <int OP>
__device__ __forceinline__ void step(int& a, int b, int c, unsigned long long msk) {
    if constexpr (OP == ADD) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == MAX) asm volatile("v_max_i32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == MAX3) asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    // DPP source b is never written inside the loop: no VALU-write -> DPP-read hazard
    if constexpr (OP == DPP) asm volatile("v_max_i32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a) : "v"(b));
    if constexpr (OP == SDWA)
        asm volatile("v_sub_u32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
                     : "+v"(a) : "v"(b), "v"(c));
    if constexpr (OP == CNDMASK) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(msk));
    if constexpr (OP == SUB) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == ADDC) {
        unsigned long long k;
        asm volatile("v_addc_co_u32 %0, %1, %0, %0, %2" : "+v"(a), "=s"(k) : "s"(msk));
    }
    if constexpr (OP == BFE) asm volatile("v_bfe_i32 %0, %1, %0, 8" : "+v"(a) : "v"(b));
    if constexpr (OP == PK_MAX) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == PK_ADD) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == PK_SUB) asm volatile("v_pk_sub_i16 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (OP == BFI) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (OP == MOV_DPP) asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a) : "v"(b));
    if constexpr (OP == ADD3) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (OP == MOV) asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(b));
    if constexpr (OP == CMP) {
        unsigned long long k;
        asm volatile("v_cmp_gt_i32 %0, %1, %2" : "=s"(k) : "v"(a), "v"(b));
        asm volatile("" :: "s"(k));
    }
}
template <>
__device__ __forceinline__ void step<MIX_ADD_MAX>(int& a, int b, int c, unsigned long long msk) {
    asm volatile("v_add_u32 %0, %0, %1\n\tv_max_i32 %0, %0, %2" : "+v"(a) : "v"(b), "v"(c));
}

template <int OP>
__global__ __launch_bounds__(256) void probe(long long* __restrict__ cyc, long long* __restrict__ rt,
                                             int* __restrict__ sink, int seed) {
    int a[kChains];
#pragma unroll
    for (int k = 0; k < kChains; ++k) a[k] = (int)threadIdx.x * (k + 3) + seed;
    const int b = seed ^ (int)threadIdx.x, c = seed + 7;
    const unsigned long long msk = 0x5555555555555555ull ^ (unsigned long long)seed;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
            for (int k = 0; k < kChains; ++k) step<OP>(a[k], b, c, msk);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    int acc = 0;
#pragma unroll
    for (int k = 0; k < kChains; ++k) acc ^= a[k];
    const int w = (int)(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
    if ((threadIdx.x & 63) == 0) {
        cyc[w] = t1 - t0;
        rt[w] = r1 - r0;
    }
    if (acc == 0x7fffffff) sink[0] = acc;   // keeps the chains live
}

template <int OP>
static void run(int cus, int k, bool first) {
    const int blocks = cus * k, waves = blocks * 4;
    long long *dc, *dr;
    int* ds;
    (void)hipMalloc(&dc, waves * sizeof(long long));
    (void)hipMalloc(&dr, waves * sizeof(long long));
    (void)hipMalloc(&ds, 64);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, dc, dr, ds, 1);   // warm-up
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, dc, dr, ds, 3);
    (void)hipEventRecord(e1, 0);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> c(waves), r(waves);
    (void)hipMemcpy(c.data(), dc, waves * sizeof(long long), hipMemcpyDeviceToHost);
    (void)hipMemcpy(r.data(), dr, waves * sizeof(long long), hipMemcpyDeviceToHost);
    std::vector<long long> cs = c;
    std::sort(cs.begin(), cs.end());
    const double med = (double)cs[cs.size() / 2], mx = (double)cs.back();
    double clk = 0;   // shader clock from the two timers (GHz)
    for (int w = 0; w < waves; ++w) clk += (double)c[w] / ((double)r[w] * 10.0);
    clk /= waves;
    const double insts = (double)kIters * kUnroll * kChains * (OP == MIX_ADD_MAX ? 2 : 1);
    // chip-wide: all waves' instructions over the kernel's wall time and every SIMD
    const double chip_cpi = (ms * 1e-3 * clk * 1e9) * (cus * 4) / (insts * waves);
    printf("%s{\"op\": \"%s\", \"waves_per_simd\": %d, \"insts_per_wave\": %.0f, \"median_wave_cycles\": %.0f, "
           "\"max_wave_cycles\": %.0f, \"cycles_per_inst_per_simd\": %.3f, \"cycles_per_inst_one_wave_view\": %.3f, "
           "\"chip_cycles_per_inst_per_simd\": %.3f, \"kernel_ms\": %.4f, \"clock_ghz\": %.3f}",
           first ? "  " : ",\n  ", kNames[OP], k, insts, med, mx, med / (insts * k), med / insts, chip_cpi, ms, clk);
    (void)hipFree(dc);
    (void)hipFree(dr);
    (void)hipFree(ds);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

template <int OP>
static void sweep(int cus, bool& first) {
    for (int k : {1, 2, 4, 8}) {
        run<OP>(cus, k, first);
        first = false;
    }
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    printf("{\"device\": \"%s\", \"cus\": %d, \"probe\": \"tools/valu_probe.hip\", \"results\": [\n", prop.gcnArchName, cus);
    bool first = true;
    sweep<ADD>(cus, first);
    sweep<MAX>(cus, first);
    sweep<MAX3>(cus, first);
    sweep<DPP>(cus, first);
    sweep<SDWA>(cus, first);
    sweep<CNDMASK>(cus, first);
    sweep<SUB>(cus, first);
    sweep<ADDC>(cus, first);
    sweep<BFE>(cus, first);
    sweep<PK_MAX>(cus, first);
    sweep<PK_ADD>(cus, first);
    sweep<PK_SUB>(cus, first);
    sweep<BFI>(cus, first);
    sweep<MOV_DPP>(cus, first);
    sweep<ADD3>(cus, first);
    sweep<MIX_ADD_MAX>(cus, first);
    sweep<CMP>(cus, first);
    sweep<MOV>(cus, first);
    printf("\n]}\n");
    return 0;
}
