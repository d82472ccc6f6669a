// lcs_step_probe: cycles per step of the LCS sweep's inner loop (gx_lcs.h
// lcs_block4), one wave alone: K0 the asm steps only (masks in registers),
// K1 + one mask buffer load a step (three groups ahead, four sets in
// rotation), K2 + one lane-63 store a step, K3 + a full-wave store a step,
// K4 = K2 with each lane's mask row one of four (as for DNA: scattered
// loads), K5 = K4 + the producer's LDS ring writes and counter each group;
// K6 = K4 with five waves in the workgroup (one SIMD holds two); K7 = K4,
// K8 = K2 and K9 = K0 with four waves (one a SIMD).  Reports
// cycles (s_memtime) and ns (s_memrealtime, 100 MHz) per step.
//   hipcc --offload-arch=gfx950 -O3 -I genomics-rs_amd/csrc -o var/lcs_step_probe tools/lcs_step_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "gx_lcs.h"
using namespace gx;
typedef int v2i __attribute__((ext_vector_type(2)));

template <int K>
__global__ void probe(unsigned long long* masks, unsigned long long* out, long long* cyc, int groups) {
    const int lane = threadIdx.x & 63;
    __shared__ unsigned long long ring[5][264];
    __shared__ int pubc[8];
    const __amdgpu_buffer_rsrc_t mrs = rsrc_of(masks, 1 << 20);
    const __amdgpu_buffer_rsrc_t ors = rsrc_of(out, 1 << 26);
    uint32_t c = 0, vl = ~0u, vh = ~0u;
    v2i mA[8], mB[8], mC[8], mD[8];
    for (int k = 0; k < 8; ++k) {
        mA[k] = v2i{(int)(0x12345 * (lane + k)), k}; mB[k] = mA[k] ^ 5; mC[k] = mA[k] ^ 9; mD[k] = mA[k] ^ 3;
    }
    const uint32_t vb = (uint32_t)(((K >= 4 && K != 8 && K != 9) ? (lane & 3) * 640 : 0) + 64 - lane) * 8u;
    const int wv = threadIdx.x >> 6;
    auto grp = [&](int t0, const v2i (&mc)[8], v2i (&mn)[8]) __attribute__((always_inline)) {
        if (K >= 1 && K != 9) {
#pragma unroll
            for (int k = 0; k < 8; ++k) mn[k] = __builtin_amdgcn_raw_buffer_load_b64(mrs, (int)vb, ((t0 + 24 + k) & 1023) * 8, 0);
        }
        uint32_t ol[8], oh[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint32_t a[4], bh[4], ml[4], mh[4], o1[4], o2[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) { a[k] = ~0u; bh[k] = ~0u; ml[k] = (uint32_t)mc[4 * h + k][0]; mh[k] = (uint32_t)mc[4 * h + k][1]; }
            lcs_block4(a, bh, ml, mh, o1, o2, vl, vh, c);
#pragma unroll
            for (int k = 0; k < 4; ++k) { ol[4 * h + k] = o1[k]; oh[4 * h + k] = o2[k]; }
            vl = o1[3]; vh = o2[3];
        }
        if (K == 5 && lane == 63) {
#pragma unroll
            for (int k = 0; k < 8; ++k) ring[wv][(t0 + k) & 255] = ((unsigned long long)oh[k] << 32) | ol[k];
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            __hip_atomic_store(pubc + wv, t0 + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (K >= 2 && K != 3 && K != 9 && lane == 63) {
#pragma unroll
            for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b64(v2i{(int)ol[k], (int)oh[k]}, ors, 0, ((t0 + k) & 65535) * 8, 0);
        }
        if (K == 3) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                __builtin_amdgcn_raw_buffer_store_b64(v2i{(int)ol[k], (int)oh[k]}, ors, lane * 8, ((t0 + k) & 16383) * 512, 0);
        }
    };
    const long long t0c = clock64();
    const long long r0c = __builtin_amdgcn_s_memrealtime();
    for (int g = 0; g < groups; g += 4) {
        const int t0 = g * 8;
        grp(t0, mA, mD); grp(t0 + 8, mB, mA); grp(t0 + 16, mC, mB); grp(t0 + 24, mD, mC);
    }
    const long long t1c = clock64();
    const long long r1c = __builtin_amdgcn_s_memrealtime();
    out[(1 << 23) + threadIdx.x] = ((unsigned long long)vh << 32) | vl | c;
    if (threadIdx.x == 0) { cyc[0] = t1c - t0c; cyc[1] = r1c - r0c; }
}
int main() {
    unsigned long long *m, *o; long long* c;
    hipMalloc(&m, 1 << 20); hipMalloc(&o, (1 << 26) + (1 << 23) * 8 + 4096); hipMalloc(&c, 16);
    hipMemset(m, 0x5A, 1 << 20);
    const int groups = 4096;
    long long h[2] = {0, 0};
    printf("{");
    for (int k = 0; k <= 9; ++k) {
        for (int rep = 0; rep < 2; ++rep) {
            if (k == 0) hipLaunchKernelGGL(probe<0>, dim3(1), dim3(64), 0, 0, m, o, c, groups);
            if (k == 1) hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, m, o, c, groups);
            if (k == 2) hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64), 0, 0, m, o, c, groups);
            if (k == 3) hipLaunchKernelGGL(probe<3>, dim3(1), dim3(64), 0, 0, m, o, c, groups);
            if (k == 4) hipLaunchKernelGGL(probe<4>, dim3(1), dim3(64), 0, 0, m, o, c, groups);
            if (k == 5) hipLaunchKernelGGL(probe<5>, dim3(1), dim3(64), 0, 0, m, o, c, groups);
            if (k == 6) hipLaunchKernelGGL(probe<6>, dim3(1), dim3(320), 0, 0, m, o, c, groups);
            if (k == 7) hipLaunchKernelGGL(probe<7>, dim3(1), dim3(256), 0, 0, m, o, c, groups);
            if (k == 8) hipLaunchKernelGGL(probe<8>, dim3(1), dim3(256), 0, 0, m, o, c, groups);
            if (k == 9) hipLaunchKernelGGL(probe<9>, dim3(1), dim3(256), 0, 0, m, o, c, groups);
            hipDeviceSynchronize();
        }
        hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
        printf("%s\"K%d\": [%.1f, %.1f]", k ? ", " : "", k, (double)h[0] / (groups * 8), (double)h[1] * 10.0 / (groups * 8));
    }
    printf("}\n");
    return 0;
}
