// lat_probe2: what a lone wave64 pays per step of the split column step's
// dependent chains (gx_cs2.hip), 16-deep unrolled, one wave on one SIMD:
//   chain kinds: a dependent v_add / v_max chain; a row_shr DPP max chain;
//   the same DPP chain with 1, 2 or 4 independent VALU ops per step (do the
//   wait states hide them?); two independent DPP chains interleaved; a DPP
//   chain with an LDS store per step (push) or per 4 steps.
//   hipcc --offload-arch=gfx950 -O3 -o var/lat_probe2 tools/lat_probe2.hip
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdio>
#include <unistd.h>

__device__ __forceinline__ int dmax(int x) {
    return max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x111, 0xF, 0xF, false));
}

__device__ __forceinline__ int scan64(int x) {
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x111, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x112, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x114, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x118, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x142, 0xA, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x143, 0xC, 0xF, false));
    return x;
}
__device__ __forceinline__ int shr1(int old, int src) {
    return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xF, 0xF, false);
}

// the split column step's core recurrence for one column (gx_cs2.hip
// cs2_core_step, GX_CS2_ASM = 0 form), registers only
__device__ __forceinline__ void core_col(int& I, int& SDh, int& SM, int psm, int dd, int sc, int h, int& out) {
    const int In = max(I, SDh);
    const int Sn = shr1(psm, SM) + sc;
    const int IS = max(In, Sn);
    const int Y = IS + h;
    int Z = shr1(dd, Y);
    Z = scan64(Z);
    SM = max(IS, Z);
    SDh = max(Sn, Z) + h;
    out ^= max(Z, Y);
    I = In;
}
// the side's landing-column chain for one column
__device__ __forceinline__ void side_col(int In, int Sn, int Dn, int t, int kl, int& Ek, unsigned& cI, unsigned& cD) {
    const int IS = max(In, Sn);
    const bool m1 = In > Sn, m2 = Dn > IS;
    const int etl = shr1(t + 64, Ek);
    int key = (int)((((unsigned)(m1 ? Ek : etl)) & 0xFFFFFFu) | (unsigned)kl);
    key = m2 ? t + 65 : key;
    cI = cI + cI + (m1 ? 1u : 0u);
    cD = cD + cD + (m2 ? 1u : 0u);
    Ek = scan64(key);
}

template <int K>
__global__ void probe(int* out, long long* cyc, int iters) {
    __shared__ int lds[1024];
    int x = threadIdx.x, y = threadIdx.x * 3 + 1, z = threadIdx.x * 7 + 5, w = threadIdx.x ^ 9, v = 1, u2 = 2;
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            if (K == 0) x = x + y;                                   // dependent add
            if (K == 1) x = max(x, y) + 1;                           // dependent max + add (2 ops)
            if (K == 2) x = dmax(x);                                 // dependent row_shr max
            if (K == 3) { x = dmax(x); y = y + z; }                  // + 1 independent op
            if (K == 4) { x = dmax(x); y = y + z; w = w ^ v; }       // + 2 independent ops
            if (K == 5) { x = dmax(x); y = y + z; w = w ^ v; z = z - 3; u2 = u2 * 3; }   // + 4
            if (K == 6) { x = dmax(x); y = dmax(y); }                // two independent DPP chains
            if (K == 7) { x = dmax(x); lds[threadIdx.x + 64 * (u & 7)] = x; }            // + LDS store per step
            if (K == 8) { x = dmax(x); if ((u & 3) == 3) lds[threadIdx.x + 64 * (u & 7)] = x; }   // per 4 steps
            if (K == 9) { x = dmax(x); y = dmax(y); z = dmax(z); }   // three chains
            if (K == 10) core_col(x, y, z, w + u, v + u, (u & 3) - 1, -5, u2);          // one core column
            if (K == 11) { unsigned a = (unsigned)y, b = (unsigned)z;                  // one side column
                           side_col(w + u, v - u, u2 + u, it * 16 + u, (threadIdx.x + 1) << 24, x, a, b);
                           y = (int)a; z = (int)b; }
        }
    }
    const long long t1 = clock64();
    out[threadIdx.x] = x + y + z + w + v + u2 + lds[threadIdx.x];
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
// the core column with the kernel's LDS traffic (a record pushed per column,
// four records read per 4 columns), in a workgroup of `nw` waves where waves
// 1.. poll an LDS counter with s_sleep(1) as the kernel's waiting waves do
template <int POLL>
__global__ void probe_wg(int* out, long long* cyc, int iters) {
    __shared__ int ring[4096];
    __shared__ volatile int flag;
    const int wave = threadIdx.x / 64, lane = threadIdx.x & 63;
    if (threadIdx.x == 0) flag = 0;
    __syncthreads();
    if (wave > 0) {
        int seen = 0;
        if (POLL) while (flag == 0) { __builtin_amdgcn_s_sleep(1); ++seen; }
        out[threadIdx.x] = seen;
        return;
    }
    int I = lane, SDh = lane * 3, SM = lane * 7, acc = 0;
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
        int dd[4], sm[4], c2[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) { dd[k] = ring[(it * 4 + k) & 1023]; sm[k] = ring[1024 + ((it * 4 + k) & 1023)]; c2[k] = ring[2048 + k]; }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            int o;
            core_col(I, SDh, SM, sm[u], dd[u], c2[u] & 3, -5, o);
            acc ^= o;
            ring[3072 + lane * 4 + u] = o;   // the push (a lane's own slot)
        }
    }
    const long long t1 = clock64();
    flag = 1;
    out[threadIdx.x] = I + SDh + SM + acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
template <int POLL>
static double run_wg(int* d, long long* c, int iters, int nw) {
    for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(probe_wg<POLL>, dim3(1), dim3(64 * nw), 0, 0, d, c, iters); (void)hipDeviceSynchronize(); }
    long long h = 0;
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    return (double)h / iters / 4;
}

template <int K>
static double run(int* d, long long* c, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int r = 0; r < 2; ++r) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(probe<K>, dim3(1), dim3(64), 0, 0, d, c, iters);
        (void)hipEventRecord(e1, 0);
        (void)hipDeviceSynchronize();
    }
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long h = 0;
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("    [%d: %.2f ns per step real time, %.0f MHz]\n", K, ms * 1e6 / iters / 16, (double)h / (ms * 1e3));
    return (double)h / iters / 16;
}
// one short run (m = 30,000 columns) after the GPU has idled: is the clock
// ramped down for a brief single-wave kernel?
static void cold_run(int* d, long long* c, int reps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int r = 0; r < reps; ++r) {
        usleep(200000);
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(probe<10>, dim3(1), dim3(64), 0, 0, d, c, 30000 / 16);
        (void)hipEventRecord(e1, 0);
        (void)hipDeviceSynchronize();
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        long long h = 0;
        (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        printf("  cold core run %d: %.3f ms, %.1f ns/col, %.1f memtime ticks/col\n", r, ms, ms * 1e6 / 30000, (double)h / 30000);
    }
    for (int r = 0; r < 3; ++r) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(probe<10>, dim3(1), dim3(64), 0, 0, d, c, 30000 / 16);
        (void)hipEventRecord(e1, 0);
        (void)hipDeviceSynchronize();
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        long long h = 0;
        (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        printf("  back-to-back core run %d: %.3f ms, %.1f ns/col, %.1f ticks/col\n", r, ms, ms * 1e6 / 30000, (double)h / 30000);
    }
}

int main() {
    int* d; long long* c;
    (void)hipMalloc(&d, 256 * 4); (void)hipMalloc(&c, 8);
    cold_run(d, c, 3);
    const int it = 20000;
    printf("cycles per step (one wave64):\n");
    printf("  dependent v_add                 %.1f\n", run<0>(d, c, it));
    printf("  dependent v_max + v_add         %.1f\n", run<1>(d, c, it));
    printf("  dependent row_shr DPP max       %.1f\n", run<2>(d, c, it));
    printf("  DPP chain + 1 independent op    %.1f\n", run<3>(d, c, it));
    printf("  DPP chain + 2 independent ops   %.1f\n", run<4>(d, c, it));
    printf("  DPP chain + 4 independent ops   %.1f\n", run<5>(d, c, it));
    printf("  two DPP chains interleaved      %.1f\n", run<6>(d, c, it));
    printf("  three DPP chains interleaved    %.1f\n", run<9>(d, c, it));
    printf("  DPP chain + LDS store per step  %.1f\n", run<7>(d, c, it));
    printf("  DPP chain + LDS store per 4     %.1f\n", run<8>(d, c, it));
    printf("  core column (cs2, registers)    %.1f\n", run<10>(d, c, it));
    printf("  side column (cs2, registers)    %.1f\n", run<11>(d, c, it));
    printf("  core column + LDS, alone         %.1f\n", run_wg<0>(d, c, it / 4, 1));
    printf("  core column + LDS, 4 idle waves  %.1f\n", run_wg<0>(d, c, it / 4, 5));
    printf("  core column + LDS, 4 polling     %.1f\n", run_wg<1>(d, c, it / 4, 5));
    printf("  core column + LDS, 1 polling     %.1f\n", run_wg<1>(d, c, it / 4, 2));
    return 0;
}
