// dpp_probe: cycles per wave64 prefix-max scan (6 DPP v_max steps), one wave
// per SIMD: a single dependent chain vs two or three independent chains
// interleaved (diagnostic for the column-step fill's per-column latency).
//   hipcc --offload-arch=gfx950 -O3 -o var/dpp_probe tools/dpp_probe.hip
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdio>

template <int CTRL, int RM, int BM>
__device__ __forceinline__ int dpp_max(int x) {
    return max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, CTRL, RM, BM, false));
}
__device__ __forceinline__ int scan(int x) {
    x = dpp_max<0x111, 0xF, 0xF>(x);
    x = dpp_max<0x112, 0xF, 0xF>(x);
    x = dpp_max<0x114, 0xF, 0xF>(x);
    x = dpp_max<0x118, 0xF, 0xF>(x);
    x = dpp_max<0x142, 0xA, 0xF>(x);
    x = dpp_max<0x143, 0xC, 0xF>(x);
    return x;
}
// the landing-column chain of one column (layout 1): E(t) from E(t-1) and the
// column's code bits (ib, db per lane)
__device__ __forceinline__ int e_step(int E, int t, int ib, int db, int kl) {
    const int etl = __builtin_amdgcn_update_dpp(t, E, 0x138, 0xF, 0xF, false);
    int key = ib ? E : etl;
    key = (key + 64) | kl;
    key = db ? -1 : key;
    key = scan(key);
    return key < 0 ? t + 1 : (key & 0x1FFFFFF) - 64;
}
template <int K>
__global__ void probe(int* out, long long* cyc, int iters) {
    int x = threadIdx.x, y = threadIdx.x * 3, z = threadIdx.x * 5, u = threadIdx.x * 7;
    const long long t0 = clock64();
    const int kl = (int)threadIdx.x << 25;
    const unsigned bits = 0x9E3779B9u * (threadIdx.x + 1);
    for (int it = 0; it < iters; ++it) {
        if (K == 7) { x = __builtin_amdgcn_update_dpp(y, x, 0x138, 0xF, 0xF, false) + 1; continue; }   // wave_shr:1
        if (K == 8) { x = __builtin_amdgcn_update_dpp(y, x, 0x111, 0xF, 0xF, false) + 1; continue; }   // row_shr:1
        if (K == 9) { x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x142, 0xA, 0xF, false)) + 1; continue; }  // row_bcast:15
        if (K == 10) { x = (x ^ y) + 1; x = max(x, y) + 3; continue; }   // four dependent plain VALU
        if (K == 5 || K == 6) {
            const int ib = (bits >> (it & 31)) & 1, db = (bits >> ((it + 7) & 31)) & (threadIdx.x & 1);
            x = e_step(x, it, ib, db, kl);
            if (K == 6) y = e_step(y, it, db, ib, kl);
            continue;
        }
        if (K == 0) { x = x + 1; x = max(x, y); }                       // plain dependent VALU pair
        if (K >= 1) x = scan(x) + 1;
        if (K >= 2) y = scan(y) + 1;
        if (K >= 3) z = scan(z) + 1;
        if (K >= 4) u = scan(u) + 1;
    }
    const long long t1 = clock64();
    out[threadIdx.x] = x + y + z + u;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
    int* d; long long* c;
    hipMalloc(&d, 256 * 4); hipMalloc(&c, 8);
    const int iters = 100000;
    for (int k = 0; k <= 10; ++k) {
        for (int rep = 0; rep < 2; ++rep) {
            if (k == 0) hipLaunchKernelGGL(probe<0>, dim3(1), dim3(64), 0, 0, d, c, iters);
            if (k == 1) hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, d, c, iters);
            if (k == 2) hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64), 0, 0, d, c, iters);
            if (k == 3) hipLaunchKernelGGL(probe<3>, dim3(1), dim3(64), 0, 0, d, c, iters);
            if (k == 4) hipLaunchKernelGGL(probe<4>, dim3(1), dim3(64), 0, 0, d, c, iters);
            if (k == 5) hipLaunchKernelGGL(probe<5>, dim3(1), dim3(64), 0, 0, d, c, iters);
            if (k == 6) hipLaunchKernelGGL(probe<6>, dim3(1), dim3(64), 0, 0, d, c, iters);
            if (k == 7) hipLaunchKernelGGL(probe<7>, dim3(1), dim3(64), 0, 0, d, c, iters);
            if (k == 8) hipLaunchKernelGGL(probe<8>, dim3(1), dim3(64), 0, 0, d, c, iters);
            if (k == 9) hipLaunchKernelGGL(probe<9>, dim3(1), dim3(64), 0, 0, d, c, iters);
            if (k == 10) hipLaunchKernelGGL(probe<10>, dim3(1), dim3(64), 0, 0, d, c, iters);
            hipDeviceSynchronize();
        }
        long long h = 0;
        hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        if (k <= 4)
            printf("chains %d: %.1f cycles per iteration (%.1f per scan)\n", k, (double)h / iters,
                   k ? (double)h / iters / k : 0.0);
        else if (k <= 6)
            printf("landing-column chain x%d: %.1f cycles per column\n", k - 4, (double)h / iters);
        else
            printf("probe %d (7 wave_shr mov+add, 8 row_shr mov+add, 9 bcast max+add, 10 4 plain): %.1f cycles\n", k,
                   (double)h / iters);
    }
    return 0;
}
