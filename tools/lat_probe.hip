// lat_probe: dependent-chain latency per instruction kind, one wave64 on one
// SIMD, 16-deep unrolled chains (loop overhead amortised).
//   hipcc --offload-arch=gfx950 -O3 -o var/lat_probe tools/lat_probe.hip
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdio>

template <int K>
__device__ __forceinline__ int op(int x, int y) {
    if (K == 0) return x + y;                                                          // v_add
    if (K == 1) return max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x111, 0xF, 0xF, false));   // row_shr:1 max
    if (K == 2) return max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x142, 0xA, 0xF, false));   // row_bcast:15 max
    if (K == 3) return __builtin_amdgcn_update_dpp(y, x, 0x138, 0xF, 0xF, false);                 // wave_shr:1 mov
    if (K == 4) return max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x143, 0xC, 0xF, false));   // row_bcast:31 max
    if (K == 5) return __builtin_amdgcn_update_dpp(y, x, 0x111, 0xF, 0xF, false) + y;             // row_shr:1 mov + add
    return x;
}
template <int K>
__global__ void probe(int* out, long long* cyc, int iters) {
    int x = threadIdx.x, y = threadIdx.x * 3 + 1;
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 16; ++u) x = op<K>(x, y);
    }
    const long long t1 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
template <int K>
static double run(int* d, long long* c, int iters) {
    for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(probe<K>, dim3(1), dim3(64), 0, 0, d, c, iters); (void)hipDeviceSynchronize(); }
    long long h = 0;
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    return (double)h / iters / 16;
}
int main() {
    int* d; long long* c;
    (void)hipMalloc(&d, 256 * 4); (void)hipMalloc(&c, 8);
    const int it = 20000;
    printf("cycles per dependent op: add %.1f | row_shr max %.1f | row_bcast15 max %.1f | bcast31 max %.1f | "
           "wave_shr mov %.1f | row_shr mov+add %.1f\n", run<0>(d, c, it), run<1>(d, c, it), run<2>(d, c, it),
           run<4>(d, c, it), run<3>(d, c, it), run<5>(d, c, it));
    return 0;
}
