// store_probe: HBM write bandwidth of the fill's store pattern (diagnostic).
// Each wave owns a "strip" and, per 4-step group, stores S streams x 2 rows of
// 1 KiB (16 B per lane) -- the score-plane pattern -- either to S separate
// planes (strip-major per plane, as the fill does) or interleaved in one
// plane (the S x 2 KiB of a group contiguous).  Prints GB/s per layout.
//   hipcc --offload-arch=gfx950 -O3 -o store_probe tools/store_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));

template <int S, bool INTERLEAVED>
__global__ __launch_bounds__(512) void probe(int* base, long long plane_ints, int groups, int strips) {
    const int wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const int lane = threadIdx.x & 63;
    if (wave >= strips) return;
    const long long strip_ints = (long long)groups * 512;   // per plane
    v4i v = {lane, wave, 1, 2};
    for (int g = 0; g < groups; ++g) {
#pragma unroll
        for (int k = 0; k < S; ++k)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                long long o;
                if (INTERLEAVED)
                    o = ((long long)wave * groups + g) * (512LL * S) + k * 512 + h * 256 + lane * 4;
                else
                    o = k * plane_ints + (long long)wave * strip_ints + (long long)g * 512 + h * 256 + lane * 4;
                *(v4i*)(base + o) = v;
                v.z += 1;
            }
    }
}

template <int S, bool IL>
static double run(int* d, long long plane_ints, int groups, int strips, int wpb) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int blocks = (strips + wpb - 1) / wpb;
    for (int it = 0; it < 2; ++it)
        hipLaunchKernelGGL((probe<S, IL>), dim3(blocks), dim3(wpb * 64), 0, 0, d, plane_ints, groups, strips);
    hipEventRecord(a);
    const int reps = 5;
    for (int it = 0; it < reps; ++it)
        hipLaunchKernelGGL((probe<S, IL>), dim3(blocks), dim3(wpb * 64), 0, 0, d, plane_ints, groups, strips);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double bytes = (double)reps * strips * groups * S * 2 * 1024.0;
    return bytes / (ms * 1e-3) / 1e9;
}

int main(int argc, char** argv) {
    const int strips = argc > 1 ? atoi(argv[1]) : 1880;
    const int groups = argc > 2 ? atoi(argv[2]) : 2048;     // 8192 steps
    const long long plane_ints = (long long)strips * groups * 512;
    int* d = nullptr;
    if (hipMalloc(&d, plane_ints * 3 * sizeof(int)) != hipSuccess) { printf("alloc failed\n"); return 1; }
    printf("strips %d groups %d  (%.1f GB per pass)\n", strips, groups, plane_ints * 3 * 4.0 / 1e9);
    for (int wpb : {8, 4}) {
        printf("waves/block %d: 3 planes separate %.0f GB/s | interleaved %.0f GB/s | 1 plane %.0f GB/s\n", wpb,
               run<3, false>(d, plane_ints, groups, strips, wpb), run<3, true>(d, plane_ints, groups, strips, wpb),
               run<1, false>(d, plane_ints, groups, strips, wpb));
    }
    hipFree(d);
    return 0;
}
