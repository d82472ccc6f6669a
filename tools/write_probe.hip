// HBM write-stream probe: each wave writes 256-B rows (64 lanes x 4 B) round-robin
// into S private streams, 2 rows per stream per round (the compact-plane fill's
// store pattern: 3 planes x 2 pairs = 6 streams per wave).  Prints one JSON
// line per (S, waves) with the achieved write bandwidth.
//   hipcc --offload-arch=gfx950 -O3 -o tools/write_probe tools/write_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512) void write_streams(unsigned* out, size_t per_stream_words, int S, int rounds) {
    const int lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    unsigned* base = out + wave * S * per_stream_words;
    unsigned v = (unsigned)wave * 2654435761u + lane;
    for (int r = 0; r < rounds; ++r) {
        for (int s = 0; s < S; ++s) {
            unsigned* p = base + s * per_stream_words + (size_t)r * 128;
            p[lane] = v + r;                                 // row A
            p[64 + lane] = v ^ r;                            // row B
        }
        v = v * 1664525u + 1013904223u;
    }
}

int main() {
    const size_t total = 24ull << 30;   // bytes written per launch
    unsigned* d = nullptr;
    if (hipMalloc(&d, total) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int waves_per_cu : {8, 16}) {
        for (int S : {1, 3, 6, 12}) {
            const int blocks = 256 * waves_per_cu / 8;   // 8 waves per block
            const size_t nw = (size_t)blocks * 8;
            const size_t per_stream_words = total / 4 / nw / S / 128 * 128;
            const int rounds = (int)(per_stream_words / 128);
            for (int it = 0; it < 3; ++it) {
                hipEventRecord(a);
                write_streams<<<blocks, 512>>>(d, per_stream_words, S, rounds);
                hipEventRecord(b);
                hipEventSynchronize(b);
            }
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double bytes = (double)nw * S * rounds * 512;
            printf("{\"streams_per_wave\": %d, \"waves_per_cu\": %d, \"GBps\": %.1f, \"ms\": %.3f}\n", S, waves_per_cu,
                   bytes / (ms * 1e-3) / 1e9, ms);
        }
    }
    hipFree(d);
    return 0;
}
