// pace_probe: cycles per anti-diagonal step of ONE compute wave running the
// fill's cell arithmetic with no memory, rings or waits (diagnostic; the
// lone-wave "free pace" that sets a single pair's time).  Variants drop
// parts of the step to price them.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I genomics-rs_amd/csrc -o var/pace_probe tools/pace_probe.hip
#include "../genomics-rs_amd/csrc/gx_kernels.hip"
#include <stdio.h>

namespace gx {

// VARIANT 0: full dp_step (codes + E, TBL); 1: no codes/E; 2: rows computed
// but no DPP (lane-local inputs); 3: full step + one 4-step group's worth of
// plane-value packing (as the fill keeps them)
template <int VARIANT>
__global__ __launch_bounds__(64) void pace_kernel(int steps, const Scores32 sc, long long* out, int* sink) {
    const int lane = threadIdx.x;
    LaneState st;
    init_row(st.a, 2 * lane + 1, true, sc);
    init_row(st.b, 2 * lane + 2, true, sc);
    st.c2c = 0;
    st.a.E = -1; st.b.E = -2; st.b.Etl = -1; st.a.Etl = 0;
    const int c1a = score_table(lane & 3, sc), c1b = score_table((lane >> 2) & 3, sc);
    int acc = 0;
    Rec r{0, 0, 0, 0};
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_sched_barrier(0);
    const long long t0 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    for (int t = 0; t < steps; t += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            int oI[2], oD[2], oS[2], oL[2];
            r.c2 = ((t + u) * 7) & 24;     // code * 8
            r.dd = t; r.sm = t;
            if (VARIANT == 1) {
                dp_step<false, false, false, false, true>(st, r, t + u, lane, steps, c1a, c1b, sc, oI, oD, oS, oL);
            } else if (VARIANT == 2) {
                // same arithmetic, inputs from the lane itself (no cross-lane move)
                cell<false, false, true, false, true>(st.a, st.b.Dd, st.b.SM, 0, st.b.E, r.c2, c1a, true, t + u, sc,
                                                      oI[0], oD[0], oS[0], oL[0]);
                cell<false, false, true, false, true>(st.b, st.a.Dd, st.a.SM, 0, st.a.E, r.c2, c1b, true, t + u, sc,
                                                      oI[1], oD[1], oS[1], oL[1]);
            } else {
                dp_step<false, false, true, false, true>(st, r, t + u, lane, steps, c1a, c1b, sc, oI, oD, oS, oL);
            }
            acc += oI[0] ^ oD[1] ^ oS[u & 1];
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    const long long t1 = __builtin_amdgcn_s_memtime();
    sink[lane] = acc ^ st.a.SM ^ st.b.SM ^ (int)st.a.cI ^ (int)st.b.cD ^ st.b.E;
    if (lane == 0) out[0] = t1 - t0;
}

}  // namespace gx

int main() {
    using namespace gx;
    Scores32 sc{1, -2, -1, -5, -6, kNeg, 0, {'A', 'C', 'G', 'T'}};
    long long* d_out;
    int* d_sink;
    (void)hipMalloc(&d_out, 8);
    (void)hipMalloc(&d_sink, 256);
    const int steps = 1 << 16;
    auto run = [&](auto kern, const char* name) {
        long long cyc = 0;
        for (int it = 0; it < 3; ++it) {
            hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, steps, sc, d_out, d_sink);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(&cyc, d_out, 8, hipMemcpyDeviceToHost);
        }
        printf("%-34s %7.1f cycles/step\n", name, (double)cyc / steps);
    };
    run(pace_kernel<0>, "full step (codes + E, table score)");
    run(pace_kernel<1>, "no codes / landing column");
    run(pace_kernel<2>, "full arithmetic, no DPP");
    return 0;
}
