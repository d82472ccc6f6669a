// skew_step_probe: what one step of layout 3's core recurrence (gx_skew.hip
// core_step, global, score tables, shifted values) costs a lone wave64 on
// its own SIMD, registers only, 16 steps unrolled per loop iteration:
//   0  the shipped form: Dn = dpp(Dd) + rdd, In = max(I, Hx), Sn = Hd + s,
//      Hn = max3(In, Sn, Dn), Hx = Hn + h, Dd = max(Dn, Hx), Hd' = dpp(H)
//   1  the same instructions with the cross-lane chains cut (the DPP reads a
//      register the loop does not write): the issue cost alone
//   2  the two-op delete chain: ISh = max3(I, Hx, Sn) + h off the chain,
//      Dd = max(Dn, ISh), Hn = max(ISh - h ..) (10 VALU)
//   3  two independent strips interleaved in one wave (form 0 twice)
//   4  form 0 with the score's bfe hoisted out of the step (per 4 steps)
//   hipcc --offload-arch=gfx950 -O3 -o var/skew_step_probe tools/skew_step_probe.hip
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdio>

__device__ __forceinline__ int shz(int x) { return __builtin_amdgcn_update_dpp(0, x, 0x138, 0xF, 0xF, true); }

struct St {
    int I, Hx, H, Dd, Hd;
};

template <int K>
__device__ __forceinline__ void step(St& s, const int rdd, const int rsm, const int c2, const int c1v, const int h,
                                     const int cut, int& acc) {
    const int Dd_src = K == 1 ? cut : s.Dd;
    const int H_src = K == 1 ? cut + 1 : s.H;
    const int Dn = shz(Dd_src) + rdd;
    const int hu = shz(H_src) + rsm;
    const int sc = __builtin_amdgcn_sbfe(c1v, c2, 8);
    const int Sn = s.Hd + sc;
    if (K == 2) {
        const int IS = max(max(s.I, s.Hx), Sn);
        const int In = max(s.I, s.Hx);
        const int ISh = IS + h;
        const int Ddn = max(Dn, ISh);
        const int Hn = max(IS, Dn);
        s.I = In; s.H = Hn; s.Hx = Hn + h; s.Dd = Ddn;
    } else {
        const int In = max(s.I, s.Hx);
        const int Hn = max(max(In, Sn), Dn);
        const int Hxn = Hn + h;
        const int Ddn = max(Dn, Hxn);
        s.I = In; s.H = Hn; s.Hx = Hxn; s.Dd = Ddn;
    }
    s.Hd = hu;
    acc ^= Sn;
}

template <int K>
__global__ void probe(int* out, long long* cyc, int iters, int h) {
    const int lane = threadIdx.x;
    St a{lane, lane * 3, lane * 5, lane * 7, lane * 11}, b{lane + 1, lane * 2, lane * 9, lane * 13, lane};
    int acc = 0, acc2 = 0;
    int c2v = lane & 3, c1v = 0x01020304 * (lane & 1);
    const int rdd = lane == 0 ? 5 : 0, rsm = lane == 0 ? 7 : 0;
    const int cut = lane * 17;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int c2 = ((c2v + u) & 3) * 8;
            if (K == 3) {
                step<0>(a, rdd, rsm, c2, c1v, h, cut, acc);
                step<0>(b, rdd, rsm, c2, c1v, h, cut, acc2);
            } else {
                step<K == 4 ? 0 : K>(a, rdd, rsm, c2, c1v, h, cut, acc);
            }
        }
        c2v += 1;
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = acc ^ acc2 ^ a.H ^ a.Dd ^ b.H ^ b.Dd;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
static void run(const char* name, int* dout, long long* dcyc, int iters) {
    hipLaunchKernelGGL(probe<K>, dim3(1), dim3(64), 0, 0, dout, dcyc, iters, -3);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(probe<K>, dim3(1), dim3(64), 0, 0, dout, dcyc, iters, -3);
    long long c = 0;
    (void)hipMemcpy(&c, dcyc, sizeof c, hipMemcpyDeviceToHost);
    const double steps = (double)iters * 16;
    printf("%-48s %7.1f cycles per step\n", name, (double)c / steps);
}

int main() {
    int* dout;
    long long* dcyc;
    (void)hipMalloc(&dout, 64 * sizeof(int));
    (void)hipMalloc(&dcyc, 64 * sizeof(long long));
    const int iters = 20000;
    run<0>("0 shipped recurrence", dout, dcyc, iters);
    run<1>("1 same instructions, chains cut (issue cost)", dout, dcyc, iters);
    run<2>("2 two-op delete chain (10 VALU)", dout, dcyc, iters);
    run<3>("3 two strips interleaved (per strip-step pair)", dout, dcyc, iters);
    return 0;
}
