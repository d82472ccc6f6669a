// gx_io.h -- the I/O wave of a fill band (gx_kernels.hip fill_kernel, gx_cs2.hip
// fill_cs2_kernel): feeds the band's first LDS ring (row 0, analytic, or the
// previous band's published bottom row from HBM) and drains its last ring to
// HBM for the next band.
#pragma once
#include "gx_device.h"

namespace gx {

#ifndef GX_IO_SLEEP
#define GX_IO_SLEEP 1
#endif
// I/O wave of a band: feeds ring 0 (row 0 analytic, or the previous band's
// published bottom row) and drains ring W to HBM for the next band.
// ADAPT (layout 1, whose strips run a few columns apart): the input side
// moves every published column it can (up to 64 per pass) instead of fixed
// chunks; the output side frees the ring as soon as it has read the records
// and publishes a chunk's progress one pass later, after its stores have
// drained, so a store round trip overlaps the next pass instead of stalling it.
template <bool TBL, int CHUNK, bool ADAPT, int SLEEP>
__device__ void io_wave(const PairDev& P, const int lb, const int lane, const Scores32& sc,
                        Rec* ring0, const Rec* ringW, lds_int* wcnt0, lds_int* rcnt0,
                        lds_int* wcntW, lds_int* rcntW, const bool do_out, int* status) {
    const int m = P.m;
    int in_next = 0, out_next = 0;
    int pend_out = -1;   // ADAPT: columns stored to HBM, progress not yet published
    const Rec* feed_in = lb > 0 ? P.feed + (size_t)(lb - 1) * P.feed_stride : nullptr;
    Rec* feed_out = do_out ? P.feed + (size_t)lb * P.feed_stride : nullptr;
    const int* prog_in = lb > 0 ? P.progress + (size_t)(lb - 1) * kProgStride : nullptr;
    int* prog_out = do_out ? P.progress + (size_t)lb * kProgStride : nullptr;
    unsigned idle = 0;
    while (in_next <= m || (do_out && (out_next <= m || pend_out >= 0))) {
        bool moved = false;
        if (in_next <= m) {
            int chunk;
            bool ok;
            if (ADAPT) {
                int lim = min(m + 1, *rcnt0 + kRing);
                if (lb > 0) lim = min(lim, ld_agent(prog_in));
                chunk = min(lim - in_next, kWave);
                ok = chunk > 0;
            } else {
                chunk = min(CHUNK, m + 1 - in_next);
                ok = in_next + chunk - 1 < *rcnt0 + kRing;
                if (ok && lb > 0) ok = ld_agent(prog_in) > in_next + chunk - 1;
            }
            const int last = in_next + chunk - 1;
            if (ok) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const int j = in_next + lane;
                if (lane < chunk) {
                    Rec r;
                    if (lb == 0) {
                        // row 0 (algo.rs:195-202, 213-220): I = h + j g, D = S = neg_inf
                        if (j == 0) { r.dd = 0; r.sm = 0; r.l = 0; r.c2 = 0; }
                        else {
                            const int I0 = sc.h + j * sc.g;
                            r.dd = max(I0 + sc.hg, sc.floor_);
                            r.sm = max(I0, sc.floor_);
                            if (sc.shift) { r.dd -= (1 + j) * sc.g; r.sm -= j * sc.g; }
                            r.l = 0;
                            r.c2 = TBL ? sym_code(P.c2[j - 1], sc) * 8 : (int)P.c2[j - 1];
                        }
                    } else {
                        r = ld_rec_agent(feed_in + j);
                    }
                    ring0[ring_slot(j)] = r;
                }
                lds_wait();
                if (lane == 0) *wcnt0 = last + 1;
                in_next = last + 1;
                moved = true;
            }
        }
        if (ADAPT && do_out) {
            if (pend_out >= 0) {   // the previous pass's stores: drained -> publish
                vm_wait();
                if (lane == 0) st_agent(prog_out, pend_out);
                pend_out = -1;
                moved = true;
            }
            if (out_next <= m) {
                const int avail = *wcntW;
                const int chunk = min(avail - out_next, kWave);
                if (chunk >= CHUNK || (avail == m + 1 && chunk > 0)) {
                    const int j = out_next + lane;
                    Rec r{};
                    if (lane < chunk) r = ringW[ring_slot(j)];
                    lds_wait();
                    if (lane == 0) *rcntW = out_next + chunk;   // ring slots free again
                    if (lane < chunk) st_rec_agent(feed_out + j, r);
                    out_next += chunk;
                    pend_out = out_next;
                    moved = true;
                }
            }
        } else if (do_out && out_next <= m) {
            const int avail = *wcntW;
            const int chunk = min(CHUNK, avail - out_next);
            if (chunk == CHUNK || (avail == m + 1 && chunk > 0)) {
                const int j = out_next + lane;
                if (lane < chunk) st_rec_agent(feed_out + j, ringW[ring_slot(j)]);
                vm_wait();
                lds_wait();
                if (lane == 0) {
                    *rcntW = out_next + chunk;
                    st_agent(prog_out, out_next + chunk);
                }
                out_next += chunk;
                moved = true;
            }
        }
        if (moved) idle = 0;
        else if (++idle > kSpinLimit ||
                 ((idle & 4095u) == 4095u &&
                  __hip_atomic_load((gint*)status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            __hip_atomic_store((gint*)status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        } else {
            __builtin_amdgcn_s_sleep(SLEEP);
        }
    }
}


}  // namespace gx
