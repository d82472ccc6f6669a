// gx_api_batch.cpp -- batches of independent pairs (BASELINE configs 4 / 5):
// one-pass and pipelined multi-pass batches, the overlapped two-group
// pipeline, gx_align_batch and the multi-context gx_align_batch_multi.
#include "gx_api.h"

// A batch through the int64 fill (jobs outside the exact-int32 range): fill,
// host start cells, device traceback, host labelling.  Synchronous, one pass.
int batch_core_wide(gx_context* ctx, const std::vector<PairHost>& ph,
                    const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc, const HostScores& hs,
                    int is_local, bool planes, bool track, std::vector<Walk>& walks, double* fill_ms) {
    const size_t P = ph.size();
    std::vector<size_t> idx;
    for (size_t p = 0; p < P; ++p) if (ph[p].n >= 1 && ph[p].m >= 1) idx.push_back(p);
    std::vector<PairHost> dph;
    std::vector<std::pair<const uint8_t*, const uint8_t*>> dproc;
    for (size_t p : idx) { dph.push_back(ph[p]); dproc.push_back(proc[p]); }
    FillJob job;
    std::vector<PairRes> res(P, PairRes{});
    std::vector<StartIn> sin(P, StartIn{0, 0, 0, 0});
    std::vector<uint64_t> si(P), sj(P);
    std::vector<int64_t> score(P);
    TbOut& tb = ctx->tb_cache;
    tb.ms = 0;
    int rc = GX_OK;
    if (!idx.empty()) {
        rc = run_fill_wide(ctx, dproc, dph, hs, is_local, planes, track, false, job);
        if (rc) { job_release(ctx, job); return rc; }
        for (size_t k = 0; k < idx.size(); ++k) { res[idx[k]] = job.res[k]; sin[idx[k]] = start_in(job, k); }
    }
    for (size_t p = 0; p < P; ++p) start_cell_common(hs, is_local, ph[p].n, ph[p].m, sin[p], &si[p], &sj[p], &score[p]);
    if (!idx.empty()) {
        std::vector<TbStart> starts(idx.size());
        for (size_t k = 0; k < idx.size(); ++k) {
            const size_t p = idx[k];
            starts[k] = (si[p] >= 1 && sj[p] >= 1)
                            ? TbStart{(int)si[p], (int)sj[p], is_local ? res[p].lmax_E : res[p].end_E}
                            : TbStart{0, 0, 0};
        }
        rc = run_traceback(ctx, job, starts, tb);
    }
    if (fill_ms) *fill_ms = job.fill_ms;
    const double fms = job.fill_ms;
    job_release(ctx, job);
    if (rc) return rc;
    std::vector<int> dev_of(P, -1);
    for (size_t k = 0; k < idx.size(); ++k) dev_of[idx[k]] = (int)k;
    return label_batch(ctx, ph, hs, is_local, track, dev_of, si, sj, score, res, tb, fms, walks);
}

static int batch_core(gx_context* ctx, const std::vector<PairHost>& ph,
                      const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc, const HostScores& hs,
                      const Scores32& sc, int is_local, bool planes, bool track, std::vector<Walk>& walks,
                      double* fill_ms, const uint8_t* chars_dev = nullptr, const std::vector<size_t>* off1 = nullptr,
                      const std::vector<size_t>* off2 = nullptr, const SmallAlpha* staged_alpha = nullptr) {
    const size_t P = ph.size();
    // pairs with an interior go to the device
    std::vector<size_t> idx;
    for (size_t p = 0; p < P; ++p) if (ph[p].n >= 1 && ph[p].m >= 1) idx.push_back(p);
    std::vector<PairHost> dph;
    std::vector<std::pair<const uint8_t*, const uint8_t*>> dproc;
    std::vector<size_t> o1, o2;
    for (size_t p : idx) {
        dph.push_back(ph[p]);
        dproc.push_back(proc[p]);
        if (chars_dev) { o1.push_back((*off1)[p]); o2.push_back((*off2)[p]); }
    }
    FillJob job;
    std::vector<PairRes> res(P, PairRes{});
    TbOut& tb = ctx->tb_cache;
    std::vector<TbStart> starts(idx.size());
    std::vector<uint64_t> si(P), sj(P);
    std::vector<int64_t> score(P);
    int rc = GX_OK;
    using clk = std::chrono::steady_clock;
    const auto c0 = clk::now();
    if (!idx.empty()) {
        SmallAlpha alpha;
        if (staged_alpha) alpha = *staged_alpha;
        else
            for (size_t k = 0; k < dproc.size() && alpha.n <= 4; ++k) {
                alpha.add(dproc[k].first, dph[k].n);
                alpha.add(dproc[k].second, dph[k].m);
            }
        rc = run_fill(ctx, dproc, dph, sc, is_local, planes, track, false, job, chars_dev, chars_dev ? &o1 : nullptr,
                      chars_dev ? &o2 : nullptr, &alpha);
        if (rc) { job_release(ctx, job); return rc; }
        for (size_t k = 0; k < idx.size(); ++k) res[idx[k]] = job.res[k];
    }
    const auto c1 = clk::now();
    for (size_t p = 0; p < P; ++p) start_cell_common(hs, is_local, ph[p].n, ph[p].m, start_in(res[p]), &si[p], &sj[p], &score[p]);
    if (!idx.empty()) {
        for (size_t k = 0; k < idx.size(); ++k) {
            const size_t p = idx[k];
            starts[k] = (si[p] >= 1 && sj[p] >= 1)
                            ? TbStart{(int)si[p], (int)sj[p], is_local ? res[p].lmax_E : res[p].end_E}
                            : TbStart{0, 0, 0};
        }
        rc = run_traceback(ctx, job, starts, tb);
    }
    const auto c2 = clk::now();
    if (fill_ms) *fill_ms = job.fill_ms;
    bool held = false;
    if (rc) job_release(ctx, job);
    else release_or_hold(ctx, job, true, &held);
    if (rc) return rc;
    if (held) {
        (void)hipStreamSynchronize(ctx->stream);
        std::vector<int> kdev(P, -1);
        for (size_t k = 0; k < idx.size(); ++k) kdev[idx[k]] = (int)k;
        keep_job(ctx, job, kdev);
    }
    struct PhaseLog {   // GX_LOG=debug: host-side phase times of the batch path
        clk::time_point c0, c1, c2;
        double fill_ms, tb_ms;
        size_t P;
        ~PhaseLog() {
            const char* e = getenv("GX_LOG");
            if (!e || strcmp(e, "debug")) return;
            auto ms = [](clk::time_point a, clk::time_point b) {
                return std::chrono::duration<double, std::milli>(b - a).count();
            };
            fprintf(stderr, "[gx DEBUG] batch P=%zu fill %.3f ms (kernel %.3f) traceback %.3f ms (kernel %.3f) "
                            "label %.3f ms\n", P, ms(c0, c1), fill_ms, ms(c1, c2), tb_ms, ms(c2, clk::now()));
        }
    } plog{c0, c1, c2, job.fill_ms, tb.ms, P};
    std::vector<int> dev_of(P, -1);
    for (size_t k = 0; k < idx.size(); ++k) dev_of[idx[k]] = (int)k;
    return label_batch(ctx, ph, hs, is_local, track, dev_of, si, sj, score, res, tb, job.fill_ms, walks);
}

// `nsteps` passes over the same batch (the staged benchmark path), pipelined
// one batch deep: batch k+1's fill is queued behind batch k's traceback, so
// the host labels batch k while the device fills batch k+1.  Device buffers
// go back to the pool as soon as their last user is queued (everything runs on
// one stream); pinned staging and events alternate between two slots.  Walks
// and results are those of the last pass; *fill_ms is the mean fill time.
// Overlapped pipeline for a global untracked batch on the twin fill without
// landing columns (the sequential strip walk, tb_seq_kernel, ~5 ms for a 30k
// pair, uses a few CUs): the pairs are split into group A (half of them;
// local batches a fifth) and group B, each filled by its own launch on its
// own stream.
// Step k's walk (stream tstream, after both fills) then runs beside step k+1's
// group-A fill, whose plane codes go to a second A buffer (two A buffers, one
// B buffer: the device holds P + |A| <= 1.5 P pairs' planes, <= 3 B a cell
// of twin codes, within the 3.25 B a cell the chunk plan budgets for a pair
// of a compact-plane batch); step k+1's group-B fill
// waits on the device for step k's walk before it reuses B's buffers.  Only
// buffers no pending work uses go back to the pool (a walk's fills after it
// was collected; B's before its next fill, which waits for the walk that
// reads them), so any stream may take them.  Returns GX_EAGAIN (nothing
// left enqueued) when the two groups' fills do not both take the twin fill
// without landing columns: the caller then runs the plain pipeline.
static constexpr int kOverlapNo = -1000;
static int batch_core_overlap(gx_context* ctx, const std::vector<PairHost>& ph,
                              const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc, const HostScores& hs,
                              const Scores32& sc, int is_local, bool planes, int nsteps, std::vector<Walk>& walks, double* fill_ms,
                              const uint8_t* chars_dev, const std::vector<size_t>* off1,
                              const std::vector<size_t>* off2, const SmallAlpha& alpha,
                              const std::vector<size_t>& idx, const PassSet* alt) {
    const size_t P = ph.size(), Q = idx.size();
    // group A: half the pairs (global), even (twins).  Two equal launches
    // fill the chip better than a small A beside a large B: 80 x 30k, fill ms
    // a pass by A's pairs 8 / 16 / 24 / 32 / 40 = 33.7 / 29.9 / 29.0 / 27.0 /
    // 26.5 (the one-launch pass 27.8); all-vs-all with planes 20.4 -> 17.0 ms,
    // 1024 x 16k 100.4 -> 99.4.  Local batches keep a fifth (64 related local
    // pairs 26.9 ms against 27.9 at half; profiles/r05_overlap_split.txt).
    // GX_OVERLAP_A sets A's pair count.
    // (half rounded up: a chunked batch's 19- and 20-pair chunks then both
    // split 10 + 9 / 10 + 10 and reuse the same cached plane buffers)
    size_t G = std::max<size_t>(2, (is_local ? Q / 5 : (Q + 1) / 2) & ~(size_t)1);
    if (const char* e = getenv("GX_OVERLAP_A"); e && atoi(e) >= 2 && (size_t)atoi(e) + 2 <= Q)
        G = (size_t)atoi(e) & ~(size_t)1;
    std::vector<size_t> gi[2];
    gi[0].assign(idx.begin(), idx.begin() + (long)G);
    gi[1].assign(idx.begin() + (long)G, idx.end());
    // [pair set][group] (one set unless alt: pass k runs set k & 1)
    const std::vector<PairHost>* const PH[2] = {&ph, alt ? alt->ph : &ph};
    const std::vector<std::pair<const uint8_t*, const uint8_t*>>* const PR[2] = {&proc, alt ? alt->proc : &proc};
    const std::vector<size_t>* const O1[2] = {off1, alt ? alt->off1 : off1};
    const std::vector<size_t>* const O2[2] = {off2, alt ? alt->off2 : off2};
    std::vector<Walk>* const WK[2] = {&walks, alt ? alt->walks : &walks};
    const size_t poff[2] = {ctx->pass_off, alt ? alt->pass_off : ctx->pass_off};
    std::vector<PairHost> dph[2][2];
    std::vector<std::pair<const uint8_t*, const uint8_t*>> dproc[2][2];
    std::vector<size_t> o1[2][2], o2[2][2];
    for (int v = 0; v < 2; ++v)
        for (int g = 0; g < 2; ++g)
            for (size_t p : gi[g]) {
                dph[v][g].push_back((*PH[v])[p]);
                dproc[v][g].push_back((*PR[v])[p]);
                if (chars_dev) { o1[v][g].push_back((*O1[v])[p]); o2[v][g].push_back((*O2[v])[p]); }
            }
    for (hipStream_t* st : {&ctx->stream2, &ctx->tstream})
        if (!*st) HIPCHK(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
    hipStream_t const sA = ctx->stream, sB = ctx->stream2, sT = ctx->tstream;
    FillJob jA[2], jB;
    bool jb_live = false;
    std::vector<int> dev_of(P, -1);
    for (size_t q = 0; q < Q; ++q) dev_of[q < G ? gi[0][q] : gi[1][q - G]] = (int)q;
    std::vector<TbStart> starts(Q);
    for (size_t q = 0; q < Q; ++q) {
        const PairHost& h = q < G ? dph[0][0][q] : dph[0][1][q - G];
        starts[q] = TbStart{(int)h.n, (int)h.m, 0};
    }
    std::vector<PairRes> res(P, PairRes{});
    std::vector<uint64_t> si(P), sj(P);
    std::vector<int64_t> score(P);
    double fsum = 0;
    auto fill = [&](int g, int k) {
        FillJob& j = g == 0 ? jA[k & 1] : jB;
        j.stream = g == 0 ? sA : sB;
        const int v = k & 1;
        return run_fill(ctx, dproc[v][g], dph[v][g], sc, is_local, planes, false, false, j, chars_dev,
                        chars_dev ? &o1[v][g] : nullptr, chars_dev ? &o2[v][g] : nullptr, &alpha, 2 * g + (k & 1), false);
    };
    auto trace = [&](int k) {
        HIPCHK(hipStreamWaitEvent(sT, ctx->slots[k & 1].fdone, 0));
        HIPCHK(hipStreamWaitEvent(sT, ctx->slots[2 + (k & 1)].fdone, 0));
        // (local: the start cells are read on the device, TbDev.start_ij_dev)
        return run_traceback(ctx, std::vector<const FillJob*>{&jA[k & 1], &jB}, starts, ctx->slots[k & 1].out, k & 1,
                             false, is_local != 0, sT);
    };
    auto take = [&](const FillJob& j, const std::vector<size_t>& g) {
        for (size_t q = 0; q < g.size(); ++q) res[g[q]] = j.res[q];
    };
    // the fills' time per step: one step's fills overlap the next step's and
    // the walks, so the whole fill pipeline (the first fill's start to the
    // last fill's end, ev0..ev1) over the steps
    auto drain = [&]() {
        (void)hipStreamSynchronize(sA); (void)hipStreamSynchronize(sB); (void)hipStreamSynchronize(sT);
        (void)hipStreamSynchronize(ctx->cstream);
        for (auto& j : jA) job_release(ctx, j);
        job_release(ctx, jB);
        release_slots(ctx);
    };
    {   // both groups must take the twin fill without landing columns: decided before anything is enqueued
        FillJob pa, pb;
        pa.plan_only = pb.plan_only = true;
        int prc = run_fill(ctx, dproc[0][0], dph[0][0], sc, is_local, planes, false, false, pa, chars_dev,
                           chars_dev ? &o1[0][0] : nullptr, chars_dev ? &o2[0][0] : nullptr, &alpha, 0, false);
        if (!prc)
            prc = run_fill(ctx, dproc[0][1], dph[0][1], sc, is_local, planes, false, false, pb, chars_dev,
                           chars_dev ? &o1[0][1] : nullptr, chars_dev ? &o2[0][1] : nullptr, &alpha, 2, false);
        if (prc || !(pa.noskel && pb.noskel && pa.twin && pb.twin && pa.lay == pb.lay)) return kOverlapNo;
    }
    unsigned long long* const sums0 = ctx->sums_dst;
    HIPCHK(hipEventRecord(ctx->ev0, sA));
    int rc = fill(0, 0);
    if (!rc) { rc = fill(1, 0); jb_live = !rc; }
    if (!rc && !(jA[0].noskel && jB.noskel && jA[0].lay == jB.lay && jA[0].twin && jB.twin)) {
        drain();
        ctx->sums_dst = sums0;   // (the plain pipeline writes this pass's checksums again)
        return kOverlapNo;
    }
    if (!rc) rc = trace(0);
    for (int k = 0; k < nsteps && !rc; ++k) {
        const int a = k & 1;
        if (k + 1 < nsteps) {
            if ((rc = fill(0, k + 1))) break;                 // beside step k's walk (its buffers: step k-1's, collected)
            if ((rc = fill_collect(ctx, jB))) break;          // step k's group B, before jB is refilled
            take(jB, gi[1]);
            job_release(ctx, jB);                             // read by step k's walk: the next B fill waits for it
            HIPCHK(hipStreamWaitEvent(sB, ctx->slots[a].te, 0));
            if ((rc = fill(1, k + 1))) break;
            if (k + 2 == nsteps) {                            // behind the last fill (B's comes after A's, below)
                HIPCHK(hipStreamWaitEvent(sB, ctx->slots[(k + 1) & 1].fdone, 0));
                HIPCHK(hipEventRecord(ctx->ev1, sB));
            }
            if (!(jA[(k + 1) & 1].noskel && jB.noskel)) { rc = fail(GX_EHIP, "overlapped batch: fill formats changed"); break; }
            if ((rc = trace(k + 1))) break;
        } else {
            if ((rc = fill_collect(ctx, jB))) break;
            take(jB, gi[1]);
        }
        if ((rc = fill_collect(ctx, jA[a]))) break;
        take(jA[a], gi[0]);
        if (k + 1 == nsteps) {
            HIPCHK(hipEventSynchronize(ctx->ev1));
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
            fsum = ms;
        }
        if ((rc = tb_collect(ctx, a, Q, ctx->slots[a].out))) break;
        job_release(ctx, jA[a]);                              // its walk is done
        for (size_t p = 0; p < P; ++p)
            start_cell_common(hs, is_local, ph[p].n, ph[p].m, start_in(res[p]), &si[p], &sj[p], &score[p]);
        ctx->pass_off = poff[a];
        if ((rc = label_batch(ctx, *PH[a], hs, is_local, false, dev_of, si, sj, score, res, ctx->slots[a].out,
                              jA[a].fill_ms + jB.fill_ms, *WK[a])))
            break;
    }
    drain();
    (void)jb_live;
    ctx->pass_off = poff[0];
    if (rc) return rc;
    ctx->last_groups = 2;
    if (fill_ms) *fill_ms = fsum / nsteps;
    return GX_OK;
}

int batch_core_steps(gx_context* ctx, const std::vector<PairHost>& ph,
                     const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc, const HostScores& hs,
                     const Scores32& sc, int is_local, bool planes, bool track, int nsteps,
                     std::vector<Walk>& walks, double* fill_ms, const uint8_t* chars_dev,
                     const std::vector<size_t>* off1, const std::vector<size_t>* off2,
                     const SmallAlpha* staged_alpha, const PassSet* alt) {
    const size_t P = ph.size();
    ctx->last_groups = 1;
    std::vector<size_t> idx;
    for (size_t p = 0; p < P; ++p) if (ph[p].n >= 1 && ph[p].m >= 1) idx.push_back(p);
    // the pair sets by pass parity (one set unless alt)
    const std::vector<PairHost>* const PH[2] = {&ph, alt ? alt->ph : &ph};
    const std::vector<std::pair<const uint8_t*, const uint8_t*>>* const PR[2] = {&proc, alt ? alt->proc : &proc};
    const std::vector<size_t>* const O1[2] = {off1, alt ? alt->off1 : off1};
    const std::vector<size_t>* const O2[2] = {off2, alt ? alt->off2 : off2};
    std::vector<Walk>* const WK[2] = {&walks, alt ? alt->walks : &walks};
    const size_t poff[2] = {ctx->pass_off, alt ? alt->pass_off : ctx->pass_off};
    struct OffBack {   // (the caller's pass offset back on every return)
        gx_context* c;
        size_t v;
        ~OffBack() { c->pass_off = v; }
    } off_back{ctx, poff[0]};
    if (nsteps <= 1 || idx.empty() || getenv("GX_TRACE_FILE")) {
        double f = 0, fsum = 0;
        for (int s = 0; s < std::max(nsteps, 1); ++s) {
            const int v = s & 1;
            ctx->pass_off = poff[v];
            const int rc = batch_core(ctx, *PH[v], *PR[v], hs, sc, is_local, planes, track, *WK[v], &f, chars_dev,
                                      O1[v], O2[v], staged_alpha);
            if (rc) return rc;
            fsum += f;
        }
        if (fill_ms) *fill_ms = fsum / std::max(nsteps, 1);
        return GX_OK;
    }
    int rc = slots_ready(ctx);
    if (rc) return fail(rc, "pipeline events");
    std::vector<PairHost> dph_s[2];
    std::vector<std::pair<const uint8_t*, const uint8_t*>> dproc_s[2];
    std::vector<size_t> o1_s[2], o2_s[2];
    for (int v = 0; v < 2; ++v)
        for (size_t p : idx) {
            dph_s[v].push_back((*PH[v])[p]);
            dproc_s[v].push_back((*PR[v])[p]);
            if (chars_dev) { o1_s[v].push_back((*O1[v])[p]); o2_s[v].push_back((*O2[v])[p]); }
        }
    const std::vector<PairHost>& dph = dph_s[0];
    const std::vector<std::pair<const uint8_t*, const uint8_t*>>& dproc = dproc_s[0];
    SmallAlpha alpha;
    if (staged_alpha) alpha = *staged_alpha;
    else
        for (size_t q = 0; q < dproc.size() && alpha.n <= 4; ++q) {
            alpha.add(dproc[q].first, dph[q].n);
            alpha.add(dproc[q].second, dph[q].m);
        }
    FillJob jobs[3];
    std::vector<PairRes> res(P, PairRes{});
    std::vector<TbStart> starts(idx.size());
    std::vector<uint64_t> si(P), sj(P);
    std::vector<int64_t> score(P);
    std::vector<int> dev_of(P, -1);
    for (size_t q = 0; q < idx.size(); ++q) dev_of[idx[q]] = (int)q;
    double fsum = 0;
    auto fill_at = [&](int s, int v) {   // slot s (pinned staging, events, job), pair set v
        return run_fill(ctx, dproc_s[v], dph_s[v], sc, is_local, planes, track, false, jobs[s], chars_dev,
                        chars_dev ? &o1_s[v] : nullptr, chars_dev ? &o2_s[v] : nullptr, &alpha, s, false);
    };
    auto fill = [&](int s) { return fill_at(s, s); };   // slot s = the pass's parity = its pair set
    // results of slot s's fill -> start cells -> its traceback queued; the fill
    // buffers return to the pool (their last user, the traceback, is queued)
    int pl_pass = 0;
    bool pl_held[2] = {false, false};
    auto trace = [&](int s) {
        int r = fill_collect(ctx, jobs[s]);
        if (r) return r;
        fsum += jobs[s].fill_ms;
        for (size_t q = 0; q < idx.size(); ++q) res[idx[q]] = jobs[s].res[q];
        for (size_t p = 0; p < P; ++p)
            start_cell_common(hs, is_local, ph[p].n, ph[p].m, start_in(res[p]), &si[p], &sj[p], &score[p]);
        for (size_t q = 0; q < idx.size(); ++q) {
            const size_t p = idx[q];
            starts[q] = (si[p] >= 1 && sj[p] >= 1)
                            ? TbStart{(int)si[p], (int)sj[p], is_local ? res[p].lmax_E : res[p].end_E}
                            : TbStart{0, 0, 0};
        }
        r = run_traceback(ctx, jobs[s], starts, ctx->slots[s].out, s, false);
        release_or_hold(ctx, jobs[s], pl_pass++ == nsteps - 1, &pl_held[s]);
        return r;
    };
    using clk = std::chrono::steady_clock;
    auto since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    double t_fill = 0, t_tbwait = 0, t_label = 0, t_trace = 0;   // host time per phase (GX_LOG=debug)
    const auto t_all = clk::now();
    size_t nmax_b = 0;
    for (const PairHost& h : dph) nmax_b = std::max(nmax_b, h.n);
    // (long pairs only: a short pair's walk is short; and both groups must
    // fill the grid on the twin fill, or the attempt falls back.  1024 x 4k:
    // 14.9 ms a step overlapped against 10.8 plain; 1024 x 16k 116.8 against
    // 145, measured in round 4 (those records were replaced by the round-5
    // ones on the same rule, profiles/r05_config5_*.json; the plain-pipeline
    // side: profiles/r02k_config5_*.json))
    // (local batches from 64 pairs: at 32 related 30k pairs the split launches
    // fill worse than the walk they hide, 27.2 vs 21.6 ms a step; GX_OVERLAP=1
    // forces it from 16 pairs, GX_OVERLAP=0 turns it off)
    const char* ov = getenv("GX_OVERLAP");
    const bool ov_force = ov && !strcmp(ov, "1");
    if (!track && planes && idx.size() >= 16 && (nmax_b >= 16384 || ov_force) && !ctx->keep_capture &&
        !(ov && !strcmp(ov, "0")) && (!is_local || idx.size() >= 64 || ov_force)) {
        const int orc = batch_core_overlap(ctx, ph, proc, hs, sc, is_local, planes, nsteps, walks, fill_ms, chars_dev, off1, off2,
                                           alpha, idx, alt);
        if (orc != kOverlapNo) return orc;
    }
    if (!is_local) {
        // global: every start cell is (n, m) and its landing column is read
        // on the device, so each step's traceback is queued right behind its
        // fill; the fill results (with a tracked fill's max cell and
        // matches_at_max, which do not move the start) are collected on the
        // host only for the labelling (no host round trip between fill and
        // traceback; tracked Covid 5.10 -> 4.89 ms a step at a 4.74 ms fill)
        for (size_t q = 0; q < idx.size(); ++q) starts[q] = TbStart{dph[q].n >= 1 && dph[q].m >= 1 ? (int)dph[q].n : 0,
                                                                     (int)dph[q].m, 0};
        // the walk stays on the fill's stream: the fill's buffers return to
        // the pool right behind it (stream-ordered reuse).  (A walk on its own
        // stream beside the next step's fill, its buffers released once the
        // walk is collected, measured in round 5 (tools/walk_stream_sweep.sh,
        // 3 alternating runs a size): 1024 x 1k 0.99 -> 1.06 ms a step,
        // 1024 x 4k 8.35 -> 8.17, 128 x 16k 17.5 -> 17.6: the walk and the
        // fill slow each other down on shared CUs (fill 0.56 -> 0.67 ms beside
        // a walk stretched from 0.30 to 0.82), and the host's labelling then
        // leaves the device idle between pairs of steps.)
        //
        // Three slots in flight: pass k+2's fill and walk are queued before
        // the host waits for pass k's records, so the record copy (4.3 MB on
        // a 1024 x 1k pass, ~0.22 ms on the copy engine after the walk) and
        // the labelling (~0.52 ms) of pass k run beside passes k+1 and k+2 on
        // the device.  One slot ahead, the next fill was queued only after
        // the labelling: the device sat idle ~0.2 ms a pass (rocprofv3
        // timeline, 1024 x 1k).  A slot's pinned buffers are rewritten when
        // pass k+3 is queued, after pass k was labelled; its device
        // descriptor caches on the fill stream, in stream order.
        int tr_pass = 0;
        bool held[3] = {false, false, false};
        // the walk on its own stream beside the next pass's fill, when the
        // two more passes' fill buffers this holds (a walk keeps its fill's
        // buffers until it is collected) fit the free HBM as it is -- not by
        // evicting the pool's cached buffers, whose re-allocation costs far
        // more (hipMalloc of an 86 GB plane buffer ~2.4 s: a 4-pair 64k batch
        // that evicted them cost the next 1024 x 64k batch 7 s).  1024 x 1k
        // 0.94 -> 0.84 ms a pass, 1024 x 4k 7.93 -> 7.57 (tools/walk_prio_ab.sh).
        // (With one slot ahead it was slower: the labelling, not the device,
        // then set the pace.)  GX_TB_OWN_STREAM=0 keeps the walk on the fill's
        // stream.
        bool wstream = !ctx->keep_capture && !(getenv("GX_TB_OWN_STREAM") && !strcmp(getenv("GX_TB_OWN_STREAM"), "0"));
        if (wstream) {
            double need = 0;
            for (const PairHost& h : dph) need += pair_device_bytes(h.n, h.m, 2.0);
            size_t fr = 0, tot = 0;
            wstream = hipMemGetInfo(&fr, &tot) == hipSuccess && 2.0 * need <= (double)fr - 4.0 * (1ull << 30);
        }
        if (wstream && !ctx->tstream && hipStreamCreateWithFlags(&ctx->tstream, hipStreamNonBlocking) != hipSuccess)
            return fail(GX_EHIP, "walk stream");
        bool jheld[3] = {false, false, false};
        auto trace_dev = [&](int s) {
            if (wstream) {   // the walk on its own stream; the fill's buffers held until it is collected
#ifndef GX_MUT_NO_FDONE_WAIT   // (mutation build only: tests/test_gpu_atsize.py must catch its absence)
                // (on the fill kernel's own end event: the walk needs its planes
                // and end cell only, not the reductions queued after it -- a
                // tracked fill's max column and matches_at_max -- nor the
                // checksums of a staged parity pass)
                if (hipStreamWaitEvent(ctx->tstream, ctx->slots[s].fe, 0) != hipSuccess) return fail(GX_EHIP, "walk stream wait");
#endif
                jheld[s] = true;
                const int r = run_traceback(ctx, std::vector<const FillJob*>{&jobs[s]}, starts, ctx->slots[s].out, s, false,
                                            true, ctx->tstream);
#ifdef GX_MUT_EARLY_RELEASE   // (mutation build only: the fill's buffers back to the pool while the walk may read them)
                job_release(ctx, jobs[s]);
                jheld[s] = false;
#endif
                return r;
            }
            int r = run_traceback(ctx, jobs[s], starts, ctx->slots[s].out, s, false, true);
            release_or_hold(ctx, jobs[s], tr_pass++ == nsteps - 1, &held[s]);   // stream order: later users come after the traceback
            return r;
        };
        auto results = [&](int s) {
            int r = fill_collect(ctx, jobs[s]);
            if (r) return r;
            fsum += jobs[s].fill_ms;
            for (size_t q = 0; q < idx.size(); ++q) res[idx[q]] = jobs[s].res[q];
            for (size_t p = 0; p < P; ++p)
                start_cell_common(hs, is_local, ph[p].n, ph[p].m, start_in(res[p]), &si[p], &sj[p], &score[p]);
            return GX_OK;
        };
        using clk = std::chrono::steady_clock;
        const auto t_all = clk::now();
        double h_enq = 0, h_tbw = 0, h_res = 0, h_lab = 0;   // host time per phase (GX_LOG=debug)
        int queued = 0;   // passes whose fill and walk are queued
        for (int k = 0; k < nsteps && !rc; ++k) {
            const int s = k % 3, v = k & 1;
            auto t = clk::now();
            while (!rc && queued < std::min(nsteps, k + 3)) {
                const int q = queued++;
                // (a pass's reductions beside the next fill only once the walk's
                // stream is settled: it holds the pass's buffers until collected)
                ctx->post_aside = wstream && q > 0;
                rc = fill_at(q % 3, q & 1);
                ctx->post_aside = false;
                if (rc) break;
                // two fill workgroups a CU (7-wave bands, run_fill) leave the
                // walks no room beside the fill: the walk stays on its stream
                if (q == 0 && ctx->last_W == 7) wstream = false;
                rc = trace_dev(q % 3);
            }
            if (rc) break;
            h_enq += since(t); t = clk::now();
            if ((rc = tb_collect(ctx, s, idx.size(), ctx->slots[s].out))) break;
            h_tbw += since(t); t = clk::now();
            if ((rc = results(s))) break;
            if (jheld[s]) { job_release(ctx, jobs[s]); jheld[s] = false; }   // its walk has ended
            h_res += since(t); t = clk::now();
            ctx->pass_off = poff[v];
            if ((rc = label_batch(ctx, *PH[v], hs, is_local, track, dev_of, si, sj, score, res, ctx->slots[s].out,
                                  jobs[s].fill_ms, *WK[v])))
                break;
            h_lab += since(t);
        }
        if (const char* e = getenv("GX_LOG"); e && !strcmp(e, "debug"))
            fprintf(stderr, "[gx DEBUG] pipelined %d steps P=%zu (device traceback starts): %.3f ms/step; host per step: "
                    "enqueue fill+traceback %.3f, traceback wait %.3f, fill results %.3f, labelling %.3f ms\n", nsteps, P,
                    std::chrono::duration<double, std::milli>(clk::now() - t_all).count() / nsteps, h_enq / nsteps,
                    h_tbw / nsteps, h_res / nsteps, h_lab / nsteps);
        if (rc) {
            (void)hipStreamSynchronize(ctx->stream);
            if (ctx->tstream) (void)hipStreamSynchronize(ctx->tstream);
            for (auto& j : jobs) job_release(ctx, j);
            release_slots(ctx);
            return rc;
        }
        for (int s = 0; s < 3; ++s)
            if (held[s]) { (void)hipStreamSynchronize(ctx->stream); keep_job(ctx, jobs[s], dev_of); }
        if (fill_ms) *fill_ms = fsum / nsteps;
        return GX_OK;
    }
    if (!(rc = fill(0))) rc = trace(0);
    for (int k = 0; k < nsteps && !rc; ++k) {
        const int s = k & 1;
        auto t = clk::now();
        if (k + 1 < nsteps && (rc = fill(s ^ 1))) break;       // queued behind batch k's traceback
        t_fill += since(t); t = clk::now();
        if ((rc = tb_collect(ctx, s, idx.size(), ctx->slots[s].out))) break;
        t_tbwait += since(t); t = clk::now();
        ctx->pass_off = poff[s];
        if ((rc = label_batch(ctx, *PH[s], hs, is_local, track, dev_of, si, sj, score, res, ctx->slots[s].out,
                              jobs[s].fill_ms, *WK[s])))
            break;
        t_label += since(t); t = clk::now();
        if (k + 1 < nsteps && (rc = trace(s ^ 1))) break;
        t_trace += since(t);
    }
    if (const char* e = getenv("GX_LOG"); e && !strcmp(e, "debug"))
        fprintf(stderr, "[gx DEBUG] pipelined %d steps P=%zu: %.3f ms/step; host per step: fill enqueue %.3f, "
                        "traceback wait %.3f, label %.3f, fill wait + traceback enqueue %.3f ms\n",
                nsteps, P, since(t_all) / nsteps, t_fill / nsteps, t_tbwait / nsteps, t_label / nsteps,
                t_trace / nsteps);
    if (rc) {
        (void)hipStreamSynchronize(ctx->stream);
        for (auto& j : jobs) job_release(ctx, j);
        release_slots(ctx);
        return rc;
    }
    for (int s = 0; s < 2; ++s)
        if (pl_held[s]) { (void)hipStreamSynchronize(ctx->stream); keep_job(ctx, jobs[s], dev_of); }
    if (fill_ms) *fill_ms = fsum / nsteps;
    return GX_OK;
}

extern "C" int gx_align_batch(gx_context* ctx, const uint8_t* const* s1, const size_t* n, const uint8_t* const* s2,
                              const size_t* m, size_t npairs, const gx_scores* scores, int is_local,
                              uint32_t flags, gx_step* const* steps, const size_t* caps, gx_result* out) {
    if (!ctx || !s1 || !n || !s2 || !m || !out) return fail(GX_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    HIPCHK(hipSetDevice(ctx->device));
    size_t nmax = 0, mmax = 0;
    for (size_t p = 0; p < npairs; ++p) { nmax = std::max(nmax, n[p]); mmax = std::max(mmax, m[p]); }
    HostScores hs;
    Scores32 sc;
    bool wide = false;
    int rc = check_scores(scores, nmax, mmax, &hs, &sc, is_local, &wide);
    if (rc) return rc;
    std::vector<PairHost> ph(npairs);
    std::vector<std::pair<const uint8_t*, const uint8_t*>> proc(npairs);
    for (size_t p = 0; p < npairs; ++p) {
        ph[p] = PairHost{s1[p], s2[p], n[p], m[p]};
        proc[p] = {s1[p], s2[p]};
    }
    // traceback codes only (no planes); batches beyond the free HBM run in
    // chunks.  Local batches that a plan of the whole batch puts on the local
    // twin fill keep its plane codes as scratch for the walk
    // (2 B/cell; chunks planned at the scalar byte format's 3 B/cell, should a
    // chunk fall back)
    bool lplanes = false;
    if (is_local && !wide && !(flags & GX_ALIGN_MAX_CELL)) {
        std::vector<PairHost> nz;
        std::vector<std::pair<const uint8_t*, const uint8_t*>> np;
        for (size_t p = 0; p < npairs; ++p)
            if (n[p] && m[p]) { nz.push_back(ph[p]); np.push_back(proc[p]); }
        FillJob pj;
        pj.plan_only = true;
        lplanes = !nz.empty() && !run_fill(ctx, np, nz, sc, is_local, true, false, false, pj) && pj.twin;
    }
    const auto chunks = plan_chunks(ctx, ph, lplanes ? 3.0 : 0.0);
    ctx->last_chunks = (int)chunks.size();
    std::vector<Walk> walks;
    for (const auto& c : chunks) {
        std::vector<PairHost> phc(ph.begin() + c.first, ph.begin() + c.second);
        std::vector<std::pair<const uint8_t*, const uint8_t*>> pc(proc.begin() + c.first, proc.begin() + c.second);
        rc = wide ? batch_core_wide(ctx, phc, pc, hs, is_local, false, (flags & GX_ALIGN_MAX_CELL) != 0, walks, nullptr)
                  : batch_core(ctx, phc, pc, hs, sc, is_local, lplanes, (flags & GX_ALIGN_MAX_CELL) != 0, walks,
                               nullptr);
        if (rc) return rc;
        for (size_t k = 0; k < phc.size(); ++k) {
            const size_t p = c.first + k;
            out[p] = walks[k].res;
            if (steps && steps[p]) {
                rc = copy_steps(walks[k], steps[p], caps ? caps[p] : 0);
                if (rc) return rc;
            }
        }
    }
    return GX_OK;
}

// Many independent pairs over several GPUs (one context each): the pairs are
// shared out by longest-processing-time on n * m cells (the heaviest pair to
// the least-loaded context), and each share runs as one gx_align_batch on its
// own host thread -- no device-to-device traffic, the shares are independent.
// The reference's multi-worker driver is the rayon pool over all pairs of
// compare (main.rs:245-261); this is its multi-GPU counterpart.
static std::vector<std::vector<size_t>> lpt_shares(const size_t* n, const size_t* m, size_t npairs, int parts) {
    std::vector<size_t> order(npairs);
    for (size_t p = 0; p < npairs; ++p) order[p] = p;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
        return (double)n[a] * (double)m[a] > (double)n[b] * (double)m[b];
    });
    std::vector<std::vector<size_t>> bins((size_t)parts);
    std::vector<double> load((size_t)parts, 0.0);
    for (size_t p : order) {
        size_t b = 0;
        for (size_t k = 1; k < bins.size(); ++k)
            if (load[k] < load[b]) b = k;
        bins[b].push_back(p);
        load[b] += (double)n[p] * (double)m[p] + (double)(n[p] + m[p]);
    }
    for (auto& b : bins) std::sort(b.begin(), b.end());
    return bins;
}

extern "C" int gx_align_batch_multi(gx_context* const* ctxs, int nctx, const uint8_t* const* s1, const size_t* n,
                                    const uint8_t* const* s2, const size_t* m, size_t npairs,
                                    const gx_scores* scores, int is_local, uint32_t flags, gx_step* const* steps,
                                    const size_t* caps, gx_result* out) {
    if (!ctxs || nctx < 1 || !s1 || !n || !s2 || !m || !out) return fail(GX_EINVAL, "NULL argument");
    for (int k = 0; k < nctx; ++k)
        if (!ctxs[k]) return fail(GX_EINVAL, "NULL context");
    if (nctx == 1)
        return gx_align_batch(ctxs[0], s1, n, s2, m, npairs, scores, is_local, flags, steps, caps, out);
    const auto bins = lpt_shares(n, m, npairs, nctx);
    std::vector<int> rc((size_t)nctx, GX_OK);
    std::vector<std::string> err((size_t)nctx);
    std::vector<std::thread> th;
    for (int k = 0; k < nctx; ++k) {
        if (bins[(size_t)k].empty()) continue;
        th.emplace_back([&, k] {
            const auto& b = bins[(size_t)k];
            const size_t q = b.size();
            std::vector<const uint8_t*> a1(q), a2(q);
            std::vector<size_t> an(q), am(q), acap(q);
            std::vector<gx_step*> ast(q, nullptr);
            std::vector<gx_result> ares(q);
            for (size_t x = 0; x < q; ++x) {
                const size_t p = b[x];
                a1[x] = s1[p]; a2[x] = s2[p]; an[x] = n[p]; am[x] = m[p];
                ast[x] = steps ? steps[p] : nullptr;
                acap[x] = caps ? caps[p] : 0;
            }
            rc[(size_t)k] = gx_align_batch(ctxs[k], a1.data(), an.data(), a2.data(), am.data(), q, scores, is_local,
                                           flags, steps ? ast.data() : nullptr, caps ? acap.data() : nullptr,
                                           ares.data());
            if (rc[(size_t)k]) err[(size_t)k] = g_err;   // g_err is thread-local
            else
                for (size_t x = 0; x < q; ++x) out[b[x]] = ares[x];
        });
    }
    for (auto& t : th) t.join();
    for (int k = 0; k < nctx; ++k)
        if (rc[(size_t)k]) return fail(rc[(size_t)k], "context " + std::to_string(k) + ": " + err[(size_t)k]);
    return GX_OK;
}
