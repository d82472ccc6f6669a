// gx_api_walk.cpp -- retrace (algo.rs:287-441): the device walk launch and
// its row records, start cells (algo.rs:306-331), and the labelling of the
// walk into AlignmentChoice steps (algo.rs:339-422) on host worker threads.
#include "gx_api.h"

StartIn start_in(const FillJob& job, size_t p) {
    if (job.wide) return StartIn{job.wres[p].end_SM, job.wres[p].lmax_val, (uint64_t)job.wres[p].lmax_i,
                                 (uint64_t)job.wres[p].lmax_j};
    const PairRes& r = job.res[p];
    return StartIn{r.end_SM, r.lmax_val, (uint64_t)r.lmax_i, (uint64_t)r.lmax_j};
}
StartIn start_in(const PairRes& r) { return StartIn{r.end_SM, r.lmax_val, (uint64_t)r.lmax_i, (uint64_t)r.lmax_j}; }

// The boundary part of a walk from (i, j) on: the reference loop on analytic
// cells (algo.rs:339-422), appending to w.steps and counting into w.res.
int label_boundary(const HostScores& hs, int is_local, const uint8_t* s1, size_t n, const uint8_t* s2,
                   size_t m, uint64_t i, uint64_t j, int last, Walk& w) {
    gx_result& r = w.res;
    for (;;) {
        int64_t I, D, S;
        boundary_cell(hs, i, j, &I, &D, &S);
        const int64_t mx = smax(I, S, D, is_local);
        gx_step st{};
        st.i = i; st.j = j;
        bool di, dj;
        if (mx == S) {
            const bool mt = tb_match(s1, n, s2, m, i, j);
            st.choice = mt ? GX_MATCH : GX_MISMATCH;
            if (mt) r.matches++; else r.mismatches++;
            last = st.choice;
            di = dj = true;
        } else if (mx == I) {
            if (last == GX_INSERT) { st.choice = GX_INSERT; r.gap_extensions++; }
            else { st.choice = GX_OPEN_INSERT; r.opening_gaps++; }
            last = GX_INSERT;
            di = false; dj = true;
        } else if (mx == D) {
            if (last == GX_DELETE) { st.choice = GX_DELETE; r.gap_extensions++; }
            else { st.choice = GX_OPEN_DELETE; r.opening_gaps++; }
            last = GX_DELETE;
            di = true; dj = false;
        } else {
            if (is_local && mx == 0) {
                if (log_info())   // algo.rs:403
                    fprintf(stderr, "[gx INFO] Ending local alignment at (%llu, %llu)\n", (unsigned long long)i,
                            (unsigned long long)j);
                break;
            }
            return fail(GX_EPANIC, "Unexpected score during retrace: " + std::to_string(mx) + " at (" +
                                       std::to_string(i) + ", " + std::to_string(j) + ")");
        }
        if (!w.steps.push_back(st)) return fail(GX_ENOMEM, "step buffer");
        const bool inone = di && i == 0, jnone = dj && j == 0;
        if (inone && jnone) break;
        i = inone ? 0 : i - (di ? 1 : 0);
        j = jnone ? 0 : j - (dj ? 1 : 0);
        if (i == 0 && j == 0) break;
    }
    return GX_OK;
}

// One labelled step as three 8-B non-temporal stores: a batch's step buffers
// are far larger than the caches, so this skips each line's read for
// ownership (label_walk_records ends with an sfence).
static inline void put_step(gx_step* o, int choice, uint64_t i, uint64_t j) {
    _mm_stream_si64((long long*)o, (long long)(unsigned)choice);
    _mm_stream_si64((long long*)o + 1, (long long)i);
    _mm_stream_si64((long long*)o + 2, (long long)j);
}

// label_walk on the device walk's per-row records (tb_strip_kernel /
// tb_seq_kernel: each row's insert run, then its diagonal or delete move, or
// the run's end at column 0), written straight into the step buffer: a run of
// L inserts is one open-or-extend step and L - 1 extensions.  The same steps
// and statistics as label_walk over RecordsSrc.
int label_walk_records(const HostScores& hs, int is_local, const uint8_t* s1, size_t n, const uint8_t* s2,
                       size_t m, uint64_t si, uint64_t sj, const TbOut& tb, size_t p, Walk& w) {
    uint64_t i = si, j = sj;
    int last = GX_MATCH;
    uint64_t nmat = 0, nmis = 0, next = 0, nopen = 0;
    const size_t cap = (size_t)si + (size_t)sj + 2;   // every move lowers i + j
    w.steps.clear();
    if (!w.steps.reserve(cap)) return fail(GX_ENOMEM, "step buffer");
    gx_step* const o = w.steps.data();
    size_t k = 0;
    bool done = false;
    for (int s = tb.c[4 * p + 2]; s >= 0 && !done; --s) {
        const int* g = &tb.sg[4 * (tb.so[p] + s)];
        if (!g[3]) break;
        const uint32_t* rr = &tb.hr[(tb.so[p] + s) * tb.srows];
        for (int q = 0; q < g[2]; ++q) {
            const uint32_t rec = rr[q], L = rec >> 2, c = rec & 3u;
            if (k + L + 1 > cap || L > j) { _mm_sfence(); return fail(GX_EPANIC, "device walk record out of range"); }
            if (L) {
                const bool ext = last == GX_INSERT;
                put_step(o + k, ext ? GX_INSERT : GX_OPEN_INSERT, i, j);
                next += ext + (L - 1); nopen += !ext;
                ++k; --j;
                for (uint32_t t = 1; t < L; ++t) { put_step(o + k, GX_INSERT, i, j); ++k; --j; }
                last = GX_INSERT;
            }
            if (c == 0u) {
                const bool mt = tb_match(s1, n, s2, m, i, j);
                put_step(o + k, mt ? GX_MATCH : GX_MISMATCH, i, j);
                nmat += mt; nmis += !mt;
                last = mt ? GX_MATCH : GX_MISMATCH;
                ++k; --i; --j;
            } else if (c != 1u) {
                const bool ext = last == GX_DELETE;
                put_step(o + k, ext ? GX_DELETE : GX_OPEN_DELETE, i, j);
                next += ext; nopen += !ext;
                last = GX_DELETE;
                ++k; --i;
            }
            if (i == 0 && j == 0) { done = true; break; }   // (only a diagonal move from (1, 1) gets here)
        }
    }
    _mm_sfence();
    w.steps.set_size(k);
    gx_result& r = w.res;
    r.matches = nmat; r.mismatches = nmis; r.gap_extensions = next; r.opening_gaps = nopen;
    if (!done) {
        const int rc = label_boundary(hs, is_local, s1, n, s2, m, i, j, last, w);
        if (rc) return rc;
    }
    r.n_steps = w.steps.size();
    return GX_OK;
}

// dev_end_E: take each start cell's landing column from the fill's device
// results (global mode, start (n, m)), so the traceback can be queued right
// behind the fill without waiting for its results on the host.
// The traceback of the pairs of one or more fills (jv: their pairs in order,
// `starts` over all of them; the fills share layout and code format), its
// kernels on stream ts (nullptr: the context's stream).
int run_traceback(gx_context* ctx, const std::vector<const FillJob*>& jv, const std::vector<TbStart>& starts,
                  TbOut& out, int slot, bool collect, bool dev_end_E, hipStream_t ts) {
    const size_t P = starts.size();
    const FillJob& job = *jv[0];
    std::vector<const PairDev*> pdv;
    std::vector<const PairRes*> presv;
    for (const FillJob* j : jv)
        for (size_t q = 0; q < j->pd.size(); ++q) { pdv.push_back(&j->pd[q]); presv.push_back((const PairRes*)j->pres.p + q); }
    // (starts may cover a prefix: a table filled as a twin of itself walks its first pair only)
    if (pdv.size() < P) return fail(GX_EINVAL, "traceback: more starts than the fills' pairs");
    if (!ts) ts = ctx->stream;
    std::vector<TbDev> jobs(P);
    std::vector<size_t> so(P);
    size_t stot = 0;   // strips over all pairs
    int max_strips = 1;
    for (size_t p = 0; p < P; ++p) {
        so[p] = stot;
        stot += (size_t)pdv[p]->strips;
        max_strips = std::max(max_strips, pdv[p]->strips);
    }
    // one device block cnt | seg | recs, as the pinned host block it is
    // copied into (one copy: each small copy on a stream costs a runtime
    // round trip, ~100 us between a short batch's walk and its records)
    DevBuf tbb, jb;
    int rc;
    auto cleanup = [&]() { pool_put(ctx, tbb); pool_put(ctx, jb); };
    const int SR = strip_rows(job.lay);
    const size_t nc = 4 * P, nsg = 4 * std::max<size_t>(stot, 1), nhr = std::max<size_t>(stot, 1) * SR;
    if ((rc = pool_get(ctx, (nc + nsg) * sizeof(int) + nhr * sizeof(uint32_t), &tbb, ts)) ||
        (slot < 0 && (rc = pool_get(ctx, P * sizeof(TbDev), &jb, ts)))) {
        cleanup();
        return rc;
    }
    int* const cnt_d = (int*)tbb.p;
    int* const seg_d = cnt_d + nc;
    uint32_t* const recs_d = (uint32_t*)(seg_d + nsg);
    for (size_t p = 0; p < P; ++p) {
        TbDev& t = jobs[p];
        const PairDev& d = *pdv[p];
        t.codes = d.codes;
        t.skel = d.skel;
        t.skel_stride = d.skel_stride;
        t.n = d.n; t.m = d.m; t.t16 = d.t16; t.strips = d.strips;
        t.start_i = starts[p].i; t.start_j = starts[p].j; t.start_E = starts[p].E;
        t.start_E_dev = (dev_end_E && starts[p].i >= 1) ? &presv[p]->end_E : nullptr;
        t.start_ij_dev = (dev_end_E && job.local_on && starts[p].i >= 1) ? &presv[p]->lmax_i : nullptr;
        t.seg = seg_d + 4 * so[p];
        t.recs = recs_d + so[p] * SR;
        t.srows = SR;
        t.skew = job.lay == 3 ? 1 : 0;
        t.skel_half = job.twin ? d.twin_half : -1;
        t.end_ij = cnt_d + 4 * p;
        t.w16 = job.nocodes ? (const uint8_t*)d.pI : nullptr;   // the twin's code plane (shared by its pairs)
        t.w16_half = d.twin_half;
        t.t4 = d.t4;
    }
    (void)presv;
    const size_t jbytes = P * sizeof(TbDev);
    void* jdev = jb.p;
    bool upload = true;
    if (slot >= 0) {   // the slot's table: uploaded again only when it changed (the slot's last walk has ended)
        auto& sl = ctx->slots[slot];
        if (sl.tjob_cap < jbytes) {
            if (sl.tjob) (void)hipFree(sl.tjob);
            sl.tjob = nullptr; sl.tjob_cap = 0; sl.tjob_last.clear();
            if (hipMalloc(&sl.tjob, jbytes) != hipSuccess) { sl.tjob = nullptr; cleanup(); return fail(GX_ENOMEM, "traceback jobs"); }
            sl.tjob_cap = jbytes;
        }
        upload = !(sl.tjob_last.size() == P && !memcmp(sl.tjob_last.data(), jobs.data(), jbytes));
        jdev = sl.tjob;
    }
    hipError_t e = hipSuccess;
    if (upload) {
        TbDev* pin_jobs = (TbDev*)(slot >= 0 ? pinned_grow(ctx->slots[slot].tjpin, jbytes) : io_pinned(ctx, jbytes));
        if (!pin_jobs) { cleanup(); return fail(GX_ENOMEM, "pinned staging buffer"); }
        memcpy(pin_jobs, jobs.data(), jbytes);
        e = hipMemcpyAsync(jdev, pin_jobs, jbytes, hipMemcpyHostToDevice, ts);
        if (slot >= 0) {   // (what the slot's table holds: only an upload that was issued counts)
            if (e == hipSuccess) ctx->slots[slot].tjob_last = jobs;
            else ctx->slots[slot].tjob_last.clear();
        }
    }
    if (e == hipSuccess) e = hipMemsetAsync(seg_d, 0, nsg * sizeof(int), ts);
    hipEvent_t evb = slot >= 0 ? ctx->slots[slot].tb : ctx->ev1, eve = slot >= 0 ? ctx->slots[slot].te : ctx->ev2;
    if (e == hipSuccess) e = hipEventRecord(evb, ts);
    if (e == hipSuccess) e = launch_traceback((const TbDev*)jdev, (int)P, max_strips, job.nocodes, job.noskel, ts);
    if (e == hipSuccess) e = hipEventRecord(eve, ts);
    // one pinned host block: c | sg | hr
    const size_t bytes = (nc + nsg) * sizeof(int) + nhr * sizeof(uint32_t);
    PinnedBuf& recpin = slot >= 0 ? ctx->slots[slot].tbpin : ctx->tb_pin;
    if (e == hipSuccess && !pinned_grow(recpin, bytes)) e = hipErrorOutOfMemory;
    int* c = (int*)recpin.p;
    int* sg = c + nc;
    uint32_t* hr = (uint32_t*)(sg + nsg);
    using clk = std::chrono::steady_clock;
    const auto q0 = clk::now();
    // pipelined: the record copies go on the copy stream after the traceback
    // kernels, so the next fill (queued on the fill stream) starts as soon as
    // the kernels end; the buffers stay held until tb_collect
    hipStream_t cs = collect ? ts : ctx->cstream;
    if (!collect && e == hipSuccess) e = hipStreamWaitEvent(cs, eve, 0);
    if (e == hipSuccess) e = hipMemcpyAsync(c, tbb.p, bytes, hipMemcpyDeviceToHost, cs);
    const auto q1 = clk::now();
    out.c = c; out.sg = sg; out.hr = hr;
    out.so = so;
    out.srows = SR;
    if (!collect) {   // pipelined: tb_collect() waits for the records later
        if (e == hipSuccess) e = hipEventRecord(ctx->slots[slot].tdone, cs);
        DevBuf* h = ctx->slots[slot].held;
        h[0] = tbb; h[1] = DevBuf{}; h[2] = jb; h[3] = DevBuf{};
        if (e != hipSuccess) return fail(GX_EHIP, std::string("traceback: ") + hipGetErrorString(e));
        return GX_OK;
    }
    if (e == hipSuccess) e = hipEventSynchronize(eve);
    const auto q2 = clk::now();
    if (e == hipSuccess) e = hipStreamSynchronize(ts);
    if (const char* lg = getenv("GX_LOG"); lg && !strcmp(lg, "debug"))
        fprintf(stderr, "[gx DEBUG] traceback: D2H enqueue %.3f ms, kernels done +%.3f ms, copies done +%.3f ms\n",
                std::chrono::duration<double, std::milli>(q1 - q0).count(),
                std::chrono::duration<double, std::milli>(q2 - q1).count(),
                std::chrono::duration<double, std::milli>(clk::now() - q2).count());
    cleanup();
    if (e != hipSuccess) return fail(GX_EHIP, std::string("traceback: ") + hipGetErrorString(e));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, evb, eve);
    out.ms = ms;
    out.end_i.resize(P);
    out.end_j.resize(P);
    for (size_t p = 0; p < P; ++p) {
        out.end_i[p] = c[4 * p + 0];
        out.end_j[p] = c[4 * p + 1];
        if (out.end_i[p] < 0) return fail(GX_EHIP, "traceback: landing column out of range (incomplete fill)");
    }
    return GX_OK;
}

int run_traceback(gx_context* ctx, const FillJob& job, const std::vector<TbStart>& starts, TbOut& out,
                  int slot, bool collect, bool dev_end_E) {
    return run_traceback(ctx, std::vector<const FillJob*>{&job}, starts, out, slot, collect, dev_end_E, nullptr);
}

int tb_collect(gx_context* ctx, int slot, size_t P, TbOut& out) {
    auto& s = ctx->slots[slot];
    HIPCHK(hipEventSynchronize(s.tdone));
    release_held(ctx, slot);   // the copies that read them are done
    float ms = 0;
    (void)hipEventElapsedTime(&ms, s.tb, s.te);
    out.ms = ms;
    out.end_i.resize(P);
    out.end_j.resize(P);
    for (size_t p = 0; p < P; ++p) {
        out.end_i[p] = out.c[4 * p + 0];
        out.end_j[p] = out.c[4 * p + 1];
        if (out.end_i[p] < 0) return fail(GX_EHIP, "traceback: landing column out of range (incomplete fill)");
    }
    if (const char* lg = getenv("GX_LOG"); lg && !strcmp(lg, "debug") && P)
        fprintf(stderr, "[gx DEBUG] traceback %.3f ms; pair 0 diag word %u (%u cycles per block, %u walking)\n", ms,
                (unsigned)out.c[3], (unsigned)out.c[3] >> 16, (unsigned)out.c[3] & 0xFFFFu);
    return GX_OK;
}

// Start cell + score (algo.rs:306-331).
int start_cell_common(const HostScores& hs, int is_local, size_t n, size_t m, const StartIn& r,
                      uint64_t* si, uint64_t* sj, int64_t* score) {
    if (!is_local) {
        *si = n; *sj = m;
        if (n >= 1 && m >= 1) *score = r.end_SM;
        else {
            int64_t I, D, S;
            boundary_cell(hs, n, m, &I, &D, &S);
            *score = smax(I, S, D, 0);
        }
        return GX_OK;
    }
    // local: LAST maximum of score_max over all cells in row-major order
    int64_t best = INT64_MIN;
    uint64_t bi = 0, bj = 0;
    auto consider = [&](int64_t v, uint64_t i, uint64_t j) {
        if (v > best || (v == best && (i > bi || (i == bi && j > bj)))) { best = v; bi = i; bj = j; }
    };
    for (uint64_t j = 0; j <= m; ++j) {  // row 0
        int64_t I, D, S;
        boundary_cell(hs, 0, j, &I, &D, &S);
        consider(smax(I, S, D, 1), 0, j);
    }
    for (uint64_t i = 1; i <= n; ++i) {  // column 0
        int64_t I, D, S;
        boundary_cell(hs, i, 0, &I, &D, &S);
        consider(smax(I, S, D, 1), i, 0);
    }
    if (n >= 1 && m >= 1) consider(r.lmax_val, r.lmax_i, r.lmax_j);
    *si = bi; *sj = bj; *score = best;
    return GX_OK;
}

int copy_steps(const Walk& w, gx_step* steps, size_t cap) {
    if (!steps) return GX_OK;
    if (w.steps.size() > cap) return fail(GX_ECAP, "steps capacity " + std::to_string(cap) + " < " +
                                                       std::to_string(w.steps.size()));
    memcpy(steps, w.steps.data(), w.steps.size() * sizeof(gx_step));
    return GX_OK;
}

// ---------------------------------------------------------------------------
// batch of independent pairs (config 4 / 5)

// Labels one batch's walks (host, algo.rs:339-422), pairs on the worker pool:
// interior moves from the device's row records (dev_of[p] >= 0), then the
// analytic boundary; fills walks[p].res.
int label_batch(gx_context* ctx, const std::vector<PairHost>& ph, const HostScores& hs, int is_local, bool track,
                const std::vector<int>& dev_of, const std::vector<uint64_t>& si,
                const std::vector<uint64_t>& sj, const std::vector<int64_t>& score,
                const std::vector<PairRes>& res, const TbOut& tb, double fill_ms, std::vector<Walk>& walks) {
    const size_t P = ph.size();
    walks.resize(P);   // keeps the step buffers of a reused vector
    std::vector<int> prc(P, GX_OK);
    std::vector<std::string> perr(P);
    const std::function<void(size_t)> label_one = [&](size_t p) {
        if (dev_of[p] >= 0)
            prc[p] = label_walk_records(hs, is_local, ph[p].s1, ph[p].n, ph[p].s2, ph[p].m, si[p], sj[p], tb,
                                        (size_t)dev_of[p], walks[p]);
        else
            prc[p] = label_walk(hs, is_local, ph[p].s1, ph[p].n, ph[p].s2, ph[p].m, si[p], sj[p], 0,
                                MovesSrc{nullptr, 0}, walks[p]);
        if (prc[p]) perr[p] = g_err;   // g_err is thread-local
    };
    // the calling thread plus up to 15 pool workers: the 16 CPUs a process
    // gets on the box (1024 x 1k, GCUPS a step by threads: 4 502, 8 707,
    // 12 817, 14 872, 16 906; the labelling writes 24-B gx_steps, ~48 MB a
    // pass, and is on the step's critical path)
    size_t cap = 16;
    if (const char* e = getenv("GX_LABEL_THREADS"); e && atoi(e) > 0) cap = (size_t)atoi(e);
    const size_t nthreads = std::min<size_t>({P, (size_t)std::max(1u, std::thread::hardware_concurrency()), cap});
    if (nthreads <= 1) {
        for (size_t p = 0; p < P; ++p) label_one(p);
    } else {
        ctx->workers.run(P, nthreads - 1, label_one);
    }
    for (size_t p = 0; p < P; ++p) {
        if (prc[p]) return fail(prc[p], perr[p]);
        Walk& w = walks[p];
        const bool interior = ph[p].n >= 1 && ph[p].m >= 1 && track;
        w.res.score = score[p];
        w.res.start_i = si[p]; w.res.start_j = sj[p];
        w.res.max_cell_i = interior ? (uint64_t)res[p].max_i : 0;
        w.res.max_cell_j = interior ? (uint64_t)res[p].max_j : 0;
        w.res.matches_at_max = interior ? (uint64_t)res[p].mam : 0;
        w.res.fill_us = (int64_t)(fill_ms * 1000.0);
        w.res.retrace_us = (int64_t)(tb.ms * 1000.0);
    }
    if (ctx->pass_rec) {   // a staged run keeps every pass's results (this chunk's pairs)
        const size_t base = (size_t)ctx->pass_k * ctx->pass_P + ctx->pass_off;
        if (base + P <= ctx->pass_res.size())
            for (size_t p = 0; p < P; ++p) ctx->pass_res[base + p] = walks[p].res;
        ++ctx->pass_k;
    }
    return GX_OK;
}
