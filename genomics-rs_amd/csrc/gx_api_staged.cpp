// gx_api_staged.cpp -- staged batches (inputs resident in HBM): the
// benchmark path gx_run_staged_steps with its per-pass results, plane
// checksums, alternating pair sets and kept planes (gx_staged_table).
#include "gx_api.h"

// ---------------------------------------------------------------------------
// staged (device-resident inputs) path for benchmarking

extern "C" int gx_stage_pairs(gx_context* ctx, const uint8_t* const* s1, const size_t* n, const uint8_t* const* s2,
                              const size_t* m, size_t npairs) {
    if (!ctx || !s1 || !n || !s2 || !m) return fail(GX_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    HIPCHK(hipSetDevice(ctx->device));
    ctx->st_s1.assign(npairs, {});
    ctx->st_s2.assign(npairs, {});
    ctx->st_off1.assign(npairs, 0);
    ctx->st_off2.assign(npairs, 0);
    ctx->st_alpha = SmallAlpha{};
    for (size_t p = 0; p < npairs; ++p) {
        if (n[p] && m[p]) { ctx->st_alpha.add(s1[p], n[p]); ctx->st_alpha.add(s2[p], m[p]); }
    }
    size_t tot = 0;
    for (size_t p = 0; p < npairs; ++p) {
        ctx->st_s1[p].assign(s1[p], s1[p] + n[p]);
        ctx->st_s2[p].assign(s2[p], s2[p] + m[p]);
        ctx->st_off1[p] = tot; tot += align_up(n[p], 64);
        ctx->st_off2[p] = tot; tot += align_up(m[p], 64);
    }
    std::vector<uint8_t> hc(std::max<size_t>(tot, 1), 0);
    for (size_t p = 0; p < npairs; ++p) {
        if (n[p]) memcpy(&hc[ctx->st_off1[p]], s1[p], n[p]);
        if (m[p]) memcpy(&hc[ctx->st_off2[p]], s2[p], m[p]);
    }
    if (ctx->st_chars.p) { (void)hipFree(ctx->st_chars.p); ctx->st_chars = DevBuf{}; }
    HIPCHK(hipMalloc(&ctx->st_chars.p, hc.size()));
    ctx->st_chars.cap = hc.size();
    HIPCHK(hipMemcpy(ctx->st_chars.p, hc.data(), hc.size(), hipMemcpyHostToDevice));
    return GX_OK;
}

// GX_STAGED_ALTERNATE (gx.h): pass k over staged pairs k % 2 * H .. + H - 1.
static int run_staged_alternate(gx_context* ctx, const std::vector<PairHost>& ph,
                                const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc,
                                const HostScores& hs, const Scores32& sc, int is_local, bool planes, bool track,
                                bool want_sums, int passes, gx_result* out, double* fill_ms_out) {
    const size_t P = ph.size(), H = P / 2;
    if (P == 0 || P % 2) return fail(GX_EINVAL, "alternating sets: an even, non-zero number of staged pairs");
    for (size_t p = 0; p < H; ++p)
        if (ph[p].n != ph[p + H].n || ph[p].m != ph[p + H].m)
            return fail(GX_EINVAL, "alternating sets: pair " + std::to_string(p) + " and " + std::to_string(p + H) +
                                       " differ in shape");
    const double bpc = planes ? ((!track && !getenv("GX_PLANES32") && d8_planes_ok(sc, is_local)) ? 3.0 : 12.0) : 0.0;
    std::vector<PairHost> ph0(ph.begin(), ph.begin() + (long)H), ph1(ph.begin() + (long)H, ph.end());
    if (plan_chunks(ctx, ph0, bpc).size() != 1) return fail(GX_EINVAL, "alternating sets must fit one chunk");
    std::vector<std::pair<const uint8_t*, const uint8_t*>> pr0(proc.begin(), proc.begin() + (long)H),
        pr1(proc.begin() + (long)H, proc.end());
    std::vector<size_t> a1(ctx->st_off1.begin(), ctx->st_off1.begin() + (long)H),
        a2(ctx->st_off2.begin(), ctx->st_off2.begin() + (long)H), b1(ctx->st_off1.begin() + (long)H, ctx->st_off1.end()),
        b2(ctx->st_off2.begin() + (long)H, ctx->st_off2.end());
    // checksum records in the order the fills write them: pass, then its set's pairs with an interior
    std::vector<std::pair<int, size_t>> sum_order;
    for (int k = 0; k < passes; ++k)
        for (size_t p = 0; p < H; ++p)
            if (ph[p].n >= 1 && ph[p].m >= 1) sum_order.emplace_back(k, (size_t)(k & 1) * H + p);
    ctx->sums_host.clear();
    if (want_sums && !sum_order.empty()) {
        const size_t bytes = sum_order.size() * 3 * sizeof(unsigned long long);
        if (ctx->sums_dev.cap < bytes) {
            if (ctx->sums_dev.p) (void)hipFree(ctx->sums_dev.p);
            ctx->sums_dev = DevBuf{};
            HIPCHK(hipMalloc(&ctx->sums_dev.p, bytes));
            ctx->sums_dev.cap = bytes;
        }
        HIPCHK(hipMemsetAsync(ctx->sums_dev.p, 0, bytes, ctx->stream));
        ctx->sums_dst = (unsigned long long*)ctx->sums_dev.p;
    }
    std::vector<Walk> w0, w1;
    PassSet alt{&ph1, &pr1, &b1, &b2, &w1, H};
    ctx->pass_off = 0;
    double fms = 0;
    int rc = batch_core_steps(ctx, ph0, pr0, hs, sc, is_local, planes, track, passes, w0, &fms,
                              (const uint8_t*)ctx->st_chars.p, &a1, &a2, &ctx->st_alpha, &alt);
    ctx->last_chunks = 1;
    const size_t filled = ctx->sums_dst ? (size_t)(ctx->sums_dst - (unsigned long long*)ctx->sums_dev.p) : 0;
    ctx->sums_dst = nullptr;
    if (rc) return rc;
    if (want_sums) {
        ctx->sums_host.assign((size_t)passes * P * 3, 0);
        if (!sum_order.empty()) {
            if (filled != sum_order.size() * 3)
                return fail(GX_EHIP, "plane sums: " + std::to_string(filled / 3) + " pair records, expected " +
                                         std::to_string(sum_order.size()));
            std::vector<uint64_t> dev(filled);
            HIPCHK(hipStreamSynchronize(ctx->stream));
            HIPCHK(hipMemcpy(dev.data(), ctx->sums_dev.p, filled * sizeof(uint64_t), hipMemcpyDeviceToHost));
            for (size_t r = 0; r < sum_order.size(); ++r)
                for (int c = 0; c < 3; ++c)
                    ctx->sums_host[((size_t)sum_order[r].first * P + sum_order[r].second) * 3 + c] = dev[r * 3 + c];
        }
    }
    std::vector<Walk>& walks = ctx->walk_cache;
    walks.resize(P);
    for (size_t p = 0; p < H; ++p) {
        if (p < w0.size()) std::swap(walks[p], w0[p]);
        if (p < w1.size()) std::swap(walks[H + p], w1[p]);
    }
    for (size_t p = 0; p < P; ++p) out[p] = walks[p].res;
    if (fill_ms_out) *fill_ms_out = fms;
    return GX_OK;
}

extern "C" int gx_run_staged_steps(gx_context* ctx, const gx_scores* scores, int is_local, int keep_planes,
                                   uint32_t flags, int nsteps, gx_result* out, double* fill_ms_out) {
    if (!ctx || !out) return fail(GX_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    HIPCHK(hipSetDevice(ctx->device));
    const size_t P = ctx->st_s1.size();
    size_t nmax = 0, mmax = 0;
    for (size_t p = 0; p < P; ++p) { nmax = std::max(nmax, ctx->st_s1[p].size()); mmax = std::max(mmax, ctx->st_s2[p].size()); }
    HostScores hs;
    Scores32 sc;
    bool wide = false;
    int rc = check_scores(scores, nmax, mmax, &hs, &sc, is_local, &wide);
    if (rc) return rc;
    std::vector<PairHost> ph(P);
    std::vector<std::pair<const uint8_t*, const uint8_t*>> proc(P);
    for (size_t p = 0; p < P; ++p) {
        ph[p] = PairHost{ctx->st_s1[p].data(), ctx->st_s2[p].data(), ctx->st_s1[p].size(), ctx->st_s2[p].size()};
        proc[p] = {ph[p].s1, ph[p].s2};
    }
    const bool track = (flags & GX_ALIGN_MAX_CELL) != 0;
    // every pass's results (label_batch records them; chunks set pass_off)
    struct PassRec {
        gx_context* c;
        ~PassRec() { c->pass_rec = false; c->keep_capture = false; }
    } pass_guard{ctx};
    ctx->kept.reset();   // (a previous run's kept planes: their tables hold their own reference)
    if (flags & GX_STAGED_KEEP_PLANES) {
        if (!keep_planes) return fail(GX_EINVAL, "GX_STAGED_KEEP_PLANES needs keep_planes");
        if (flags & GX_STAGED_ALTERNATE) return fail(GX_EINVAL, "GX_STAGED_KEEP_PLANES with alternating sets");
        ctx->keep_capture = true;
        ctx->kept_hs = hs;
        ctx->kept_sc = sc;
    }
    ctx->pass_res.assign((size_t)std::max(nsteps, 1) * P, gx_result{});
    ctx->pass_rec = true;
    ctx->pass_P = P;
    ctx->pass_off = 0;
    ctx->pass_k = 0;
    if (wide && (flags & GX_STAGED_ALTERNATE)) return fail(GX_EINVAL, "alternating sets: not on the int64 fill");
    if (wide && ctx->keep_capture) return fail(GX_EINVAL, "GX_STAGED_KEEP_PLANES: not on the int64 fill");
    if (wide) {   // int64 fill: one synchronous pass at a time (a rare path, no pipelining or chunking)
        std::vector<Walk>& walks = ctx->walk_cache;
        const int passes = std::max(nsteps, 1);
        const bool want_sums = (flags & GX_STAGED_PLANE_SUMS) && keep_planes;
        size_t nint = 0;
        for (size_t p = 0; p < P; ++p) nint += (ph[p].n >= 1 && ph[p].m >= 1);
        ctx->sums_host.clear();
        if (want_sums && nint) {
            const size_t bytes = (size_t)passes * nint * 3 * sizeof(unsigned long long);
            if (ctx->sums_dev.cap < bytes) {
                if (ctx->sums_dev.p) (void)hipFree(ctx->sums_dev.p);
                ctx->sums_dev = DevBuf{};
                HIPCHK(hipMalloc(&ctx->sums_dev.p, bytes));
                ctx->sums_dev.cap = bytes;
            }
            ctx->sums_dst = (unsigned long long*)ctx->sums_dev.p;
        }
        double fsum = 0;
        for (int k = 0; k < passes && !rc; ++k) {
            double f = 0;
            rc = batch_core_wide(ctx, ph, proc, hs, is_local, keep_planes != 0, track, walks, &f);
            fsum += f;
        }
        ctx->sums_dst = nullptr;
        ctx->last_chunks = 1;
        if (rc) return rc;
        if (want_sums) {
            ctx->sums_host.assign((size_t)passes * P * 3, 0);
            if (nint) {
                std::vector<uint64_t> dev((size_t)passes * nint * 3);
                HIPCHK(hipMemcpy(dev.data(), ctx->sums_dev.p, dev.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
                size_t r = 0;
                for (int k = 0; k < passes; ++k)
                    for (size_t p = 0; p < P; ++p)
                        if (ph[p].n >= 1 && ph[p].m >= 1) {
                            for (int c = 0; c < 3; ++c) ctx->sums_host[((size_t)k * P + p) * 3 + c] = dev[r * 3 + c];
                            ++r;
                        }
            }
        }
        for (size_t p = 0; p < P; ++p) out[p] = walks[p].res;
        if (fill_ms_out) *fill_ms_out = fsum / passes;
        return GX_OK;
    }
    std::vector<Walk>& walks = ctx->walk_cache;
    // GX_STAGED_PLANE_SUMS: every pass's fill is followed by the plane
    // checksum kernel (stream order, before the planes return to the pool)
    const bool want_sums = (flags & GX_STAGED_PLANE_SUMS) && keep_planes;
    const int passes = std::max(nsteps, 1);
    if (flags & GX_STAGED_ALTERNATE)
        return run_staged_alternate(ctx, ph, proc, hs, sc, is_local, keep_planes != 0, track, want_sums, passes, out,
                                    fill_ms_out);
    // chunks: each runs its `passes` passes pipelined (pass k's labelling
    // beside pass k+1's fill); a step is still one pass over every pair
    const double bpc = keep_planes ? ((!track && !getenv("GX_PLANES32") && d8_planes_ok(sc, is_local)) ? 3.0 : 12.0)
                                   : 0.0;
    const auto chunks = plan_chunks(ctx, ph, bpc);
    if (ctx->keep_capture && chunks.size() != 1) return fail(GX_EINVAL, "GX_STAGED_KEEP_PLANES needs one chunk");
    // the order in which the fills write their checksum records: chunk, pass, pair with an interior
    std::vector<std::pair<int, size_t>> sum_order;
    for (const auto& c : chunks)
        for (int k = 0; k < passes; ++k)
            for (size_t p = c.first; p < c.second; ++p)
                if (ph[p].n >= 1 && ph[p].m >= 1) sum_order.emplace_back(k, p);
    ctx->sums_host.clear();
    if (want_sums && !sum_order.empty()) {
        const size_t bytes = sum_order.size() * 3 * sizeof(unsigned long long);
        if (ctx->sums_dev.cap < bytes) {
            if (ctx->sums_dev.p) (void)hipFree(ctx->sums_dev.p);
            ctx->sums_dev = DevBuf{};
            HIPCHK(hipMalloc(&ctx->sums_dev.p, bytes));
            ctx->sums_dev.cap = bytes;
        }
        HIPCHK(hipMemsetAsync(ctx->sums_dev.p, 0, bytes, ctx->stream));
        ctx->sums_dst = (unsigned long long*)ctx->sums_dev.p;
    }
    double fms = 0;
    if (chunks.size() == 1) {
        rc = batch_core_steps(ctx, ph, proc, hs, sc, is_local, keep_planes != 0, track, passes, walks, &fms,
                              (const uint8_t*)ctx->st_chars.p, &ctx->st_off1, &ctx->st_off2, &ctx->st_alpha);
    } else {
        walks.resize(P);
        std::vector<Walk> wc;
        for (const auto& c : chunks) {
            const size_t a = c.first, b = c.second;
            std::vector<PairHost> phc(ph.begin() + a, ph.begin() + b);
            std::vector<std::pair<const uint8_t*, const uint8_t*>> pc(proc.begin() + a, proc.begin() + b);
            std::vector<size_t> o1(ctx->st_off1.begin() + a, ctx->st_off1.begin() + b),
                o2(ctx->st_off2.begin() + a, ctx->st_off2.begin() + b);
            ctx->pass_off = a;
            ctx->pass_k = 0;
            double f = 0;
            rc = batch_core_steps(ctx, phc, pc, hs, sc, is_local, keep_planes != 0, track, passes, wc, &f,
                                  (const uint8_t*)ctx->st_chars.p, &o1, &o2, &ctx->st_alpha);
            if (rc) break;
            fms += f;   // a pass over every pair = one pass of each chunk
            for (size_t k = 0; k < b - a; ++k) std::swap(walks[a + k], wc[k]);
        }
    }
    ctx->last_chunks = (int)chunks.size();
    const size_t filled = ctx->sums_dst ? (size_t)(ctx->sums_dst - (unsigned long long*)ctx->sums_dev.p) : 0;
    ctx->sums_dst = nullptr;
    if (rc) return rc;
    if (want_sums) {
        ctx->sums_host.assign((size_t)passes * P * 3, 0);
        if (!sum_order.empty()) {
            if (filled != sum_order.size() * 3)
                return fail(GX_EHIP, "plane sums: " + std::to_string(filled / 3) + " pair records, expected " +
                                         std::to_string(sum_order.size()));
            std::vector<uint64_t> dev(filled);
            HIPCHK(hipStreamSynchronize(ctx->stream));
            HIPCHK(hipMemcpy(dev.data(), ctx->sums_dev.p, filled * sizeof(uint64_t), hipMemcpyDeviceToHost));
            for (size_t r = 0; r < sum_order.size(); ++r)
                for (int c = 0; c < 3; ++c)
                    ctx->sums_host[((size_t)sum_order[r].first * P + sum_order[r].second) * 3 + c] = dev[r * 3 + c];
        }
    }
    for (size_t p = 0; p < P; ++p) out[p] = walks[p].res;
    if (fill_ms_out) *fill_ms_out = fms;
    return GX_OK;
}

extern "C" int gx_staged_table(gx_context* ctx, size_t pair, gx_table** table_out) {
    if (!ctx || !table_out) return fail(GX_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    HIPCHK(hipSetDevice(ctx->device));
    const std::shared_ptr<KeptFill> k = ctx->kept;
    if (!k) return fail(GX_EINVAL, "no kept planes: run gx_run_staged_steps with GX_STAGED_KEEP_PLANES");
    if (pair >= ctx->st_s1.size() || pair >= k->dev_of.size()) return fail(GX_EINVAL, "no such staged pair");
    const size_t n = ctx->st_s1[pair].size(), m = ctx->st_s2[pair].size();
    gx_table* t = new gx_table();
    t->ctx = ctx;
    t->is_local = k->job.local_on ? 1 : 0;
    t->flags = GX_TABLE_PLANES;
    t->hs = ctx->kept_hs;
    t->sc = ctx->kept_sc;
    t->s1 = ctx->st_s1[pair];
    t->s2 = ctx->st_s2[pair];
    int rc = processed_chars(t->s1.data(), n, t->s2.data(), m, 0, t->c1, t->c2);
    if (rc) { delete t; return rc; }
    // a view of the kept job: its flags and this pair's descriptor and
    // results; the device buffers stay the kept job's (t->share), but for a
    // descriptor block of its own (the plane checksum kernel reads it)
    FillJob& j = t->job;
    const FillJob& kj = k->job;
    j.lay = kj.lay; j.W = kj.W; j.planes_on = kj.planes_on; j.d8 = kj.d8; j.shift = kj.shift; j.twin = kj.twin;
    j.w16 = kj.w16; j.nocodes = kj.nocodes; j.noskel = kj.noskel; j.local_on = kj.local_on; j.g = kj.g;
    j.fill_ms = kj.fill_ms; j.table = true;
    const int q = k->dev_of[pair];
    if (q >= 0) {
        j.pd.assign(1, kj.pd[(size_t)q]);
        j.res.assign(1, (size_t)q < kj.res.size() ? kj.res[(size_t)q] : PairRes{});
        if ((rc = pool_get(ctx, sizeof(PairDev), &j.pairs))) { delete t; return rc; }
        HIPCHK(hipMemcpy(j.pairs.p, &j.pd[0], sizeof(PairDev), hipMemcpyHostToDevice));
    } else {
        j.pd.assign(1, PairDev{});
        j.pd[0].n = (int)n; j.pd[0].m = (int)m;
        j.res.assign(1, PairRes{});
    }
    t->share = k;
    *table_out = t;
    return GX_OK;
}

extern "C" int gx_staged_plane_sums(const gx_context* ctx, uint64_t* out, size_t cap, size_t* n_values) {
    if (!ctx) return fail(GX_EINVAL, "context is NULL");
    if (n_values) *n_values = ctx->sums_host.size();
    if (!out) return GX_OK;
    if (cap < ctx->sums_host.size()) return fail(GX_ECAP, "out too small");
    std::copy(ctx->sums_host.begin(), ctx->sums_host.end(), out);
    return GX_OK;
}

extern "C" int gx_staged_pass_results(const gx_context* ctx, gx_result* out, size_t cap, size_t* n_values) {
    if (!ctx) return fail(GX_EINVAL, "context is NULL");
    if (n_values) *n_values = ctx->pass_res.size();
    if (!out) return GX_OK;
    if (cap < ctx->pass_res.size()) return fail(GX_ECAP, "out too small");
    std::copy(ctx->pass_res.begin(), ctx->pass_res.end(), out);
    return GX_OK;
}

extern "C" int gx_staged_steps(const gx_context* ctx, size_t pair, gx_step* steps, size_t cap, size_t* n_steps) {
    if (!ctx) return fail(GX_EINVAL, "context is NULL");
    if (pair >= ctx->walk_cache.size() || pair >= ctx->st_s1.size())
        return fail(GX_EINVAL, "no such staged pair in the last run");
    const Walk& w = ctx->walk_cache[pair];
    if (n_steps) *n_steps = w.steps.size();
    if (!steps) return GX_OK;
    return copy_steps(w, steps, cap);
}

extern "C" int gx_batch_chunks(const gx_context* ctx) { return ctx ? ctx->last_chunks : -1; }
extern "C" int gx_fill_twin(const gx_context* ctx) { return ctx ? ctx->last_twin : -1; }
extern "C" int gx_fill_groups(const gx_context* ctx) { return ctx ? ctx->last_groups : -1; }
extern "C" int gx_fill_plane_bits(const gx_context* ctx) { return ctx ? ctx->last_pbits : -1; }

extern "C" int gx_fill_info(const gx_context* ctx, int* layout, int* band_waves, int* plane_bytes_per_cell) {
    if (!ctx) return fail(GX_EINVAL, "context is NULL");
    if (layout) *layout = ctx->last_lay;
    if (band_waves) *band_waves = ctx->last_W;
    if (plane_bytes_per_cell) *plane_bytes_per_cell = ctx->last_pbytes;
    return GX_OK;
}

extern "C" int gx_run_staged(gx_context* ctx, const gx_scores* scores, int is_local, int keep_planes, uint32_t flags,
                             gx_result* out, double* fill_ms_out) {
    return gx_run_staged_steps(ctx, scores, is_local, keep_planes, flags, 1, out, fill_ms_out);
}
