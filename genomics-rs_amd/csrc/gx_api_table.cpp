// gx_api_table.cpp -- the reference's alignment API on one pair:
//   alignment_table  src/alignment/algo.rs:151-282  -> gx_alignment_table
//   retrace          src/alignment/algo.rs:287-441  -> gx_retrace
// plus the table's exports (planes, rows, cells, checksums) and gx_align.
#include "gx_api.h"

static int start_cell(const gx_table* t, const StartIn& r, uint64_t* si, uint64_t* sj, int64_t* score) {
    return start_cell_common(t->hs, t->is_local, t->s1.size(), t->s2.size(), r, si, sj, score);
}

extern "C" int gx_alignment_table(gx_context* ctx, const uint8_t* s1, size_t n, const uint8_t* s2, size_t m,
                                  const gx_scores* scores, int is_local, int reverse_sequences, uint32_t flags,
                                  gx_table** table_out, uint64_t* matches_at_max) {
    if (!ctx || !table_out) return fail(GX_EINVAL, "ctx/table_out is NULL");
    if ((n && !s1) || (m && !s2)) return fail(GX_EINVAL, "sequence pointer is NULL");
    std::lock_guard<std::mutex> lk(ctx->mu);
    HIPCHK(hipSetDevice(ctx->device));
    gx_table* t = new gx_table();
    t->ctx = ctx;
    t->is_local = is_local;
    t->flags = flags;
    bool wide = false;
    int rc = check_scores(scores, n, m, &t->hs, &t->sc, is_local, &wide);
    if (!rc) rc = processed_chars(s1, n, s2, m, reverse_sequences, t->c1, t->c2);
    if (rc) { delete t; return rc; }
    t->s1.assign(s1, s1 + n);
    t->s2.assign(s2, s2 + m);
    if (log_info()) {
        fprintf(stderr, "[gx INFO] Sequence table shape: [%zu, %zu]\n", n + 1, m + 1);
    }
    std::vector<PairHost> ph{PairHost{t->s1.data(), t->s2.data(), n, m}};
    std::vector<std::pair<const uint8_t*, const uint8_t*>> proc{{t->c1.data(), t->c2.data()}};
    // GX_TABLE_TWIN=1 (verification): fill the table with the twin fill, the
    // pair beside a copy of itself, so that its planes can be exported
    if (const char* e = getenv("GX_TABLE_TWIN"); e && !strcmp(e, "1") && !wide) {
        ph.push_back(ph[0]);
        proc.push_back(proc[0]);
    }
    const bool planes = (flags & (GX_TABLE_PLANES | GX_TABLE_MATCHES)) != 0;
    const bool lcs = (flags & GX_TABLE_MATCHES) != 0;
    if (n >= 1 && m >= 1) {
        t->job.table = true;   // exportable planes: the per-pair formats only
        SmallAlpha alpha;      // (the batch paths' small-alphabet score table)
        alpha.add(t->c1.data(), n);
        alpha.add(t->c2.data(), m);
        rc = wide ? run_fill_wide(ctx, proc, ph, t->hs, is_local, planes, matches_at_max != nullptr, lcs, t->job)
                  : run_fill(ctx, proc, ph, t->sc, is_local, planes, matches_at_max != nullptr, lcs, t->job, nullptr,
                             nullptr, nullptr, &alpha);
        if (rc) { job_release(ctx, t->job); delete t; return rc; }
    } else {
        t->job.res.assign(1, PairRes{});
        t->job.pd.assign(1, PairDev{});
        t->job.pd[0].n = (int)n; t->job.pd[0].m = (int)m;
    }
    if (log_info())
        fprintf(stderr, "[gx INFO] Table initialization complete, time taken: %lldus\n",
                (long long)(t->job.fill_ms * 1000.0));
    if (matches_at_max)
        *matches_at_max = (n >= 1 && m >= 1) ? (t->job.wide ? t->job.wres[0].mam : (uint64_t)t->job.res[0].mam) : 0;
    *table_out = t;
    return GX_OK;
}

extern "C" int gx_table_info(const gx_table* t, uint64_t* n_rows, uint64_t* n_cols, uint64_t* max_cell_i,
                             uint64_t* max_cell_j, int64_t* fill_us) {
    if (!t) return fail(GX_EINVAL, "table is NULL");
    const bool interior = t->s1.size() >= 1 && t->s2.size() >= 1 && t->job.track_on;
    if (n_rows) *n_rows = t->s1.size() + 1;
    if (n_cols) *n_cols = t->s2.size() + 1;
    if (max_cell_i) *max_cell_i = interior ? (uint64_t)t->job.res[0].max_i : 0;
    if (max_cell_j) *max_cell_j = interior ? (uint64_t)t->job.res[0].max_j : 0;
    if (fill_us) *fill_us = (int64_t)(t->job.fill_ms * 1000.0);
    return GX_OK;
}

// Interior of rows row0 .. row0 + rows - 1 of one plane as int32, row-major
// rows x (m+1) (slots of row 0 and column 0 undefined).
static int fetch_rows32(const gx_table* t, int which, size_t row0, size_t rows, std::vector<int32_t>& out) {
    const size_t n = t->s1.size(), m = t->s2.size();
    out.assign(rows * (m + 1), 0);
    if (n == 0 || m == 0 || rows == 0) return GX_OK;
    const PairDev& d = t->job.pd[0];
    const int32_t* src = which == 0 ? d.pI : which == 1 ? d.pD : which == 2 ? d.pS : d.pL;
    if (t->job.w16) src = which <= 2 ? d.pI : nullptr;   // (one code plane holds all three)
    if (!src) return fail(GX_EINVAL, "plane not kept: build the table with GX_TABLE_PLANES / GX_TABLE_MATCHES");
    gx_context* ctx = t->ctx;
    DevBuf tmp;
    int rc = pool_get(ctx, out.size() * sizeof(int32_t), &tmp);
    if (rc) return rc;
    hipError_t e;
    if (t->job.w16)   // twin plane codes (staged tables): this pair's half of the twin's code plane
        e = launch_export_w16((const uint8_t*)d.pI, d.twin_half, which, (int32_t*)tmp.p, (int)n, (int)m, d.t4,
                              t->sc.h, t->sc.g, t->sc.floor_, t->sc.g, (int)row0, (int)rows, ctx->stream);
    else if (t->job.d8)   // compact planes: rebuilt from the insert plane's running sum (+ this plane's x)
        e = launch_export_d8((const uint8_t*)d.pI, which == 0 ? nullptr : (const uint8_t*)src, (int32_t*)tmp.p,
                             (int)n, (int)m, d.t4, t->sc.h, t->sc.g, t->sc.floor_, t->job.shift ? t->sc.g : 0,
                             (int)row0, (int)rows, ctx->stream);
    else
        e = launch_export(src, (int32_t*)tmp.p, (int)n, (int)m, d.t4, t->job.lay, t->job.shift ? t->sc.g : 0,
                          (int)row0, (int)rows, ctx->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(out.data(), tmp.p, out.size() * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    pool_put(ctx, tmp);
    if (e != hipSuccess) return fail(GX_EHIP, std::string("export: ") + hipGetErrorString(e));
    return GX_OK;
}

// Interior of one plane as int32 row-major (n+1)x(m+1) (boundary slots undefined).
static int fetch_plane32(const gx_table* t, int which, std::vector<int32_t>& out) {
    return fetch_rows32(t, which, 0, t->s1.size() + 1, out);
}

// max_matches of the interior cells of rows row0 .. row0 + rows - 1,
// row-major rows x (m+1) (row 0 and column 0: 0), from a layout-3 fill's LCS
// bit rows (gx_lcs.h): LM(i, j) = j - popcount(V_i & (2^j - 1)).
static int fetch_lcs_rows(const gx_table* t, size_t row0, size_t rows, std::vector<int32_t>& out) {
    const size_t n = t->s1.size(), m = t->s2.size();
    out.assign(rows * (m + 1), 0);
    const PairDev& d = t->job.pd[0];
    if (n == 0 || m == 0 || rows == 0) return GX_OK;
    if (!d.lbits || d.lwords <= 0 || !((d.lcs_waves >> 16) & 1))
        return fail(GX_EINVAL, "LCS rows not kept: build the table with GX_TABLE_MATCHES");
    const size_t i0 = std::max<size_t>(row0, 1), i1 = std::min(row0 + rows, n + 1);
    if (i1 <= i0) return GX_OK;
    // (the rows' strips: bits[strip][step][lane], gx_lcs.h lcs_word_index)
    const size_t s0 = (i0 - 1) / kWave, s1 = (i1 - 2) / kWave + 1, T = (size_t)lcs_steps(d.lwords);
    std::vector<unsigned long long> bits((s1 - s0) * T * kWave);
    HIPCHK(hipMemcpy(bits.data(), d.lbits + s0 * T * kWave, bits.size() * sizeof(unsigned long long),
                     hipMemcpyDeviceToHost));
    const size_t base = s0 * T * kWave;
    for (size_t i = i0; i < i1; ++i) {
        int32_t* o = &out[(i - row0) * (m + 1)];
        int32_t ones = 0;
        for (size_t j = 1; j <= m; ++j) {
            const unsigned long long wv = bits[lcs_word_index((int)i, (int)((j - 1) / kLcsBits), d.lwords) - base];
            ones += (int32_t)((wv >> ((j - 1) % kLcsBits)) & 1u);
            o[j] = (int32_t)j - ones;
        }
    }
    return GX_OK;
}
static int fetch_lcs_plane(const gx_table* t, std::vector<int32_t>& out) {
    return fetch_lcs_rows(t, 0, t->s1.size() + 1, out);
}

// The int64 fill's planes: rows row0 .. row0 + rows - 1 of plane `which`
// (0-2; 3 = the LCS plane) as int64, rows x (m+1) (column 0 and row 0 undefined).
static int fetch_rows_wide(const gx_table* t, int which, size_t row0, size_t rows, std::vector<int64_t>& out) {
    const size_t n = t->s1.size(), m = t->s2.size();
    out.assign(rows * (m + 1), 0);
    if (n == 0 || m == 0 || rows == 0) return GX_OK;
    const WideDev& w = t->job.wd[0];
    if (!w.pI || (which == 3 && !w.pL))
        return fail(GX_EINVAL, "plane not kept: build the table with GX_TABLE_PLANES / GX_TABLE_MATCHES");
    const size_t i0 = std::max<size_t>(row0, 1), i1 = std::min(row0 + rows, n + 1);
    if (i1 <= i0) return GX_OK;
    std::vector<int64_t> tmp((i1 - i0) * m);
    std::vector<unsigned> tl;
    hipError_t e;
    if (which == 3) {
        tl.resize((i1 - i0) * m);
        e = hipMemcpy(tl.data(), w.pL + (i0 - 1) * m, tl.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
        for (size_t k = 0; k < tl.size(); ++k) tmp[k] = tl[k];
    } else {
        const long long* src = which == 0 ? w.pI : which == 1 ? w.pD : w.pS;
        e = hipMemcpy(tmp.data(), src + (i0 - 1) * m, tmp.size() * sizeof(int64_t), hipMemcpyDeviceToHost);
    }
    if (e != hipSuccess) return fail(GX_EHIP, std::string("export: ") + hipGetErrorString(e));
    for (size_t i = i0; i < i1; ++i)
        memcpy(&out[(i - row0) * (m + 1) + 1], &tmp[(i - i0) * m], m * sizeof(int64_t));
    return GX_OK;
}

// Rows row0 .. row0 + rows - 1 of plane `which` as int64 into out (row-major
// rows x (m+1), or column-major with leading dimension ld_rows when colmajor).
static int export_rows(const gx_table* t, int which, size_t row0, size_t rows, int64_t* out, int colmajor,
                       size_t ld_rows) {
    const size_t m = t->s2.size();
    std::vector<int32_t> p32;
    std::vector<int64_t> p64;
    if (which == 3 && !t->job.lcs_on)
        return fail(GX_EINVAL, "max_matches not kept: build the table with GX_TABLE_MATCHES");
    int rc = t->job.wide ? fetch_rows_wide(t, which, row0, rows, p64)
             : (which == 3 && t->job.lcs_rows) ? fetch_lcs_rows(t, row0, rows, p32)
                                               : fetch_rows32(t, which, row0, rows, p32);
    if (rc) return rc;
    for (size_t r = 0; r < rows; ++r) {
        const size_t i = row0 + r;
        for (size_t j = 0; j <= m; ++j) {
            int64_t v;
            if (which == 3 && (i == 0 || j == 0)) {
                v = 0;   // (boundary cells match nothing, algo.rs:195-220)
            } else if (i == 0 || j == 0) {
                int64_t I, D, S;
                boundary_cell(t->hs, i, j, &I, &D, &S);
                v = which == 0 ? I : which == 1 ? D : S;
            } else {
                v = t->job.wide ? p64[r * (m + 1) + j] : p32[r * (m + 1) + j];
            }
            out[colmajor ? r + j * ld_rows : r * (m + 1) + j] = v;
        }
    }
    return GX_OK;
}

extern "C" int gx_table_export_plane(const gx_table* t, int which, int64_t* out, size_t out_cells, int colmajor) {
    if (!t || !out) return fail(GX_EINVAL, "NULL argument");
    if (which < 0 || which > 2) return fail(GX_EINVAL, "which must be 0 (insert), 1 (delete) or 2 (sub)");
    const size_t n = t->s1.size(), m = t->s2.size();
    if (out_cells < (n + 1) * (m + 1)) return fail(GX_ECAP, "out too small");
    std::lock_guard<std::mutex> lk(t->ctx->mu);
    HIPCHK(hipSetDevice(t->ctx->device));
    return export_rows(t, which, 0, n + 1, out, colmajor, n + 1);
}

extern "C" int gx_table_export_rows(const gx_table* t, int which, size_t row0, size_t rows, int64_t* out,
                                    size_t out_cells) {
    if (!t || (!out && rows)) return fail(GX_EINVAL, "NULL argument");
    if (which < 0 || which > 3)
        return fail(GX_EINVAL, "which must be 0 (insert), 1 (delete), 2 (sub) or 3 (max_matches)");
    const size_t n = t->s1.size(), m = t->s2.size();
    if (row0 > n + 1 || rows > n + 1 - row0) return fail(GX_EINVAL, "row range outside the table");
    if (out_cells < rows * (m + 1)) return fail(GX_ECAP, "out too small");
    if (rows == 0) return GX_OK;
    std::lock_guard<std::mutex> lk(t->ctx->mu);
    HIPCHK(hipSetDevice(t->ctx->device));
    return export_rows(t, which, row0, rows, out, 0, rows);
}

extern "C" int gx_table_plane_sums(const gx_table* t, uint64_t* sums) {
    if (!t || !sums) return fail(GX_EINVAL, "NULL argument");
    const size_t n = t->s1.size(), m = t->s2.size();
    sums[0] = sums[1] = sums[2] = 0;
    if (n == 0 || m == 0) return GX_OK;
    if (t->job.wide ? !t->job.wd[0].pI : !t->job.pd[0].pI)
        return fail(GX_EINVAL, "planes not kept: build the table with GX_TABLE_PLANES / GX_TABLE_MATCHES");
    gx_context* ctx = t->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    HIPCHK(hipSetDevice(ctx->device));
    DevBuf buf;
    // (a GX_TABLE_TWIN table holds the pair twice: room for both; pair 0's are returned)
    const size_t np = t->job.wide ? 1 : std::max<size_t>(t->job.pd.size(), 1);
    int rc = pool_get(ctx, 3 * np * sizeof(unsigned long long), &buf);
    if (rc) return rc;
    const WideDev* w = t->job.wide ? &t->job.wd[0] : nullptr;
    hipError_t e = w ? launch_wide_plane_sums((const int64_t*)w->pI, (const int64_t*)w->pD, (const int64_t*)w->pS,
                                              w->n, w->m, (unsigned long long*)buf.p, ctx->stream)
                     : enqueue_plane_sums(ctx, t->job, t->sc, (unsigned long long*)buf.p);
    if (e == hipSuccess) e = hipMemcpyAsync(sums, buf.p, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    pool_put(ctx, buf);
    if (e != hipSuccess) return fail(GX_EHIP, std::string("plane sums: ") + hipGetErrorString(e));
    return GX_OK;
}

extern "C" int gx_table_export(const gx_table* t, gx_cell* out, size_t out_cells) {
    if (!t || !out) return fail(GX_EINVAL, "NULL argument");
    const size_t n = t->s1.size(), m = t->s2.size();
    if (out_cells < (n + 1) * (m + 1)) return fail(GX_ECAP, "out too small");
    std::lock_guard<std::mutex> lk(t->ctx->mu);
    HIPCHK(hipSetDevice(t->ctx->device));
    const bool have_l = t->job.lcs_on;
    int rc;
    if (t->job.wide) {   // int64 planes (gx_wide.hip)
        std::vector<int64_t> wI, wD, wS, wL;
        if ((rc = fetch_rows_wide(t, 0, 0, n + 1, wI)) || (rc = fetch_rows_wide(t, 1, 0, n + 1, wD)) ||
            (rc = fetch_rows_wide(t, 2, 0, n + 1, wS)))
            return rc;
        if (have_l && (rc = fetch_rows_wide(t, 3, 0, n + 1, wL))) return rc;
        auto Lw = [&](size_t i, size_t j) -> uint64_t {
            return (i == 0 || j == 0 || !have_l) ? 0 : (uint64_t)wL[i * (m + 1) + j];
        };
        for (size_t i = 0; i <= n; ++i)
            for (size_t j = 0; j <= m; ++j) {
                gx_cell c{};
                if (i == 0 || j == 0) {
                    boundary_cell(t->hs, i, j, &c.insert_score, &c.delete_score, &c.sub_score);
                } else {
                    const size_t o = i * (m + 1) + j;
                    c.insert_score = wI[o]; c.delete_score = wD[o]; c.sub_score = wS[o];
                    if (have_l) {
                        c.insert_matches = Lw(i, j - 1);
                        c.delete_matches = Lw(i - 1, j);
                        c.sub_matches = Lw(i - 1, j - 1) + (t->c1[i - 1] == t->c2[j - 1] ? 1 : 0);
                    }
                }
                out[i + j * (n + 1)] = c;
            }
        return GX_OK;
    }
    std::vector<int32_t> pI, pD, pS, pL;
    if ((rc = fetch_plane32(t, 0, pI)) || (rc = fetch_plane32(t, 1, pD)) || (rc = fetch_plane32(t, 2, pS))) return rc;
    if (have_l && (rc = t->job.lcs_rows ? fetch_lcs_plane(t, pL) : fetch_plane32(t, 3, pL))) return rc;
    auto L = [&](size_t i, size_t j) -> uint64_t {
        if (i == 0 || j == 0 || !have_l) return 0;
        return (uint64_t)pL[i * (m + 1) + j];
    };
    for (size_t i = 0; i <= n; ++i)
        for (size_t j = 0; j <= m; ++j) {
            gx_cell c{};
            if (i == 0 || j == 0) {
                boundary_cell(t->hs, i, j, &c.insert_score, &c.delete_score, &c.sub_score);
            } else {
                const size_t o = i * (m + 1) + j;
                c.insert_score = pI[o]; c.delete_score = pD[o]; c.sub_score = pS[o];
                if (have_l) {
                    // A.5: Im = L(i,j-1), Dm = L(i-1,j), Sm = L(i-1,j-1) + is_match(i-1,j-1)
                    c.insert_matches = L(i, j - 1);
                    c.delete_matches = L(i - 1, j);
                    c.sub_matches = L(i - 1, j - 1) + (t->c1[i - 1] == t->c2[j - 1] ? 1 : 0);
                }
            }
            out[i + j * (n + 1)] = c;   // column-major, algo.rs:172 `.f()`
        }
    return GX_OK;
}

extern "C" void gx_table_free(gx_table* t) {
    if (!t) return;
    if (t->ctx) {
        std::lock_guard<std::mutex> lk(t->ctx->mu);
        job_release(t->ctx, t->job);
        t->share.reset();   // (the kept fill's buffers go back to the pool with its last table)
    }
    delete t;
}

extern "C" void gx_table_free(gx_table* t);
extern "C" int gx_retrace(gx_table* t, int is_local, gx_step* steps, size_t cap, gx_result* out) {
    if (!t) return fail(GX_EINVAL, "table is NULL");
    if (t->share) {   // (consumed whatever the return code, gx.h)
        gx_table_free(t);
        return fail(GX_EINVAL, "a staged table has no retrace (its alignment: gx_staged_steps)");
    }
    gx_context* ctx = t->ctx;
    int rc = GX_OK;
    Walk w;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        (void)hipSetDevice(ctx->device);
        const size_t n = t->s1.size(), m = t->s2.size();
        const auto t0 = std::chrono::steady_clock::now();
        t->is_local = is_local;
        uint64_t si, sj;
        int64_t score;
        const PairRes r = t->job.res[0];
        start_cell(t, start_in(t->job, 0), &si, &sj, &score);
        if (log_info()) fprintf(stderr, "[gx INFO] Starting at (%llu, %llu)\n", (unsigned long long)si,
                                (unsigned long long)sj);
        TbOut tb;
        if (si >= 1 && sj >= 1 && n >= 1 && m >= 1) {
            rc = run_traceback(ctx, t->job, {TbStart{(int)si, (int)sj, is_local ? r.lmax_E : r.end_E}}, tb);
            if (!rc) rc = label_walk(t->hs, is_local, t->s1.data(), n, t->s2.data(), m, si, sj, n + m,
                                     RecordsSrc{&tb, 0}, w);
        } else {
            rc = label_walk(t->hs, is_local, t->s1.data(), n, t->s2.data(), m, si, sj, 0, MovesSrc{nullptr, 0}, w);
        }
        const auto t1 = std::chrono::steady_clock::now();
        w.res.score = score;
        w.res.start_i = si; w.res.start_j = sj;
        const bool interior = n >= 1 && m >= 1 && t->job.track_on;
        w.res.max_cell_i = interior ? (uint64_t)r.max_i : 0;
        w.res.max_cell_j = interior ? (uint64_t)r.max_j : 0;
        w.res.matches_at_max = interior ? (uint64_t)r.mam : 0;
        w.res.fill_us = (int64_t)(t->job.fill_ms * 1000.0);
        w.res.retrace_us = std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count();
        if (log_info()) {
            fprintf(stderr, "[gx INFO] Retrace complete, time taken: %lldus\n", (long long)w.res.retrace_us);
            fprintf(stderr, "[gx INFO] Retrace alignment size: %zu\n", w.steps.size());
        }
        job_release(ctx, t->job);
    }
    delete t;  // consumed, like the by-value Array2 in the reference
    if (rc) return rc;
    if (out) *out = w.res;
    return copy_steps(w, steps, cap);
}

extern "C" int gx_align(gx_context* ctx, const uint8_t* s1, size_t n, const uint8_t* s2, size_t m,
                        const gx_scores* scores, int is_local, int reverse_sequences, uint32_t flags,
                        gx_step* steps, size_t cap, gx_result* out) {
    gx_table* t = nullptr;
    uint64_t mam = 0;
    int rc = gx_alignment_table(ctx, s1, n, s2, m, scores, is_local, reverse_sequences, 0, &t,
                                (flags & GX_ALIGN_MAX_CELL) ? &mam : nullptr);
    if (rc) return rc;
    return gx_retrace(t, is_local, steps, cap, out);
}
