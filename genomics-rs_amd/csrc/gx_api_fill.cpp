// gx_api_fill.cpp -- the DP fill (alignment_table's table fill,
// algo.rs:151-282) as device launches: descriptors, buffers and launch of
// the int32 layouts (gx_kernels.hip, gx_cs2.hip, gx_skew.hip), the twin fill
// (gx_fill_pk.hip) and the int64 fill (gx_wide.hip), their results, and the
// on-device plane checksums.
#include "gx_api.h"

// Shifted fills (Scores32.shift) report score_max(n, m) as H - (n + m) g.
void unshift_results(FillJob& j) {
    if (!j.shift) return;
    for (size_t p = 0; p < j.res.size() && p < j.pd.size(); ++p)
        if (j.pd[p].n >= 1 && j.pd[p].m >= 1) j.res[p].end_SM += (j.pd[p].n + j.pd[p].m) * j.g;
}

void job_release(gx_context* ctx, FillJob& j) {
    if (j.pairs_borrowed) { j.pairs = DevBuf{}; j.pairs_borrowed = false; }
    if (j.pres_held) { j.pres = DevBuf{}; j.pres_held = false; }
    pool_put(ctx, j.chars); pool_put(ctx, j.planes); pool_put(ctx, j.codes); pool_put(ctx, j.feed);
    pool_put(ctx, j.progress); pool_put(ctx, j.sres); pool_put(ctx, j.pres); pool_put(ctx, j.pairs);
    pool_put(ctx, j.counter); pool_put(ctx, j.skel); pool_put(ctx, j.ccodes);
    pool_put(ctx, j.wrows); pool_put(ctx, j.wdesc); pool_put(ctx, j.wres_d); pool_put(ctx, j.lcs);
}

// The pipelines' release point for a pass's fill: the last pass of a
// GX_STAGED_KEEP_PLANES run is held (*keep set) instead of released.
void release_or_hold(gx_context* ctx, FillJob& j, bool last_pass, bool* held) {
    if (ctx->keep_capture && last_pass) { *held = true; return; }
    job_release(ctx, j);
}
void keep_job(gx_context* ctx, FillJob& j, const std::vector<int>& dev_of) {
    auto k = std::make_shared<KeptFill>();
    k->ctx = ctx;
    k->dev_of = dev_of;
    std::swap(k->job, j);
    ctx->kept = std::move(k);
}

// chars_dev: if non-null, device buffer already holding the processed chars
// at offsets off1/off2 (staged path); otherwise c1/c2 are uploaded.
// track: first max cell + LCS field (alignment_table's max_cell and
// matches_at_max, algo.rs:258-262, 279); lcs: also keep the LCS plane.
int run_fill(gx_context* ctx, const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc,
             const std::vector<PairHost>& ph, const Scores32& sc, int is_local, bool planes, bool track,
             bool lcs, FillJob& job, const uint8_t* chars_dev,
             const std::vector<size_t>* off1, const std::vector<size_t>* off2,
             const SmallAlpha* alpha, int slot, bool collect) {
    const int lay = fill_layout(ph, sc, fill_grid_cap(ctx->device), track || (lcs && planes), lcs && planes);
    hipStream_t const fs = job.stream ? job.stream : ctx->stream;
    const int SR = strip_rows(lay);
    int total_strips = 0;
    for (const PairHost& h : ph) total_strips += ceil_div((int)h.n, SR);
    const bool codes = true;
    lcs = lcs && planes;
    track = track || lcs;
    int min_strips = INT_MAX;
    for (const PairHost& h : ph) min_strips = std::min(min_strips, ceil_div((int)h.n, SR));
    // the split column step (gx_cs2.hip): layout 1's formats, each strip on a
    // core and a side wave; untracked fills (global or local)
    const bool cs2 = lay == 1 && !track && cs2_enabled(is_local, sc);
    const int W = cs2         ? cs2_band_waves(total_strips, fill_grid_cap(ctx->device))
                  : lay == 3 ? skew_band_waves()
                             : fill_band_waves(track || is_local, total_strips, fill_grid_cap(ctx->device), lay, min_strips);
    job.lay = lay;
    job.local_on = is_local != 0;
    // layout-0 untracked global fills and the split column step keep every
    // value as V - (i + j) g (one add less per recurrence, gx_kernels.hip
    // cell; the local floor becomes -(i + j) g); the sub scores carry -2g
    Scores32 scl = sc;
    // (layout 3's global recurrence always holds shifted values; its tracked
    // fill compares them through a shifted threshold, gx_skew.hip track_step)
    const bool shift = (lay == 3 && !is_local) || (lay == 0 && !is_local && !track) || cs2;
    scl.shift = shift ? 1 : 0;
    if (shift) { scl.sm = sc.sm - 2 * sc.g; scl.smm = sc.smm - 2 * sc.g; }
    job.shift = shift; job.g = sc.g;
    // small-alphabet score table: <= 4 symbols, scores in a signed byte; untracked fills (global or
    // local), and tracked ones on layout 3 (whose max_matches comes from the LCS rows, not the fill)
    const bool tbl = alpha && alpha->n <= 4 && (!track || lay == 3) && scl.sm >= -128 && scl.sm <= 127 &&
                     scl.smm >= -128 && scl.smm <= 127 && !getenv("GX_NO_SCORE_TABLE");
    if (tbl)
        for (int k = 0; k < 4; ++k) scl.sym[k] = alpha->sym[k];
    job.planes_on = planes; job.lcs_on = lcs; job.track_on = track;
    // layout 3 keeps max_matches as bit-parallel LCS rows beside the fill (gx_lcs.h), never as a plane
    job.lcs_rows = lay == 3 && track;
    const bool d8 = planes && lay == 0 && !track && d8_planes_ok(sc, is_local);
    job.d8 = d8;
    // twin fill: half as many band jobs (each carries two pairs); the band
    // width follows the usual rule on the twins' strips (GX_BAND_WAVES forces it)
    int Wt = 0;
    int wt_want = 15;
    if (const char* e = getenv("GX_BAND_WAVES")) wt_want = atoi(e);
    else wt_want = fill_band_waves(false, total_strips / 2, fill_grid_cap(ctx->device), lay, min_strips);
    const std::vector<std::pair<int, int>> tw = twin_table(
        ph, twin_gap_cap(sc, wt_want >= 15 ? 15 : wt_want >= 8 ? 8 : wt_want >= 7 ? 7 : wt_want >= 4 ? 4 : 3,
                         is_local != 0));
    {
        const bool long_ok = planes && !job.table && w16_ok(sc);   // (the noskel rule below)
        Wt = twin_width(ph, tw, sc, is_local, track, lcs, lay, planes, d8, wt_want, long_ok);
        // auto: the twin fill once its own bands fill the grid (a twin band
        // is slower per step than a scalar one, so fewer bands than CUs
        // leave it latency-bound).  30k pairs, fill ms scalar / twin (codes,
        // tables): 4 pairs (158 twin bands) 7.2 / 8.8, 6 (237) 9.4 / 8.9,
        // 8 9.96 / 8.9, 16 14.1 / 12.9, 24 19.2 / 17.4, all-vs-all and 80
        // pairs far apart.  GX_TWIN=1 forces it.
        const char* e = getenv("GX_TWIN");
        if (Wt && !(e && !strcmp(e, "1"))) {
            long long twin_bands = 0;
            for (const auto& t : tw)
                twin_bands += ceil_div(ceil_div((int)std::max(ph[t.first].n, ph[t.second].n), SR), Wt);
            if (10 * twin_bands < 9LL * fill_grid_cap(ctx->device)) Wt = 0;
            // a pair twinned with itself does a twin band's work for one pair:
            // batches of mostly unmatched shapes stay on the scalar fill
            size_t selfs = 0;
            for (const auto& t : tw) selfs += t.first == t.second;
            if (4 * selfs > tw.size() + 3) Wt = 0;
        }
        // 7-wave bands, two workgroups per CU (16 waves: the twin fill's 128
        // VGPRs allow four a SIMD; 8-wave bands fit one), for global batches
        // of pairs of >= 32 strips (4,096 rows) with >= 1.25 such bands per
        // workgroup of that grid: the CU then holds two independent band
        // pipelines.  80 x 30k (each overlapped group 680 bands on 512
        // workgroups) fill 26.8 -> 24.6 ms a pass (2,616 -> 2,852 GCUPS),
        // 1024 x 16k (1,216) 99.5 -> 95.0, 1024 x 4k 7.59 -> 6.78 ms a pass and
        // 8k 26.7 -> 23.9 (with the walk on the fill's stream: beside the
        // fill, 1,024 walks found no room on the CUs, 4k once 72 ms a pass;
        // batch_core_steps); slower with fewer bands (all-vs-all with planes,
        // 374-408: 16.7 -> 18.5 ms), for 2k pairs (2.25 -> 2.38 ms) and for
        // the local twin (64 related 30k pairs 1,852 -> 1,359 GCUPS)
        // (profiles/r05_w7_sweep.txt)
        if (Wt == 8 && !is_local && long_ok && !getenv("GX_BAND_WAVES") && min_strips >= 32) {
            long long b7 = 0;
            for (const auto& t : tw) b7 += ceil_div(ceil_div((int)std::max(ph[t.first].n, ph[t.second].n), SR), 7);
            if (4 * b7 >= 5LL * 2 * fill_grid_cap(ctx->device)) Wt = 7;
        }
    }
    const bool twin = Wt > 0;
    job.twin = twin;
    if (twin && is_local) {   // the local twin's scores carry + K so that its score tables hold bytes >= 0
        const int K = std::max(0, -std::min(sc.sm, sc.smm));
        scl.koff = K; scl.sm = sc.sm + K; scl.smm = sc.smm + K;
    }
    const bool w16 = twin && planes && !job.table && w16_ok(sc);
    job.w16 = w16;
    // with twin plane codes the fill stores no code words (0.25 B/cell less):
    // the traceback rebuilds the words of the path's strips from the planes
    // (tb_w16_codes_kernel), and no landing columns either (a quarter of the
    // twin cell's VALU): the traceback walks the strips one after another,
    // each entered where the one below left it (tb_seq_kernel).  The byte
    // planes (tables, GX_PLANES_W16=0) keep both.
    job.nocodes = w16;
    job.noskel = job.nocodes;
    // small-alphabet twins: the match test through score tables (cell_pk; the
    // shifted scores must fit an unsigned byte);
    // the byte-plane twin (tables) keeps the plain test
    const bool twin_tbl = twin && tbl && (!planes || w16) && scl.sm >= 0 && scl.sm <= 255 && scl.smm >= 0 &&
                          scl.smm <= 255;
    ctx->last_twin = twin ? 1 : 0;
    const int Wf = twin ? Wt : W;   // band width of the launch
    const size_t plane_esz = d8 ? 1 : sizeof(int32_t);
    job.W = Wf;
    ctx->last_lay = cs2 ? 2 : lay; ctx->last_W = Wf;
    ctx->last_pbytes = planes ? (w16 ? 2 : (int)(plane_esz * 3)) : 0;   // (twin codes: 1.5, reported rounded up)
    ctx->last_pbits = planes ? (w16 ? 12 : (int)(plane_esz * 24)) : 0;
    const size_t P = ph.size();
    if (job.plan_only) { job.twin = twin; return GX_OK; }
    job.pd.assign(P, PairDev{});
    // -- sizes
    size_t chars_bytes = 0, plane_elems = 0, code_elems = 0, feed_recs = 0, prog_elems = 0, skel_elems = 0;
    std::vector<size_t> c1o(P), c2o(P), po(P), co(P), fo(P), gofs(P), so(P);
    int bands = 0, strips = 0;
    // twins: each pair's mate and its half (the first of a twin is the low half)
    std::vector<int> mate(P, -1), half(P, 0);
    if (twin)
        for (const auto& t : tw) {
            mate[t.first] = t.second; mate[t.second] = t.first;
            half[t.first] = 0;
            if (t.second != t.first) half[t.second] = 1;
        }
    for (size_t p = 0; p < P; ++p) {
        const int n = (int)ph[p].n, m = (int)ph[p].m;
        PairDev& d = job.pd[p];
        d.n = n; d.m = m;
        // the shape the pair is laid out for: its own, or its twin's larger n and m
        int ns = n, ms = m;
        if (twin) {
            const PairHost& y = ph[mate[p]];
            ns = (int)std::max(ph[p].n, y.n); ms = (int)std::max(ph[p].m, y.m);
        }
        d.strips = ceil_div(ns, SR);
        d.bands = ceil_div(d.strips, Wf);
        // steps per strip: layout 0, lane 63 pushes column m at step m + 63; layout 1, column m at step m - 1
        const int T = lay == 1 ? ms + 1 : ms + kWave;
        d.t16 = ceil_div(T, 16);
        d.t4 = d.t16 * 4;
        d.strip_base = strips;
        d.feed_stride = (int)align_up((size_t)ms + 1 + 64, 16);
        d.skel_stride = (int)align_up((size_t)ms + 1, 64);
        d.twin_half = half[p];
        strips += d.strips;
        c1o[p] = chars_bytes; chars_bytes += align_up(n, 64);
        c2o[p] = chars_bytes; chars_bytes += align_up(m, 64);
        if (!w16) { po[p] = plane_elems; plane_elems += (size_t)d.strips * d.t4 * (lay ? kGroupInts1 : kGroupInts); }
        co[p] = code_elems; code_elems += (size_t)d.strips * d.t16 * SR;
        if (!twin) {
            d.band_base = bands;
            bands += d.bands;
            so[p] = skel_elems; skel_elems += (size_t)d.strips * d.skel_stride;
            fo[p] = feed_recs; feed_recs += (size_t)std::max(d.bands - 1, 0) * d.feed_stride;
            gofs[p] = prog_elems; prog_elems += (size_t)std::max(d.bands - 1, 0) * kProgStride;
        }
    }
    // a twin's bands, skeleton (both halves' landing columns), hand-off rows
    // (32-B records, gx_fill_pk.hip RecW: two Rec slots per column) and code
    // plane (w16) are shared by its two pairs
    if (twin)
        for (const auto& t : tw) {
            PairDev& d = job.pd[t.first];
            const size_t a = t.first, b = t.second;
            d.band_base = bands; job.pd[b].band_base = bands;
            bands += d.bands;
            so[a] = so[b] = skel_elems; skel_elems += (size_t)d.strips * d.skel_stride;
            fo[a] = fo[b] = feed_recs; feed_recs += (size_t)std::max(d.bands - 1, 0) * d.feed_stride * 2;
            gofs[a] = gofs[b] = prog_elems; prog_elems += (size_t)std::max(d.bands - 1, 0) * kProgStride;
            if (w16) { po[a] = po[b] = plane_elems; plane_elems += (size_t)d.strips * d.t4 * kTwinGroupBytes; }
        }
    job.total_bands = bands;
    job.total_strips = strips;
    int rc;
    const int nplanes = w16 ? 1 : (lcs && !job.lcs_rows) ? 4 : 3;
    if (!chars_dev) {
        if ((rc = pool_get(ctx, chars_bytes, &job.chars, fs))) return rc;
    }
    if (planes && (rc = pool_get(ctx, plane_elems * plane_esz * nplanes, &job.planes, fs))) return rc;
    // (no code-word buffer for a fill that stores none: 0.25 B a cell, 21 GB of
    // a 20-pair 64k chunk, which the overlapped pipeline's second A group needs)
    const bool want_codes = codes && !job.nocodes;
    if (want_codes && (rc = pool_get(ctx, code_elems * sizeof(uint32_t), &job.codes, fs))) return rc;
    if ((rc = pool_get(ctx, std::max<size_t>(skel_elems, 1) * sizeof(int), &job.skel, fs))) return rc;
    if ((rc = pool_get(ctx, std::max<size_t>(feed_recs, 1) * sizeof(Rec), &job.feed, fs))) return rc;
    if ((rc = pool_get(ctx, std::max(strips, 1) * sizeof(StripRes), &job.sres, fs))) return rc;
    if (getenv("GX_LCS_ALONE"))   // (diagnostics: no fill writes the strip results, so they must not be pool garbage)
        HIPCHK(hipMemsetAsync(job.sres.p, 0, std::max(strips, 1) * sizeof(StripRes), fs));
    // one buffer [PairRes x P | band counter + status (64 B) | band progress]:
    // one memset before the launch, one copy of the results and status after
    // it (each small copy or memset on the stream costs a runtime round trip
    // of ~100 us between a batch's fill and its walk, profiles: r04 1024 x 1k)
    const size_t res_bytes = P * sizeof(PairRes), prog_bytes = std::max<size_t>(prog_elems, 1) * sizeof(int);
    if ((rc = pool_get(ctx, res_bytes + 64 + prog_bytes, &job.pres, fs))) return rc;
    int* const counter = (int*)((char*)job.pres.p + res_bytes);
    int* const progress = counter + 16;
    // band queue order, stored after the pair descriptors: band-major ("round"
    // order: band 0 of every pair, then band 1, ...; a band's predecessor in its
    // pair is always dequeued before it, so a waiting band is never waiting on
    // an unstarted one; pair-major order, all bands of pair 0 first, was 10-25 %
    // slower, profiles/r01o_band_order_ab.txt)
    std::vector<int> order;
    order.reserve(2 * (size_t)bands);
    if (twin) {   // band-major over the twins: entries (twin q, band), then the twin table
        int maxb = 0;
        for (const auto& t : tw) maxb = std::max(maxb, job.pd[t.first].bands);
        for (int lb = 0; lb < maxb; ++lb)
            for (size_t q = 0; q < tw.size(); ++q)
                if (lb < job.pd[tw[q].first].bands) { order.push_back((int)q); order.push_back(lb); }
        for (const auto& t : tw) { order.push_back(t.first); order.push_back(t.second); }
    } else {
        int maxb = 0;
        for (size_t p = 0; p < P; ++p) maxb = std::max(maxb, job.pd[p].bands);
        for (int lb = 0; lb < maxb; ++lb)
            for (size_t p = 0; p < P; ++p)
                if (lb < job.pd[p].bands) { order.push_back((int)p); order.push_back(lb); }
    }
    const size_t ord_bytes = align_up(order.size() * sizeof(int), 16);   // keeps the PairRes staging 16-B aligned
    if (slot < 0 && (rc = pool_get(ctx, P * sizeof(PairDev) + ord_bytes, &job.pairs, fs))) return rc;
    // -- chars upload
    const uint8_t* cbase = chars_dev;
    if (!chars_dev) {
        std::vector<uint8_t> hc(chars_bytes, 0);
        for (size_t p = 0; p < P; ++p) {
            if (ph[p].n) memcpy(&hc[c1o[p]], proc[p].first, ph[p].n);
            if (ph[p].m) memcpy(&hc[c2o[p]], proc[p].second, ph[p].m);
        }
        HIPCHK(hipMemcpyAsync(job.chars.p, hc.data(), chars_bytes, hipMemcpyHostToDevice, fs));
        HIPCHK(hipStreamSynchronize(fs));  // hc goes out of scope
        cbase = (const uint8_t*)job.chars.p;
    }
    for (size_t p = 0; p < P; ++p) {
        PairDev& d = job.pd[p];
        d.c1 = cbase + (chars_dev ? (*off1)[p] : c1o[p]);
        d.c2 = cbase + (chars_dev ? (*off2)[p] : c2o[p]);
        uint8_t* pl = (uint8_t*)job.planes.p;
        auto plane_at = [&](int k) { return (int32_t*)(pl + (k * plane_elems + po[p]) * plane_esz); };
        d.pI = planes ? plane_at(0) : nullptr;
        d.pD = (planes && !w16) ? plane_at(1) : nullptr;
        d.pS = (planes && !w16) ? plane_at(2) : nullptr;
        d.pL = (planes && lcs && !job.lcs_rows) ? plane_at(3) : nullptr;
        d.codes = want_codes ? (uint32_t*)job.codes.p + co[p] : nullptr;
        d.skel = (int*)job.skel.p + so[p];
        d.feed = (Rec*)job.feed.p + fo[p];
        d.progress = progress + gofs[p];
    }
    // layout 3 reads each lane's column symbols from an int32 copy (gx_skew.hip)
    // (with score tables: four rows per pair, one per row symbol: the scores themselves)
    if (lay == 3) {
        const size_t rows = tbl ? 4 : 1;
        size_t cc = 0;
        for (size_t p = 0; p < P; ++p) cc += rows * ((size_t)job.pd[p].m + 192);
        if ((rc = pool_get(ctx, cc * sizeof(int), &job.ccodes, fs))) return rc;
        cc = 0;
        for (size_t p = 0; p < P; ++p) {
            job.pd[p].ccodes = (const int*)job.ccodes.p + cc;
            cc += rows * ((size_t)job.pd[p].m + 192);
        }
    }
    // layout-3 tracked fills: per pair the masks 256 x (lwords + 128) (zeroed) and the bit rows
    // strips x lcs_steps(lwords) x 64 words, filled by the launch's leading LCS workgroups (gx_lcs.h)
    int lcs_blocks = 0;
    // (GX_LCS=0, diagnostics only: no LCS workgroups, so matches_at_max is
    // not computed -- the timing of the fill without them)
    if (const char* e = getenv("GX_LCS"); e && !strcmp(e, "0")) job.lcs_rows = false;
    if (job.lcs_rows) {
        std::vector<size_t> zo(P), ro(P);
        size_t zbytes = 0, rbytes = 0;
        for (size_t p = 0; p < P; ++p) {
            PairDev& d = job.pd[p];
            d.lwords = ceil_div(d.m, kLcsBits);
            // sweeping workgroups (GX_LCS_WAVES, GX_LCS_WGS override: diagnostics)
            const int nwg = getenv("GX_LCS_WGS") ? std::max(1, atoi(getenv("GX_LCS_WGS"))) : skew_lcs_blocks(W, d.n, d.m);
            d.lcs_waves = (getenv("GX_LCS_WAVES") ? atoi(getenv("GX_LCS_WAVES")) : skew_lcs_sweep(W)) | (nwg << 8) |
                          (lcs ? 1 << 16 : 0);   // every row (the matches planes of a table) or the strips' last
            d.lcs_base = lcs_blocks;
            lcs_blocks += nwg;
            const size_t feed_words = (size_t)ceil_div(d.n, kWave) * lcs_steps(d.lwords);   // (x2: tagged halves)
            zo[p] = zbytes; zbytes += (256 * ((size_t)d.lwords + 2 * kLcsMaskPad) + 2 * feed_words) * sizeof(unsigned long long);
            ro[p] = rbytes;
            rbytes += feed_words * (lcs ? kWave : 1) * sizeof(unsigned long long);
        }
        // (GX_LCS_TRACE=file, diagnostics: each strip's s_memrealtime stamps, after the zeroed region)
        const char* ltrace_file = getenv("GX_LCS_TRACE");
        size_t tbytes = 0;
        if (ltrace_file && *ltrace_file)
            for (size_t p = 0; p < P; ++p) tbytes += (size_t)ceil_div(job.pd[p].n, kWave) * 4 * sizeof(unsigned long long);
        if ((rc = pool_get(ctx, zbytes + rbytes + tbytes, &job.lcs, fs))) return rc;
        size_t to = 0;
        for (size_t p = 0; p < P; ++p) {
            PairDev& d = job.pd[p];
            d.lmask = (unsigned long long*)((char*)job.lcs.p + zo[p]);
            d.llink = d.lmask + 256 * ((size_t)d.lwords + 2 * kLcsMaskPad);
            d.lbits = (unsigned long long*)((char*)job.lcs.p + zbytes + ro[p]);
            d.ltrace = tbytes ? (unsigned long long*)((char*)job.lcs.p + zbytes + rbytes + to) : nullptr;
            if (tbytes) to += (size_t)ceil_div(d.n, kWave) * 4 * sizeof(unsigned long long);
        }
        if (tbytes) HIPCHK(hipMemsetAsync((char*)job.lcs.p + zbytes + rbytes, 0, tbytes, fs));
        job.ltrace_off = zbytes + rbytes;
        job.ltrace_bytes = tbytes;
        HIPCHK(hipMemsetAsync(job.lcs.p, 0, zbytes, fs));
    }
    const char* trace_file = slot < 0 ? getenv("GX_TRACE_FILE") : nullptr;
    if (trace_file && *trace_file && lay == 3 && !skew_traced(planes, true, track)) {
        // (layout 3 has traced instantiations for untracked fills with planes only: no file of zero stamps)
        fprintf(stderr, "[gx WARN] GX_TRACE_FILE: this layout-3 launch (planes %d, tracked %d) runs untraced; no trace written\n",
                planes ? 1 : 0, track ? 1 : 0);
        trace_file = nullptr;
    }
    DevBuf trace;
    if (trace_file && *trace_file) {
        if ((rc = pool_get(ctx, (size_t)std::max(strips, 1) * sizeof(StripTrace), &trace, fs))) return rc;
        HIPCHK(hipMemsetAsync(trace.p, 0, (size_t)std::max(strips, 1) * sizeof(StripTrace), fs));
        for (size_t p = 0; p < P; ++p) job.pd[p].trace = (StripTrace*)trace.p + job.pd[p].strip_base;
    }
    // descriptors in (and results out) through pinned staging, laid out [PairDev x P | PairRes x P | status]
    const size_t pin_bytes = P * (sizeof(PairDev) + sizeof(PairRes)) + ord_bytes + 2 * sizeof(int);
    char* pin = (char*)(slot >= 0 ? pinned_grow(ctx->slots[slot].fpin, pin_bytes) : io_pinned(ctx, pin_bytes));
    if (!pin) return fail(GX_ENOMEM, "pinned staging buffer");
    memcpy(pin, job.pd.data(), P * sizeof(PairDev));
    if (!order.empty()) memcpy(pin + P * sizeof(PairDev), order.data(), order.size() * sizeof(int));
    const size_t dbytes = P * sizeof(PairDev) + ord_bytes;
    if (slot < 0) {
        HIPCHK(hipMemcpyAsync(job.pairs.p, pin, dbytes, hipMemcpyHostToDevice, fs));
    } else {
        // pipelined passes repeat their descriptors: the slot pair's cached
        // device copies are looked up first and uploaded only on a change
        // (the copy engine serialises an upload behind the previous pass's
        // record copy, ~0.2 ms on a 1024 x 1k step).  A cache is rewritten
        // on this stream only, after every fill that read it.
        int hit = -1;
        for (int x : {slot, slot ^ 1}) {
            const auto& sl = ctx->slots[x];
            if (sl.fdesc && sl.fdesc_last.size() == dbytes && !memcmp(sl.fdesc_last.data(), pin, dbytes)) { hit = x; break; }
        }
        if (hit < 0) {
            auto& sl = ctx->slots[slot];
            if (sl.fdesc_cap < dbytes) {
                if (sl.fdesc) (void)hipFree(sl.fdesc);
                sl.fdesc = nullptr; sl.fdesc_cap = 0; sl.fdesc_last.clear();
                if (hipMalloc(&sl.fdesc, dbytes) != hipSuccess) { sl.fdesc = nullptr; return fail(GX_ENOMEM, "fill descriptors"); }
                sl.fdesc_cap = dbytes;
            }
            sl.fdesc_last.assign(pin, pin + dbytes);
            HIPCHK(hipMemcpyAsync(sl.fdesc, pin, dbytes, hipMemcpyHostToDevice, fs));
            hit = slot;
        }
        job.pairs = DevBuf{ctx->slots[hit].fdesc, ctx->slots[hit].fdesc_cap};
        job.pairs_borrowed = true;
    }
    // layout 3 hands band rows over in tagged granules (gx_skew.hip io_wave_tag): valid once written
    if (lay == 3 && feed_recs > 0) HIPCHK(hipMemsetAsync(job.feed.p, 0, feed_recs * sizeof(Rec), fs));
    HIPCHK(hipMemsetAsync(job.pres.p, 0, res_bytes + 64 + prog_bytes, fs));
    // twin workgroups: as many per CU as fit 16 waves (the global twin fill
    // holds 96 VGPRs, the local one 149: 5 and 3 waves a SIMD by registers;
    // 16 measured best for the global fill: 8-wave bands two a CU, 18
    // waves, 30.4 ms a headline pass against 25.4 at 7-wave bands two a CU
    // and 29.2 at 4-wave bands four a CU, profiles/r05_w7_sweep.txt)
    const int per_cu = (twin && !getenv("GX_FILL_GRID")) ? std::max(1, 16 / (Wf + 1)) : 1;
    const int grid = std::min(bands, fill_grid_cap(ctx->device) * per_cu);
    if (const char* lg = getenv("GX_LOG"); lg && !strcmp(lg, "debug"))
        fprintf(stderr, "[gx DEBUG] fill launch: P=%zu layout=%d W=%d twin=%d plane_bytes=%d tbl=%d grid=%d bands=%d\n", P,
                lay, Wf, twin ? 1 : 0, ctx->last_pbytes, (twin ? twin_tbl : tbl) ? 1 : 0, grid, bands);
    const auto h_launch = std::chrono::steady_clock::now();
    hipEvent_t evb = slot >= 0 ? ctx->slots[slot].fb : ctx->ev0, eve = slot >= 0 ? ctx->slots[slot].fe : ctx->ev1;
    if (bands > 0 && lay == 3) {   // the column symbols as int32 for layout 3's lanes (before the timed fill)
        int mmax = 0;
        for (size_t p = 0; p < P; ++p) mmax = std::max(mmax, job.pd[p].m);
        HIPCHK(launch_skew_codes((const PairDev*)job.pairs.p, (int)P, mmax, scl, tbl, fs));
    }
    HIPCHK(hipEventRecord(evb, fs));
    if (bands > 0 && twin)
        HIPCHK(launch_fill_pk(Wf, (planes ? (w16 ? 2 : 1) : 0) + (twin_tbl ? 4 : 0) + (job.nocodes ? 8 : 0) +
                                  (job.noskel ? 16 : 0) + (is_local ? 32 : 0),
                              (const PairDev*)job.pairs.p, (int)P, (int)tw.size(), bands, counter,
                              (PairRes*)job.pres.p, (StripRes*)job.sres.p, scl, grid, fs));
    else if (bands > 0 && lay == 3)
        HIPCHK(launch_fill_skew(W, is_local != 0, planes, tbl, trace.p != nullptr, track, (const PairDev*)job.pairs.p, (int)P,
                                // (GX_LCS_ALONE=1, diagnostics only: the LCS workgroups without the fill, to time them)
                                getenv("GX_LCS_ALONE") && lcs_blocks ? 0 : bands,
                                counter, (StripRes*)job.sres.p, (PairRes*)job.pres.p, scl, grid, lcs_blocks, fs));
    else if (bands > 0 && cs2)
        HIPCHK(launch_fill_cs2(W, is_local != 0, planes, tbl, (const PairDev*)job.pairs.p, (int)P, bands,
                               counter, (StripRes*)job.sres.p, (PairRes*)job.pres.p, scl, grid, fs));
    else if (bands > 0)
        HIPCHK(launch_fill(W, lay, is_local != 0, planes ? (d8 ? 2 : 1) : 0, track, lcs, tbl, (const PairDev*)job.pairs.p, (int)P, bands,
                           counter, (StripRes*)job.sres.p, (PairRes*)job.pres.p, scl, grid, fs));
    HIPCHK(hipEventRecord(eve, fs));   // evb..eve brackets the fill kernel alone
    // the reductions after the fill: on the fill stream, or (pipelined, the
    // walk on its own stream, gx_context.post_aside) on pstream beside the
    // next pass's fill, which would otherwise queue behind them (~50 us a
    // tracked Covid pass)
    const bool aside = !collect && slot >= 0 && ctx->post_aside && bands > 0 &&
                       ((ctx->sums_dst && planes) || track || is_local);
    hipStream_t const ps = aside ? ctx->pstream : fs;
    if (aside) HIPCHK(hipStreamWaitEvent(ps, eve, 0));
    if (ctx->sums_dst && planes && bands > 0) {   // staged checksum run: this pass's plane sums
        HIPCHK(enqueue_plane_sums(ctx, job, sc, ctx->sums_dst, ps));
        ctx->sums_dst += 3 * P;
    }
    // strip results exist only for the tracked and local fills (the untracked
    // global fill writes end_SM / end_E itself): no reduction launch otherwise
    if (bands > 0 && (track || is_local))
        HIPCHK(launch_finalize((const PairDev*)job.pairs.p, (int)P, (const StripRes*)job.sres.p,
                               (PairRes*)job.pres.p, ps));
    // tracked layout-3 fills with planes track each row's largest value only:
    // the first column holding the maximum from the planes, then matches_at_max
    if (bands > 0 && lay == 3 && track && planes) {
        int mmax = 0;
        for (size_t p = 0; p < P; ++p) mmax = std::max(mmax, job.pd[p].m);
        HIPCHK(launch_skew_max_col((const PairDev*)job.pairs.p, (int)P, mmax, (PairRes*)job.pres.p,
                                   is_local ? 0 : sc.g, ps));
    }
    if (job.ltrace_bytes) {   // (GX_LCS_TRACE: pair, strip, start / first group / end stamps (100 MHz), workgroup * 64 + wave)
        std::vector<unsigned long long> h(job.ltrace_bytes / sizeof(unsigned long long));
        HIPCHK(hipStreamSynchronize(ps));
        HIPCHK(hipMemcpy(h.data(), (char*)job.lcs.p + job.ltrace_off, job.ltrace_bytes, hipMemcpyDeviceToHost));
        if (FILE* f = fopen(getenv("GX_LCS_TRACE"), "a")) {
            size_t o = 0;
            for (size_t p = 0; p < P; ++p)
                for (int s = 0; s < ceil_div(job.pd[p].n, kWave); ++s, o += 4)
                    fprintf(f, "%zu,%d,%llu,%llu,%llu,%llu\n", p, s, h[o], h[o + 1], h[o + 2], h[o + 3]);
            fclose(f);
        }
    }
    // the local twin fill tracks each row's maximum only: the last column of
    // the chosen row from its plane codes (gx_kernels.hip local_col_kernel)
    if (bands > 0 && twin && is_local)
        HIPCHK(launch_local_col((const PairDev*)job.pairs.p, (int)P, (PairRes*)job.pres.p, sc.h, sc.g, ps));
    job.res.assign(P, PairRes{});
    int status[2] = {0, 0};
    PairRes* pin_res = (PairRes*)(pin + P * sizeof(PairDev) + ord_bytes);
    int* pin_status = (int*)(pin + P * (sizeof(PairDev) + sizeof(PairRes)) + ord_bytes);
    job.pin_res = pin_res;
    job.pin_status = pin_status;
    job.slot = slot;
    if (!collect) {   // pipelined: fill_collect() waits for the results later
        // the results (+ status) go on the copy stream, so the walk queued
        // behind this fill does not wait for a device-to-host copy (~0.12 ms
        // on the copy engine after a long transfer, 1024 x 1k); the block
        // stays held by the slot until that copy is collected
        auto& sl = ctx->slots[slot];
        HIPCHK(hipEventRecord(sl.fdone, ps));   // (the fill and its reductions)
        HIPCHK(hipStreamWaitEvent(ctx->cstream, sl.fdone, 0));
        HIPCHK(hipMemcpyAsync(pin_res, job.pres.p, res_bytes + sizeof status, hipMemcpyDeviceToHost, ctx->cstream));
        HIPCHK(hipEventRecord(sl.fres, ctx->cstream));
        pool_put(ctx, sl.held_pres);   // (collected already: fill_collect released it)
        sl.held_pres = job.pres;
        job.pres_held = true;
        return GX_OK;
    }
    HIPCHK(hipMemcpyAsync(pin_res, job.pres.p, res_bytes + sizeof status, hipMemcpyDeviceToHost, fs));   // (+ status)
    HIPCHK(hipStreamSynchronize(fs));
    memcpy(job.res.data(), pin_res, P * sizeof(PairRes));
    unshift_results(job);
    memcpy(status, pin_status, sizeof status);
    if (const char* lg = getenv("GX_LOG"); lg && !strcmp(lg, "debug"))
        fprintf(stderr, "[gx DEBUG] fill: launch..sync %.3f ms\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h_launch).count());
    if (status[1] != 0)
        return fail(GX_EHIP, "fill kernel: inter-wave wait timed out (status " + std::to_string(status[1]) + ")");
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, evb, eve));
    job.fill_ms = ms;
    if (trace.p) {
        std::vector<StripTrace> tr((size_t)strips);
        HIPCHK(hipMemcpy(tr.data(), trace.p, tr.size() * sizeof(StripTrace), hipMemcpyDeviceToHost));
        pool_put(ctx, trace);
        if (FILE* f = fopen(trace_file, "w")) {
            fprintf(f, "pair,strip,band,t_start,t_first,t_end,clk,wait_in,wait_out,W,fill_ms");
            for (int q = 0; q < kTraceQ; ++q) fprintf(f, ",q%d", q + 1);
            for (int q = 0; q < kTraceTL; ++q) fprintf(f, ",tl%d", q);
            for (int q = 0; q < kTraceTL; ++q) fprintf(f, ",tc%d", q);
            for (int q = 0; q < kTraceTL; ++q) fprintf(f, ",ts%d", q);
            fprintf(f, "\n");
            for (size_t p = 0; p < P; ++p)
                for (int s = 0; s < job.pd[p].strips; ++s) {
                    const StripTrace& t = tr[job.pd[p].strip_base + s];
                    fprintf(f, "%zu,%d,%d,%lld,%lld,%lld,%lld,%d,%d,%d,%.4f", p, s, job.pd[p].band_base + s / W,
                            t.t_start, t.t_first, t.t_end, t.clk, t.wait_in, t.wait_out, W, ms);
                    for (int q = 0; q < kTraceQ; ++q) fprintf(f, ",%lld", t.t_q[q]);
                    for (int q = 0; q < kTraceTL; ++q) fprintf(f, ",%lld", t.tl[q]);
                    for (int q = 0; q < kTraceTL; ++q) fprintf(f, ",%lld", t.tc[q]);
                    for (int q = 0; q < kTraceTL; ++q) fprintf(f, ",%lld", t.ts[q]);
                    fprintf(f, "\n");
                }
            fclose(f);
        }
    }
    return GX_OK;
}

// Results of a fill enqueued with collect = false (pipelined path).
int fill_collect(gx_context* ctx, FillJob& job) {
    auto& s = ctx->slots[job.slot];
    HIPCHK(hipEventSynchronize(s.fres));
    pool_put(ctx, s.held_pres);   // its copy is done (the walk that reads it is ordered before any reuse: see callers)
    const size_t P = job.pd.size();
    job.res.assign(P, PairRes{});
    memcpy(job.res.data(), job.pin_res, P * sizeof(PairRes));
    unshift_results(job);
    if (job.pin_status[1] != 0)
        return fail(GX_EHIP, "fill kernel: inter-wave wait timed out (status " + std::to_string(job.pin_status[1]) + ")");
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, s.fb, s.fe));
    job.fill_ms = ms;
    return GX_OK;
}

// The int64 fill (gx_wide.hip) of jobs outside the exact-int32 range: one
// wave per pair, outputs in the column-step layout's code / skeleton formats
// (job.lay = 1), int64 planes row-major.  Synchronous.
int run_fill_wide(gx_context* ctx, const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc,
                  const std::vector<PairHost>& ph, const HostScores& hs, int is_local, bool planes, bool track,
                  bool lcs, FillJob& job) {
    const size_t P = ph.size();
    job.wide = true;
    job.lay = 1;
    job.W = 1;
    lcs = lcs && planes;
    track = track || lcs;
    job.planes_on = planes; job.lcs_on = lcs; job.track_on = track;
    ctx->last_lay = 1; ctx->last_W = 1; ctx->last_pbytes = planes ? 24 : 0; ctx->last_pbits = planes ? 192 : 0;
    job.pd.assign(P, PairDev{});
    job.wd.assign(P, WideDev{});
    size_t chars = 0, codes = 0, skel = 0, rows = 0, cells = 0;
    std::vector<size_t> c1o(P), c2o(P), co(P), so(P), ro(P), po(P);
    for (size_t p = 0; p < P; ++p) {
        const int n = (int)ph[p].n, m = (int)ph[p].m;
        PairDev& d = job.pd[p];
        d.n = n; d.m = m;
        d.strips = ceil_div(n, kStripRows1);
        d.t16 = ceil_div(m + 1, 16);
        d.t4 = d.t16 * 4;
        d.skel_stride = (int)align_up((size_t)m + 1, 64);
        c1o[p] = chars; chars += align_up(n, 64);
        c2o[p] = chars; chars += align_up(m, 64);
        co[p] = codes; codes += (size_t)d.strips * d.t16 * kWave;
        so[p] = skel; skel += (size_t)d.strips * d.skel_stride;
        ro[p] = rows; rows += (size_t)d.strips * (m + 1);
        po[p] = cells; cells += (size_t)n * m;
    }
    int rc;
    if ((rc = pool_get(ctx, std::max<size_t>(chars, 1), &job.chars)) ||
        (rc = pool_get(ctx, std::max<size_t>(codes, 1) * sizeof(uint32_t), &job.codes)) ||
        (rc = pool_get(ctx, std::max<size_t>(skel, 1) * sizeof(int), &job.skel)) ||
        (rc = pool_get(ctx, std::max<size_t>(rows, 1) * sizeof(WideRow), &job.wrows)) ||
        (rc = pool_get(ctx, P * sizeof(WideDev), &job.wdesc)) || (rc = pool_get(ctx, P * sizeof(WideRes), &job.wres_d)))
        return rc;
    const size_t nplane = lcs ? 3 * sizeof(int64_t) + sizeof(unsigned) : 3 * sizeof(int64_t);
    if (planes && (rc = pool_get(ctx, std::max<size_t>(cells, 1) * nplane, &job.planes))) return rc;
    std::vector<uint8_t> hc(std::max<size_t>(chars, 1), 0);
    for (size_t p = 0; p < P; ++p) {
        if (ph[p].n) memcpy(&hc[c1o[p]], proc[p].first, ph[p].n);
        if (ph[p].m) memcpy(&hc[c2o[p]], proc[p].second, ph[p].m);
    }
    for (size_t p = 0; p < P; ++p) {
        PairDev& d = job.pd[p];
        WideDev& w = job.wd[p];
        d.codes = (uint32_t*)job.codes.p + co[p];
        d.skel = (int*)job.skel.p + so[p];
        w.c1 = (const uint8_t*)job.chars.p + c1o[p];
        w.c2 = (const uint8_t*)job.chars.p + c2o[p];
        w.n = d.n; w.m = d.m; w.strips = d.strips; w.t16 = d.t16;
        w.codes = d.codes; w.skel = d.skel; w.skel_stride = d.skel_stride;
        w.rows = (WideRow*)job.wrows.p + ro[p];
        if (planes) {
            int64_t* base = (int64_t*)job.planes.p;
            w.pI = (long long*)(base + po[p]);
            w.pD = (long long*)(base + cells + po[p]);
            w.pS = (long long*)(base + 2 * cells + po[p]);
            w.pL = lcs ? (unsigned*)(base + 3 * cells) + po[p] : nullptr;
        }
    }
    HIPCHK(hipMemcpyAsync(job.chars.p, hc.data(), hc.size(), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(job.wdesc.p, job.wd.data(), P * sizeof(WideDev), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemsetAsync(job.wres_d.p, 0, P * sizeof(WideRes), ctx->stream));
    const WideScores ws{hs.sm, hs.smm, hs.g, hs.h, hs.neg_inf};
    HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
    HIPCHK(launch_fill_wide((const WideDev*)job.wdesc.p, (int)P, ws, (WideRes*)job.wres_d.p, is_local ? 1 : 0,
                            track ? 1 : 0, ctx->stream));
    HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
    if (ctx->sums_dst && planes) {   // staged checksum run
        for (size_t p = 0; p < P; ++p) {
            HIPCHK(launch_wide_plane_sums((const int64_t*)job.wd[p].pI, (const int64_t*)job.wd[p].pD,
                                          (const int64_t*)job.wd[p].pS, job.wd[p].n, job.wd[p].m, ctx->sums_dst,
                                          ctx->stream));
            ctx->sums_dst += 3;
        }
    }
    job.wres.assign(P, WideRes{});
    HIPCHK(hipMemcpyAsync(job.wres.data(), job.wres_d.p, P * sizeof(WideRes), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    job.fill_ms = ms;
    // the traceback's start columns and the tables' max cell in the PairRes view
    job.res.assign(P, PairRes{});
    for (size_t p = 0; p < P; ++p) {
        job.res[p].max_i = job.wres[p].max_i; job.res[p].max_j = job.wres[p].max_j;
        job.res[p].mam = (int)job.wres[p].mam;
        job.res[p].lmax_i = job.wres[p].lmax_i; job.res[p].lmax_j = job.wres[p].lmax_j;
        job.res[p].end_E = job.wres[p].end_E; job.res[p].lmax_E = job.wres[p].lmax_E;
    }
    return GX_OK;
}

// Plane checksums of job `job`'s pairs into the device buffer out[P][3].
hipError_t enqueue_plane_sums(gx_context* ctx, const FillJob& job, const Scores32& sc,
                              unsigned long long* out, hipStream_t st) {
    int max_strips = 0;
    for (const PairDev& d : job.pd) max_strips = std::max(max_strips, d.strips);
    return launch_plane_sums((const PairDev*)job.pairs.p, (int)job.pd.size(), max_strips, job.lay,
                             job.w16 ? 3 : job.d8 ? 2 : 1,
                             sc.h, sc.g, sc.floor_, (job.shift || job.w16) ? sc.g : 0, out, st ? st : ctx->stream);
}

KeptFill::~KeptFill() { job_release(ctx, job); }
