// gx-align -- the reference CLI (src/main.rs) on top of the C ABI.
//
//   gx-align [-c config.toml] align [-a local|global|1] -f pair.fasta
//       main.rs:27-37, 77-84, 86-153: load config (config.rs) and FASTA
//       (sequence.rs), align the first two records on the GPU, print the
//       sequence table for small inputs (retrace -> print_alignment_table,
//       algo.rs:438, display.rs:131-220) and the AlignedSequences Display
//       (display.rs:9-127).
//
//   gx-align [-c config.toml] all-vs-all -d fasta_dir [-a global|local]
//            [-o similarity_matrix.tsv] [-g N_GPUS] [--no-self]
//       BASELINE config 4: every pair (i, j), i <= j, of the
//       records of all *.fasta files in fasta_dir aligned on the GPU(s), with
//       the matrix layout and TSV writer of the reference's `compare` mode
//       (main.rs:216-378: row r, column c filled for c <= r, written as
//       "r\t v\t v\t ..."), carrying the alignment score instead of the suffix
//       tree's LCS score.  Pairs are sharded over the GPUs by longest-
//       processing-time on n*m, one host thread and gx_context per GPU, one
//       batched launch per GPU.  Files are read in name order (the reference
//       uses fs::read_dir order, which the OS leaves unspecified).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "../../include/gx.h"

namespace {

void usage() {
    fprintf(stderr,
            "Usage: gx-align [-c|--config-path <CONFIG>] align [-a|--alignment-type <TYPE>] -f|--fasta-path <FASTA>\n"
            "       gx-align [-c|--config-path <CONFIG>] all-vs-all -d|--fasta-dir <DIR> [-a <TYPE>] "
            "[-o <TSV>] [-g|--gpus <N>] [--no-self]\n");
}

struct Records {
    std::vector<uint8_t> buf;
    std::vector<uint64_t> no, nl, so, sl;
    size_t size() const { return so.size(); }
    const uint8_t* seq(size_t k) const { return buf.data() + so[k]; }
    std::string name(size_t k) const { return std::string((const char*)buf.data() + no[k], nl[k]); }
};

// from_fasta (sequence.rs:45-95) appending to `r`
void load_fasta(const std::string& path, Records& r) {
    size_t nrec = 0, need = 0;
    gx_fasta_load(path.c_str(), nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, &nrec, &need);
    if (!nrec) return;
    std::vector<uint8_t> buf(need + 1);
    std::vector<uint64_t> no(nrec), nl(nrec), so(nrec), sl(nrec);
    gx_fasta_load(path.c_str(), buf.data(), buf.size(), no.data(), nl.data(), so.data(), sl.data(), nrec, &nrec,
                  &need);
    const uint64_t base = r.buf.size();
    r.buf.insert(r.buf.end(), buf.begin(), buf.begin() + need);
    for (size_t k = 0; k < nrec; ++k) {
        r.no.push_back(base + no[k]);
        r.nl.push_back(nl[k]);
        r.so.push_back(base + so[k]);
        r.sl.push_back(sl[k]);
    }
}

bool stdout_color() {
    // the `colored` crate: CLICOLOR_FORCE forces, NO_COLOR / CLICOLOR=0 disable, else a terminal
    if (const char* f = getenv("CLICOLOR_FORCE"); f && strcmp(f, "0")) return true;
    if (const char* nc = getenv("NO_COLOR"); nc && *nc) return false;
    if (const char* c = getenv("CLICOLOR"); c && !strcmp(c, "0")) return false;
    return isatty(1);
}

int fail_msg(const char* what, int rc) {
    fprintf(stderr, "[ERROR] %s: %s\n", what, gx_last_error());
    return rc == GX_EPANIC ? 101 : 1;
}

int run_align(const gx_scores& sc, const std::string& type, const std::string& fasta) {
    Records r;
    load_fasta(fasta, r);
    const size_t nrec = r.size();
    if (nrec < 2) {
        fprintf(stderr, "thread 'main' panicked: index out of bounds: the len is %zu but the index is %zu\n", nrec,
                nrec);
        return 101;  // algo.rs:169 panics on fewer than two sequences
    }
    if (nrec > 2) fprintf(stderr, "[WARN] More than two sequences found. Only the first two will be used.\n");
    fprintf(stderr, "[INFO] Using the following values for scoring:\n[INFO] Match: %lld\n[INFO] Mismatch: %lld\n"
                    "[INFO] Gap: %lld\n[INFO] Opening Gap: %lld\n[INFO] Alignment Type: %s\n",
            (long long)sc.s_match, (long long)sc.s_mismatch, (long long)sc.g, (long long)sc.h, type.c_str());
    const int is_local = (type == "local" || type == "1") ? 1 : 0;  // main.rs:142
    gx_context* ctx = nullptr;
    if (gx_context_create(0, &ctx) != GX_OK) return fail_msg("context", 1);
    const uint8_t* s1 = r.seq(0);
    const uint8_t* s2 = r.seq(1);
    const size_t n = r.sl[0], m = r.sl[1];
    std::vector<gx_step> steps(n + m + 2);
    gx_result res{};
    std::string table_txt;
    if (n < 200 && m < 2000) {
        // small input: keep the planes so that the sequence table can be printed (algo.rs:438)
        gx_table* t = nullptr;
        uint64_t mam = 0;
        int rc = gx_alignment_table(ctx, s1, n, s2, m, &sc, is_local, 0, GX_TABLE_PLANES, &t, &mam);
        if (rc != GX_OK) { gx_context_destroy(ctx); return fail_msg("alignment_table", rc); }
        const size_t cells = (n + 1) * (m + 1);
        std::vector<int64_t> pl(3 * cells);
        for (int k = 0; k < 3 && rc == GX_OK; ++k) rc = gx_table_export_plane(t, k, pl.data() + k * cells, cells, 0);
        if (rc != GX_OK) { gx_table_free(t); gx_context_destroy(ctx); return fail_msg("export", rc); }
        rc = gx_retrace(t, is_local, steps.data(), steps.size(), &res);
        if (rc != GX_OK) { gx_context_destroy(ctx); return fail_msg("retrace", rc); }
        size_t need = 0;
        const int color = stdout_color();
        gx_format_table(s1, n, s2, m, steps.data(), res.n_steps, pl.data(), pl.data() + cells,
                        pl.data() + 2 * cells, color, nullptr, 0, &need);
        table_txt.resize(need);
        rc = gx_format_table(s1, n, s2, m, steps.data(), res.n_steps, pl.data(), pl.data() + cells,
                             pl.data() + 2 * cells, color, table_txt.data(), need, nullptr);
        if (rc != GX_OK) { gx_context_destroy(ctx); return fail_msg("print_alignment_table", rc); }
        table_txt.resize(need ? need - 1 : 0);
    } else {
        int rc = gx_align(ctx, s1, n, s2, m, &sc, is_local, 0, 0, steps.data(), steps.size(), &res);
        if (rc != GX_OK) { gx_context_destroy(ctx); return fail_msg("align", rc); }
        fprintf(stderr, "[WARN] Sequence table too large to visualize\n");
    }
    // (the library logs the table shape, its fill time, the start cell and the
    // retrace lines of algo.rs:175-179, 274-277, 325, 428-436 under GX_LOG=info)
    fputs(table_txt.c_str(), stdout);
    size_t need_txt = 0;
    gx_format_alignment(s1, n, s2, m, steps.data(), res.n_steps, &res, nullptr, 0, &need_txt);
    std::vector<char> txt(need_txt);
    gx_format_alignment(s1, n, s2, m, steps.data(), res.n_steps, &res, txt.data(), txt.size(), nullptr);
    fputs(txt.data(), stdout);
    gx_context_destroy(ctx);
    return 0;
}

// Longest-processing-time partition of `w` over `parts` bins.
std::vector<std::vector<size_t>> lpt(const std::vector<double>& w, int parts) {
    std::vector<size_t> order(w.size());
    for (size_t k = 0; k < w.size(); ++k) order[k] = k;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return w[a] > w[b]; });
    std::vector<std::vector<size_t>> bins(parts);
    std::vector<double> load(parts, 0.0);
    for (size_t k : order) {
        int b = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        bins[b].push_back(k);
        load[b] += w[k];
    }
    for (auto& b : bins) std::sort(b.begin(), b.end());
    return bins;
}

int run_all_vs_all(const gx_scores& sc, const std::string& type, const std::string& dir, const std::string& tsv,
                   int ngpu, bool with_self) {
    namespace fs = std::filesystem;
    std::vector<std::string> files;
    std::error_code ec;
    for (const auto& e : fs::directory_iterator(dir, ec))
        if (e.path().extension() == ".fasta") files.push_back(e.path().string());
    if (ec) { fprintf(stderr, "[ERROR] cannot read directory %s: %s\n", dir.c_str(), ec.message().c_str()); return 1; }
    std::sort(files.begin(), files.end());
    fprintf(stderr, "[INFO] Loading sequences from %s\n", dir.c_str());
    Records r;
    for (const auto& f : files) load_fasta(f, r);
    const size_t K = r.size();
    fprintf(stderr, "[INFO] Number of sequences: %zu\n", K);
    const int is_local = (type == "local" || type == "1") ? 1 : 0;
    std::vector<std::pair<size_t, size_t>> pairs;
    for (size_t j = 0; j < K; ++j)
        for (size_t i = 0; i <= j; ++i)
            if (i < j || with_self) pairs.push_back({i, j});
    std::vector<double> w(pairs.size());
    double cells = 0;
    for (size_t p = 0; p < pairs.size(); ++p) {
        w[p] = (double)r.sl[pairs[p].first] * (double)r.sl[pairs[p].second];
        cells += w[p];
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        fprintf(stderr, "[ERROR] no HIP device\n");
        return 1;
    }
    // GX_DEVICE_MAP=d0,d1,...: logical shard g runs on device map[g % len]
    // (e.g. "0,0,0,0" runs a 4-shard plan on one GPU: the multi-GPU code path
    // with several contexts on one device); without it shards clamp to the
    // visible devices
    std::vector<int> devmap;
    if (const char* dm = getenv("GX_DEVICE_MAP"); dm && *dm) {
        for (const char* q = dm; *q;) {
            char* end = nullptr;
            const long d = strtol(q, &end, 10);
            if (end == q) break;
            if (d < 0 || d >= ndev) { fprintf(stderr, "[ERROR] GX_DEVICE_MAP: no HIP device %ld\n", d); return 1; }
            devmap.push_back((int)d);
            q = *end == ',' ? end + 1 : end;
        }
    }
    if (devmap.empty()) {
        if (ngpu <= 0 || ngpu > ndev) ngpu = ndev;
        for (int g = 0; g < ngpu; ++g) devmap.push_back(g);
    } else if (ngpu <= 0) {
        ngpu = (int)devmap.size();
    }
    auto bins = lpt(w, ngpu);
    std::vector<gx_result> res(pairs.size());
    std::vector<int> rcs(ngpu, GX_OK);
    std::vector<std::string> errs(ngpu);
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int g = 0; g < ngpu; ++g) {
        th.emplace_back([&, g] {
            const auto& b = bins[g];
            if (b.empty()) return;
            gx_context* ctx = nullptr;
            int rc = gx_context_create(devmap[g % devmap.size()], &ctx);
            if (rc == GX_OK) {
                std::vector<const uint8_t*> a1, a2;
                std::vector<size_t> n1, n2;
                for (size_t p : b) {
                    a1.push_back(r.seq(pairs[p].first)); n1.push_back(r.sl[pairs[p].first]);
                    a2.push_back(r.seq(pairs[p].second)); n2.push_back(r.sl[pairs[p].second]);
                }
                std::vector<gx_result> out(b.size());
                rc = gx_align_batch(ctx, a1.data(), n1.data(), a2.data(), n2.data(), b.size(), &sc, is_local, 0,
                                    nullptr, nullptr, out.data());
                if (rc == GX_OK)
                    for (size_t k = 0; k < b.size(); ++k) res[b[k]] = out[k];
                gx_context_destroy(ctx);
            }
            if (rc != GX_OK) errs[g] = gx_last_error();
            rcs[g] = rc;
        });
    }
    for (auto& t : th) t.join();
    for (int g = 0; g < ngpu; ++g)
        if (rcs[g] != GX_OK) {
            fprintf(stderr, "[ERROR] GPU %d: %s\n", g, errs[g].c_str());
            return rcs[g] == GX_EPANIC ? 101 : 1;
        }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    fprintf(stderr, "[INFO] Time taken to compare: %.0f us (%.0f ms), %zu pairs on %d shard(s), %.1f GCUPS\n", us,
            us / 1e3, pairs.size(), ngpu, cells / us / 1e3);
    for (int g = 0; g < ngpu; ++g) {
        double cg = 0;
        for (size_t p : bins[g]) cg += w[p];
        fprintf(stderr, "[INFO] shard %d: device %d, %zu pairs, %.3g cells\n", g, devmap[g % devmap.size()],
                bins[g].size(), cg);
    }
    // matrix in the reference's layout: row j, column i filled for i <= j (main.rs:253-264)
    std::vector<const gx_result*> cellp(K * K, nullptr);
    for (size_t p = 0; p < pairs.size(); ++p) cellp[pairs[p].second * K + pairs[p].first] = &res[p];
    FILE* f = fopen(tsv.c_str(), "w");
    if (!f) { fprintf(stderr, "[ERROR] cannot write %s\n", tsv.c_str()); return 1; }
    auto table = [&](FILE* o, bool header_blank, auto field) {
        fprintf(o, header_blank ? " \t" : "\t");
        for (size_t i = 0; i < K; ++i) fprintf(o, "%zu\t", i);
        fprintf(o, "\n");
        for (size_t j = 0; j < K; ++j) {
            fprintf(o, "%zu\t", j);
            for (size_t i = 0; i < K; ++i) {
                const gx_result* c = cellp[j * K + i];
                fprintf(o, "%lld\t", c ? (long long)field(*c) : 0LL);
            }
            fprintf(o, "\n");
        }
    };
    table(f, false, [](const gx_result& c) { return c.score; });
    fclose(f);
    printf("Similarity TSV:\n");
    table(stdout, true, [](const gx_result& c) { return c.score; });
    printf("\nMatches TSV:\n");
    table(stdout, true, [](const gx_result& c) { return (int64_t)c.matches; });
    printf("\nSequences:\n");
    for (size_t k = 0; k < K; ++k) printf("%zu\t%s\t%llu\n", k, r.name(k).c_str(), (unsigned long long)r.sl[k]);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    // main.rs:91-96: the CLI logs at info unless told otherwise
    setenv("GX_LOG", getenv("GX_LOG") ? getenv("GX_LOG") : "info", 1);
    std::string config = "config.toml", type, fasta, dir, tsv = "similarity_matrix.tsv", mode;
    int ngpu = 0;
    bool with_self = true;
    for (int k = 1; k < argc; ++k) {
        std::string a = argv[k];
        auto next = [&](std::string& dst) {
            if (k + 1 >= argc) { usage(); exit(2); }
            dst = argv[++k];
        };
        if (a == "-c" || a == "--config-path") next(config);
        else if (a == "align" || a == "all-vs-all") mode = a;
        else if (a == "-a" || a == "--alignment-type") next(type);
        else if (a == "-f" || a == "--fasta-path") next(fasta);
        else if (a == "-d" || a == "--fasta-dir") next(dir);
        else if (a == "-o" || a == "--output") next(tsv);
        else if (a == "-g" || a == "--gpus") { std::string v; next(v); ngpu = atoi(v.c_str()); }
        else if (a == "--no-self") with_self = false;
        else if (a == "-h" || a == "--help") { usage(); return 0; }
        else { usage(); return 2; }
    }
    if (mode.empty() || (mode == "align" && fasta.empty()) || (mode == "all-vs-all" && dir.empty())) {
        usage();
        return 2;
    }
    gx_scores sc;
    if (gx_config_load(config.c_str(), &sc) != GX_OK) {
        fprintf(stderr, "[ERROR] %s\n", gx_last_error());
        return 1;  // config.rs: exit(1)
    }
    if (mode == "align") return run_align(sc, type.empty() ? "local" : type, fasta);  // main.rs:35 default "local"
    return run_all_vs_all(sc, type.empty() ? "global" : type, dir, tsv, ngpu, with_self);
}
