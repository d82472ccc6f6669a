// gx-align -- the reference CLI's `align` mode (src/main.rs:27-37, 77-84,
// 86-153) on top of the C ABI:
//     gx-align [-c config.toml] align [-a local|global|1] -f pair.fasta
// Loads the config (config.rs), the FASTA (sequence.rs), aligns the first two
// records on the GPU and prints the AlignedSequences Display (display.rs).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gx.h"

static void usage() {
    fprintf(stderr,
            "Usage: gx-align [-c|--config-path <CONFIG>] align [-a|--alignment-type <TYPE>] "
            "-f|--fasta-path <FASTA>\n");
}

int main(int argc, char** argv) {
    std::string config = "config.toml", type = "local", fasta;
    bool have_align = false;
    for (int k = 1; k < argc; ++k) {
        std::string a = argv[k];
        auto next = [&](std::string& dst) {
            if (k + 1 >= argc) { usage(); exit(2); }
            dst = argv[++k];
        };
        if (a == "-c" || a == "--config-path") next(config);
        else if (a == "align") have_align = true;
        else if (a == "-a" || a == "--alignment-type") next(type);
        else if (a == "-f" || a == "--fasta-path") next(fasta);
        else if (a == "-h" || a == "--help") { usage(); return 0; }
        else { usage(); return 2; }
    }
    if (!have_align || fasta.empty()) { usage(); return 2; }
    gx_scores sc;
    if (gx_config_load(config.c_str(), &sc) != GX_OK) {
        fprintf(stderr, "[ERROR] %s\n", gx_last_error());
        return 1;  // config.rs: exit(1)
    }
    size_t nrec = 0, need = 0;
    gx_fasta_load(fasta.c_str(), nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, &nrec, &need);
    std::vector<uint8_t> buf(need + 1);
    std::vector<uint64_t> no(nrec + 1), nl(nrec + 1), so(nrec + 1), sl(nrec + 1);
    if (nrec) gx_fasta_load(fasta.c_str(), buf.data(), buf.size(), no.data(), nl.data(), so.data(), sl.data(), nrec,
                            &nrec, &need);
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
    if (gx_context_create(0, &ctx) != GX_OK) {
        fprintf(stderr, "[ERROR] %s\n", gx_last_error());
        return 1;
    }
    const uint8_t* s1 = buf.data() + so[0];
    const uint8_t* s2 = buf.data() + so[1];
    const size_t n = sl[0], m = sl[1];
    std::vector<gx_step> steps(n + m + 2);
    gx_result res{};
    int rc = gx_align(ctx, s1, n, s2, m, &sc, is_local, 0, 0, steps.data(), steps.size(), &res);
    if (rc != GX_OK) {
        fprintf(stderr, "[ERROR] %s\n", gx_last_error());
        gx_context_destroy(ctx);
        return rc == GX_EPANIC ? 101 : 1;
    }
    fprintf(stderr, "[INFO] Table initialization complete, time taken: %lldus\n", (long long)res.fill_us);
    fprintf(stderr, "[INFO] Retrace complete, time taken: %lldus\n", (long long)res.retrace_us);
    size_t need_txt = 0;
    gx_format_alignment(s1, n, s2, m, steps.data(), res.n_steps, &res, nullptr, 0, &need_txt);
    std::vector<char> txt(need_txt);
    gx_format_alignment(s1, n, s2, m, steps.data(), res.n_steps, &res, txt.data(), txt.size(), nullptr);
    fputs(txt.data(), stdout);
    gx_context_destroy(ctx);
    return 0;
}
