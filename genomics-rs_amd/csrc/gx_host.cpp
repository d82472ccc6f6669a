// gx_host.cpp -- host mirrors of the reference's input/output contract:
//   from_fasta            src/sequence.rs:45-95    -> gx_fasta_load
//   get_config [scores]   src/config.rs:21-40      -> gx_config_load
//   Display for AlignedSequences  src/alignment/display.rs:9-127 -> gx_format_alignment
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gx.h"

int gx_internal_fail(int code, const std::string& msg);  // gx_api_context.cpp (shared gx_last_error state)

namespace {
int hfail(int code, const std::string& m) { return gx_internal_fail(code, m); }
// The reference's log::info! / warn! lines on the Display path, on stderr
// when GX_LOG asks for them (info / debug: both; warn: warnings only) -- the
// reference's CLI logs at info unless RUST_LOG says otherwise (main.rs:91-96).
int log_level() {
    const char* e = getenv("GX_LOG");
    if (!e) return 0;
    if (!strcmp(e, "debug")) return 3;
    if (!strcmp(e, "info")) return 2;
    if (!strcmp(e, "warn")) return 1;
    return 0;
}
void log_info_line(const std::string& m) { if (log_level() >= 2) fprintf(stderr, "[gx INFO] %s\n", m.c_str()); }
void log_warn_line(const std::string& m) { if (log_level() >= 1) fprintf(stderr, "[gx WARN] %s\n", m.c_str()); }

// ---- UTF-8 / whitespace helpers (BufRead::lines, str::trim) --------------
bool utf8_valid(const unsigned char* s, size_t len) {
    size_t i = 0;
    while (i < len) {
        unsigned char c = s[i];
        if (c < 0x80) { ++i; continue; }
        size_t need;
        unsigned cp;
        if (c >= 0xC2 && c <= 0xDF) { need = 1; cp = c & 0x1F; }
        else if (c >= 0xE0 && c <= 0xEF) { need = 2; cp = c & 0x0F; }
        else if (c >= 0xF0 && c <= 0xF4) { need = 3; cp = c & 0x07; }
        else return false;
        if (i + need >= len) return false;
        for (size_t k = 1; k <= need; ++k) {
            if ((s[i + k] & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (s[i + k] & 0x3F);
        }
        if ((need == 2 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) || (need == 3 && (cp < 0x10000 || cp > 0x10FFFF)))
            return false;
        i += need + 1;
    }
    return true;
}

// length of a leading Unicode White_Space code point at s (0 if none)
size_t ws_at(const unsigned char* s, size_t len) {
    if (len == 0) return 0;
    unsigned char c = s[0];
    if (c == ' ' || (c >= 0x09 && c <= 0x0D)) return 1;
    if (c == 0xC2 && len >= 2 && (s[1] == 0x85 || s[1] == 0xA0)) return 2;
    if (len >= 3) {
        if (c == 0xE1 && s[1] == 0x9A && s[2] == 0x80) return 3;
        if (c == 0xE2 && s[1] == 0x80 && ((s[2] >= 0x80 && s[2] <= 0x8A) || s[2] == 0xA8 || s[2] == 0xA9 || s[2] == 0xAF)) return 3;
        if (c == 0xE2 && s[1] == 0x81 && s[2] == 0x9F) return 3;
        if (c == 0xE3 && s[1] == 0x80 && s[2] == 0x80) return 3;
    }
    return 0;
}
// length of a trailing White_Space code point ending at s+len
size_t ws_before(const unsigned char* s, size_t len) {
    if (len == 0) return 0;
    unsigned char c = s[len - 1];
    if (c == ' ' || (c >= 0x09 && c <= 0x0D)) return 1;
    if (len >= 2 && s[len - 2] == 0xC2 && (c == 0x85 || c == 0xA0)) return 2;
    if (len >= 3 && ws_at(s + len - 3, 3) == 3) return 3;
    return 0;
}
void trim(const unsigned char*& s, size_t& len) {
    size_t k;
    while ((k = ws_at(s, len)) > 0) { s += k; len -= k; }
    while ((k = ws_before(s, len)) > 0) len -= k;
}
}  // namespace

extern "C" int gx_fasta_load(const char* path, uint8_t* buf, size_t cap, uint64_t* name_off, uint64_t* name_len,
                             uint64_t* seq_off, uint64_t* seq_len, size_t rec_cap, size_t* n_records,
                             size_t* bytes_needed) {
    if (!path || !n_records) return hfail(GX_EINVAL, "NULL argument");
    *n_records = 0;
    if (bytes_needed) *bytes_needed = 0;
    FILE* f = fopen(path, "rb");
    if (!f) {
        // sequence.rs:84-86: error!("Could not open file: {}") and nothing is added
        fprintf(stderr, "[gx ERROR] Could not open file: %s\n", path);
        return GX_OK;
    }
    std::vector<unsigned char> data;
    unsigned char tmp[1 << 16];
    size_t k;
    while ((k = fread(tmp, 1, sizeof tmp, f)) > 0) data.insert(data.end(), tmp, tmp + k);
    fclose(f);
    size_t used = 0, nrec = 0;
    bool have = false, overflow = false;
    size_t pos = 0;
    const size_t len = data.size();
    while (pos < len) {
        size_t e = pos;
        while (e < len && data[e] != '\n') ++e;
        const unsigned char* line = data.data() + pos;
        size_t ll = e - pos;
        if (ll > 0 && line[ll - 1] == '\r') --ll;
        if (!utf8_valid(line, ll)) break;                // lines().map_while(Result::ok)
        pos = e < len ? e + 1 : e;
        if (ll == 0) continue;                           // sequence.rs:54-56
        if (line[0] == '>') {                            // sequence.rs:58-71
            const unsigned char* nm = line + 1;
            size_t nl = ll - 1;
            trim(nm, nl);
            if (nrec < rec_cap && used + nl <= cap && buf) {
                memcpy(buf + used, nm, nl);
                name_off[nrec] = used; name_len[nrec] = nl;
                seq_off[nrec] = used + nl; seq_len[nrec] = 0;
            } else {
                overflow = true;
            }
            used += nl;
            ++nrec;
            have = true;
        } else if (have) {                               // sequence.rs:72-78
            const unsigned char* d = line;
            size_t dl = ll;
            trim(d, dl);
            if (!overflow && used + dl <= cap && buf) {
                memcpy(buf + used, d, dl);
                seq_len[nrec - 1] += dl;
            } else {
                overflow = true;
            }
            used += dl;
        } else {
            fprintf(stderr, "[gx WARN] Sequence data found without a header\n");  // sequence.rs:79-81
        }
    }
    *n_records = nrec;
    if (bytes_needed) *bytes_needed = used;
    if (overflow) return hfail(GX_ECAP, "buffer or record capacity too small");
    return GX_OK;
}

// ---- config.rs: minimal TOML for [scores] ------------------------------

namespace {
bool parse_toml_int(std::string v, int64_t* out) {
    // TOML integer: [+-]dec with '_' separators, or 0x / 0o / 0b
    size_t h = v.find('#');
    if (h != std::string::npos) v = v.substr(0, h);
    while (!v.empty() && (v.back() == ' ' || v.back() == '\t' || v.back() == '\r')) v.pop_back();
    while (!v.empty() && (v[0] == ' ' || v[0] == '\t')) v.erase(0, 1);
    if (v.empty()) return false;
    int base = 10;
    bool neg = false;
    size_t i = 0;
    if (v[0] == '+' || v[0] == '-') { neg = v[0] == '-'; i = 1; }
    if (i == 0 && v.size() > 2 && v[0] == '0' && (v[1] == 'x' || v[1] == 'o' || v[1] == 'b')) {
        base = v[1] == 'x' ? 16 : v[1] == 'o' ? 8 : 2;
        i = 2;
    }
    if (i >= v.size()) return false;
    if (base == 10 && v[i] == '0' && i + 1 < v.size()) return false;  // no leading zeros
    std::string digits;
    char prev = '_';
    for (size_t k = i; k < v.size(); ++k) {
        char c = v[k];
        if (c == '_') {
            if (prev == '_') return false;
            prev = c;
            continue;
        }
        int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : 99;
        if (d >= base) return false;
        digits.push_back(c);
        prev = c;
    }
    if (prev == '_' || digits.empty()) return false;
    errno = 0;
    unsigned long long u = strtoull(digits.c_str(), nullptr, base);
    if (errno) return false;
    if (neg) {
        if (u > (unsigned long long)INT64_MAX + 1ull) return false;
        *out = (int64_t)(0ull - u);
    } else {
        if (u > (unsigned long long)INT64_MAX) return false;
        *out = (int64_t)u;
    }
    return true;
}

std::string strip(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && (s[a] == ' ' || s[a] == '\t' || s[a] == '\r')) ++a;
    while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r')) --b;
    return s.substr(a, b - a);
}

bool assign_key(const std::string& key, const std::string& val, gx_scores* s, unsigned* seen) {
    int64_t v;
    int idx = key == "s_match" ? 0 : key == "s_mismatch" ? 1 : key == "g" ? 2 : key == "h" ? 3 : -1;
    if (idx < 0) return true;  // serde ignores unknown fields
    if (!parse_toml_int(val, &v)) return false;
    if (*seen & (1u << idx)) return false;  // duplicate key is a TOML error
    *seen |= 1u << idx;
    (idx == 0 ? s->s_match : idx == 1 ? s->s_mismatch : idx == 2 ? s->g : s->h) = v;
    return true;
}
}  // namespace

extern "C" int gx_config_load(const char* path, gx_scores* out) {
    if (!path || !out) return hfail(GX_EINVAL, "NULL argument");
    FILE* f = fopen(path, "rb");
    if (!f) return hfail(GX_EIO, std::string("Could not read config file: ") + path);  // config.rs:25-27
    std::string text;
    char tmp[4096];
    size_t k;
    while ((k = fread(tmp, 1, sizeof tmp, f)) > 0) text.append(tmp, k);
    fclose(f);
    const std::string perr = std::string("Could not parse config file: ") + path;  // config.rs:33-35
    gx_scores s{};
    unsigned seen = 0;
    bool in_scores = false, scores_defined = false;
    size_t pos = 0;
    while (pos <= text.size()) {
        size_t e = text.find('\n', pos);
        if (e == std::string::npos) e = text.size();
        std::string line = strip(text.substr(pos, e - pos));
        pos = e + 1;
        if (line.empty() || line[0] == '#') { if (e == text.size()) break; continue; }
        if (line[0] == '[') {
            size_t c = line.find(']');
            if (c == std::string::npos) return hfail(GX_EPARSE, perr);
            std::string name = strip(line.substr(1, c - 1));
            std::string rest = strip(line.substr(c + 1));
            if (!rest.empty() && rest[0] != '#') return hfail(GX_EPARSE, perr);
            if (name == "scores") {
                if (scores_defined) return hfail(GX_EPARSE, perr);
                scores_defined = true;
                in_scores = true;
            } else {
                in_scores = false;
            }
        } else {
            size_t eq = line.find('=');
            if (eq == std::string::npos) return hfail(GX_EPARSE, perr);
            std::string key = strip(line.substr(0, eq));
            std::string val = strip(line.substr(eq + 1));
            if (!in_scores && key == "scores" && !val.empty() && val[0] == '{') {
                // inline table: scores = { s_match = 1, ... }
                if (scores_defined) return hfail(GX_EPARSE, perr);
                scores_defined = true;
                size_t close = val.find('}');
                if (close == std::string::npos) return hfail(GX_EPARSE, perr);
                std::string body = val.substr(1, close - 1);
                size_t p = 0;
                while (p < body.size()) {
                    size_t comma = body.find(',', p);
                    if (comma == std::string::npos) comma = body.size();
                    std::string kv = strip(body.substr(p, comma - p));
                    p = comma + 1;
                    if (kv.empty()) continue;
                    size_t q = kv.find('=');
                    if (q == std::string::npos) return hfail(GX_EPARSE, perr);
                    if (!assign_key(strip(kv.substr(0, q)), strip(kv.substr(q + 1)), &s, &seen))
                        return hfail(GX_EPARSE, perr);
                }
            } else if (!in_scores && key.rfind("scores.", 0) == 0) {
                scores_defined = true;
                if (!assign_key(strip(key.substr(7)), val, &s, &seen)) return hfail(GX_EPARSE, perr);
            } else if (in_scores) {
                if (!assign_key(key, val, &s, &seen)) return hfail(GX_EPARSE, perr);
            }
        }
        if (e == text.size()) break;
    }
    if (seen != 0xF) return hfail(GX_EPARSE, perr);  // a missing field fails deserialization
    *out = s;
    return GX_OK;
}

// ---- display.rs:9-127 -----------------------------------------------------

namespace {
void push_char(std::string& s, unsigned char b) {
    // `byte as char` then String::push: bytes >= 0x80 are Latin-1 code points
    if (b < 0x80) s.push_back((char)b);
    else {
        s.push_back((char)(0xC0 | (b >> 6)));
        s.push_back((char)(0x80 | (b & 0x3F)));
    }
}

// Rust `{}` for f64: shortest round-trip digits, never exponent notation.
std::string rust_f64(double v) {
    if (std::isnan(v)) return "NaN";
    if (std::isinf(v)) return v > 0 ? "inf" : "-inf";
    if (v == 0.0) return std::signbit(v) ? "-0" : "0";
    char b[64];
    int prec = 1;
    for (; prec <= 17; ++prec) {
        snprintf(b, sizeof b, "%.*e", prec - 1, v);
        if (strtod(b, nullptr) == v) break;
    }
    // b = [-]d.ddde[+-]XX
    std::string s(b);
    bool neg = s[0] == '-';
    if (neg) s.erase(0, 1);
    size_t epos = s.find('e');
    int ex = atoi(s.c_str() + epos + 1);
    std::string dig;
    for (size_t k = 0; k < epos; ++k) if (s[k] != '.') dig.push_back(s[k]);
    std::string r;
    int point = ex + 1;  // digits before the decimal point
    if (point <= 0) {
        r = "0." + std::string(-point, '0') + dig;
    } else if ((size_t)point >= dig.size()) {
        r = dig + std::string(point - dig.size(), '0');
    } else {
        r = dig.substr(0, point) + "." + dig.substr(point);
    }
    return neg ? "-" + r : r;
}

std::string pct2(uint64_t a, uint64_t b) {
    double v = (double)a / (double)b * 100.0;
    if (std::isnan(v)) return "NaN";
    char buf[64];
    snprintf(buf, sizeof buf, "%.2f", v);
    return buf;
}
}  // namespace

extern "C" int gx_format_alignment(const uint8_t* s1, size_t n, const uint8_t* s2, size_t m, const gx_step* steps,
                                   size_t n_steps, const gx_result* res, char* out, size_t cap, size_t* needed) {
    if ((!s1 && n) || (!s2 && m) || (!steps && n_steps) || !res) return hfail(GX_EINVAL, "NULL argument");
    const size_t W = 200;  // DISP_MAX_WIDTH (display.rs:7)
    // display.rs:12-18 (logged once per rendering: the size query of a
    // two-call use -- out == NULL -- stays silent)
    if (out) {
        if (n <= W && m <= W) {
            log_info_line("Original Sequences:");
            log_info_line(std::string((const char*)s1, n));
            log_info_line(std::string((const char*)s2, m));
        } else {
            log_warn_line("Sequences are too long to display.");
        }
    }
    std::string f, s1o, alo, s2o;
    size_t s1i = 0, s2i = 0, hl = 0, ai = 0;
    while (ai < n_steps) {
        const int c = steps[n_steps - 1 - ai].choice;  // alignment.iter().rev()
        if (hl > W) {
            f += "\n\n" + std::to_string(ai - W) + "-" + std::to_string(ai) + ":\n\n";
            f += s1o + "\n" + alo + "\n" + s2o + "\n";
            s1o.clear(); alo.clear(); s2o.clear();
            hl = 0;
        }
        if (c == GX_INSERT || c == GX_OPEN_INSERT) s1o.push_back('-');
        else if (s1i < n) push_char(s1o, s1[s1i++]);
        switch (c) {
            case GX_MATCH: alo.push_back('|'); break;
            case GX_MISMATCH: alo.push_back('x'); break;
            case GX_INSERT: case GX_DELETE: alo.push_back(' '); break;
            default: alo.push_back('%'); break;
        }
        if (c == GX_DELETE || c == GX_OPEN_DELETE) s2o.push_back('-');
        else if (s2i < m) push_char(s2o, s2[s2i++]);
        ++hl;
        ++ai;
    }
    f += "\n\n" + std::to_string(ai - s1o.size()) + "-" + std::to_string(ai) + ":\n\n";
    f += s1o + "\n" + alo + "\n" + s2o + "\n";
    f += "\n\nAlignment Score: " + std::to_string(res->score) + "\n";
    f += "Matches: " + std::to_string(res->matches) + "/" + std::to_string(ai) + " (" + pct2(res->matches, ai) + "%)\n";
    f += "Mismatches: " + std::to_string(res->mismatches) + "/" + std::to_string(ai) + " (" + pct2(res->mismatches, ai) + "%)\n";
    f += "Gap Extensions: " + std::to_string(res->gap_extensions) + "/" + std::to_string(ai) + " (" +
         pct2(res->gap_extensions, ai) + "%)\n";
    f += "Opening Gaps: " + std::to_string(res->opening_gaps) + "/" + std::to_string(ai) + " (" +
         pct2(res->opening_gaps, ai) + "%)\n";
    f += "Percent Identity " + rust_f64((double)res->matches / (double)ai * 100.0) + "%\n";
    if (needed) *needed = f.size() + 1;
    if (!out || cap < f.size() + 1) return hfail(GX_ECAP, "output buffer too small");
    memcpy(out, f.c_str(), f.size() + 1);
    return GX_OK;
}

// ---- display.rs:131-220  print_alignment_table / print_scores_table --------
//
// The reference prints these from inside retrace (algo.rs:438) with the table
// it was handed; here the caller passes the three int64 score planes
// (row-major (n+1)x(m+1), as gx_table_export_plane writes them) and the
// alignment, and receives the text print_alignment_table writes to stdout.
// Inputs with n >= 200 or m >= 2000 produce the empty string (the reference
// warns "Sequence table too large to visualize" and prints nothing,
// display.rs:139-144).  `color` selects the `colored` crate's ANSI styling
// (it colours only when stdout is a terminal); 0 gives plain text.

namespace {
// Number of chars in a UTF-8 byte string (the reference indexes with chars().nth()).
size_t utf8_chars(const uint8_t* s, size_t len) {
    size_t c = 0;
    for (size_t k = 0; k < len; ++k) c += (s[k] & 0xC0) != 0x80;
    return c;
}

void scores_table(std::string& f, const int64_t* plane, size_t n, size_t m) {
    // display.rs:183-219
    f += ". \t";
    for (size_t j = 0; j <= m; ++j) f += std::to_string(j) + "\t";
    f += "\n";
    for (size_t i = 0; i <= n; ++i) {
        f += std::to_string(i) + "\t";
        for (size_t j = 0; j <= m; ++j) {
            const int64_t v = plane[i * (m + 1) + j];
            f += v <= -9223372036854775700LL ? std::string("-inf") : std::to_string(v);
            f += "\t";
        }
        f += "\n";
    }
}
}  // namespace

extern "C" int gx_format_table(const uint8_t* s1, size_t n, const uint8_t* s2, size_t m, const gx_step* steps,
                               size_t n_steps, const int64_t* insert_plane, const int64_t* delete_plane,
                               const int64_t* sub_plane, int color, char* out, size_t cap, size_t* needed) {
    if ((!s1 && n) || (!s2 && m) || (!steps && n_steps)) return hfail(GX_EINVAL, "NULL argument");
    const size_t W = 200;  // DISP_MAX_WIDTH (display.rs:7)
    std::string f;
    if (out) {   // display.rs:139-144
        if (n < W && m < W * 10) log_info_line("Computing sequence table visualization...");
        else log_warn_line("Sequence table too large to visualize");
    }
    if (n < W && m < W * 10) {
        if (!insert_plane || !delete_plane || !sub_plane) return hfail(GX_EINVAL, "NULL score plane");
        // chars().nth(k).unwrap() for k < byte length panics on multi-byte text
        if (utf8_chars(s1, n) != n || utf8_chars(s2, m) != m)
            return hfail(GX_EPANIC, "called `Option::unwrap()` on a `None` value (display.rs:150)");
        // path cells: .find(|(_, x, y)| x == i+1 && y == j+1) takes the first hit
        std::vector<int8_t> mark((n + 1) * (m + 1), -1);
        for (size_t k = n_steps; k-- > 0;) {
            const gx_step& s = steps[k];
            if (s.i <= n && s.j <= m) mark[s.i * (m + 1) + s.j] = (int8_t)s.choice;
        }
        static const char* glyph[6] = {"M", "X", "I", "D", "I", "D"};
        // colored 3: fg green 32, red 31, blue 34, cyan 36; bold = style 1
        static const char* style[6] = {"\x1b[32m", "\x1b[31m", "\x1b[34m", "\x1b[36m", "\x1b[1;34m", "\x1b[1;36m"};
        f += "\nSequence Table (S1 columns, S2 rows):\n\n";
        f += " ";
        f.append((const char*)s2, m);
        f += "\n";
        for (size_t i = 0; i < n; ++i) {
            f.push_back((char)s1[i]);
            for (size_t j = 0; j < m; ++j) {
                const int c = mark[(i + 1) * (m + 1) + (j + 1)];
                if (c < 0 || c > 5) { f += "."; continue; }
                if (color) f += std::string(style[c]) + glyph[c] + "\x1b[0m";
                else f += glyph[c];
            }
            f += "\n";
        }
        f += "Delete Scores\n";
        scores_table(f, delete_plane, n, m);
        f += "Insert Scores\n";
        scores_table(f, insert_plane, n, m);
        f += "Sub Scores\n";
        scores_table(f, sub_plane, n, m);
    }
    if (needed) *needed = f.size() + 1;
    if (!out || cap < f.size() + 1) return hfail(GX_ECAP, "output buffer too small");
    memcpy(out, f.c_str(), f.size() + 1);
    return GX_OK;
}
