// gx_api.h -- internal state and helpers of the host side of the C ABI
// (include/gx.h), shared by the gx_api_*.cpp files:
//   gx_api_context.cpp  contexts, errors, device buffer pool, pipeline slots
//   gx_api_plan.cpp     range guard, boundary cells, launch planning
//   gx_api_fill.cpp     fill launches (int32 layouts, twin fill, int64 fill)
//   gx_api_walk.cpp     traceback walk, start cells, labelling
//   gx_api_table.cpp    alignment_table / retrace (algo.rs:151-441), table export
//   gx_api_batch.cpp    batches of independent pairs, multi-context batches
//   gx_api_staged.cpp   device-resident (staged) batches, the benchmark path
// Not a public header: host code only, one library.
#pragma once
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gx.h"
#include "gx_internal.h"

// Everything below is internal to the library: hidden, so that only the C
// ABI (gx.h, declared above with default visibility) is exported.
#pragma GCC visibility push(hidden)

namespace gx {
hipError_t launch_fill(int W, int lay, bool local, int planes, bool track, bool lcs, bool tbl, const PairDev* d_pairs, int npairs,
                       int total_bands, int* d_counter, StripRes* d_sres, PairRes* d_pres, Scores32 sc, int grid,
                       hipStream_t st);
hipError_t launch_finalize(const PairDev* d_pairs, int npairs, const StripRes* d_sres, PairRes* d_pres,
                           hipStream_t st);
hipError_t launch_traceback(const TbDev* d_jobs, int njobs, int max_strips, bool w16, bool seq, hipStream_t st);
hipError_t launch_export(const int32_t* plane, int32_t* out, int n, int m, int t4, int lay, int gshift, int row0,
                         int rows, hipStream_t st);
hipError_t launch_export_w16(const uint8_t* codes, int half, int which, int32_t* out, int n, int m, int t4, int h,
                             int g, int floor_, int gshift, int row0, int rows, hipStream_t st);
hipError_t launch_export_d8(const uint8_t* pI, const uint8_t* px, int32_t* out, int n, int m, int t4, int h, int g,
                            int floor_, int gshift, int row0, int rows, hipStream_t st);
hipError_t launch_plane_sums(const PairDev* d_pairs, int npairs, int max_strips, int lay, int mode, int h, int g,
                             int floor_, int gshift, unsigned long long* out, hipStream_t st);
hipError_t launch_local_col(const PairDev* d_pairs, int npairs, PairRes* d_pres, int h, int g, hipStream_t st);
hipError_t launch_fill_cs2(int W, bool local, bool planes, bool tbl, const PairDev* d_pairs, int npairs,
                           int total_bands, int* d_counter, StripRes* d_sres, PairRes* d_pres, Scores32 sc, int grid,
                           hipStream_t st);
hipError_t launch_fill_skew(int W, bool local, bool planes, bool tbl, bool trace, bool track, const PairDev* d_pairs, int npairs,
                            int total_bands, int* d_counter, StripRes* d_sres, PairRes* d_pres, Scores32 sc, int grid,
                            int lcs_blocks, hipStream_t st);
int skew_lcs_blocks(int W, int n, int m);
int skew_lcs_sweep(int W);
hipError_t launch_skew_max_col(const PairDev* d_pairs, int npairs, int mmax, PairRes* d_pres, int gshift, hipStream_t st);
bool skew_traced(bool planes, bool trace, bool track);
hipError_t launch_skew_codes(const PairDev* d_pairs, int npairs, int mmax, Scores32 sc, bool tbl, hipStream_t st);
hipError_t launch_fill_pk(int W, int planes, const PairDev* d_pairs, int npairs, int ntwins, int total_bands,
                          int* d_counter, PairRes* d_pres, StripRes* d_sres, Scores32 sc, int grid, hipStream_t st);
hipError_t launch_fill_wide(const WideDev* d_pairs, int npairs, WideScores sc, WideRes* d_res, int local, int track,
                            hipStream_t st);
hipError_t launch_wide_plane_sums(const int64_t* pI, const int64_t* pD, const int64_t* pS, int n, int m,
                                  unsigned long long* out, hipStream_t st);
}  // namespace gx

using namespace gx;

extern thread_local std::string g_err;   // the calling thread's last error (gx_last_error)
int fail(int code, const std::string& msg);
#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(e_ == hipErrorOutOfMemory ? GX_ENOMEM : GX_EHIP,                       \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                   \
    } while (0)

// ---------------------------------------------------------------------------
// device buffer pool (one per context)

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

// Distinct processed bytes of a job, while there are at most 4 (the fill's
// small-alphabet score table, Scores32.sym); n = 5 means "more than 4".
struct SmallAlpha {
    int sym[4] = {-1, -1, -1, -1};
    int n = 0;
    void add(const uint8_t* p, size_t len) {
        if (n > 4) return;
        bool seen[256] = {};
        for (int k = 0; k < n; ++k) seen[sym[k]] = true;
        for (size_t i = 0; i < len; ++i) {
            if (seen[p[i]]) continue;
            if (n == 4) { n = 5; return; }
            seen[p[i]] = true;
            sym[n++] = p[i];
        }
    }
};

// A walk's labelled steps: a growable array that, unlike std::vector, does
// not zero what it reserves (the labelling writes every step, ~48 MB a pass
// of a 1024 x 1k batch, and is on the short-batch step's critical path).
class StepBuf {
public:
    StepBuf() = default;
    StepBuf(const StepBuf& o) { *this = o; }
    StepBuf(StepBuf&& o) noexcept : p_(o.p_), n_(o.n_), cap_(o.cap_) { o.p_ = nullptr; o.n_ = o.cap_ = 0; }
    StepBuf& operator=(const StepBuf& o) {   // (as std::vector: bad_alloc when the copy cannot be held)
        if (this != &o) {
            clear();
            if (!reserve(o.n_)) throw std::bad_alloc();
            if (o.n_) memcpy(p_, o.p_, o.n_ * sizeof(gx_step));
            n_ = o.n_;
        }
        return *this;
    }
    StepBuf& operator=(StepBuf&& o) noexcept {
        std::swap(p_, o.p_); std::swap(n_, o.n_); std::swap(cap_, o.cap_);
        return *this;
    }
    ~StepBuf() { free(p_); }
    void clear() { n_ = 0; }
    bool reserve(size_t c) {   // keeps the contents
        if (c <= cap_) return true;
        gx_step* q = (gx_step*)malloc(c * sizeof(gx_step));
        if (!q) return false;
        if (n_) memcpy(q, p_, n_ * sizeof(gx_step));
        free(p_);
        p_ = q; cap_ = c;
        return true;
    }
    [[nodiscard]] bool push_back(const gx_step& st) {   // false: out of host memory (nothing appended)
        if (n_ == cap_ && !reserve(std::max<size_t>(16, 2 * cap_))) return false;
        p_[n_++] = st;
        return true;
    }
    size_t size() const { return n_; }
    size_t capacity() const { return cap_; }
    gx_step* data() { return p_; }
    const gx_step* data() const { return p_; }
    void set_size(size_t n) { n_ = n; }   // (<= capacity; the steps written through data())
private:
    gx_step* p_ = nullptr;
    size_t n_ = 0, cap_ = 0;
};

// Interior walk + labelling + boundary continuation (algo.rs:306-422).
struct Walk {
    StepBuf steps;
    gx_result res{};
};

// Device walk for a set of jobs: the per-strip row records in pinned host
// memory (RecordsSrc replays one job's records as moves).
struct TbOut {
    std::vector<int> end_i, end_j;
    std::vector<size_t> so;            // job -> its first strip in sg / hr
    int srows = kStripRows;            // rows per strip of the fill layout
    const int* c = nullptr;            // [4 * jobs] end i, end j, first strip
    const int* sg = nullptr;           // [4 * strips] entry i, entry j, records, active
    const uint32_t* hr = nullptr;      // [strips * kStripRows] records
    double ms = 0;
};

// Page-locked host buffer, grown on demand (device-to-host copies DMA
// straight into it).
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
};

// Persistent host workers for the labelling of a batch's walks (spawning
// threads per call cost ~0.5 ms per batch): items are taken from an atomic
// counter by the workers and the calling thread.
struct WorkPool {
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv, done_cv;
    const std::function<void(size_t)>* fn = nullptr;
    std::atomic<size_t> next{0};
    size_t total = 0, busy = 0;
    uint64_t gen = 0;
    bool stop = false;

    void worker() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
            }
            drain();
            std::lock_guard<std::mutex> lk(m);
            if (--busy == 0) done_cv.notify_all();
        }
    }
    void drain() {
        for (size_t i; (i = next.fetch_add(1)) < total;) (*fn)(i);
    }
    // f(i) for i in [0, n) on up to `workers` pool threads plus the caller
    void run(size_t n, size_t workers, const std::function<void(size_t)>& f) {
        while (th.size() < workers) th.emplace_back([this] { worker(); });
        {
            std::lock_guard<std::mutex> lk(m);
            fn = &f;
            total = n;
            next = 0;
            busy = th.size();
            ++gen;
        }
        cv.notify_all();
        drain();
        std::unique_lock<std::mutex> lk(m);
        done_cv.wait(lk, [&] { return busy == 0; });
    }
    ~WorkPool() {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        cv.notify_all();
        // a context destroyed during interpreter teardown may find its workers
        // already gone: never let a failed join terminate the process
        for (auto& t : th) {
            try {
                if (t.joinable()) t.join();
            } catch (...) {
                if (t.joinable()) t.detach();
            }
        }
    }
};

struct HostScores {
    int64_t sm, smm, g, h;
    int64_t neg_inf;  // i64::MIN + |g + h|   (algo.rs:166)
};

struct gx_context {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t cstream = nullptr;   // pipelined path: traceback record copies (D2H) off the fill stream
    hipStream_t stream2 = nullptr;   // overlapped batches (batch_core_overlap): the second group's fills
    hipStream_t tstream = nullptr;   // ... and the walks
    // the three-slot pipeline with the walk on its own stream (which holds a
    // pass's buffers until it is collected): a fill's reductions -- strip
    // results, a tracked fill's max column and matches_at_max, a parity
    // pass's checksums -- run on pstream beside the next pass's fill
    hipStream_t pstream = nullptr;
    bool post_aside = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    std::mutex mu;
    std::vector<DevBuf> free_list;
    // staged pairs (bench path)
    std::vector<std::vector<uint8_t>> st_s1, st_s2;
    DevBuf st_chars;
    std::vector<size_t> st_off1, st_off2;
    SmallAlpha st_alpha;
    // host buffers reused across calls (no fresh, page-faulting allocations per batch)
    std::vector<Walk> walk_cache;
    TbOut tb_cache;
    PinnedBuf tb_pin;
    PinnedBuf io_pin;   // staging for the small per-launch descriptors and results (a pageable
                        // copy goes through the runtime's staging and now and then stalls ms)
    WorkPool workers;   // labelling threads (created on first use)
    // pipelined multi-step batches (gx_run_staged_steps): two slots, so batch
    // k's host labelling overlaps batch k+1's fill on the device
    struct Slot {
        PinnedBuf fpin, tjpin, tbpin;        // fill descriptors/results, traceback jobs, traceback records
        hipEvent_t fb = nullptr, fe = nullptr, tb = nullptr, te = nullptr, fdone = nullptr, tdone = nullptr;
        hipEvent_t fres = nullptr;           // the fill's results copied (copy stream)
        DevBuf held_pres;                    // the fill's results block, read by that copy (until fill_collect)
        TbOut out;
        DevBuf held[4];                      // traceback buffers the copy stream still reads (until tb_collect)
        // the walk's job table of this slot's last pass, kept on the device:
        // a staged run's passes repeat it, so later passes skip its upload
        // (a 120 KB copy cost ~130 us on the fill stream, 1024 x 1k)
        void* tjob = nullptr;
        size_t tjob_cap = 0;
        std::vector<TbDev> tjob_last;
        void* fdesc = nullptr;               // ... and the fill's descriptor block (run_fill)
        size_t fdesc_cap = 0;
        std::vector<char> fdesc_last;
    } slots[4];   // 0, 1: pipelined steps by parity (overlapped batches: group A's fills and the walks); 2, 3: group B's fills
    int last_lay = 0, last_W = 0, last_pbytes = 0;   // the last fill launch (gx_fill_info)
    int last_pbits = 0;                              // ... its plane bits per cell (gx_fill_plane_bits)
    int last_chunks = 1;                             // chunks of the last staged / batch call
    int last_twin = 0;                               // the last fill was the twin (packed 16-bit) fill
    int last_groups = 1;                             // fill launches per pass of the last staged / batch call
    // GX_STAGED_PLANE_SUMS: plane checksums of every pass of a staged run
    DevBuf sums_dev;
    unsigned long long* sums_dst = nullptr;          // where the next fill's checksums go (nullptr: off)
    std::vector<uint64_t> sums_host;                 // [passes][staged pairs][3] of the last run
    // every pass's results of a staged run (gx_staged_pass_results): label_batch
    // appends one pass of the current chunk (pairs pass_off ..) when pass_rec
    bool pass_rec = false;
    size_t pass_off = 0, pass_P = 0;
    int pass_k = 0;
    std::vector<gx_result> pass_res;                 // [passes][staged pairs]
    // GX_STAGED_KEEP_PLANES: the last pass's fill of a staged run, kept
    // (device buffers included) for the tables gx_staged_table hands out.
    // keep_capture: set while that pass runs; the pipelines then hold its
    // job back from the pool and keep_job() takes it.
    std::shared_ptr<struct KeptFill> kept;
    bool keep_capture = false;
    HostScores kept_hs{};
    Scores32 kept_sc{};
};

struct PairHost {
    const uint8_t* s1;   // original bytes (traceback labels, sequence.rs:113 with rev=false)
    const uint8_t* s2;
    size_t n, m;
};

struct FillJob {
    // device buffers (owned by the job until released)
    DevBuf chars, planes, codes, skel, feed, progress, sres, pres, pairs, counter, ccodes;
    DevBuf lcs;                    // layout-3 tracked fills: LCS masks, hand-offs and bit rows (gx_lcs.h)
    bool lcs_rows = false;         // max_matches lives in PairDev.lbits (not in an LCS plane)
    size_t ltrace_off = 0, ltrace_bytes = 0;   // (GX_LCS_TRACE diagnostics: the stamps' place in `lcs`)
    bool pairs_borrowed = false;   // pairs is a pipeline slot's cached descriptor block (not pooled)
    bool pres_held = false;        // pres is held by its pipeline slot until fill_collect
    std::vector<PairDev> pd;
    std::vector<PairRes> res;
    int W = 4;
    int lay = 0;   // 0: anti-diagonal 128-row strips, 1: column-step 64-row strips, 3: skewed 64-row strips (gx_internal.h)
    int slot = -1;                      // pipelined path: the context slot whose pinned staging / events it uses
    PairRes* pin_res = nullptr;         // results in pinned staging (collected by fill_collect)
    int* pin_status = nullptr;
    int total_bands = 0, total_strips = 0;
    bool planes_on = false, lcs_on = false, track_on = false;
    bool d8 = false;                    // compact byte planes (d8_planes_ok)
    bool shift = false;                 // values kept as V - (i + j) g (Scores32.shift)
    bool twin = false;                  // the twin fill (gx_fill_pk.hip): twin_table's pairs share every band
    bool w16 = false;                   // twin plane codes, 2 B per cell (w16_ok; batches only)
    bool nocodes = false;               // w16 without code words: the traceback derives them from the planes
    bool noskel = false;                // nocodes without landing columns: the traceback walks the strips in sequence
    bool local_on = false;              // local (Smith-Waterman) fill: the start cell is the last max (PairRes.lmax_*)
    hipStream_t stream = nullptr;       // the stream its fill runs on (nullptr: the context's)
    bool plan_only = false;             // run_fill: decide layout and formats only (no buffers, no launch)
    bool table = false;                 // an alignment table (exportable planes: never the twin codes)
    int g = 0;
    double fill_ms = 0.0;
    // the int64 fill (gx_wide.hip): its own buffers and results
    bool wide = false;
    DevBuf wrows, wdesc, wres_d;
    std::vector<WideDev> wd;
    std::vector<WideRes> wres;
};

// A staged run's last fill, kept for gx_staged_table (its buffers go back to
// the pool when the run is replaced and the last table of it is freed; the
// owner holds ctx->mu then).
struct KeptFill {
    gx_context* ctx = nullptr;
    FillJob job;
    std::vector<int> dev_of;   // staged pair -> its index in job.pd (-1: no interior, not filled)
    ~KeptFill();   // (its buffers back to the pool: gx_api_fill.cpp)
};

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------
// tables

struct gx_table {
    gx_context* ctx = nullptr;
    FillJob job;
    std::vector<uint8_t> s1, s2;      // original bytes (retrace labels)
    std::vector<uint8_t> c1, c2;      // processed chars (export of *_matches)
    HostScores hs;
    Scores32 sc;
    int is_local = 0;
    uint32_t flags = 0;
    std::shared_ptr<KeptFill> share;   // gx_staged_table: the staged run's kept fill whose planes this table views
};

// What the start cell search needs from a fill's results (int32 or int64 fill).
struct StartIn {
    int64_t end_SM, lmax_val;
    uint64_t lmax_i, lmax_j;
};

static bool tb_match(const uint8_t* s1, size_t n, const uint8_t* s2, size_t m, uint64_t i, uint64_t j) {
    // is_match(i, j, false) with unshifted indices: nth() past the end is None
    const int a = i < n ? (int)s1[i] : 0x1FF;
    const int b = j < m ? (int)s2[j] : 0x1FF;
    return a == b;
}

struct TbStart {
    int i, j;   // interior start cell, or 0 = nothing to walk
    int E;      // its landing column (PairRes.end_E / lmax_E)
};

// Move source over a plain move array.
struct MovesSrc {
    const uint8_t* mv;
    size_t n;
    template <class E> void operator()(E&& emit) const {
        for (size_t k = 0; k < n; ++k) if (!emit(mv[k])) return;
    }
};

// Move source over job p's strip row records (run of inserts, then the
// row's sub / delete move), from the start strip upwards.
struct RecordsSrc {
    const TbOut* tb;
    size_t p;
    template <class E> void operator()(E&& emit) const {
        for (int s = tb->c[4 * p + 2]; s >= 0; --s) {
            const int* g = &tb->sg[4 * (tb->so[p] + s)];
            if (!g[3]) return;
            const uint32_t* r = &tb->hr[(tb->so[p] + s) * tb->srows];
            for (int k = 0; k < g[2]; ++k) {
                for (uint32_t q = r[k] >> 2; q > 0; --q) if (!emit((uint8_t)1)) return;
                if ((r[k] & 3u) != 1u && !emit((uint8_t)(r[k] & 3u))) return;
            }
        }
    }
};

// A staged run over two alternating pair sets (GX_STAGED_ALTERNATE): pass k
// processes set k % 2.  The sets hold pairs of the same shapes (so every
// buffer, plan and launch is the same for both); `alt` describes set 1, the
// regular arguments set 0.  Each set's walks and per-pass results (pass_off
// into ctx->pass_res) are its own.
struct PassSet {
    const std::vector<PairHost>* ph;
    const std::vector<std::pair<const uint8_t*, const uint8_t*>>* proc;
    const std::vector<size_t>* off1;
    const std::vector<size_t>* off2;
    std::vector<Walk>* walks;
    size_t pass_off;
};

// ---------------------------------------------------------------------------
// functions shared across the gx_api_*.cpp files

// contexts: errors, pinned staging, the device buffer pool, pipeline slots (gx_api_context.cpp)
int fail(int code, const std::string& msg);
bool log_info();
void* pinned_grow(PinnedBuf& b, size_t bytes);
int slots_ready(gx_context* ctx);
void* io_pinned(gx_context* ctx, size_t bytes);
int pool_get(gx_context* ctx, size_t bytes, DevBuf* out, hipStream_t st = nullptr);
void pool_put(gx_context* ctx, DevBuf& b);
void release_held(gx_context* ctx, int slot);
void release_slots(gx_context* ctx);

// launch planning: exact-int32 range guard, boundary cells, layout / band width / plane format, twin pairing, chunks (gx_api_plan.cpp)
int check_scores(const gx_scores* s, size_t n, size_t m, HostScores* hs, Scores32* sc, int is_local,
                 bool* wide = nullptr);
void boundary_cell(const HostScores& hs, uint64_t i, uint64_t j, int64_t* I, int64_t* D, int64_t* S);
int64_t smax(int64_t I, int64_t S, int64_t D, int local);
int processed_chars(const uint8_t* s1, size_t n, const uint8_t* s2, size_t m, int rev,
                    std::vector<uint8_t>& c1, std::vector<uint8_t>& c2);
int fill_grid_cap(int device);
int fill_band_waves(bool track, int total_strips, int grid_cap, int lay, int min_strips);
bool d8_planes_ok(const Scores32& sc, int is_local);
bool w16_ok(const Scores32& sc);
bool cs2_enabled(int is_local, const Scores32& sc);
int skew_band_waves();
int cs2_band_waves(int total_strips, int grid_cap);
bool skew_ok(const Scores32& sc, bool lcs_plane, size_t mmax);
int fill_layout(const std::vector<PairHost>& ph, const Scores32& sc, int grid_cap, bool track, bool lcs_plane);
long long twin_bound(const Scores32& sc, int W, long long dm, bool local = false);
long long twin_gap_cap(const Scores32& sc, int W, bool local = false);
std::vector<std::pair<int, int>> twin_table(const std::vector<PairHost>& ph, long long gap_cap = 1024);
int twin_width(const std::vector<PairHost>& ph, const std::vector<std::pair<int, int>>& tw, const Scores32& sc,
               int is_local, bool track, bool lcs, int lay, bool planes, bool d8, int W_want,
               bool long_ok = false);
double pair_device_bytes(size_t n, size_t m, double plane_bpc);   // one pair's device bytes in a batch
double chunk_budget(gx_context* ctx);                             // device bytes one chunk may use
std::vector<std::pair<size_t, size_t>> plan_chunks(gx_context* ctx, const std::vector<PairHost>& ph,
                                                   double plane_bpc);

// fill launches and their results (gx_api_fill.cpp)
void unshift_results(FillJob& j);
void job_release(gx_context* ctx, FillJob& j);
void release_or_hold(gx_context* ctx, FillJob& j, bool last_pass, bool* held);
void keep_job(gx_context* ctx, FillJob& j, const std::vector<int>& dev_of);
int run_fill(gx_context* ctx, const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc,
             const std::vector<PairHost>& ph, const Scores32& sc, int is_local, bool planes, bool track,
             bool lcs, FillJob& job, const uint8_t* chars_dev = nullptr,
             const std::vector<size_t>* off1 = nullptr, const std::vector<size_t>* off2 = nullptr,
             const SmallAlpha* alpha = nullptr, int slot = -1, bool collect = true);
int fill_collect(gx_context* ctx, FillJob& job);
int run_fill_wide(gx_context* ctx, const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc,
                  const std::vector<PairHost>& ph, const HostScores& hs, int is_local, bool planes, bool track,
                  bool lcs, FillJob& job);
hipError_t enqueue_plane_sums(gx_context* ctx, const FillJob& job, const Scores32& sc,
                              unsigned long long* out, hipStream_t st = nullptr);

// traceback: device walk, start cells, labelling (gx_api_walk.cpp)
StartIn start_in(const FillJob& job, size_t p);
StartIn start_in(const PairRes& r);
int label_boundary(const HostScores& hs, int is_local, const uint8_t* s1, size_t n, const uint8_t* s2,
                   size_t m, uint64_t i, uint64_t j, int last, Walk& w);
int label_walk_records(const HostScores& hs, int is_local, const uint8_t* s1, size_t n, const uint8_t* s2,
                       size_t m, uint64_t si, uint64_t sj, const TbOut& tb, size_t p, Walk& w);
int run_traceback(gx_context* ctx, const std::vector<const FillJob*>& jv, const std::vector<TbStart>& starts,
                  TbOut& out, int slot, bool collect, bool dev_end_E, hipStream_t ts);
int run_traceback(gx_context* ctx, const FillJob& job, const std::vector<TbStart>& starts, TbOut& out,
                  int slot = -1, bool collect = true, bool dev_end_E = false);
int tb_collect(gx_context* ctx, int slot, size_t P, TbOut& out);
int start_cell_common(const HostScores& hs, int is_local, size_t n, size_t m, const StartIn& r,
                      uint64_t* si, uint64_t* sj, int64_t* score);
int copy_steps(const Walk& w, gx_step* steps, size_t cap);
int label_batch(gx_context* ctx, const std::vector<PairHost>& ph, const HostScores& hs, int is_local, bool track,
                const std::vector<int>& dev_of, const std::vector<uint64_t>& si,
                const std::vector<uint64_t>& sj, const std::vector<int64_t>& score,
                const std::vector<PairRes>& res, const TbOut& tb, double fill_ms, std::vector<Walk>& walks);

// batches of independent pairs (gx_api_batch.cpp)
int batch_core_wide(gx_context* ctx, const std::vector<PairHost>& ph,
                    const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc, const HostScores& hs,
                    int is_local, bool planes, bool track, std::vector<Walk>& walks, double* fill_ms);
int batch_core_steps(gx_context* ctx, const std::vector<PairHost>& ph,
                     const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc, const HostScores& hs,
                     const Scores32& sc, int is_local, bool planes, bool track, int nsteps,
                     std::vector<Walk>& walks, double* fill_ms, const uint8_t* chars_dev,
                     const std::vector<size_t>* off1, const std::vector<size_t>* off2,
                     const SmallAlpha* staged_alpha, const PassSet* alt = nullptr);

// Labels the walk (algo.rs:339-422).  The interior moves come from `src`,
// which calls emit(code) per move (0 sub, 1 insert, 2 delete) while emit
// returns true; the boundary part follows the reference loop.
template <class Src>
static int label_walk(const HostScores& hs, int is_local, const uint8_t* s1, size_t n, const uint8_t* s2, size_t m,
                      uint64_t si, uint64_t sj, size_t nmoves_hint, Src&& src, Walk& w) {
    uint64_t i = si, j = sj;
    int last = GX_MATCH;
    gx_result& r = w.res;
    uint64_t nmat = 0, nmis = 0, next = 0, nopen = 0;
    w.steps.clear();
    if (!w.steps.reserve(nmoves_hint + (size_t)si + (size_t)sj + 2)) return fail(GX_ENOMEM, "step buffer");
    bool done = false, oom = false;
    // interior part, decided on the device
    src([&](uint8_t c) -> bool {
        gx_step st{};
        st.i = i; st.j = j;
        if (c == 0) {
            const bool mt = tb_match(s1, n, s2, m, i, j);
            st.choice = mt ? GX_MATCH : GX_MISMATCH;
            nmat += mt; nmis += !mt;
            last = st.choice;
            --i; --j;
        } else if (c == 1) {
            const bool ext = last == GX_INSERT;
            st.choice = ext ? GX_INSERT : GX_OPEN_INSERT;
            next += ext; nopen += !ext;
            last = GX_INSERT;
            --j;
        } else {
            const bool ext = last == GX_DELETE;
            st.choice = ext ? GX_DELETE : GX_OPEN_DELETE;
            next += ext; nopen += !ext;
            last = GX_DELETE;
            --i;
        }
        if (!w.steps.push_back(st)) { oom = true; return false; }
        if (i == 0 && j == 0) { done = true; return false; }
        return true;
    });
    if (oom) return fail(GX_ENOMEM, "step buffer");
    r.matches = nmat; r.mismatches = nmis; r.gap_extensions = next; r.opening_gaps = nopen;
    if (!done) {
        const int rc = label_boundary(hs, is_local, s1, n, s2, m, i, j, last, w);
        if (rc) return rc;
    }
    r.n_steps = w.steps.size();
    return GX_OK;
}

#pragma GCC visibility pop
