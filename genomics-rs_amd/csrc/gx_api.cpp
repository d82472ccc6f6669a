// gx_api.cpp -- host side of the C ABI (include/gx.h).
//
// Mirrors the reference's alignment API (nlaha/genomics-rs):
//   alignment_table  src/alignment/algo.rs:151-282  -> gx_alignment_table
//   retrace          src/alignment/algo.rs:287-441  -> gx_retrace
// The DP fill and the interior traceback walk run on the GPU
// (gx_kernels.hip); this file owns device memory, the exact-int32 range
// guard, the boundary cells (analytic, int64, algo.rs:193-220), the local
// start search over boundary cells, and the labelling of the walk into
// AlignmentChoice values (algo.rs:351-400).
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
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
                            hipStream_t st);
hipError_t launch_skew_codes(const PairDev* d_pairs, int npairs, int mmax, Scores32 sc, bool tbl, hipStream_t st);
hipError_t launch_fill_pk(int W, int planes, const PairDev* d_pairs, int npairs, int ntwins, int total_bands,
                          int* d_counter, PairRes* d_pres, StripRes* d_sres, Scores32 sc, int grid, hipStream_t st);
hipError_t launch_fill_wide(const WideDev* d_pairs, int npairs, WideScores sc, WideRes* d_res, int local, int track,
                            hipStream_t st);
hipError_t launch_wide_plane_sums(const int64_t* pI, const int64_t* pD, const int64_t* pS, int n, int m,
                                  unsigned long long* out, hipStream_t st);
}  // namespace gx

using namespace gx;

// ---------------------------------------------------------------------------
// errors

static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(e_ == hipErrorOutOfMemory ? GX_ENOMEM : GX_EHIP,                       \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                   \
    } while (0)

int gx_internal_fail(int code, const std::string& msg) { return fail(code, msg); }

extern "C" const char* gx_last_error(void) { return g_err.c_str(); }
extern "C" const char* gx_version(void) { return "genomics-rs_amd 0.1 (gfx950)"; }

static bool log_info() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("GX_LOG");
        v = (e && (!strcmp(e, "info") || !strcmp(e, "debug"))) ? 1 : 0;
    }
    return v == 1;
}

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

static void* pinned_grow(PinnedBuf& b, size_t bytes) {
    if (b.cap < bytes) {
        if (b.p) (void)hipHostFree(b.p);
        b = PinnedBuf{};
        const size_t cap = std::max<size_t>(bytes, 1 << 16);
        if (hipHostMalloc(&b.p, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
        b.cap = cap;
    }
    return b.p;
}

static int slots_ready(gx_context* ctx) {
    for (auto& s : ctx->slots) {
        hipEvent_t* evs[] = {&s.fb, &s.fe, &s.tb, &s.te, &s.fdone, &s.tdone, &s.fres};
        for (hipEvent_t* e : evs)
            if (!*e && hipEventCreate(e) != hipSuccess) return GX_EHIP;
    }
    return GX_OK;
}

// ctx->io_pin grown to `bytes` (contents not kept); nullptr on failure.
static void* io_pinned(gx_context* ctx, size_t bytes) {
    if (ctx->io_pin.cap < bytes) {
        if (ctx->io_pin.p) (void)hipHostFree(ctx->io_pin.p);
        ctx->io_pin = PinnedBuf{};
        const size_t cap = std::max<size_t>(bytes, 1 << 16);
        if (hipHostMalloc(&ctx->io_pin.p, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
        ctx->io_pin.cap = cap;
    }
    return ctx->io_pin.p;
}

static bool pool_poison();
static int pool_take(gx_context* ctx, size_t bytes, DevBuf* out);
// `st`: the stream its new user runs on (GX_POOL_POISON fills the buffer there,
// ahead of that user's work).
static int pool_get(gx_context* ctx, size_t bytes, DevBuf* out, hipStream_t st = nullptr) {
    const int rc = pool_take(ctx, bytes, out);
    if (rc == GX_OK && pool_poison()) (void)hipMemsetAsync(out->p, 0xA5, out->cap, st ? st : ctx->stream);
    return rc;
}
static int pool_take(gx_context* ctx, size_t bytes, DevBuf* out) {
    bytes = std::max<size_t>(bytes, 256);
    size_t best = (size_t)-1;
    int bi = -1;
    for (size_t k = 0; k < ctx->free_list.size(); ++k) {
        const DevBuf& b = ctx->free_list[k];
        if (b.cap >= bytes && b.cap < best) { best = b.cap; bi = (int)k; }
    }
    // a large request does not take a cached buffer more than twice its size
    // (that buffer may fit a later, larger request of the same launch)
    if (bi >= 0 && bytes >= ((size_t)1 << 30) && best > 2 * bytes) bi = -1;
    if (bi >= 0) {
        *out = ctx->free_list[bi];
        ctx->free_list.erase(ctx->free_list.begin() + bi);
        return GX_OK;
    }
    void* p = nullptr;
    if (const char* lg = getenv("GX_LOG"); lg && !strcmp(lg, "debug"))
        fprintf(stderr, "[gx DEBUG] pool miss: hipMalloc %zu B (%zu cached)\n", bytes, ctx->free_list.size());
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
        // drop cached buffers and retry once (after the device has drained:
        // an overlapped batch returns a buffer to the pool while the walk
        // enqueued before it may still read it)
        (void)hipGetLastError();
        (void)hipDeviceSynchronize();
        for (auto& b : ctx->free_list) (void)hipFree(b.p);
        ctx->free_list.clear();
        e = hipMalloc(&p, bytes);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return fail(GX_ENOMEM, "hipMalloc(" + std::to_string(bytes) + " B) failed");
        }
    }
    out->p = p;
    out->cap = bytes;
    return GX_OK;
}
// GX_POOL_POISON=1 (debug): every buffer the pool hands out is filled with
// 0xA5 bytes on the stream of its new user, before that user's work.  A user
// that reads what it did not write (pool reuse bugs) sees garbage instead of
// the previous pass's identical data, and a buffer handed to a stream that is
// not ordered behind the buffer's previous readers (stream-order bugs, e.g. an
// overlapped pipeline's next fill and the walk still reading its planes) has
// those readers read garbage.  Poisoning at release instead would have to run
// on the last reader's stream and order every later user behind it.
static bool pool_poison() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("GX_POOL_POISON");
        v = (e && *e && strcmp(e, "0")) ? 1 : 0;
    }
    return v == 1;
}
static void pool_put(gx_context* ctx, DevBuf& b) {
    if (b.p) ctx->free_list.push_back(b);
    b = DevBuf{};
}

extern "C" int gx_context_create(int device, gx_context** out) {
    if (!out) return fail(GX_EINVAL, "out is NULL");
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(GX_EINVAL, "no HIP device " + std::to_string(device));
    HIPCHK(hipSetDevice(device));
    gx_context* c = new gx_context();
    c->device = device;
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&c->ev0));
    HIPCHK(hipEventCreate(&c->ev1));
    HIPCHK(hipEventCreate(&c->ev2));
    // Exercise the copy paths once (device->pinned host of a few MB, host->
    // device, memset): the runtime sets some of them up on first use, which
    // otherwise stalled one later batch's traceback copies by ~8 ms.
    {
        const size_t wb = 16u << 20;
        void* d = nullptr;
        if (hipMalloc(&d, wb) == hipSuccess) {
            if (void* h = io_pinned(c, wb)) {
                (void)hipMemsetAsync(d, 0, wb, c->stream);
                (void)hipMemcpyAsync(h, d, wb, hipMemcpyDeviceToHost, c->stream);
                (void)hipMemcpyAsync(d, h, 4096, hipMemcpyHostToDevice, c->stream);
                (void)hipMemcpyAsync(h, d, 4096, hipMemcpyDeviceToHost, c->stream);
                (void)hipStreamSynchronize(c->stream);
            }
            (void)hipFree(d);
        }
    }
    *out = c;
    return GX_OK;
}

extern "C" int gx_context_trim(gx_context* ctx) {
    if (!ctx) return fail(GX_EINVAL, "ctx is NULL");
    std::lock_guard<std::mutex> lk(ctx->mu);
    (void)hipSetDevice(ctx->device);
    for (auto& b : ctx->free_list) (void)hipFree(b.p);
    ctx->free_list.clear();
    return GX_OK;
}

static void release_slots(gx_context* ctx);
extern "C" void gx_context_destroy(gx_context* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    release_slots(ctx);   // (into the pool, which the trim frees)
    ctx->kept.reset();
    gx_context_trim(ctx);
    (void)hipSetDevice(ctx->device);
    if (ctx->st_chars.p) (void)hipFree(ctx->st_chars.p);
    if (ctx->sums_dev.p) (void)hipFree(ctx->sums_dev.p);
    if (ctx->tb_pin.p) (void)hipHostFree(ctx->tb_pin.p);
    if (ctx->io_pin.p) (void)hipHostFree(ctx->io_pin.p);
    for (auto& s : ctx->slots) {
        for (PinnedBuf* b : {&s.fpin, &s.tjpin, &s.tbpin})
            if (b->p) (void)hipHostFree(b->p);
        for (hipEvent_t e : {s.fb, s.fe, s.tb, s.te, s.fdone, s.tdone, s.fres})
            if (e) (void)hipEventDestroy(e);
        if (s.tjob) (void)hipFree(s.tjob);
        if (s.fdesc) (void)hipFree(s.fdesc);
    }
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->ev2) (void)hipEventDestroy(ctx->ev2);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->cstream) (void)hipStreamDestroy(ctx->cstream);
    if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
    if (ctx->tstream) (void)hipStreamDestroy(ctx->tstream);
    delete ctx;
}

// ---------------------------------------------------------------------------
// scoring: exact-int32 guard (DESIGN.md "Integer range")


static int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static int64_t wmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }

// `wide` (may be NULL): set when the job is outside the exact-int32 range of
// the main fill and must take the int64 fill (gx_wide.hip) instead; with
// wide == NULL such a job is refused with GX_ERANGE.
static int check_scores(const gx_scores* s, size_t n, size_t m, HostScores* hs, Scores32* sc, int is_local,
                        bool* wide = nullptr) {
    if (!s) return fail(GX_EINVAL, "scores is NULL");
    hs->sm = s->s_match; hs->smm = s->s_mismatch; hs->g = s->g; hs->h = s->h;
    const uint64_t ugh = (uint64_t)s->g + (uint64_t)s->h;   // g + h as the reference's release build adds it
    const int64_t gh = (int64_t)ugh;
    hs->neg_inf = wadd(INT64_MIN, gh < 0 ? (int64_t)(0 - ugh) : gh);
    if (wide) *wide = false;
    if (n >= (size_t)1 << 30 || m >= (size_t)1 << 30) return fail(GX_ERANGE, "sequence longer than 2^30");
    const char* why = nullptr;
    const uint64_t lim = (uint64_t)1 << 24;
    auto mag = [](int64_t v) { return v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v; };
    if (mag(s->s_match) > lim || mag(s->s_mismatch) > lim || mag(s->g) > lim || mag(s->h) > lim)
        why = "score magnitudes above 2^24 are outside the exact int32 device range";
    // The reference adds g and h+g to neg_inf at the boundary; when that
    // wraps (possible only for g < 0 < h with |g+h| < |g|) its release build
    // produces wrapped giants that the int32 path cannot reproduce.
    else if (s->g < 0 && mag(gh) < mag(s->g))
        why = "g < 0 < h with |g+h| < |g|: the reference's boundary arithmetic wraps";
    else {
        // every interior magnitude <= (n + m + 2) * (|sm| + |smm| + |g| + |h|) + |h|
        const double bound = (double)(n + m + 2) * (double)(mag(s->s_match) + mag(s->s_mismatch) + mag(s->g) +
                                                            mag(s->h)) + (double)mag(s->h);
        if (bound >= (double)(1 << 28)) why = "|score| bound exceeds 2^28: outside the exact int32 device range";
        else if (n > (size_t)1 << 26 || m > (size_t)1 << 26) why = "sequence longer than 2^26";
    }
    if (why) {
        if (!wide) return fail(GX_ERANGE, why);
        *wide = true;   // the int64 fill computes it
        return GX_OK;
    }
    sc->sm = (int)s->s_match; sc->smm = (int)s->s_mismatch; sc->g = (int)s->g; sc->h = (int)s->h;
    sc->hg = (int)(s->h + s->g);
    sc->floor_ = is_local ? 0 : kNeg;
    const char* dbg = getenv("GX_DEBUG_FLAGS");
    sc->dbg = dbg ? atoi(dbg) : 0;
    sc->shift = 0;
    for (int k = 0; k < 4; ++k) sc->sym[k] = -1;
    sc->koff = 0;
    return GX_OK;
}

// Boundary cell of the table (algo.rs:195-220), int64.
static void boundary_cell(const HostScores& hs, uint64_t i, uint64_t j, int64_t* I, int64_t* D, int64_t* S) {
    if (i == 0 && j == 0) { *I = 0; *D = 0; *S = 0; }
    else if (j == 0) { *I = hs.neg_inf; *D = wadd(hs.h, wmul((int64_t)i, hs.g)); *S = hs.neg_inf; }
    else { *I = wadd(hs.h, wmul((int64_t)j, hs.g)); *D = hs.neg_inf; *S = hs.neg_inf; }
}
// score_max(cell, 0, 0, 0, is_local) (algo.rs:98-107)
static int64_t smax(int64_t I, int64_t S, int64_t D, int local) {
    int64_t r = std::max(std::max(I, S), D);
    return std::max(r, local ? (int64_t)0 : INT64_MIN);
}

// Processed characters for is_match(i-1, j-1, rev) (sequence.rs:102-115).
// Without `rev` they are the bytes themselves.  With `rev`, index k of s1
// reads s1[m - k] and index k of s2 reads s2[n - k]; an index out of range
// (including a wrapped usize) is None, encoded 0xFF on both sides so that
// None == None matches.  Inputs containing 0xFF are rejected in rev mode.
static int processed_chars(const uint8_t* s1, size_t n, const uint8_t* s2, size_t m, int rev,
                           std::vector<uint8_t>& c1, std::vector<uint8_t>& c2) {
    c1.assign(s1, s1 + n);
    c2.assign(s2, s2 + m);
    if (!rev) return GX_OK;
    for (size_t k = 0; k < n; ++k) if (s1[k] == 0xFF) return fail(GX_EINVAL, "byte 0xFF is reserved in reverse mode");
    for (size_t k = 0; k < m; ++k) if (s2[k] == 0xFF) return fail(GX_EINVAL, "byte 0xFF is reserved in reverse mode");
    for (size_t k = 0; k < n; ++k) {
        // i_processed = len(s2) - k
        c1[k] = (k <= m && (m - k) < n) ? s1[m - k] : 0xFF;
    }
    for (size_t k = 0; k < m; ++k) {
        // j_processed = len(s1) - k
        c2[k] = (k <= n && (n - k) < m) ? s2[n - k] : 0xFF;
    }
    return GX_OK;
}

// ---------------------------------------------------------------------------
// fill orchestration

// Persistent fill workgroups: one per CU by default (bands beyond the grid
// are taken from the queue as earlier bands finish; a band deep in a pair
// starts late anyway, so it loses little, and no CU runs two bands' waves).
static int fill_grid_cap(int device) {
    if (const char* e = getenv("GX_FILL_GRID"); e && atoi(e) > 0) return atoi(e);
    static int cus = -1;
    if (cus < 0) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c < 1) c = 256;
        cus = c;
    }
    return cus;
}

// Band width: the narrowest instantiated width whose bands fit the grid
// (one band per workgroup, all strips in flight from the start) up to 8
// strips; beyond that 8-strip bands that queue for workgroups.  Measured on
// queued batches (profiles/r01i_widths.txt): 8 beats 11 and 15 everywhere
// (45 Covid pairs 845 -> 969 GCUPS, 20 x 30k 433 -> 496, 64 x 16k 485 -> 524)
// and ties 15 where 15 fits (16 x 30k).  GX_BAND_WAVES forces a width (if
// instantiated for the variant).
template <size_t N>
static int pick_width(const int (&ws)[N], int total_strips, int grid_cap) {
    if (const char* e = getenv("GX_BAND_WAVES")) {
        const int w = atoi(e);
        for (int x : ws) if (x == w) return w;
    }
    int queued = ws[0];
    for (int x : ws) {
        if (x > 8) break;
        if (ceil_div(total_strips, x) <= grid_cap) return x;
        queued = x;
    }
    return queued;
}
// min_strips: the fewest strips of any pair in the launch.
static int fill_band_waves(bool track, int total_strips, int grid_cap, int lay, int min_strips) {
    // layout 1 starts at 4-strip bands: fewer HBM hand-offs for the same one
    // compute wave per SIMD (the I/O wave shares a SIMD but mostly sleeps)
    static constexpr int kWidths1[] = {4, 6, 8, 11, 15};
    if (track) return pick_width(kFillWidthsTrack, total_strips, grid_cap);
    if (lay) return pick_width(kWidths1, total_strips, grid_cap);
    const int w = pick_width(kFillWidths, total_strips, grid_cap);
    // Deep queues of long pairs: 15-strip bands (four compute waves per SIMD)
    // once every pair spans >= 200 strips (25.6k rows) and the queue holds
    // >= 2.5 rounds of them: 64 x 30k 50.9 -> 49.1 ms, 45 Covid pairs 32.3 ->
    // 30.5; shallower queues (16 x 30k: 15.0 vs 22.5 ms, 12 x 64k) and shorter
    // pairs (128 x 16k, 1024 x 4k) stay faster with 8 (profiles/r01o_round_sweep.txt)
    if (w == 8 && !getenv("GX_BAND_WAVES") && min_strips >= 200 && 2 * ceil_div(total_strips, 15) >= 5 * grid_cap)
        return 15;
    return w;
}

// Compact score planes (layout 0, untracked: the batch path).  The
// fill stores per cell one signed byte each of x_I = I(i,j) - I(i,j-1),
// x_S = S(i,j) - I(i,j), x_D = D(i,j) - I(i,j) (gx_kernels.hip put_byte), 3 B
// instead of 12.  With g, h <= 0, a = h + g, smax/smin the larger/smaller of
// the match and mismatch scores and U = max(0, smax - a), every interior cell
// satisfies (DESIGN.md section 4.2 has the derivation from algo.rs:231-248)
//     a <= H(i,j) - H(i,j-1) <= U   (and the same down a column),
//     H(i,j-1) + a <= I(i,j) <= H(i,j-1),   H(i-1,j) + a <= D(i,j) <= H(i-1,j),
// so  x_I in [g, U - a],  x_S in [smin - U, smax - 2a],  x_D in [2a - U, U - 2a].
// The same holds in local mode (the 0 floor of I, D and H keeps every
// inequality; the row base is H(i, 0) + h = h).  Compact planes are used when
// those ranges fit a signed byte (the default scores give [-1, 13], [-9, 13],
// [-19, 19]); GX_PLANES32 forces int32 planes.
static bool d8_planes_ok(const Scores32& sc, int is_local) {
    (void)is_local;
    if (sc.g > 0 || sc.h > 0 || getenv("GX_PLANES32")) return false;
    const long long g = sc.g, a = (long long)sc.h + sc.g;
    const long long smax = std::max(sc.sm, sc.smm), smin = std::min(sc.sm, sc.smm);
    const long long U = std::max(0LL, smax - a);
    // (the shifted fill, Scores32.shift, stores x_I - g: in [0, U - a - g])
    const long long lo = std::min({g, smin - U, 2 * a - U}), hi = std::max({U - a - g, smax - 2 * a, U - 2 * a});
    return lo >= -128 && hi <= 127;
}

// Twin plane codes (gx_fill_pk.hip w16_code): x_I - g in [0, U - a - g] must
// fit 4 unsigned bits, x_S in [smin - U, smax - 2a] 5 signed bits and x_D in
// [2a - U, U - 2a] 7 signed bits (the bounds of d8_planes_ok); the default
// scores give [0, 14], [-9, 13], [-19, 19].  GX_PLANES_W16=0 keeps the byte
// format.
static bool w16_ok(const Scores32& sc) {
    if (sc.g > 0 || sc.h > 0 || getenv("GX_PLANES32")) return false;
    if (const char* e = getenv("GX_PLANES_W16"); e && !strcmp(e, "0")) return false;
    const long long g = sc.g, a = (long long)sc.h + sc.g;
    const long long smax = std::max(sc.sm, sc.smm), smin = std::min(sc.sm, sc.smm);
    const long long U = std::max(0LL, smax - a);
    return U - a - g <= 15 && smin - U >= -16 && smax - 2 * a <= 15 && 2 * a - U >= -64 && U - 2 * a <= 63;
}

// The split column step (gx_cs2.hip) replaces layout 1's one-wave strips for
// untracked fills; GX_CS2=0 keeps the one-wave kernel.  Band width: the
// narrowest instantiated width whose bands fit the grid (W = 2: every compute
// wave of a CU on its own SIMD), else 7-strip bands queued for workgroups
// (GX_BAND_WAVES forces an instantiated width).
// The split column step (gx_cs2.hip) by default for local fills only: on a
// 30k global pair its two-wave strips in two-strip bands lose to layout 1's
// one-wave strips in four-strip bands (more band hand-offs through HBM,
// 5.33 vs 4.53 ms; BRCA2 local 1.76 vs 1.79 ms, profiles/r03a_bench.json).
// GX_CS2=1 / 0 forces it on / off.  Local fills need g <= 0: the split
// core applies the shifted 0 floor, -(i + j) g, after the delete chain's
// prefix max, which is the reference's per-row floor (algo.rs:238-243) only
// while the floor does not decrease down the rows; with g > 0 a floor reached
// at an upper row must carry down the chain, which the one-wave column step
// does (its per-lane chain offsets) and the split core does not.
static bool cs2_enabled(int is_local, const Scores32& sc) {
    if (is_local && sc.g > 0) return false;
    const char* e = getenv("GX_CS2");
    if (e && *e) return strcmp(e, "0") != 0;
    return is_local != 0;
}
// Layout 3 (gx_skew.hip): 2-strip bands, each strip's core and side wave on
// SIMDs of their own; GX_BAND_WAVES picks another instantiated width (1-3;
// must match gx_skew.hip launch_fill_skew).
static int skew_band_waves() {
    if (const char* e = getenv("GX_BAND_WAVES")) {
        const int w = atoi(e);
        if (w >= 1 && w <= 3) return w;
    }
    return 2;
}
static int cs2_band_waves(int total_strips, int grid_cap) {
    static constexpr int kCs2Widths[] = {1, 2, 3, 4, 7};
    if (const char* e = getenv("GX_BAND_WAVES")) {
        const int w = atoi(e);
        for (int x : kCs2Widths) if (x == w) return w;
    }
    for (int x : {2, 3, 4})
        if (ceil_div(total_strips, x) <= grid_cap) return x;
    return 7;
}

struct PairHost {
    const uint8_t* s1;   // original bytes (traceback labels, sequence.rs:113 with rev=false)
    const uint8_t* s2;
    size_t n, m;
};

// Fill layout (gx_internal.h): 0 = anti-diagonal 128-row strips, 1 = column
// step over 64-row strips (delete chain as a wave prefix max; a strip follows
// the one above a few columns behind instead of 64+ steps), 3 = anti-diagonal
// 64-row strips with one row per lane (gx_skew.hip, the latency fill).
// GX_LAYOUT forces one.  Layout 1 offsets the delete chain by up to 64
// (|g| + |h|) inside the scan, so it needs that much int32 headroom above the
// range guard's 2^28.
//
// Default: a latency layout while the job is latency-bound -- its 64-row
// strips fit about two per SIMD (one to three 30k pairs); layout 0 from four
// 30k pairs on, where the band-major queue keeps every CU busy and layout 0's
// 2-row lanes issue fewer instructions per cell (four 30k pairs 7.7 vs 8.4
// ms, eight 10.6 vs 15.9 ms; profiles/r01o_round_sweep.txt,
// profiles/r01d_layouts.txt).  The latency layout is 3 for untracked fills
// with h <= 0 (its recurrences fold the gap opening onto score_max, which is
// exact only then) when it is predicted faster than the column step, else
// the column step (below: a fitted cost model per layout).
// Covid 29,903 x 29,882 global: layout 3 (4.52 vs 4.62 ms); BRCA2 11,382 x
// 10,346 local: the split column step (1.74 vs 1.79); 64 x 30,000: layout 3
// (1.5 vs 3.4).
// Layout 3 needs h <= 0 (the folded gap opening), small penalties for the
// virtual columns of its global ramp-up (values drift from -2^30 by up to 64
// steps of |g| + |h| + |s''|, s'' = s - 2g the shifted substitution score),
// and fewer than 2^24 - 128 columns: its skeleton holds E + 64 in the 24 bits
// tb_chase_kernel decodes, and a strip's int32 plane (256 (m + 64) bytes)
// must stay inside one buffer descriptor's 32-bit range.
// Tracked fills (max_cell, matches_at_max) run on it too (round 5: the side
// wave carries the first maximum and the LCS values); an LCS plane does not.
static bool skew_ok(const Scores32& sc, bool lcs_plane, size_t mmax) {
    const long long g = sc.g;
    const long long s2 = std::max(std::llabs((long long)sc.sm - 2 * g), std::llabs((long long)sc.smm - 2 * g));
    const long long drift = 64LL * (std::llabs(g) + std::llabs((long long)sc.h) + s2);
    return !lcs_plane && sc.h <= 0 && drift < (1LL << 28) && mmax + 128 < (1u << 24);
}
static int fill_layout(const std::vector<PairHost>& ph, const Scores32& sc, int grid_cap, bool track, bool lcs_plane) {
    const long long span = 65LL * (std::llabs((long long)sc.g) + std::llabs((long long)sc.h));
    size_t mmax = 0;
    long long strips64 = 0;
    for (const PairHost& h : ph) {
        mmax = std::max(mmax, h.m);
        strips64 += ceil_div((int)h.n, kStripRows1);
    }
    const bool cs_ok = span < (1LL << 29) && mmax + 128 < (1u << 24);   // landing keys hold E + 64 in 24 bits
    // a pair's fill time ~ m x (a strip's pace per column) + S x (a strip's
    // start lag), fitted per layout on a lone 64-row strip and on the
    // BASELINE pairs (round 4, profiles/r04_layout_fit.json): layout 3 50 ns
    // + 6.46 us global, 57.5 ns + 6.66 us local; the column step 113 ns +
    // 2.66 us (global), split for local fills 110 ns + 3.37 us
    const bool local = sc.floor_ == 0;
    (void)track;
    double est1 = 0, est3 = 0;   // the launch's slowest pair on each layout (ns)
    for (const PairHost& h : ph) {
        const double S = (double)ceil_div((int)h.n, kStripRows1), m = (double)h.m;
        est1 = std::max(est1, local ? m * 110.0 + S * 3370.0 : m * 113.0 + S * 2660.0);
        est3 = std::max(est3, local ? m * 57.5 + S * 6660.0 : m * 50.0 + S * 6460.0);
    }
    const bool sk_ok = skew_ok(sc, lcs_plane, mmax);
    const int lat = sk_ok && (!cs_ok || est3 < est1) ? 3 : cs_ok ? 1 : 0;
    if (const char* e = getenv("GX_LAYOUT"); e && *e) {
        const int want = atoi(e);
        if (want == 3) return sk_ok ? 3 : cs_ok ? 1 : 0;
        return (want == 1 && cs_ok) ? 1 : 0;
    }
    return strips64 <= 6LL * grid_cap ? lat : 0;
}

struct FillJob {
    // device buffers (owned by the job until released)
    DevBuf chars, planes, codes, skel, feed, progress, sres, pres, pairs, counter, ccodes;
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

// Shifted fills (Scores32.shift) report score_max(n, m) as H - (n + m) g.
static void unshift_results(FillJob& j) {
    if (!j.shift) return;
    for (size_t p = 0; p < j.res.size() && p < j.pd.size(); ++p)
        if (j.pd[p].n >= 1 && j.pd[p].m >= 1) j.res[p].end_SM += (j.pd[p].n + j.pd[p].m) * j.g;
}

static void job_release(gx_context* ctx, FillJob& j) {
    if (j.pairs_borrowed) { j.pairs = DevBuf{}; j.pairs_borrowed = false; }
    if (j.pres_held) { j.pres = DevBuf{}; j.pres_held = false; }
    pool_put(ctx, j.chars); pool_put(ctx, j.planes); pool_put(ctx, j.codes); pool_put(ctx, j.feed);
    pool_put(ctx, j.progress); pool_put(ctx, j.sres); pool_put(ctx, j.pres); pool_put(ctx, j.pairs);
    pool_put(ctx, j.counter); pool_put(ctx, j.skel); pool_put(ctx, j.ccodes);
    pool_put(ctx, j.wrows); pool_put(ctx, j.wdesc); pool_put(ctx, j.wres_d);
}

// A staged run's last fill, kept for gx_staged_table (its buffers go back to
// the pool when the run is replaced and the last table of it is freed; the
// owner holds ctx->mu then).
struct KeptFill {
    gx_context* ctx = nullptr;
    FillJob job;
    std::vector<int> dev_of;   // staged pair -> its index in job.pd (-1: no interior, not filled)
    ~KeptFill() { job_release(ctx, job); }
};
// The pipelines' release point for a pass's fill: the last pass of a
// GX_STAGED_KEEP_PLANES run is held (*keep set) instead of released.
static void release_or_hold(gx_context* ctx, FillJob& j, bool last_pass, bool* held) {
    if (ctx->keep_capture && last_pass) { *held = true; return; }
    job_release(ctx, j);
}
static void keep_job(gx_context* ctx, FillJob& j, const std::vector<int>& dev_of) {
    auto k = std::make_shared<KeptFill>();
    k->ctx = ctx;
    k->dev_of = dev_of;
    std::swap(k->job, j);
    ctx->kept = std::move(k);
}

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// chars_dev: if non-null, device buffer already holding the processed chars
// at offsets off1/off2 (staged path); otherwise c1/c2 are uploaded.
// track: first max cell + LCS field (alignment_table's max_cell and
// matches_at_max, algo.rs:258-262, 279); lcs: also keep the LCS plane.
static hipError_t enqueue_plane_sums(gx_context* ctx, const FillJob& job, const Scores32& sc, unsigned long long* out,
                                     hipStream_t st = nullptr);

// The twin fill (gx_fill_pk.hip): two pairs per band, one in each 16-bit
// half.  Its values are kept relative to bases that a band's
// strips inherit from its top row (see the file header); a value of strip k
// of a W-strip band lies within D (192 (k + 1) + 16) + 2 (|a| + |smax| + |smin|)
// of its base, D = max |V''(i,j) - V''(i',j')| over neighbours = max(|a - g|,
// |U - g|) (the range proof of d8_planes_ok).  Returns the widest admissible
// band width <= W_want from {3, 4, 7, 8, 15}, or 0 when the twin fill does not apply
// (shape, mode, scores, GX_TWIN=0; run_fill also skips it for short queues).
// The twins (twin_table) pair the batch's pairs by shape whatever their
// order; the sweep covers the larger n and m of a twin, the shorter pair's
// state stays at its last column (its values beyond lie in the row above's
// range, but the bound takes the column difference anyway); an odd last pair
// is twinned with itself.
// The admission bound of a W-strip twin band whose twins' column counts
// differ by up to dm: the largest |value - base| any state of the band can
// reach (see the comment above twin_table).
// Local twins (plain values, no shift) take D = max(|a|, U), the neighbour
// bound of d8_planes_ok itself (the 0 floor keeps it), and their score
// offsets carry + K (K = max(0, -s_min), run_fill) and the floor's -g term.
constexpr long long kTwinBoundLimit = 30000;   // < 2^15 with room for the derived offsets
static long long twin_step(const Scores32& sc, bool local) {
    const long long g = sc.g, a = (long long)sc.h + sc.g;
    const long long smax = std::max(sc.sm, sc.smm);
    const long long U = std::max(0LL, smax - a);
    return local ? std::max({std::llabs(a), U, 1LL}) : std::max({std::llabs(a - g), std::llabs(U - g), 1LL});
}
static long long twin_const(const Scores32& sc, bool local) {
    const long long g = sc.g, a = (long long)sc.h + sc.g;
    const long long smax = std::max(sc.sm, sc.smm), smin = std::min(sc.sm, sc.smm);
    return 2 * (std::llabs(a) + std::llabs(smax) + std::llabs(smin)) + 64 +
           (local ? std::max(0LL, -smin) + std::llabs(g) : 0);
}
static long long twin_bound(const Scores32& sc, int W, long long dm, bool local = false) {
    return twin_step(sc, local) * (192LL * W + 16 + dm) + twin_const(sc, local);
}
// Largest column gap between twins that keeps band width W admissible under
// twin_width's bound (capped at 1,024): twin_table pairs no wider gaps, so one
// ill-matched twin never narrows the band width of a whole batch.
static long long twin_gap_cap(const Scores32& sc, int W, bool local = false) {
    const long long rest = kTwinBoundLimit - 1 - twin_const(sc, local);
    return std::max(0LL, std::min(1024LL, rest / twin_step(sc, local) - 192LL * W - 16));
}
static std::vector<std::pair<int, int>> twin_table(const std::vector<PairHost>& ph, long long gap_cap = 1024) {
    std::vector<int> idx(ph.size());
    for (size_t p = 0; p < ph.size(); ++p) idx[p] = (int)p;
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) {
        return ph[a].m != ph[b].m ? ph[a].m > ph[b].m : ph[a].n > ph[b].n;
    });
    // neighbours in that order, unless their column counts lie more than
    // gap_cap apart (the admission bound's column margin): such a pair is
    // twinned with itself
    std::vector<std::pair<int, int>> tw;
    for (size_t k = 0; k < idx.size();) {
        if (k + 1 < idx.size() && (long long)(ph[idx[k]].m - ph[idx[k + 1]].m) <= gap_cap) {
            tw.emplace_back(idx[k], idx[k + 1]);
            k += 2;
        } else {
            tw.emplace_back(idx[k], idx[k]);
            k += 1;
        }
    }
    return tw;
}
// long_ok: the launch will be the twin fill without landing columns (twin
// plane codes, no code words, no skeleton): no int16 column quantity is
// left, so the 31,920-column limit of the int16 landing columns is lifted.
// The local twin fill (gx_fill_pk.hip LOCAL) keeps plain values relative to
// the same per-block bases, under the same bound (twin_step's local D); its
// row maxima fold into int32 at each base change, and it tracks no columns,
// so neither the magnitude of its values nor the column count is limited.
// Only as the launch without code words or skeleton (twin plane codes, the
// sequential walk): long_ok.
static int twin_width(const std::vector<PairHost>& ph, const std::vector<std::pair<int, int>>& tw, const Scores32& sc,
                      int is_local, bool track, bool lcs, int lay, bool planes, bool d8, int W_want,
                      bool long_ok = false) {
    if (const char* e = getenv("GX_TWIN"); e && !strcmp(e, "0")) return 0;
    if (lay != 0 || track || lcs || (planes && !d8) || sc.g > 0 || sc.h > 0) return 0;
    if (ph.empty()) return 0;
    if (is_local && (!planes || !long_ok)) return 0;
    long long dm = 0;
    for (const auto& t : tw) {
        const PairHost& x = ph[t.first];
        const PairHost& y = ph[t.second];
        if (!x.n || !x.m || !y.n || !y.m) return 0;
        if (std::max(x.m, y.m) + 80 > 32000 && !long_ok) return 0;
        dm = std::max(dm, std::llabs((long long)x.m - (long long)y.m));
    }
    for (int W : {15, 8, 7, 4, 3}) {
        if (W > W_want && W != 3) continue;
        if (twin_bound(sc, W, dm, is_local != 0) < kTwinBoundLimit) return W;
    }
    return 0;
}

static int run_fill(gx_context* ctx, const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc,
                    const std::vector<PairHost>& ph, const Scores32& sc, int is_local, bool planes, bool track,
                    bool lcs, FillJob& job, const uint8_t* chars_dev = nullptr,
                    const std::vector<size_t>* off1 = nullptr, const std::vector<size_t>* off2 = nullptr,
                    const SmallAlpha* alpha = nullptr, int slot = -1, bool collect = true) {
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
    // small-alphabet score table: untracked fill (global or local), <= 4 symbols, scores in a signed byte
    const bool tbl = alpha && alpha->n <= 4 && !track && scl.sm >= -128 && scl.sm <= 127 &&
                     scl.smm >= -128 && scl.smm <= 127 && !getenv("GX_NO_SCORE_TABLE");
    if (tbl)
        for (int k = 0; k < 4; ++k) scl.sym[k] = alpha->sym[k];
    job.planes_on = planes; job.lcs_on = lcs; job.track_on = track;
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
    ctx->last_pbytes = planes ? (w16 ? 2 : (int)(plane_esz * 3)) : 0;
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
    const int nplanes = w16 ? 1 : lcs ? 4 : 3;
    if (!chars_dev) {
        if ((rc = pool_get(ctx, chars_bytes, &job.chars, fs))) return rc;
    }
    if (planes && (rc = pool_get(ctx, plane_elems * plane_esz * nplanes, &job.planes, fs))) return rc;
    if (codes && (rc = pool_get(ctx, code_elems * sizeof(uint32_t), &job.codes, fs))) return rc;
    if ((rc = pool_get(ctx, std::max<size_t>(skel_elems, 1) * sizeof(int), &job.skel, fs))) return rc;
    if ((rc = pool_get(ctx, std::max<size_t>(feed_recs, 1) * sizeof(Rec), &job.feed, fs))) return rc;
    if ((rc = pool_get(ctx, std::max(strips, 1) * sizeof(StripRes), &job.sres, fs))) return rc;
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
        d.pL = (planes && lcs) ? plane_at(3) : nullptr;
        d.codes = codes ? (uint32_t*)job.codes.p + co[p] : nullptr;
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
    const char* trace_file = slot < 0 ? getenv("GX_TRACE_FILE") : nullptr;
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
    // twin workgroups: as many per CU as fit 16 waves (the twin kernels hold
    // up to 128 VGPRs: 4 waves per SIMD)
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
        HIPCHK(launch_fill_skew(W, is_local != 0, planes, tbl, trace.p != nullptr, track, (const PairDev*)job.pairs.p, (int)P, bands,
                                counter, (StripRes*)job.sres.p, (PairRes*)job.pres.p, scl, grid, fs));
    else if (bands > 0 && cs2)
        HIPCHK(launch_fill_cs2(W, is_local != 0, planes, tbl, (const PairDev*)job.pairs.p, (int)P, bands,
                               counter, (StripRes*)job.sres.p, (PairRes*)job.pres.p, scl, grid, fs));
    else if (bands > 0)
        HIPCHK(launch_fill(W, lay, is_local != 0, planes ? (d8 ? 2 : 1) : 0, track, lcs, tbl, (const PairDev*)job.pairs.p, (int)P, bands,
                           counter, (StripRes*)job.sres.p, (PairRes*)job.pres.p, scl, grid, fs));
    HIPCHK(hipEventRecord(eve, fs));   // evb..eve brackets the fill kernel alone
    if (ctx->sums_dst && planes && bands > 0) {   // staged checksum run: this pass's plane sums
        HIPCHK(enqueue_plane_sums(ctx, job, sc, ctx->sums_dst, fs));
        ctx->sums_dst += 3 * P;
    }
    // strip results exist only for the tracked and local fills (the untracked
    // global fill writes end_SM / end_E itself): no reduction launch otherwise
    if (bands > 0 && (track || is_local))
        HIPCHK(launch_finalize((const PairDev*)job.pairs.p, (int)P, (const StripRes*)job.sres.p,
                               (PairRes*)job.pres.p, fs));
    // the local twin fill tracks each row's maximum only: the last column of
    // the chosen row from its plane codes (gx_kernels.hip local_col_kernel)
    if (bands > 0 && twin && is_local)
        HIPCHK(launch_local_col((const PairDev*)job.pairs.p, (int)P, (PairRes*)job.pres.p, sc.h, sc.g, fs));
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
        HIPCHK(hipEventRecord(sl.fdone, fs));
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
static int fill_collect(gx_context* ctx, FillJob& job) {
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
static int run_fill_wide(gx_context* ctx, const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc,
                         const std::vector<PairHost>& ph, const HostScores& hs, int is_local, bool planes, bool track,
                         bool lcs, FillJob& job) {
    const size_t P = ph.size();
    job.wide = true;
    job.lay = 1;
    job.W = 1;
    lcs = lcs && planes;
    track = track || lcs;
    job.planes_on = planes; job.lcs_on = lcs; job.track_on = track;
    ctx->last_lay = 1; ctx->last_W = 1; ctx->last_pbytes = planes ? 24 : 0;
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
static StartIn start_in(const FillJob& job, size_t p) {
    if (job.wide) return StartIn{job.wres[p].end_SM, job.wres[p].lmax_val, (uint64_t)job.wres[p].lmax_i,
                                 (uint64_t)job.wres[p].lmax_j};
    const PairRes& r = job.res[p];
    return StartIn{r.end_SM, r.lmax_val, (uint64_t)r.lmax_i, (uint64_t)r.lmax_j};
}
static StartIn start_in(const PairRes& r) { return StartIn{r.end_SM, r.lmax_val, (uint64_t)r.lmax_i, (uint64_t)r.lmax_j}; }
static int start_cell(const gx_table* t, const StartIn& r, uint64_t* si, uint64_t* sj, int64_t* score);


static bool tb_match(const uint8_t* s1, size_t n, const uint8_t* s2, size_t m, uint64_t i, uint64_t j) {
    // is_match(i, j, false) with unshifted indices: nth() past the end is None
    const int a = i < n ? (int)s1[i] : 0x1FF;
    const int b = j < m ? (int)s2[j] : 0x1FF;
    return a == b;
}

// The boundary part of a walk from (i, j) on: the reference loop on analytic
// cells (algo.rs:339-422), appending to w.steps and counting into w.res.
static int label_boundary(const HostScores& hs, int is_local, const uint8_t* s1, size_t n, const uint8_t* s2,
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
static int label_walk_records(const HostScores& hs, int is_local, const uint8_t* s1, size_t n, const uint8_t* s2,
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

struct TbStart {
    int i, j;   // interior start cell, or 0 = nothing to walk
    int E;      // its landing column (PairRes.end_E / lmax_E)
};

// dev_end_E: take each start cell's landing column from the fill's device
// results (global mode, start (n, m)), so the traceback can be queued right
// behind the fill without waiting for its results on the host.
// The traceback of the pairs of one or more fills (jv: their pairs in order,
// `starts` over all of them; the fills share layout and code format), its
// kernels on stream ts (nullptr: the context's stream).
static int run_traceback(gx_context* ctx, const std::vector<const FillJob*>& jv, const std::vector<TbStart>& starts,
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

static int run_traceback(gx_context* ctx, const FillJob& job, const std::vector<TbStart>& starts, TbOut& out,
                         int slot = -1, bool collect = true, bool dev_end_E = false) {
    return run_traceback(ctx, std::vector<const FillJob*>{&job}, starts, out, slot, collect, dev_end_E, nullptr);
}

// Records of a traceback enqueued with collect = false (pipelined path).
static void release_held(gx_context* ctx, int slot) {
    for (DevBuf& b : ctx->slots[slot].held) { pool_put(ctx, b); b = DevBuf{}; }
}
// After a pipeline drained (its streams and the copy stream synchronised),
// or on its error path: every slot's traceback buffers and fill results block
// back to the pool (a fill's held_pres is otherwise released only by its
// fill_collect or the slot's next fill).
static void release_slots(gx_context* ctx) {
    (void)hipStreamSynchronize(ctx->cstream);
    for (int k = 0; k < 4; ++k) {
        release_held(ctx, k);
        pool_put(ctx, ctx->slots[k].held_pres);
    }
}

static int tb_collect(gx_context* ctx, int slot, size_t P, TbOut& out) {
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


// Start cell + score (algo.rs:306-331).
static int start_cell_common(const HostScores& hs, int is_local, size_t n, size_t m, const StartIn& r,
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
    int rc = t->job.wide ? fetch_rows_wide(t, which, row0, rows, p64) : fetch_rows32(t, which, row0, rows, p32);
    if (rc) return rc;
    for (size_t r = 0; r < rows; ++r) {
        const size_t i = row0 + r;
        for (size_t j = 0; j <= m; ++j) {
            int64_t v;
            if (i == 0 || j == 0) {
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
    if (which < 0 || which > 2) return fail(GX_EINVAL, "which must be 0 (insert), 1 (delete) or 2 (sub)");
    const size_t n = t->s1.size(), m = t->s2.size();
    if (row0 > n + 1 || rows > n + 1 - row0) return fail(GX_EINVAL, "row range outside the table");
    if (out_cells < rows * (m + 1)) return fail(GX_ECAP, "out too small");
    if (rows == 0) return GX_OK;
    std::lock_guard<std::mutex> lk(t->ctx->mu);
    HIPCHK(hipSetDevice(t->ctx->device));
    return export_rows(t, which, row0, rows, out, 0, rows);
}

// Plane checksums of job `job`'s pairs into the device buffer out[P][3].
static hipError_t enqueue_plane_sums(gx_context* ctx, const FillJob& job, const Scores32& sc,
                                     unsigned long long* out, hipStream_t st) {
    int max_strips = 0;
    for (const PairDev& d : job.pd) max_strips = std::max(max_strips, d.strips);
    return launch_plane_sums((const PairDev*)job.pairs.p, (int)job.pd.size(), max_strips, job.lay,
                             job.w16 ? 3 : job.d8 ? 2 : 1,
                             sc.h, sc.g, sc.floor_, (job.shift || job.w16) ? sc.g : 0, out, st ? st : ctx->stream);
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
    if (have_l && (rc = fetch_plane32(t, 3, pL))) return rc;
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

static int copy_steps(const Walk& w, gx_step* steps, size_t cap) {
    if (!steps) return GX_OK;
    if (w.steps.size() > cap) return fail(GX_ECAP, "steps capacity " + std::to_string(cap) + " < " +
                                                       std::to_string(w.steps.size()));
    memcpy(steps, w.steps.data(), w.steps.size() * sizeof(gx_step));
    return GX_OK;
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

// ---------------------------------------------------------------------------
// chunked batches: a batch whose device footprint exceeds the free HBM runs
// as contiguous chunks of pairs through the same (reused) device buffers

// Device bytes a fill + traceback of pair (n, m) holds: score planes
// (plane_bpc per cell), traceback codes (0.25 B/cell), skeleton and hand-off
// rows, traceback records.
static double pair_device_bytes(size_t n, size_t m, double plane_bpc) {
    const double cells = (double)(n + 128) * (double)(m + 64);
    return cells * (plane_bpc + 0.25) + 64.0 * (double)(m + 64) * (double)(n / 64 + 2) / 8.0 + 65536.0;
}

// Budget for one chunk: GX_CHUNK_BYTES if set, else the free device memory
// plus the context's cached buffers, less 4 GiB of headroom.
static double chunk_budget(gx_context* ctx) {
    if (const char* e = getenv("GX_CHUNK_BYTES"); e && *e) return atof(e);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 64e9;
    double cached = 0;
    for (const DevBuf& b : ctx->free_list) cached += (double)b.cap;
    return std::max(1e9, (double)fr + cached - 4.0 * (1ull << 30));
}

// Contiguous [begin, end) ranges of the pairs, each within the budget (a pair
// larger than the budget runs alone), balanced: the fewest chunks the budget
// allows, each near total / chunks (1024 x 16k: 4 x 256 pairs, not 3 x 330 +
// 34, whose short last chunk would lose the twin fill and leave CUs idle).
// (Twins are formed inside each chunk by twin_table, by shape, so a chunk's
// pair count need not be even.)
static std::vector<std::pair<size_t, size_t>> plan_chunks_within(const std::vector<PairHost>& ph, double plane_bpc,
                                                                 double budget) {
    std::vector<std::pair<size_t, size_t>> out;
    auto bytes = [&](size_t p) { return (ph[p].n && ph[p].m) ? pair_device_bytes(ph[p].n, ph[p].m, plane_bpc) : 0.0; };
    size_t b = 0;
    double acc = 0;
    for (size_t p = 0; p < ph.size(); ++p) {
        const double x = bytes(p);
        if (p > b && acc + x > budget) {
            out.emplace_back(b, p);
            b = p;
            acc = 0.0;
        }
        acc += x;
    }
    out.emplace_back(b, ph.size());
    return out;
}
static std::vector<std::pair<size_t, size_t>> plan_chunks(gx_context* ctx, const std::vector<PairHost>& ph,
                                                          double plane_bpc) {
    const double budget = chunk_budget(ctx);
    auto out = plan_chunks_within(ph, plane_bpc, budget);
    if (out.size() > 1) {
        double total = 0;
        for (size_t p = 0; p < ph.size(); ++p)
            total += (ph[p].n && ph[p].m) ? pair_device_bytes(ph[p].n, ph[p].m, plane_bpc) : 0.0;
        // the same number of chunks with a smaller target, if the greedy split allows it
        for (double f : {1.0, 1.02, 1.05, 1.1}) {
            const double target = std::min(budget, f * total / (double)out.size());
            auto bal = plan_chunks_within(ph, plane_bpc, target);
            if (bal.size() <= out.size()) return bal;
        }
    }
    return out;
}

// ---------------------------------------------------------------------------
// batch of independent pairs (config 4 / 5)

// Labels one batch's walks (host, algo.rs:339-422), pairs on the worker pool:
// interior moves from the device's row records (dev_of[p] >= 0), then the
// analytic boundary; fills walks[p].res.
static int label_batch(gx_context* ctx, const std::vector<PairHost>& ph, const HostScores& hs, int is_local, bool track,
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

// A batch through the int64 fill (jobs outside the exact-int32 range): fill,
// host start cells, device traceback, host labelling.  Synchronous, one pass.
static int batch_core_wide(gx_context* ctx, const std::vector<PairHost>& ph,
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

// `nsteps` passes over the same batch (the staged benchmark path), pipelined
// one batch deep: batch k+1's fill is queued behind batch k's traceback, so
// the host labels batch k while the device fills batch k+1.  Device buffers
// go back to the pool as soon as their last user is queued (everything runs on
// one stream); pinned staging and events alternate between two slots.  Walks
// and results are those of the last pass; *fill_ms is the mean fill time.
// Overlapped pipeline for a global untracked batch on the twin fill without
// landing columns (the sequential strip walk, tb_seq_kernel, ~5 ms for a 30k
// pair, uses a few CUs): the pairs are split into a small group A (about a
// fifth) and the rest, B, each filled by its own launch on its own stream.
// Step k's walk (stream tstream, after both fills) then runs beside step k+1's
// group-A fill, whose plane codes go to a second A buffer (two A buffers, one
// B buffer: the device holds P + |A| pairs' planes); step k+1's group-B fill
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
    const size_t G = std::max<size_t>(2, (Q / 5) & ~(size_t)1);   // group A: about a fifth, even (twins)
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

static int batch_core_steps(gx_context* ctx, const std::vector<PairHost>& ph,
                            const std::vector<std::pair<const uint8_t*, const uint8_t*>>& proc, const HostScores& hs,
                            const Scores32& sc, int is_local, bool planes, bool track, int nsteps,
                            std::vector<Walk>& walks, double* fill_ms, const uint8_t* chars_dev,
                            const std::vector<size_t>* off1, const std::vector<size_t>* off2,
                            const SmallAlpha* staged_alpha, const PassSet* alt = nullptr) {
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
    FillJob jobs[2];
    std::vector<PairRes> res(P, PairRes{});
    std::vector<TbStart> starts(idx.size());
    std::vector<uint64_t> si(P), sj(P);
    std::vector<int64_t> score(P);
    std::vector<int> dev_of(P, -1);
    for (size_t q = 0; q < idx.size(); ++q) dev_of[idx[q]] = (int)q;
    double fsum = 0;
    auto fill = [&](int s) {   // slot s = the pass's parity = its pair set
        return run_fill(ctx, dproc_s[s], dph_s[s], sc, is_local, planes, track, false, jobs[s], chars_dev,
                        chars_dev ? &o1_s[s] : nullptr, chars_dev ? &o2_s[s] : nullptr, &alpha, s, false);
    };
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
    // 145: profiles/r04_config5_*.json, r02k_config5_*.json)
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
    if (!is_local && !track) {
        // global untracked: every start cell is (n, m) and its landing column
        // is read on the device, so each step's traceback is queued right
        // behind its fill; the fill results are collected on the host only
        // for the labelling (no host round trip between fill and traceback)
        for (size_t q = 0; q < idx.size(); ++q) starts[q] = TbStart{dph[q].n >= 1 && dph[q].m >= 1 ? (int)dph[q].n : 0,
                                                                     (int)dph[q].m, 0};
        // the walk stays on the fill's stream: the fill's buffers return to
        // the pool right behind it (stream-ordered reuse).  (A walk on its own
        // stream beside the next step's fill measured 1024 x 4k +6 % but made
        // 1024 x 1k 2.5x slower: the host's enqueue of the next fill stalled
        // behind the running walk.)
        int tr_pass = 0;
        bool held[2] = {false, false};
        auto trace_dev = [&](int s) {
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
        if (!(rc = fill(0))) rc = trace_dev(0);
        for (int k = 0; k < nsteps && !rc; ++k) {
            const int s = k & 1;
            auto t = clk::now();
            if (k + 1 < nsteps && ((rc = fill(s ^ 1)) || (rc = trace_dev(s ^ 1)))) break;
            h_enq += since(t); t = clk::now();
            if ((rc = tb_collect(ctx, s, idx.size(), ctx->slots[s].out))) break;
            h_tbw += since(t); t = clk::now();
            if ((rc = results(s))) break;
            h_res += since(t); t = clk::now();
            ctx->pass_off = poff[s];
            if ((rc = label_batch(ctx, *PH[s], hs, is_local, track, dev_of, si, sj, score, res, ctx->slots[s].out,
                                  jobs[s].fill_ms, *WK[s])))
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
            for (auto& j : jobs) job_release(ctx, j);
            release_slots(ctx);
            return rc;
        }
        for (int s = 0; s < 2; ++s)
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

extern "C" int gx_fill_info(const gx_context* ctx, int* layout, int* band_waves, int* plane_bytes_per_cell) {
    if (!ctx) return fail(GX_EINVAL, "context is NULL");
    if (layout) *layout = ctx->last_lay;
    if (band_waves) *band_waves = ctx->last_W;
    if (plane_bytes_per_cell) *plane_bytes_per_cell = ctx->last_pbytes;
    return GX_OK;
}

extern "C" int gx_twin_admission(const gx_scores* scores, int band_waves, int64_t col_gap, int64_t* bound) {
    if (!scores || band_waves < 1 || col_gap < 0) return -1;
    HostScores hs;
    Scores32 sc;
    if (check_scores(scores, 1, 1, &hs, &sc, 0, nullptr) != GX_OK) return -1;
    const long long b = twin_bound(sc, band_waves, col_gap);
    if (bound) *bound = b;
    return (sc.g <= 0 && sc.h <= 0 && b < kTwinBoundLimit) ? 1 : 0;
}

extern "C" int gx_twin_admission_mode(const gx_scores* scores, int is_local, int band_waves, int64_t col_gap,
                                      int64_t* bound) {
    if (!scores || band_waves < 1 || col_gap < 0) return -1;
    HostScores hs;
    Scores32 sc;
    if (check_scores(scores, 1, 1, &hs, &sc, is_local, nullptr) != GX_OK) return -1;
    const long long b = twin_bound(sc, band_waves, col_gap, is_local != 0);
    if (bound) *bound = b;
    return (sc.g <= 0 && sc.h <= 0 && b < kTwinBoundLimit) ? 1 : 0;
}

extern "C" int gx_plan_layout(const gx_scores* scores, int is_local, const int64_t* n, const int64_t* m,
                              size_t npairs, int track, int grid_cap) {
    if (!scores || !n || !m || npairs == 0) return -1;
    int64_t nmax = 0, mmax = 0;
    for (size_t p = 0; p < npairs; ++p) {
        if (n[p] < 0 || m[p] < 0) return -1;
        nmax = std::max(nmax, n[p]); mmax = std::max(mmax, m[p]);
    }
    HostScores hs;
    Scores32 sc;
    if (check_scores(scores, (size_t)nmax, (size_t)mmax, &hs, &sc, is_local, nullptr) != GX_OK) return -1;
    std::vector<PairHost> ph(npairs);
    for (size_t p = 0; p < npairs; ++p) ph[p] = PairHost{nullptr, nullptr, (size_t)n[p], (size_t)m[p]};
    return fill_layout(ph, sc, grid_cap > 0 ? grid_cap : 256, track != 0, false);
}

extern "C" int gx_plane_bytes_per_cell(const gx_scores* scores, int is_local) {
    HostScores hs;
    Scores32 sc;
    if (check_scores(scores, 1, 1, &hs, &sc, is_local)) return -1;
    return d8_planes_ok(sc, is_local) ? 3 : 12;
}

extern "C" int gx_run_staged(gx_context* ctx, const gx_scores* scores, int is_local, int keep_planes, uint32_t flags,
                             gx_result* out, double* fill_ms_out) {
    return gx_run_staged_steps(ctx, scores, is_local, keep_planes, flags, 1, out, fill_ms_out);
}
