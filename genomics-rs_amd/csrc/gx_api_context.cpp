// gx_api_context.cpp -- contexts (gx_context_create / trim / destroy), the
// thread's last error, pinned host staging, the per-context device buffer
// pool and the pipeline slots' held buffers.
#include "gx_api.h"

// ---------------------------------------------------------------------------
// errors

thread_local std::string g_err;
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int gx_internal_fail(int code, const std::string& msg) { return fail(code, msg); }

extern "C" const char* gx_last_error(void) { return g_err.c_str(); }
extern "C" const char* gx_version(void) { return "genomics-rs_amd 0.1 (gfx950)"; }

bool log_info() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("GX_LOG");
        v = (e && (!strcmp(e, "info") || !strcmp(e, "debug"))) ? 1 : 0;
    }
    return v == 1;
}

void* pinned_grow(PinnedBuf& b, size_t bytes) {
    if (b.cap < bytes) {
        if (b.p) (void)hipHostFree(b.p);
        b = PinnedBuf{};
        const size_t cap = std::max<size_t>(bytes, 1 << 16);
        if (hipHostMalloc(&b.p, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
        b.cap = cap;
    }
    return b.p;
}

int slots_ready(gx_context* ctx) {
    for (auto& s : ctx->slots) {
        hipEvent_t* evs[] = {&s.fb, &s.fe, &s.tb, &s.te, &s.fdone, &s.tdone, &s.fres};
        for (hipEvent_t* e : evs)
            if (!*e && hipEventCreate(e) != hipSuccess) return GX_EHIP;
    }
    return GX_OK;
}

// ctx->io_pin grown to `bytes` (contents not kept); nullptr on failure.
void* io_pinned(gx_context* ctx, size_t bytes) {
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
int pool_get(gx_context* ctx, size_t bytes, DevBuf* out, hipStream_t st) {
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
    // no request takes a cached buffer of 1 GiB or more that is over twice
    // its size (that buffer may fit a later, larger request of the same
    // launch; 1024 x 64k chunks ran out of HBM when the 0.7 GB skeleton and
    // hand-off requests of an overlapped pass took the two 34 GB plane
    // buffers a smaller batch had left cached.  A tighter 1.25x made the
    // chunks' alternating 86 / 69 / 95 GB plane requests miss and re-map the
    // HBM: 1024 x 64k fill 2.0 -> 4.8 s a pass)
    if (bi >= 0 && best >= ((size_t)1 << 30) && best / 2 > bytes) bi = -1;
    if (bi >= 0) {
        if (const char* lg = getenv("GX_LOG"); lg && !strcmp(lg, "debug") && bytes >= ((size_t)1 << 30))
            fprintf(stderr, "[gx DEBUG] pool hit: %zu B from a cached %zu B\n", bytes, best);
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
            size_t fr = 0, tot = 0;
            (void)hipMemGetInfo(&fr, &tot);
            return fail(GX_ENOMEM, "hipMalloc(" + std::to_string(bytes) + " B) failed (" + std::to_string(fr) +
                                       " B free of " + std::to_string(tot) + ")");
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
void pool_put(gx_context* ctx, DevBuf& b) {
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
    // every stream of the context up front, in this order: HIP maps streams
    // onto its hardware queues (GPU_MAX_HW_QUEUES, 4 by default) round robin
    // at creation, and two streams on one queue run in order.  Created on
    // first use instead, the walk stream of a short batch ahead of the second
    // fill stream put that stream on the fill stream's queue: a later
    // overlapped batch (1024 x 64k) then ran its two fill groups and the walk
    // in series, fill 1.9 -> 5.4 s a pass.
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->tstream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->pstream, hipStreamNonBlocking));
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
    if (ctx->pstream) (void)hipStreamDestroy(ctx->pstream);
    delete ctx;
}

// Records of a traceback enqueued with collect = false (pipelined path).
void release_held(gx_context* ctx, int slot) {
    for (DevBuf& b : ctx->slots[slot].held) { pool_put(ctx, b); b = DevBuf{}; }
}
// After a pipeline drained (its streams and the copy stream synchronised),
// or on its error path: every slot's traceback buffers and fill results block
// back to the pool (a fill's held_pres is otherwise released only by its
// fill_collect or the slot's next fill).
void release_slots(gx_context* ctx) {
    (void)hipStreamSynchronize(ctx->cstream);
    for (int k = 0; k < 4; ++k) {
        release_held(ctx, k);
        pool_put(ctx, ctx->slots[k].held_pres);
    }
}
