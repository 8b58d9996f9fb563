// rsk_runtime.hip — contexts, errors, staging and kernel timing for librsk.so.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "rsk_common.h"

namespace rsk {

int DevBuf::reserve(size_t need) {
    if (need <= bytes && ptr) return RSK_OK;
    release();
    size_t n = need < 256 ? 256 : need;
    RSK_HIP(hipMalloc(&ptr, n));
    bytes = n;
    return RSK_OK;
}

void DevBuf::release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
}

int activate(rsk_ctx *ctx) {
    RSK_CHECK(ctx, "null context");
    RSK_HIP(hipSetDevice(ctx->device));
    return check_dev_err(ctx);
}

unsigned *dev_err(rsk_ctx *ctx) {
    if (!ctx->errw.host) {
        if (ctx->errw.reserve(64) != RSK_OK) return nullptr;
        *static_cast<volatile unsigned *>(ctx->errw.host) = 0u;
    }
    return static_cast<unsigned *>(ctx->errw.dev);
}

int check_dev_err(rsk_ctx *ctx) {
    if (!ctx->errw.host) return RSK_OK;
    volatile unsigned *w = static_cast<volatile unsigned *>(ctx->errw.host);
    const unsigned e = *w;
    if (!e) return RSK_OK;
    *w = 0u;
    set_error("device write guard: %s%s(offsets from an earlier launch's counts exceeded the buffer; the stores "
              "were skipped and the results are invalid)",
              (e & kErrNrPlace) ? "nr_place record offset past its buffer " : "",
              (e & kErrListFill) ? "list_fill base-list offset past P " : "");
    return RSK_EHIP;
}

static hipEvent_t pooled_event(rsk_ctx *ctx) {
    if (!ctx->event_pool.empty()) {
        hipEvent_t e = ctx->event_pool.back();
        ctx->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}

ScopedTimer::ScopedTimer(rsk_ctx *c, const char *n, hipStream_t s) : ctx(c), name(n), stream(s ? s : c->stream) {
    if (!ctx->profiling) return;
    if (!ctx->profile_only.empty() && ctx->profile_only != name) return;
    a = pooled_event(ctx);
    b = pooled_event(ctx);
    if (!a || !b) {
        if (a) ctx->event_pool.push_back(a);
        if (b) ctx->event_pool.push_back(b);
        a = b = nullptr;
        return;
    }
    (void)hipEventRecord(a, stream);
}

ScopedTimer::~ScopedTimer() {
    if (!a) return;
    (void)hipEventRecord(b, stream);
    ctx->pending[name].push_back({a, b});
}

int aux_fork(rsk_ctx *ctx, int k) {
    if (!ctx->fork) RSK_HIP(hipEventCreateWithFlags(&ctx->fork, hipEventDisableTiming));
    RSK_HIP(hipEventRecord(ctx->fork, ctx->stream));
    for (int i = 0; i < k; ++i) {
        if (!ctx->aux[i]) {
            // (a high-priority side stream measured no change)
            RSK_HIP(hipStreamCreateWithFlags(&ctx->aux[i], hipStreamNonBlocking));
            RSK_HIP(hipEventCreateWithFlags(&ctx->join[i], hipEventDisableTiming));
        }
        RSK_HIP(hipStreamWaitEvent(ctx->aux[i], ctx->fork, 0));
    }
    return RSK_OK;
}

int aux_join(rsk_ctx *ctx, int k) {
    for (int i = 0; i < k; ++i) {
        RSK_HIP(hipEventRecord(ctx->join[i], ctx->aux[i]));
        RSK_HIP(hipStreamWaitEvent(ctx->stream, ctx->join[i], 0));
    }
    return RSK_OK;
}

int PinBuf::reserve(size_t need) {
    if (need <= bytes) return RSK_OK;
    release();
    size_t n = 4096;
    while (n < need) n <<= 1;
    RSK_HIP(hipHostMalloc(&host, n, hipHostMallocMapped));
    if (hipHostGetDevicePointer(&dev, host, 0) != hipSuccess) {
        (void)hipHostFree(host);
        host = nullptr;
        set_error("hipHostGetDevicePointer failed");
        return RSK_EHIP;
    }
    bytes = n;
    return RSK_OK;
}

void PinBuf::release() {
    if (host) (void)hipHostFree(host);
    host = dev = nullptr;
    bytes = 0;
}

int stage_in(rsk_ctx *ctx, int slot, const void *src, size_t bytes, bool device, const void **out) {
    if (device || bytes == 0) { *out = src; return RSK_OK; }
    RSK_CHECK(src, "null input pointer");
    RSK_TRY(ctx->host_stage[slot].reserve(bytes));
    RSK_HIP(hipMemcpyAsync(ctx->host_stage[slot].ptr, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    *out = ctx->host_stage[slot].ptr;
    return RSK_OK;
}

int stage_out(rsk_ctx *ctx, int slot, void *dst, size_t bytes, bool device, void **out) {
    if (device || bytes == 0) { *out = dst; return RSK_OK; }
    RSK_TRY(ctx->host_stage[slot].reserve(bytes));
    *out = ctx->host_stage[slot].ptr;
    return RSK_OK;
}

int copy_back(rsk_ctx *ctx, void *host_dst, const void *dev_src, size_t bytes, bool device) {
    if (device || bytes == 0 || !host_dst) return RSK_OK;
    RSK_HIP(hipMemcpyAsync(host_dst, dev_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    return RSK_OK;
}

int ws_u64_layout(int64_t N, int64_t S, int64_t H, U64Slice *out) {
    int n = 0;
    auto add = [&](const char *name, uint64_t off) { out[n++] = U64Slice{name, off}; };
    const uint64_t nbs = (uint64_t)S * blk_nb(N);
    add("plan.zc zc_key half 0", 0);
    add("plan.zc zc_key half 1", zc_half_bytes(S));
    add("rounds.key_ws kdet", 0);
    add("rounds.key_ws kpick", (uint64_t)S * 8);
    add("rounds.key_ws zc_key", (uint64_t)S * 16);
    add("blk bm", 0);
    add("blk bz", nbs * 8);
    add("move table red64", (uint64_t)H * 8);
    add("move global area 1", move_tab_bytes(H));
    add("persist LDS bm", move_tab_bytes(H));
    add("persist LDS bz", move_tab_bytes(H) + (uint64_t)blk_nb(N) * 8);
    return n;
}

int ws_check_u64(int64_t N, int64_t S, int64_t H) {
    U64Slice sl[kMaxU64Slices];
    const int n = ws_u64_layout(N, S, H, sl);
    for (int i = 0; i < n; ++i)
        RSK_CHECK(sl[i].off % 8 == 0, "workspace slice '%s' at byte %llu is not 8-B aligned (N=%lld S=%lld H=%lld)",
                  sl[i].name, (unsigned long long)sl[i].off, (long long)N, (long long)S, (long long)H);
    return RSK_OK;
}

int ws_check_ptr(const void *p, const char *name) {
    RSK_CHECK(((uintptr_t)p & 7) == 0, "u64 buffer '%s' at %p is not 8-B aligned", name, p);
    return RSK_OK;
}

}  // namespace rsk

using namespace rsk;

extern "C" {

int rsk_version(void) { return 105; }  // 1.05: rsk_check_ws_layout

int rsk_check_ws_layout(int32_t N, int32_t S, int32_t H) {
    RSK_CHECK(N > 0 && S > 0 && H >= 0, "bad sizes N=%d S=%d H=%d", N, S, H);
    return ws_check_u64(N, S, H);
}


int rsk_ctx_create(int device, rsk_ctx **out) {
    RSK_CHECK(out, "null output pointer");
    *out = nullptr;
    int n = 0;
    RSK_HIP(hipGetDeviceCount(&n));
    RSK_CHECK(device >= 0 && device < n, "device %d out of range (%d visible)", device, n);
    RSK_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    RSK_HIP(hipGetDeviceProperties(&prop, device));
    RSK_CHECK(std::strncmp(prop.gcnArchName, "gfx950", 6) == 0,
              "librsk is built for gfx950 (MI355X); device %d is %s", device, prop.gcnArchName);
    rsk_ctx *c = new rsk_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        set_error("hipStreamCreateWithFlags failed");
        return RSK_EHIP;
    }
    c->stream = c->own_stream;
    *out = c;
    return RSK_OK;
}

int rsk_ctx_destroy(rsk_ctx *ctx) {
    if (!ctx) return RSK_OK;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto &kv : ctx->pending)
        for (auto &e : kv.second) { (void)hipEventDestroy(e.start); (void)hipEventDestroy(e.stop); }
    for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
    for (auto &b : ctx->host_stage) b.release();
    for (auto &b : ctx->work) b.release();
    ctx->pin.release();
    ctx->errw.release();
    for (int i = 0; i < rsk_ctx::kAux; ++i)
        if (ctx->aux[i]) {
            (void)hipStreamSynchronize(ctx->aux[i]);
            (void)hipStreamDestroy(ctx->aux[i]);
            (void)hipEventDestroy(ctx->join[i]);
        }
    if (ctx->fork) (void)hipEventDestroy(ctx->fork);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
    return RSK_OK;
}

int rsk_ctx_set_stream(rsk_ctx *ctx, void *hip_stream) {
    RSK_CHECK(ctx, "null context");
    ctx->stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->own_stream;
    return RSK_OK;
}

int rsk_ctx_synchronize(rsk_ctx *ctx) {
    RSK_TRY(activate(ctx));
    RSK_HIP(hipStreamSynchronize(ctx->stream));
    return check_dev_err(ctx);
}

int rsk_ctx_set_profiling(rsk_ctx *ctx, int on) {
    RSK_CHECK(ctx, "null context");
    ctx->profiling = on != 0;
    return RSK_OK;
}

int rsk_ctx_kernel_time(rsk_ctx *ctx, const char *kernel, double *total_ms, int64_t *launches) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(kernel && total_ms && launches, "null argument");
    auto it = ctx->pending.find(kernel);
    if (it != ctx->pending.end()) {
        auto &acc = ctx->totals[kernel];
        for (auto &e : it->second) {
            RSK_HIP(hipEventSynchronize(e.stop));
            float ms = 0.f;
            RSK_HIP(hipEventElapsedTime(&ms, e.start, e.stop));
            acc.first += ms;
            acc.second += 1;
            ctx->event_pool.push_back(e.start);
            ctx->event_pool.push_back(e.stop);
        }
        it->second.clear();
    }
    auto t = ctx->totals.find(kernel);
    *total_ms = t == ctx->totals.end() ? 0.0 : t->second.first;
    *launches = t == ctx->totals.end() ? 0 : t->second.second;
    return RSK_OK;
}

int rsk_ctx_reset_profiling(rsk_ctx *ctx) {
    RSK_TRY(activate(ctx));
    RSK_HIP(hipStreamSynchronize(ctx->stream));
    for (auto &kv : ctx->pending)
        for (auto &e : kv.second) { ctx->event_pool.push_back(e.start); ctx->event_pool.push_back(e.stop); }
    ctx->pending.clear();
    ctx->totals.clear();
    return RSK_OK;
}

int rsk_ctx_set_profile_only(rsk_ctx *ctx, const char *kernel) {
    RSK_CHECK(ctx, "null context");
    ctx->profile_only = kernel ? kernel : "";
    return RSK_OK;
}

}  // extern "C"
