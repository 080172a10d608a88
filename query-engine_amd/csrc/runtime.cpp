// Context, caching device pool, per-thread errors and per-kernel timing of the
// qeh C ABI (include/qeh.h).  The reference executor takes no configuration and
// owns no device state (executor.rs:12-17); everything here is new runtime that
// an MI355X backend needs around its kernels.
#include "qeh_internal.h"

#include <cstdio>

namespace qeh {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int status, const std::string &msg) {
    g_last_error = msg;
    return status;
}

// ---- DevicePool ---------------------------------------------------------------
size_t DevicePool::size_class(size_t bytes) {
    if (bytes <= 256) return 256;
    if (bytes >= (size_t(1) << 30)) return (bytes + 0xFFFFF) & ~size_t(0xFFFFF);  // 1 MiB granules
    size_t c = 256;
    while (c < bytes) c <<= 1;
    return c;
}

DevicePool::~DevicePool() { trim(); }

int DevicePool::alloc(size_t bytes, void **out) {
    size_t cls = size_class(bytes);
    {
        std::lock_guard<std::mutex> g(mu_);
        auto it = free_.find(cls);
        if (it != free_.end()) {
            void *p = it->second;
            free_.erase(it);
            live_[p] = cls;
            in_use_ += cls;
            *out = p;
            return QEH_OK;
        }
    }
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, cls);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        trim();  // give cached blocks back and retry once
        e = hipMalloc(&p, cls);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return fail(QEH_E_OOM, "device allocation of " + std::to_string(bytes) + " bytes failed");
        }
    }
    std::lock_guard<std::mutex> g(mu_);
    live_[p] = cls;
    in_use_ += cls;
    *out = p;
    return QEH_OK;
}

int DevicePool::free(void *p) {
    if (!p) return QEH_OK;
    std::lock_guard<std::mutex> g(mu_);
    auto it = live_.find(p);
    if (it == live_.end()) return fail(QEH_E_INVALID, "qeh_device_free: pointer not owned by this context");
    free_.emplace(it->second, p);
    in_use_ -= it->second;
    live_.erase(it);
    return QEH_OK;
}

void DevicePool::trim() {
    std::lock_guard<std::mutex> g(mu_);
    for (auto &kv : free_) hipFree(kv.second);
    free_.clear();
}

// ---- timing --------------------------------------------------------------------
static hipEvent_t take_event(qeh_ctx *ctx) {
    if (!ctx->event_free.empty()) {
        hipEvent_t e = ctx->event_free.back();
        ctx->event_free.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    hipEventCreate(&e);
    return e;
}

KernelTimer::KernelTimer(qeh_ctx *c, const char *n, hipStream_t s) : ctx(c), name(n), stream(s ? s : c->stream) {
    if (!ctx->timing) return;
    a = take_event(ctx);
    b = take_event(ctx);
    hipEventRecord(a, stream);
}

KernelTimer::~KernelTimer() {
    if (!ctx->timing || !a) return;
    hipEventRecord(b, stream);
    ctx->timing_pending.push_back({name, a, b});
}

hipStream_t aux_stream(qeh_ctx *ctx) {
    if (!ctx->aux_stream) (void)hipStreamCreateWithFlags(&ctx->aux_stream, hipStreamNonBlocking);
    return ctx->aux_stream;
}

static void drain_timing(qeh_ctx *ctx) {
    for (auto &r : ctx->timing_pending) {
        hipEventSynchronize(r.stop);
        float ms = 0.f;
        hipEventElapsedTime(&ms, r.start, r.stop);
        auto &slot = ctx->timing_done[r.name];
        slot.first += ms;
        slot.second += 1;
        ctx->event_free.push_back(r.start);
        ctx->event_free.push_back(r.stop);
    }
    ctx->timing_pending.clear();
}

int read_small(qeh_ctx *ctx, void *host_dst, const void *dev_src, size_t bytes) {
    if (bytes == 0) return QEH_OK;
    if (bytes > ctx->pinned_bytes) {
        if (ctx->pinned) hipHostFree(ctx->pinned);
        ctx->pinned = nullptr;
        size_t n = bytes < 65536 ? 65536 : bytes;
        QEH_HIP(hipHostMalloc(&ctx->pinned, n, hipHostMallocDefault));
        ctx->pinned_bytes = n;
    }
    QEH_HIP(hipMemcpyAsync(ctx->pinned, dev_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    std::memcpy(host_dst, ctx->pinned, bytes);
    return QEH_OK;
}

int scratch_zeroed(qeh_ctx *ctx, size_t bytes, void **out) {
    bytes = (bytes + 255) & ~size_t(255);
    if (bytes > ctx->scratch_bytes) {
        if (ctx->scratch) ctx->pool->free(ctx->scratch);
        ctx->scratch = nullptr;
        size_t n = bytes < (1 << 20) ? (1 << 20) : bytes;
        QEH_TRY(ctx->pool->alloc(n, &ctx->scratch));
        ctx->scratch_bytes = n;
    }
    QEH_HIP(hipMemsetAsync(ctx->scratch, 0, bytes, ctx->stream));
    *out = ctx->scratch;
    return QEH_OK;
}

size_t dtype_size(int dt) {
    switch (dt) {
        case QEH_DT_INT32: return 4;
        case QEH_DT_UINT32: return 4;
        case QEH_DT_FLOAT32: return 4;
        case QEH_DT_INT64: return 8;
        case QEH_DT_FLOAT64: return 8;
        default: return 0;  // BOOL bit-packed, UTF8 variable, NULL none
    }
}

int alloc_column(qeh_ctx *ctx, int dtype, int64_t length, bool with_validity, qeh_column *out) {
    std::memset(out, 0, sizeof(*out));
    out->dtype = dtype;
    out->owned = 1;
    out->length = length;
    out->null_count = with_validity ? -1 : 0;
    size_t bytes;
    if (dtype == QEH_DT_BOOL) bytes = (size_t)((length + 63) / 64) * 8;
    else bytes = (size_t)length * dtype_size(dtype);
    if (bytes == 0) bytes = 8;
    QEH_TRY(ctx->pool->alloc(bytes, &out->values));
    if (with_validity) {
        size_t vb = (size_t)((length + 63) / 64) * 8;
        if (vb == 0) vb = 8;
        void *v = nullptr;
        int s = ctx->pool->alloc(vb, &v);
        if (s != QEH_OK) {
            ctx->pool->free(out->values);
            out->values = nullptr;
            return s;
        }
        out->validity = (uint8_t *)v;
    }
    return QEH_OK;
}

}  // namespace qeh

using namespace qeh;

extern "C" {

int qeh_abi_version(void) { return QEH_ABI_VERSION; }

const char *qeh_last_error(void) { return g_last_error.c_str(); }

int qeh_init(int device, qeh_ctx **out) {
    if (!out) return fail(QEH_E_INVALID, "qeh_init: out is NULL");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(QEH_E_HIP, "qeh_init: no HIP device available (" +
                                   std::string(hipGetErrorString(e)) + ")");
    if (device < 0 || device >= n) return fail(QEH_E_INVALID, "qeh_init: device out of range");
    QEH_HIP(hipSetDevice(device));
    qeh_ctx *ctx = new qeh_ctx();
    ctx->device = device;
    if (hipGetDeviceProperties(&ctx->props, device) != hipSuccess) {
        delete ctx;
        return fail(QEH_E_HIP, "qeh_init: hipGetDeviceProperties failed");
    }
    if (hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return fail(QEH_E_HIP, "qeh_init: stream creation failed");
    }
    ctx->stream = ctx->own_stream;
    ctx->pool = new DevicePool(device);
    *out = ctx;
    return QEH_OK;
}

int qeh_shutdown(qeh_ctx *ctx) {
    if (!ctx) return QEH_OK;
    DeviceGuard dg(ctx->device);
    hipStreamSynchronize(ctx->stream);
    for (auto &r : ctx->timing_pending) {
        hipEventDestroy(r.start);
        hipEventDestroy(r.stop);
    }
    for (auto e : ctx->event_free) hipEventDestroy(e);
    if (ctx->scratch) ctx->pool->free(ctx->scratch);
    // a prelaunched phase A may still have its plan's copy into pinned_plan queued: wait for it (and
    // return its buffers to the pool) before the pinned buffers go
    ctx->pending_slice.reset();
    if (ctx->aux_stream) hipStreamSynchronize(ctx->aux_stream);
    if (ctx->pinned_plan) hipHostFree(ctx->pinned_plan);
    if (ctx->pinned) hipHostFree(ctx->pinned);
    ctx->source_cache.reset();  // its columns go back to the pool first
    delete ctx->pool;
    if (ctx->own_stream) hipStreamDestroy(ctx->own_stream);
    if (ctx->aux_stream) {
        hipStreamSynchronize(ctx->aux_stream);
        hipStreamDestroy(ctx->aux_stream);
    }
    delete ctx;
    return QEH_OK;
}

int qeh_set_stream(qeh_ctx *ctx, void *hip_stream) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    ctx->stream = hip_stream ? (hipStream_t)hip_stream : ctx->own_stream;
    return QEH_OK;
}

void *qeh_get_stream(qeh_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int qeh_synchronize(qeh_ctx *ctx) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    DeviceGuard dg(ctx->device);
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    return QEH_OK;
}

int qeh_device_alloc(qeh_ctx *ctx, size_t bytes, void **out) {
    if (!ctx || !out) return fail(QEH_E_INVALID, "qeh_device_alloc: bad argument");
    DeviceGuard dg(ctx->device);
    return ctx->pool->alloc(bytes, out);
}

int qeh_device_free(qeh_ctx *ctx, void *ptr) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    return ctx->pool->free(ptr);
}

int qeh_pool_trim(qeh_ctx *ctx) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    DeviceGuard dg(ctx->device);
    hipStreamSynchronize(ctx->stream);
    ctx->pool->trim();
    return QEH_OK;
}

int qeh_memcpy_h2d(qeh_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    if (!bytes) return QEH_OK;
    DeviceGuard dg(ctx->device);
    QEH_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    return QEH_OK;
}

int qeh_memcpy_d2h(qeh_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    if (!bytes) return QEH_OK;
    DeviceGuard dg(ctx->device);
    QEH_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    return QEH_OK;
}

int qeh_memcpy_d2d(qeh_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    if (!bytes) return QEH_OK;
    DeviceGuard dg(ctx->device);
    QEH_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    return QEH_OK;
}

int qeh_memset(qeh_ctx *ctx, void *dst, int value, size_t bytes) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    DeviceGuard dg(ctx->device);
    QEH_HIP(hipMemsetAsync(dst, value, bytes, ctx->stream));
    return QEH_OK;
}

int qeh_column_release(qeh_ctx *ctx, qeh_column *col) {
    if (!ctx || !col) return fail(QEH_E_INVALID, "qeh_column_release: bad argument");
    if (col->owned) {
        if (col->values) ctx->pool->free(col->values);
        if (col->validity) ctx->pool->free(col->validity);
        if (col->offsets) ctx->pool->free(col->offsets);
    }
    std::memset(col, 0, sizeof(*col));
    return QEH_OK;
}

int qeh_timing_enable(qeh_ctx *ctx, int enable) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    ctx->timing = enable != 0;
    return QEH_OK;
}

int qeh_timing_reset(qeh_ctx *ctx) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    DeviceGuard dg(ctx->device);
    drain_timing(ctx);
    ctx->timing_done.clear();
    return QEH_OK;
}

int qeh_kernel_time(qeh_ctx *ctx, const char *name, double *total_ms, int64_t *launches) {
    if (!ctx || !name) return fail(QEH_E_INVALID, "qeh_kernel_time: bad argument");
    DeviceGuard dg(ctx->device);
    drain_timing(ctx);
    auto it = ctx->timing_done.find(name);
    if (total_ms) *total_ms = it == ctx->timing_done.end() ? 0.0 : it->second.first;
    if (launches) *launches = it == ctx->timing_done.end() ? 0 : it->second.second;
    return QEH_OK;
}

}  // extern "C"
