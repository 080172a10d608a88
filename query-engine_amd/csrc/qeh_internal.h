// Internal host-side runtime of the qeh backend: context, caching device pool,
// per-thread error string, launch/timing helpers.  Not part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/qeh.h"

namespace qeh {

// ---- errors ----------------------------------------------------------------
void set_error(const std::string &msg);
int fail(int status, const std::string &msg);

#define QEH_HIP(expr)                                                                       \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return ::qeh::fail(QEH_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

#define QEH_TRY(expr)               \
    do {                            \
        int _s = (expr);            \
        if (_s != QEH_OK) return _s; \
    } while (0)

// ---- caching device pool ----------------------------------------------------
// Size-class free lists (powers of two >= 256 B, exact size above 1 GiB).
// Freed blocks are kept for reuse so steady-state queries never call
// hipMalloc / hipFree (which would also serialise the device).
class DevicePool {
  public:
    explicit DevicePool(int device) : device_(device) {}
    int device() const { return device_; }
    ~DevicePool();
    int alloc(size_t bytes, void **out);
    int free(void *p);
    void trim();
    size_t bytes_in_use() const { return in_use_; }

  private:
    static size_t size_class(size_t bytes);
    int device_;
    std::mutex mu_;
    std::multimap<size_t, void *> free_;        // class size -> block
    std::unordered_map<void *, size_t> live_;   // block -> class size
    size_t in_use_ = 0;
};

// ---- per-kernel timing --------------------------------------------------------
struct TimingRecord {
    std::string name;
    hipEvent_t start, stop;
};

}  // namespace qeh

namespace qeh {
struct SourceCache;  // device-resident Scan inputs (executor.hip)
}

struct qeh_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    hipStream_t aux_stream = nullptr;  // second queue for overlapped pipeline stages (created on first use)
    qeh::DevicePool *pool = nullptr;
    hipDeviceProp_t props{};
    // small scratch (status words, counters, flags), zeroed per call
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
    // pinned host staging for small device->host results
    void *pinned = nullptr;
    size_t pinned_bytes = 0;
    // pinned host copy of a device-planned phase A's plan (queued ahead of phase A, so reading it
    // back does not wait behind work queued after phase A)
    void *pinned_plan = nullptr;
    // timing
    bool timing = false;
    std::vector<qeh::TimingRecord> timing_pending;
    std::vector<hipEvent_t> event_free;
    std::map<std::string, std::pair<double, int64_t>> timing_done;
    // Scan inputs kept on the device between queries (qeh_source.cache_key)
    std::shared_ptr<qeh::SourceCache> source_cache;
    // integer-column min/max already read during the current operator call (its input
    // columns are immutable for the call); on only inside a qeh::MinMaxMemoScope
    struct MinMaxMemoEntry {
        const void *values, *validity;
        int64_t offset, length;
        int32_t dtype;
        int64_t mn, mx, cnt;
    };
    bool mm_memo_on = false;
    int mm_memo_n = 0;
    MinMaxMemoEntry mm_memo[4];
    // set by the fused join-aggregate while its build runs beside a prelaunched phase A: probe
    // rows streaming meanwhile (build_join_table picks the XCD-split insert when it is long)
    int64_t build_beside_rows = 0;
    // phase A launched ahead by qeh_join_filter_aggregate_prelaunch (build-side ranges given by the
    // caller while the build columns are still in flight); adopted or discarded by the next
    // qeh_join_filter_aggregate (a qeh::PendingSlice)
    std::shared_ptr<void> pending_slice;
};

namespace qeh {

// Scoped device selection for every entry point.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

// Enables ctx->mm_memo for one operator call, so the build side reads each key column's
// range once (the prelaunch, the group table and the join table all need it).
struct MinMaxMemoScope {
    qeh_ctx *c;
    explicit MinMaxMemoScope(qeh_ctx *ctx) : c(ctx) { c->mm_memo_on = true, c->mm_memo_n = 0; }
    ~MinMaxMemoScope() { c->mm_memo_on = false, c->mm_memo_n = 0; }
};

// RAII device buffer from the pool.
struct DevBuf {
    qeh_ctx *ctx = nullptr;
    void *p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { reset(); }
    int alloc(qeh_ctx *c, size_t bytes) {
        reset();
        ctx = c;
        n = bytes;
        return c->pool->alloc(bytes ? bytes : 1, &p);
    }
    void reset() {
        if (p && ctx) ctx->pool->free(p);
        p = nullptr;
        n = 0;
    }
    void *release() {
        void *r = p;
        p = nullptr;
        return r;
    }
    template <class T>
    T *as() const { return reinterpret_cast<T *>(p); }
};

// Event bracketing for named kernels (only when ctx->timing).
struct KernelTimer {
    qeh_ctx *ctx;
    const char *name;
    hipStream_t stream;
    hipEvent_t a = nullptr, b = nullptr;
    KernelTimer(qeh_ctx *c, const char *n, hipStream_t s = nullptr);  // s: ctx->stream when null
    ~KernelTimer();
};

// The context's second queue (created on first use) for pipeline stages that overlap the main one.
hipStream_t aux_stream(qeh_ctx *ctx);

// Pinned staging for small D2H results.
int read_small(qeh_ctx *ctx, void *host_dst, const void *dev_src, size_t bytes);
// Zeroed scratch words (status / counters) valid until the next call.
int scratch_zeroed(qeh_ctx *ctx, size_t bytes, void **out);

// Grid sizing: persistent-ish grids of `per_cu` blocks per CU.
inline int grid_for(qeh_ctx *ctx, int64_t work_items, int items_per_block, int per_cu = 8) {
    int64_t want = (work_items + items_per_block - 1) / items_per_block;
    int64_t cap = (int64_t)ctx->props.multiProcessorCount * per_cu;
    if (want > cap) want = cap;
    if (want < 1) want = 1;
    return (int)want;
}

size_t dtype_size(int dt);
int alloc_column(qeh_ctx *ctx, int dtype, int64_t length, bool with_validity, qeh_column *out);

}  // namespace qeh
