// Shared kernels and host helpers: column views, device-wide scan, gather.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "device_common.h"
#include "ops.h"

namespace qeh {

ColRef make_colref(const qeh_column &c) {
    ColRef r{};
    r.dtype = c.dtype;
    r.validity = c.validity;
    r.vbit0 = c.offset;
    size_t es = dtype_size(c.dtype);
    if (c.dtype == QEH_DT_BOOL || c.dtype == QEH_DT_UTF8 || es == 0)
        r.values = c.values;  // bit-addressed (BOOL) or offsets-addressed (UTF8)
    else
        r.values = (const char *)c.values + (size_t)c.offset * es;
    return r;
}

int check_column(const qeh_column &c, const char *what) {
    if (c.length < 0) return fail(QEH_E_INVALID, std::string(what) + ": negative length");
    if (c.length > 0 && !c.values) return fail(QEH_E_INVALID, std::string(what) + ": null values pointer");
    if (c.length >= (int64_t)0xFFFFFFFFll)
        return fail(QEH_E_UNSUPPORTED, std::string(what) + ": more than 2^32-1 rows per column");
    switch (c.dtype) {
        case QEH_DT_BOOL: case QEH_DT_INT32: case QEH_DT_INT64: case QEH_DT_FLOAT32:
        case QEH_DT_FLOAT64: case QEH_DT_UINT32:
            return QEH_OK;
        case QEH_DT_UTF8:
            return QEH_OK;
        default:
            return fail(QEH_E_UNSUPPORTED, std::string(what) + ": unsupported column type");
    }
}

int make_colset(const qeh_column *cols, int n, ColSet *out) {
    if (n > kMaxCols)
        return fail(QEH_E_UNSUPPORTED, "too many columns for one device operator (max " +
                                           std::to_string(kMaxCols) + ")");
    std::memset(out, 0, sizeof(*out));
    out->n = n;
    for (int i = 0; i < n; ++i) {
        QEH_TRY(check_column(cols[i], "column"));
        out->c[i] = make_colref(cols[i]);
    }
    return QEH_OK;
}

int kernel_error_status(uint32_t err, const char *op) {
    if (err & kErrDiv0) return fail(QEH_E_DIV0, "Arrow error: Divide by zero error");
    if (err & kErrModOverflow)
        return fail(QEH_E_OVERFLOW, "attempt to calculate the remainder with overflow (the reference aborts here, operators.rs:720)");
    if (err & kErrOverflow) return fail(QEH_E_OVERFLOW, "Arrow error: Arithmetic overflow");
    if (err & kErrSpin) return fail(QEH_E_INTERNAL, std::string(op) + ": device protocol timeout");
    return QEH_OK;
}

int forced_table_kind() {
    const char *e = std::getenv("QEH_FORCE_TABLE");
    if (!e) return -1;
    if (!std::strcmp(e, "direct")) return TK_DIRECT;
    if (!std::strcmp(e, "packed")) return TK_PACKED;
    if (!std::strcmp(e, "wide")) return TK_WIDE;
    if (!std::strcmp(e, "bucket")) return TK_BUCKET;
    return -1;
}

// ---- exclusive scan --------------------------------------------------------------
constexpr int kScanItems = 4;                    // per thread
constexpr int kScanTile = kBlock * kScanItems;   // 1024 per block

__device__ __forceinline__ uint64_t block_excl_scan_u64(uint64_t v, uint64_t *lds_wave, uint64_t *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t t = __shfl_up(x, d, 64);
        if (lane >= d) x += t;
    }
    if (lane == 63) lds_wave[w] = x;
    __syncthreads();
    uint64_t base = 0, tot = 0;
    for (int i = 0; i < kBlock / 64; ++i) {
        if (i < w) base += lds_wave[i];
        tot += lds_wave[i];
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

__global__ void k_scan_partials(const uint32_t *__restrict__ in, int64_t n, uint64_t *__restrict__ partial) {
    __shared__ uint64_t lw[kBlock / 64];
    int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i)
        if (base + i < n) s += in[base + i];
    uint64_t tot;
    block_excl_scan_u64(s, lw, &tot);
    if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

// single block: exclusive scan of partial[0..nb) in place, total -> *total
__global__ void k_scan_top(uint64_t *partial, int64_t nb, uint64_t *total) {
    __shared__ uint64_t lw[kBlock / 64];
    uint64_t carry = 0;
    for (int64_t b0 = 0; b0 < nb; b0 += kBlock) {
        int64_t i = b0 + threadIdx.x;
        uint64_t v = i < nb ? partial[i] : 0;
        uint64_t tot;
        uint64_t ex = block_excl_scan_u64(v, lw, &tot);
        if (i < nb) partial[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ void k_scan_apply(const uint32_t *__restrict__ in, int64_t n, const uint64_t *__restrict__ partial,
                             uint64_t *__restrict__ out) {
    __shared__ uint64_t lw[kBlock / 64];
    int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        v[i] = base + i < n ? in[base + i] : 0;
        s += v[i];
    }
    uint64_t tot;
    uint64_t ex = block_excl_scan_u64(s, lw, &tot) + partial[blockIdx.x];
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        if (base + i < n) out[base + i] = ex;
        ex += v[i];
    }
}

// As exclusive_scan_u32, the total written to device memory (no host read); n > 0.
int exclusive_scan_u32_dev(qeh_ctx *ctx, const uint32_t *in, uint64_t *out, int64_t n, uint64_t *total_dev) {
    const int64_t nb = (n + kScanTile - 1) / kScanTile;
    DevBuf part;
    QEH_TRY(part.alloc(ctx, (size_t)nb * 8));
    {
        KernelTimer kt(ctx, "scan");
        hipLaunchKernelGGL(k_scan_partials, dim3((unsigned)nb), dim3(kBlock), 0, ctx->stream, in, n, part.as<uint64_t>());
        hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kBlock), 0, ctx->stream, part.as<uint64_t>(), nb, total_dev);
        hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)nb), dim3(kBlock), 0, ctx->stream, in, n, part.as<uint64_t>(), out);
    }
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

int exclusive_scan_u32(qeh_ctx *ctx, const uint32_t *in, uint64_t *out, int64_t n, uint64_t *total) {
    if (n <= 0) {
        if (total) *total = 0;
        return QEH_OK;
    }
    int64_t nb = (n + kScanTile - 1) / kScanTile;
    DevBuf part, tot;
    QEH_TRY(part.alloc(ctx, (size_t)nb * 8));
    QEH_TRY(tot.alloc(ctx, 8));
    {
        KernelTimer kt(ctx, "scan");
        hipLaunchKernelGGL(k_scan_partials, dim3((unsigned)nb), dim3(kBlock), 0, ctx->stream, in, n, part.as<uint64_t>());
        hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kBlock), 0, ctx->stream, part.as<uint64_t>(), nb, tot.as<uint64_t>());
        hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)nb), dim3(kBlock), 0, ctx->stream, in, n, part.as<uint64_t>(), out);
    }
    QEH_HIP(hipGetLastError());
    if (total) QEH_TRY(read_small(ctx, total, tot.p, 8));
    return QEH_OK;
}

// ---- gather --------------------------------------------------------------------
// out[i] = src[idx[i]]; one wave writes 64 consecutive rows so that the
// validity / boolean words are produced by a single ballot.
template <typename T>
__global__ void k_gather(ColRef src, const uint32_t *__restrict__ idx, int64_t m, T *__restrict__ out,
                         uint64_t *__restrict__ out_valid) {
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
    const int lane = threadIdx.x & 63;
    for (int64_t w = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); w * 64 < m; w += nwaves) {
        int64_t i = w * 64 + lane;
        bool live = i < m;
        uint32_t j = live ? idx[i] : 0;
        const bool hit = live && j != kNullRow;  // kNullRow: outer-join filler -> NULL
        bool valid = hit && col_valid(src, j);
        if (live) out[i] = hit ? ((const T *)src.values)[j] : T(0);
        if (out_valid) {
            uint64_t b = __ballot(valid);
            if (lane == 0) out_valid[w] = b;
        }
    }
}

__global__ void k_gather_bool(ColRef src, const uint32_t *__restrict__ idx, int64_t m, uint64_t *__restrict__ out,
                              uint64_t *__restrict__ out_valid) {
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
    const int lane = threadIdx.x & 63;
    for (int64_t w = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); w * 64 < m; w += nwaves) {
        int64_t i = w * 64 + lane;
        bool live = i < m;
        uint32_t j = live ? idx[i] : 0;
        const bool hit = live && j != kNullRow;
        bool v = hit && bit_at((const uint8_t *)src.values, src.vbit0 + j);
        bool valid = hit && col_valid(src, j);
        uint64_t bv = __ballot(v), bn = __ballot(valid);
        if (lane == 0) {
            out[w] = bv;
            if (out_valid) out_valid[w] = bn;
        }
    }
}

// ---- Utf8 gather: lengths -> scan -> offsets -> byte copy --------------------------
__global__ void k_utf8_lengths(const int32_t *__restrict__ offs, int64_t off0, const uint32_t *__restrict__ idx, int64_t m,
                               uint32_t *__restrict__ len) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        if (idx[i] == kNullRow) {
            len[i] = 0;
            continue;
        }
        const int64_t r = off0 + idx[i];
        len[i] = (uint32_t)(offs[r + 1] - offs[r]);
    }
}

__global__ void k_utf8_offsets(const uint64_t *__restrict__ excl, int64_t m, uint64_t total, int32_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= m; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (int32_t)(i < m ? excl[i] : total);
}

// one wave per row: lanes copy the row's bytes
__global__ void k_utf8_copy(const int32_t *__restrict__ offs, int64_t off0, const uint8_t *__restrict__ data,
                            const uint32_t *__restrict__ idx, int64_t m, const int32_t *__restrict__ out_offs,
                            uint8_t *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t w = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); w < m; w += nw) {
        if (idx[w] == kNullRow) continue;
        const int64_t r = off0 + idx[w];
        const int32_t s = offs[r], e = offs[r + 1], d = out_offs[w];
        for (int32_t b = lane; b < e - s; b += 64) out[d + b] = data[s + b];
    }
}

// validity bits of gathered rows (kNullRow -> NULL)
__global__ void k_gather_valid(ColRef src, const uint32_t *__restrict__ idx, int64_t m, uint64_t *__restrict__ out_valid) {
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
    const int lane = threadIdx.x & 63;
    for (int64_t w = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); w * 64 < m; w += nwaves) {
        const int64_t i = w * 64 + lane;
        const uint32_t j = i < m ? idx[i] : kNullRow;
        const uint64_t b = __ballot(j != kNullRow && col_valid(src, j));
        if (lane == 0) out_valid[w] = b;
    }
}

static int gather_utf8(qeh_ctx *ctx, const qeh_column &src, const uint32_t *idx, int64_t m, qeh_column *out,
                       bool nullable_idx) {
    std::memset(out, 0, sizeof(*out));
    out->dtype = QEH_DT_UTF8;
    out->owned = 1;
    out->length = m;
    DevBuf len, excl;
    QEH_TRY(len.alloc(ctx, (size_t)std::max<int64_t>(m, 1) * 4));
    QEH_TRY(excl.alloc(ctx, (size_t)std::max<int64_t>(m, 1) * 8));
    const int grid = grid_for(ctx, m + 1, kBlock * 4, 8);
    if (m > 0)
        hipLaunchKernelGGL(k_utf8_lengths, dim3(grid), dim3(kBlock), 0, ctx->stream, src.offsets, src.offset, idx, m,
                           len.as<uint32_t>());
    uint64_t total = 0;
    QEH_TRY(exclusive_scan_u32(ctx, len.as<uint32_t>(), excl.as<uint64_t>(), m, &total));
    if (total > 0x7FFFFFFFull) return fail(QEH_E_UNSUPPORTED, "Utf8 output larger than 2 GiB (Arrow Utf8 uses int32 offsets)");
    void *o = nullptr, *d = nullptr;
    QEH_TRY(ctx->pool->alloc((size_t)(m + 1) * 4, &o));
    int s = ctx->pool->alloc(std::max<size_t>(total, 8), &d);
    if (s != QEH_OK) {
        ctx->pool->free(o);
        return s;
    }
    out->offsets = (int32_t *)o;
    out->values = d;
    out->values_bytes = (int64_t)total;
    hipLaunchKernelGGL(k_utf8_offsets, dim3(grid), dim3(kBlock), 0, ctx->stream, excl.as<uint64_t>(), m, total, out->offsets);
    if (m > 0)
        hipLaunchKernelGGL(k_utf8_copy, dim3(grid_for(ctx, m, kBlock / 64, 8)), dim3(kBlock), 0, ctx->stream, src.offsets,
                           src.offset, (const uint8_t *)src.values, idx, m, out->offsets, (uint8_t *)out->values);
    if (src.validity || nullable_idx) {
        void *v = nullptr;
        const size_t vb = std::max<size_t>(((size_t)(m + 63) / 64) * 8, 8);
        QEH_TRY(ctx->pool->alloc(vb, &v));
        out->validity = (uint8_t *)v;
        out->null_count = -1;
        if (m > 0)
            hipLaunchKernelGGL(k_gather_valid, dim3(grid_for(ctx, (m + 63) / 64, kBlock / 64, 8)), dim3(kBlock), 0,
                               ctx->stream, make_colref(src), idx, m, (uint64_t *)out->validity);
    } else {
        out->null_count = 0;
    }
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

int gather_column(qeh_ctx *ctx, const qeh_column &src, const uint32_t *idx, int64_t m, qeh_column *out,
                  bool nullable_idx) {
    QEH_TRY(check_column(src, "gather"));
    if (src.dtype == QEH_DT_UTF8) return gather_utf8(ctx, src, idx, m, out, nullable_idx);
    bool with_valid = src.validity != nullptr || nullable_idx;
    QEH_TRY(alloc_column(ctx, src.dtype, m, with_valid, out));
    if (m == 0) return QEH_OK;
    ColRef s = make_colref(src);
    int grid = grid_for(ctx, (m + 63) / 64, kBlock / 64, 8);
    KernelTimer kt(ctx, "gather");
    switch (src.dtype) {
        case QEH_DT_BOOL:
            hipLaunchKernelGGL(k_gather_bool, dim3(grid), dim3(kBlock), 0, ctx->stream, s, idx, m,
                               (uint64_t *)out->values, (uint64_t *)out->validity);
            break;
        case QEH_DT_INT32: case QEH_DT_FLOAT32: case QEH_DT_UINT32:
            hipLaunchKernelGGL(k_gather<uint32_t>, dim3(grid), dim3(kBlock), 0, ctx->stream, s, idx, m,
                               (uint32_t *)out->values, (uint64_t *)out->validity);
            break;
        default:
            hipLaunchKernelGGL(k_gather<uint64_t>, dim3(grid), dim3(kBlock), 0, ctx->stream, s, idx, m,
                               (uint64_t *)out->values, (uint64_t *)out->validity);
            break;
    }
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

}  // namespace qeh

namespace qeh {
__global__ void k_valid_bytes(ColRef c, int64_t n, uint8_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = col_valid(c, i) ? 1 : 0;
}

__global__ void k_bytes_valid(const uint8_t *__restrict__ in, int64_t n, uint64_t *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t w = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); w * 64 < n; w += nw) {
        const int64_t i = w * 64 + lane;
        const uint64_t b = __ballot(i < n && in[i] != 0);
        if (lane == 0) out[w] = b;
    }
}
}  // namespace qeh

extern "C" int qeh_validity_to_bytes(qeh_ctx *ctx, const qeh_column *col, uint8_t *out_bytes) {
    using namespace qeh;
    if (!ctx || !col || (col->length > 0 && !out_bytes)) return fail(QEH_E_INVALID, "qeh_validity_to_bytes: bad argument");
    DeviceGuard dg(ctx->device);
    if (col->length == 0) return QEH_OK;
    hipLaunchKernelGGL(k_valid_bytes, dim3(grid_for(ctx, col->length, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream,
                       make_colref(*col), col->length, out_bytes);
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

extern "C" int qeh_bytes_to_validity(qeh_ctx *ctx, const uint8_t *bytes, int64_t n, uint8_t *out_bitmap) {
    using namespace qeh;
    if (!ctx || (n > 0 && (!bytes || !out_bitmap))) return fail(QEH_E_INVALID, "qeh_bytes_to_validity: bad argument");
    DeviceGuard dg(ctx->device);
    if (n == 0) return QEH_OK;
    hipLaunchKernelGGL(k_bytes_valid, dim3(grid_for(ctx, (n + 63) / 64, kBlock / 64, 8)), dim3(kBlock), 0, ctx->stream,
                       bytes, n, (uint64_t *)out_bitmap);
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

namespace qeh {

// ---- self-check of the stable LDS-atomic tile ranking -----------------------------------------
// The stable partition passes (k_rs_scatter, k_part_scatter_small, the window passes) rank a tile's
// rows per digit with one returning LDS atomic per row; that rank is stable only if ds_add_rtn serves
// the lanes of one instruction that hit the same word in lane order.  This kernel checks exactly that
// on the running device, in both forms the passes use (a u32 counter per digit, and two u16 counters
// packed per word), against ranks computed by ballot matching; the host falls back to the ballot
// ranking when any rank differs.
namespace {
constexpr int kRcBlock = 512, kRcRounds = 8, kRcDig = 1024;
__device__ __forceinline__ uint32_t rc_digit(int pat, int w, int j, int lane) {
    uint64_t z = ((uint64_t)pat << 48) ^ ((uint64_t)w << 24) ^ ((uint64_t)j << 8) ^ (uint64_t)lane;
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const uint32_t masks[4] = {kRcDig - 1, 63u, 3u, 0u};  // uniform, narrow, hot and single-digit patterns
    return (uint32_t)z & masks[pat & 3];
}
}  // namespace

__global__ __launch_bounds__(kRcBlock) void k_lds_rank_check(uint32_t *__restrict__ bad) {
    __shared__ uint32_t c32[kRcBlock / 64][kRcDig];       // u32 counter per digit (k_rs_scatter form)
    __shared__ uint32_t c16[kRcBlock / 64][kRcDig / 2];   // u16 halves packed per word (window form)
    __shared__ uint32_t ref[kRcBlock / 64][kRcDig];       // rows of each digit ranked so far (ballot)
    __shared__ uint32_t nbad;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) nbad = 0;
    uint32_t miss = 0;
    for (int pat = 0; pat < 4; ++pat) {
        for (int i = lane; i < kRcDig; i += 64) c32[wave][i] = 0, ref[wave][i] = 0;
        for (int i = lane; i < kRcDig / 2; i += 64) c16[wave][i] = 0;
        __syncthreads();
        for (int j = 0; j < kRcRounds; ++j) {
            const uint32_t d = rc_digit(pat, blockIdx.x * (kRcBlock / 64) + wave, j, lane);
            const uint32_t r32 = atomicAdd(&c32[wave][d], 1u);
            const uint32_t sh = (d & 1u) * 16u;
            const uint32_t r16 = (atomicAdd(&c16[wave][d >> 1], 1u << sh) >> sh) & 0xFFFFu;
            // lanes of this round with the same digit, by ballot over the digit bits
            uint64_t m = ~0ull;
            for (int b = 0; b < 10; ++b) {
                const uint64_t bl = __ballot(((d >> b) & 1u) != 0);
                m &= ((d >> b) & 1u) ? bl : ~bl;
            }
            const uint32_t before = ref[wave][d];
            const uint32_t want = before + mbcnt(m);
            __builtin_amdgcn_s_waitcnt(0xc07f);  // every lane read ref before the group's last lane updates it
            __builtin_amdgcn_wave_barrier();
            if (mbcnt(m) + 1u == (uint32_t)popc64(m)) ref[wave][d] = before + (uint32_t)popc64(m);
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            miss += (r32 != want) + (r16 != want);
        }
        __syncthreads();
    }
    if (miss) atomicAdd(&nbad, miss);
    __syncthreads();
    if (threadIdx.x == 0) bad[blockIdx.x] = nbad;
}

// true when the device ranks stably by LDS atomics; checked once per process (first caller's device)
bool lds_atomic_rank_ok(qeh_ctx *ctx) {
    // cached per device, and only once the check kernel has run to the end: a failed allocation,
    // launch or sync returns false for this call and leaves the next call to retry
    constexpr int kMaxDev = 64;
    static int state[kMaxDev];  // 0 unknown, 1 fall back to ballot, 2 atomics are lane-ordered
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    const int dev = ctx->device >= 0 && ctx->device < kMaxDev ? ctx->device : 0;
    if (state[dev]) return state[dev] == 2;
    constexpr int blocks = 64;
    DevBuf bad;
    if (bad.alloc(ctx, blocks * 4) != QEH_OK) return false;
    hipLaunchKernelGGL(k_lds_rank_check, dim3(blocks), dim3(kRcBlock), 0, ctx->stream, bad.as<uint32_t>());
    uint32_t h[blocks];
    if (hipGetLastError() != hipSuccess || hipMemcpyAsync(h, bad.p, sizeof h, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess)
        return false;
    uint64_t tot = 0;
    for (int i = 0; i < blocks; ++i) tot += h[i];
    state[dev] = tot == 0 ? 2 : 1;
    return state[dev] == 2;
}

}  // namespace qeh

extern "C" int qeh_lds_atomic_rank_ok(qeh_ctx *ctx) {
    using namespace qeh;
    if (!ctx) return fail(QEH_E_INVALID, "qeh_lds_atomic_rank_ok: bad argument");
    DeviceGuard dg(ctx->device);
    return lds_atomic_rank_ok(ctx) ? 1 : 0;
}
