// Merge of partition results (crates/query-distributed/src/operators.rs:75-224).
//
// Merge::execute combines the batches every partition produced: Concat
// flattens them (:139-141), SortedMerge concatenates (arrow concat_batches,
// :206-216) and lexsorts the result by the named columns with per-column
// descending / nulls_first options (:143-193), UnionDistinct is a plain
// concatenation in the reference (:196-204).  On the device a partition's
// columns are HBM-resident qeh_columns; the concatenation is one copy per
// buffer (values with a device memcpy, validity / boolean bits re-aligned by a
// word kernel, Utf8 offsets re-based), the sort is the LSD radix sort of
// k_sort.hip with the per-key NULL placement, and the rows leave through one
// gather per column.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "device_common.h"
#include "ops.h"

namespace qeh {

// dst bits [dst0, dst0 + n) = src bits [src0, src0 + n) (src NULL: all ones).  One thread per
// 32-bit destination word; the first and last word may be shared with the neighbouring parts
// (atomicOr into a zeroed bitmap), interior words are stored whole.
__global__ void k_concat_bits(const uint8_t *__restrict__ src, int64_t src0, int64_t n, uint32_t *__restrict__ dst,
                              int64_t dst0) {
    const int64_t w0 = dst0 >> 5, w1 = (dst0 + n - 1) >> 5;
    for (int64_t w = w0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w <= w1; w += (int64_t)gridDim.x * blockDim.x) {
        uint32_t v = 0;
        for (int b = 0; b < 32; ++b) {
            const int64_t d = (w << 5) + b;
            if (d < dst0 || d >= dst0 + n) continue;
            if (!src || bit_at(src, src0 + (d - dst0))) v |= 1u << b;
        }
        if (w == w0 || w == w1) atomicOr(&dst[w], v);
        else dst[w] = v;
    }
}

__global__ void k_rebase_offsets(const int32_t *__restrict__ src, int64_t n, int32_t base, int32_t *__restrict__ dst) {
    const int32_t s0 = src[0];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[i] - s0 + base;
}

int concat_columns(qeh_ctx *ctx, const qeh_column *const *parts, int n_parts, qeh_column *out) {
    std::memset(out, 0, sizeof(*out));
    if (n_parts <= 0) return fail(QEH_E_INVALID, "concat: no parts");
    const int dt = parts[0]->dtype;
    int64_t total = 0, nulls = 0;
    bool any_valid = false, nulls_known = true;
    for (int p = 0; p < n_parts; ++p) {
        QEH_TRY(check_column(*parts[p], "concat"));
        if (parts[p]->dtype != dt) return fail(QEH_E_INVALID, "concat: parts have different types");
        total += parts[p]->length;
        if (parts[p]->validity) {
            any_valid = true;
            if (parts[p]->null_count < 0) nulls_known = false;
            else nulls += parts[p]->null_count;
        }
    }
    if (dt == QEH_DT_UTF8) {
        out->dtype = QEH_DT_UTF8;
        out->owned = 1;
        out->length = total;
        std::vector<int64_t> lo(n_parts), hi(n_parts);
        int64_t bytes = 0;
        for (int p = 0; p < n_parts; ++p) {
            int32_t e[2] = {0, 0};
            if (parts[p]->length > 0) {
                QEH_TRY(read_small(ctx, &e[0], parts[p]->offsets + parts[p]->offset, 4));
                QEH_TRY(read_small(ctx, &e[1], parts[p]->offsets + parts[p]->offset + parts[p]->length, 4));
            }
            lo[p] = e[0];
            hi[p] = e[1];
            bytes += e[1] - e[0];
        }
        if (bytes > 0x7FFFFFFF) return fail(QEH_E_UNSUPPORTED, "Utf8 output larger than 2 GiB (Arrow Utf8 uses int32 offsets)");
        void *o = nullptr, *d = nullptr;
        QEH_TRY(ctx->pool->alloc((size_t)(total + 1) * 4, &o));
        int s = ctx->pool->alloc(std::max<size_t>((size_t)bytes, 8), &d);
        if (s != QEH_OK) {
            ctx->pool->free(o);
            return s;
        }
        out->offsets = (int32_t *)o;
        out->values = d;
        out->values_bytes = bytes;
        QEH_HIP(hipMemsetAsync(o, 0, 4, ctx->stream));  // offsets[0] = 0 (also for total == 0)
        int64_t row = 0, at = 0;
        for (int p = 0; p < n_parts; ++p) {
            const qeh_column &c = *parts[p];
            if (c.length > 0) {
                hipLaunchKernelGGL(k_rebase_offsets, dim3(grid_for(ctx, c.length + 1, kBlock * 4, 8)), dim3(kBlock), 0,
                                   ctx->stream, c.offsets + c.offset, c.length, (int32_t)at, out->offsets + row);
                if (hi[p] > lo[p])
                    QEH_HIP(hipMemcpyAsync((uint8_t *)d + at, (const uint8_t *)c.values + lo[p], (size_t)(hi[p] - lo[p]),
                                           hipMemcpyDeviceToDevice, ctx->stream));
            }
            row += c.length;
            at += hi[p] - lo[p];
        }
    } else {
        QEH_TRY(alloc_column(ctx, dt, total, any_valid, out));
        const size_t words = ((size_t)(total + 63) / 64) * 8;
        if (dt == QEH_DT_BOOL) QEH_HIP(hipMemsetAsync(out->values, 0, std::max<size_t>(words, 8), ctx->stream));
        const size_t es = dtype_size(dt);
        int64_t row = 0;
        for (int p = 0; p < n_parts; ++p) {
            const qeh_column &c = *parts[p];
            if (c.length > 0) {
                if (dt == QEH_DT_BOOL)
                    hipLaunchKernelGGL(k_concat_bits, dim3(grid_for(ctx, c.length / 32 + 2, kBlock, 8)), dim3(kBlock), 0,
                                       ctx->stream, (const uint8_t *)c.values, c.offset, c.length, (uint32_t *)out->values,
                                       row);
                else
                    QEH_HIP(hipMemcpyAsync((uint8_t *)out->values + (size_t)row * es,
                                           (const uint8_t *)c.values + (size_t)c.offset * es, (size_t)c.length * es,
                                           hipMemcpyDeviceToDevice, ctx->stream));
            }
            row += c.length;
        }
    }
    if (any_valid) {
        if (!out->validity) {
            void *v = nullptr;
            QEH_TRY(ctx->pool->alloc(std::max<size_t>(((size_t)(total + 63) / 64) * 8, 8), &v));
            out->validity = (uint8_t *)v;
        }
        QEH_HIP(hipMemsetAsync(out->validity, 0, std::max<size_t>(((size_t)(total + 63) / 64) * 8, 8), ctx->stream));
        int64_t row = 0;
        for (int p = 0; p < n_parts; ++p) {
            const qeh_column &c = *parts[p];
            if (c.length > 0)
                hipLaunchKernelGGL(k_concat_bits, dim3(grid_for(ctx, c.length / 32 + 2, kBlock, 8)), dim3(kBlock), 0,
                                   ctx->stream, c.validity, c.offset, c.length, (uint32_t *)out->validity, row);
            row += c.length;
        }
        out->null_count = nulls_known ? nulls : -1;
    } else {
        out->null_count = 0;
    }
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

}  // namespace qeh

using namespace qeh;

extern "C" int qeh_concat(qeh_ctx *ctx, const qeh_column *parts, int n_parts, qeh_column *out) {
    if (!ctx || !parts || !out || n_parts <= 0) return fail(QEH_E_INVALID, "qeh_concat: bad argument");
    DeviceGuard dg(ctx->device);
    std::vector<const qeh_column *> pp(n_parts);
    for (int p = 0; p < n_parts; ++p) pp[p] = &parts[p];
    QEH_TRY(concat_columns(ctx, pp.data(), n_parts, out));
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    return QEH_OK;
}

extern "C" int qeh_merge_sorted(qeh_ctx *ctx, const qeh_column *parts, int n_parts, int n_cols, const int32_t *key_idx,
                                const int8_t *ascending, const int8_t *nulls_first, int n_keys, qeh_column *out,
                                int64_t *out_rows) {
    if (!ctx || !out_rows || n_parts < 0 || n_cols <= 0 || !out || (n_parts > 0 && !parts) || (n_keys > 0 && !key_idx))
        return fail(QEH_E_INVALID, "qeh_merge_sorted: bad argument");
    *out_rows = 0;
    if (n_parts == 0) return fail(QEH_E_INVALID, "qeh_merge_sorted: no partitions (the reference returns no batches)");
    for (int k = 0; k < n_keys; ++k)
        if (key_idx[k] < 0 || key_idx[k] >= n_cols) return fail(QEH_E_INVALID, "qeh_merge_sorted: sort column out of range");
    DeviceGuard dg(ctx->device);
    if (n_keys == 1 && n_cols == 2 && n_parts <= 16) {
        // one key and one 8-byte payload: the payload rides through the radix passes (no gathers), and the
        // first pass reads the partitions in place -- the concatenation (operators.rs:206-216) is never
        // materialised
        const int kj = key_idx[0], vj = 1 - key_idx[0];
        std::vector<qeh_column> kp(n_parts), vp(n_parts);
        bool ok = true;
        for (int p = 0; p < n_parts; ++p) {
            kp[p] = parts[(size_t)p * n_cols + kj];
            vp[p] = parts[(size_t)p * n_cols + vj];
            ok = ok && check_column(kp[p], "merge key") == QEH_OK && check_column(vp[p], "merge column") == QEH_OK;
        }
        qeh_column ok_{}, ov{};
        const int ps = ok ? sort_pairs_payload_parts(ctx, kp.data(), vp.data(), n_parts, ascending ? ascending[0] != 0 : true,
                                                     nulls_first ? nulls_first[0] != 0 : true, &ok_, &ov)
                          : kPayloadSortNotEligible;
        if (ps != kPayloadSortNotEligible) {
            QEH_TRY(ps);
            out[kj] = ok_;
            out[vj] = ov;
            *out_rows = ok_.length;
            return QEH_OK;
        }
    }
    // concat_batches (operators.rs:206-216): parts is [n_parts][n_cols], row-major by partition
    std::vector<qeh_column> cat(n_cols);
    int made = 0, s = QEH_OK;
    {
        KernelTimer kt(ctx, "merge_concat");  // (part of Merge::sorted's device time: tools/bench_configs.py cfg_merge)
        for (int j = 0; j < n_cols && s == QEH_OK; ++j) {
            std::vector<const qeh_column *> pp(n_parts);
            for (int p = 0; p < n_parts; ++p) pp[p] = &parts[(size_t)p * n_cols + j];
            s = concat_columns(ctx, pp.data(), n_parts, &cat[j]);
            if (s == QEH_OK) ++made;
        }
    }
    auto release_cat = [&]() {
        for (int j = 0; j < made; ++j) qeh_column_release(ctx, &cat[j]);
    };
    if (s != QEH_OK) {
        release_cat();
        return s;
    }
    const int64_t n = cat[0].length;
    if (n_keys == 0) {  // no named sort column resolved: the concatenation (operators.rs:181-183)
        for (int j = 0; j < n_cols; ++j) out[j] = cat[j];
        QEH_HIP(hipStreamSynchronize(ctx->stream));
        *out_rows = n;
        return QEH_OK;
    }
    if (n_keys == 1 && n_cols == 2) {
        // one key and one 8-byte payload: the payload rides through the radix passes (no gathers)
        const int kj = key_idx[0], vj = 1 - key_idx[0];
        qeh_column ok{}, ov{};
        const int ps = sort_pairs_payload(ctx, cat[kj], cat[vj], ascending ? ascending[0] != 0 : true,
                                          nulls_first ? nulls_first[0] != 0 : true, &ok, &ov);
        if (ps != kPayloadSortNotEligible) {
            release_cat();
            QEH_TRY(ps);
            out[kj] = ok;
            out[vj] = ov;
            *out_rows = n;
            return QEH_OK;
        }
    }
    std::vector<qeh_column> keys(n_keys);
    for (int k = 0; k < n_keys; ++k) keys[k] = cat[key_idx[k]];
    qeh_column perm{};
    s = qeh_sort_indices_nulls(ctx, keys.data(), n_keys, ascending, nulls_first, &perm);
    int taken = 0;
    for (int j = 0; j < n_cols && s == QEH_OK; ++j) {
        s = gather_column(ctx, cat[j], (const uint32_t *)perm.values, n, &out[j]);
        if (s == QEH_OK) ++taken;
    }
    if (s == QEH_OK) {
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) s = fail(QEH_E_HIP, std::string("merge: ") + hipGetErrorString(e));
    }
    if (perm.owned) qeh_column_release(ctx, &perm);
    release_cat();
    if (s != QEH_OK) {
        for (int j = 0; j < taken; ++j) qeh_column_release(ctx, &out[j]);
        return s;
    }
    *out_rows = n;
    return QEH_OK;
}
