// Result encoding after the path: PostgreSQL DataRow
// messages in text format, as the reference's pgwire front end builds them
// (crates/query-pgwire/src/result.rs:56-176: one DataRowEncoder per row,
// encode_value per cell; pgwire 0.28.0 renders each value with Rust's
// Display, fmt_float.h).  Message: 'D', Int32 length (self-inclusive), Int16
// field count, then per field Int32 length (-1 = NULL) and the text, all
// big-endian.
//
// Two passes over the rows: every thread measures its row (the formatter
// runs in length-only mode), an exclusive scan places the rows, and the same
// code writes them.  The output is one Utf8 column whose i-th string is row
// i's complete DataRow message, so the buffer can go to the socket as is.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "device_common.h"
#include "fmt_float.h"
#include "ops.h"

namespace qeh {

constexpr int kEncMaxCols = 32;

struct EncCol {
    ColRef c;
    const int32_t *offs;  // Utf8: offsets (already advanced by the column offset)
    const uint8_t *data;
};
struct EncCols {
    EncCol col[kEncMaxCols];
    int32_t n;
};

__device__ inline void put_be32(char *p, int32_t v) {
    p[0] = (char)((uint32_t)v >> 24);
    p[1] = (char)((uint32_t)v >> 16);
    p[2] = (char)((uint32_t)v >> 8);
    p[3] = (char)(uint32_t)v;
}

// text of one cell at out (nullptr: length only); -1 for NULL
__device__ inline int enc_cell(const EncCol &e, int64_t row, char *out) {
    if (!col_valid(e.c, row)) return -1;
    switch (e.c.dtype) {
        case QEH_DT_BOOL:
            if (out) out[0] = bit_at((const uint8_t *)e.c.values, e.c.vbit0 + row) ? 't' : 'f';
            return 1;
        case QEH_DT_INT32: case QEH_DT_INT64: case QEH_DT_UINT32:
            return fmt_i64(out, load_i64(e.c, row));
        case QEH_DT_FLOAT32:
            return fmt_f32(out, ((const float *)e.c.values)[row]);
        case QEH_DT_FLOAT64:
            return fmt_f64(out, ((const double *)e.c.values)[row]);
        case QEH_DT_UTF8: {
            const int32_t s = e.offs[row], t = e.offs[row + 1];
            if (out)
                for (int32_t i = s; i < t; ++i) out[i - s] = (char)e.data[i];
            return t - s;
        }
        default: return 0;
    }
}

__global__ void k_pg_row_len(EncCols cols, int64_t n, uint32_t *__restrict__ len) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        uint32_t l = 1 + 4 + 2;
        for (int j = 0; j < cols.n; ++j) {
            const int c = enc_cell(cols.col[j], r, nullptr);
            l += 4 + (c > 0 ? (uint32_t)c : 0u);
        }
        len[r] = l;
    }
}

__device__ inline void pg_write_row(const EncCols &cols, int64_t r, char *p, uint32_t bytes) {
    p[0] = 'D';
    put_be32(p + 1, (int32_t)(bytes - 1));
    p[5] = (char)(cols.n >> 8);
    p[6] = (char)cols.n;
    char *q = p + 7;
    for (int j = 0; j < cols.n; ++j) {
        const int c = enc_cell(cols.col[j], r, q + 4);
        put_be32(q, c);
        q += 4 + (c > 0 ? c : 0);
    }
}

// One workgroup per 256 rows: the rows are rendered into LDS at their relative offsets, then the
// workgroup's contiguous byte range leaves with coalesced 4-byte stores (a row-per-thread direct
// write would scatter ~50-byte pieces).  Ranges larger than the LDS stage are written directly.
// LDS = the stage's bytes: 16 KB (rows averaging <= 56 B: more workgroups per CU for the formatting
// work; a workgroup whose rows overflow it writes directly) or 48 KB.
template <int LDS>
__global__ __launch_bounds__(kBlock, 6) void k_pg_row_write(EncCols cols, int64_t n, const uint64_t *__restrict__ at,
                                                         const uint32_t *__restrict__ len, char *__restrict__ out,
                                                         int32_t *__restrict__ out_offs, uint64_t total) {
    constexpr int kEncLds = LDS;
    __shared__ __attribute__((aligned(16))) char stage[kEncLds + 16];
    for (int64_t b0 = (int64_t)blockIdx.x * kBlock; b0 < n; b0 += (int64_t)gridDim.x * kBlock) {
        const int64_t r = b0 + threadIdx.x;
        const uint64_t base = at[b0];
        const uint64_t end = b0 + kBlock < n ? at[b0 + kBlock] : total;
        const uint64_t span = end - base;
        if (r < n) out_offs[r] = (int32_t)at[r];
        if (r == n - 1) out_offs[n] = (int32_t)total;
        if (span > (uint64_t)kEncLds) {  // wide rows: direct
            if (r < n) pg_write_row(cols, r, out + at[r], len[r]);
            continue;
        }
        // stage at the destination's 16-B alignment so that whole 16-B pieces can be stored
        const uint32_t lead = (uint32_t)(base & 15);
        if (r < n) pg_write_row(cols, r, stage + lead + (at[r] - base), len[r]);
        __syncthreads();
        const uint32_t head = lead ? 16 - lead : 0;  // bytes before the first aligned 16-B piece
        const uint32_t h = (uint32_t)(head < span ? head : span);
        if (threadIdx.x < h) out[base + threadIdx.x] = stage[lead + threadIdx.x];
        const uint32_t body = (uint32_t)(span - h) / 16;
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        v4u *dst = (v4u *)(out + base + h);
        const v4u *src = (const v4u *)(stage + lead + h);
        for (uint32_t i = threadIdx.x; i < body; i += kBlock) dst[i] = src[i];
        for (uint32_t i = h + body * 16 + threadIdx.x; i < span; i += kBlock) out[base + i] = stage[lead + i];
        __syncthreads();
    }
}

}  // namespace qeh

using namespace qeh;

extern "C" int qeh_encode_pg_datarows(qeh_ctx *ctx, const qeh_column *cols, int n_cols, qeh_column *out) {
    if (!ctx || !out || n_cols < 0 || (n_cols > 0 && !cols)) return fail(QEH_E_INVALID, "qeh_encode_pg_datarows: bad argument");
    if (n_cols > kEncMaxCols) return fail(QEH_E_UNSUPPORTED, "DataRow encoding: at most 32 columns per call");
    DeviceGuard dg(ctx->device);
    std::memset(out, 0, sizeof(*out));
    const int64_t n = n_cols > 0 ? cols[0].length : 0;
    EncCols ec{};
    ec.n = n_cols;
    for (int j = 0; j < n_cols; ++j) {
        QEH_TRY(check_column(cols[j], "encode"));
        if (cols[j].length != n) return fail(QEH_E_INVALID, "encode: columns have different lengths");
        switch (cols[j].dtype) {
            case QEH_DT_BOOL: case QEH_DT_INT32: case QEH_DT_INT64: case QEH_DT_UINT32: case QEH_DT_FLOAT32:
            case QEH_DT_FLOAT64: case QEH_DT_UTF8: break;
            default: return fail(QEH_E_UNSUPPORTED, "encode: unsupported column type");
        }
        ec.col[j].c = make_colref(cols[j]);
        if (cols[j].dtype == QEH_DT_UTF8) {
            ec.col[j].offs = cols[j].offsets + cols[j].offset;
            ec.col[j].data = (const uint8_t *)cols[j].values;
        }
    }
    DevBuf len, at;
    QEH_TRY(len.alloc(ctx, (size_t)std::max<int64_t>(n, 1) * 4));
    QEH_TRY(at.alloc(ctx, (size_t)std::max<int64_t>(n, 1) * 8));
    const int grid = grid_for(ctx, n, kBlock, 8);
    uint64_t total = 0;
    if (n > 0) {
        KernelTimer kt(ctx, "encode_len");
        hipLaunchKernelGGL(k_pg_row_len, dim3(grid), dim3(kBlock), 0, ctx->stream, ec, n, len.as<uint32_t>());
    }
    QEH_HIP(hipGetLastError());
    QEH_TRY(exclusive_scan_u32(ctx, len.as<uint32_t>(), at.as<uint64_t>(), n, &total));
    if (total > 0x7FFFFFFFull)
        return fail(QEH_E_UNSUPPORTED, "DataRow encoding beyond 2 GiB per call: encode the batch in slices");
    out->dtype = QEH_DT_UTF8;
    out->owned = 1;
    out->length = n;
    void *o = nullptr, *d = nullptr;
    QEH_TRY(ctx->pool->alloc((size_t)(n + 1) * 4, &o));
    int s = ctx->pool->alloc(std::max<size_t>((size_t)total, 8), &d);
    if (s != QEH_OK) {
        ctx->pool->free(o);
        return s;
    }
    out->offsets = (int32_t *)o;
    out->values = d;
    out->values_bytes = (int64_t)total;
    if (n == 0) QEH_HIP(hipMemsetAsync(o, 0, 4, ctx->stream));
    else {
        KernelTimer kt(ctx, "encode_write");
        const char *ek = std::getenv("QEH_ENC_LDS_KB");  // (A/B)
        const bool small = ek ? atoi(ek) == 16 : total <= (uint64_t)n * 56;
        auto wk = small ? k_pg_row_write<16 * 1024> : k_pg_row_write<48 * 1024>;
        hipLaunchKernelGGL(wk, dim3(grid), dim3(kBlock), 0, ctx->stream, ec, n, at.as<uint64_t>(),
                           len.as<uint32_t>(), (char *)d, (int32_t *)o, total);
    }
    QEH_HIP(hipGetLastError());
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    return QEH_OK;
}
