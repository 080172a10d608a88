// HashJoinExec (INNER, equi-join on one Int32/Int64 key), materialising.
//
// Reference: execute_join / execute_inner_join / join_batches
// (crates/query-executor/src/executor.rs:343-381, 500-540) ignore `on` and
// emit every (left row, right row) pair of every batch pair, left row-major,
// with schema left ++ right.  The intended semantics keep
// exactly the pairs of that product on which `left.key = right.key` is TRUE;
// NULL keys never match.  We build on the right input (the dimension in the
// BASELINE configs) and probe with the left, so for a unique build key the
// output is in left-row order — the order of the reference's filtered product.
//
// Device plan: build (k_build.hip) -> one probe pass that ranks every probe
// tile's matches and learns its output offset by decoupled look-back
// (lookback.h), writing (probe row, build row) index pairs -> gather of the
// requested payload columns (late materialisation).  Build keys with
// duplicates take one extra counting pass to size the output.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "expr_device.h"
#include "lookback.h"
#include "ops.h"

namespace qeh {

constexpr int kJR = 8;
constexpr int kJTile = kBlock * kJR;

template <bool UNIQUE>
__global__ __launch_bounds__(kBlock) void k_join_probe(ColRef key, int64_t n, int64_t n_tiles, HashTable t,
                                                       uint64_t *__restrict__ status, unsigned long long *__restrict__ ticket,
                                                       uint32_t *__restrict__ out_probe, uint32_t *__restrict__ out_build,
                                                       uint64_t cap, uint32_t *__restrict__ errp,
                                                       uint64_t *__restrict__ total_out) {
    __shared__ uint32_t wave_cnt[kJR][kBlock / 64];
    __shared__ uint32_t wave_off[kJR][kBlock / 64];
    __shared__ int64_t s_tile;
    __shared__ uint64_t s_prefix;
    __shared__ uint32_t s_total;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (;;) {
        if (threadIdx.x == 0) s_tile = (int64_t)atomicAdd(ticket, 1ull);
        __syncthreads();
        const int64_t tile = s_tile;
        if (tile >= n_tiles) break;
        const int64_t row0 = tile * kJTile + threadIdx.x;
        int64_t kv[kJR];
        uint32_t kvalid;
        load_rows<kJR>(key, row0, kBlock, n, kv, kvalid);
        uint32_t cnt[kJR], first[kJR];
#pragma unroll
        for (int r = 0; r < kJR; ++r) {
            cnt[r] = 0;
            first[r] = 0;
            if ((kvalid >> r) & 1) {
                uint32_t c = 0, f = 0;
                table_probe(t, kv[r], [&](uint32_t p) {
                    if (c == 0) f = p;
                    ++c;
                });
                cnt[r] = c;
                first[r] = f;
            }
        }
        uint32_t excl[kJR];
#pragma unroll
        for (int r = 0; r < kJR; ++r) {
            const uint32_t inc = wave_incl_scan(cnt[r]);
            excl[r] = inc - cnt[r];
            if (lane == 63) wave_cnt[r][wave] = inc;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            for (int r = 0; r < kJR; ++r)
                for (int w = 0; w < kBlock / 64; ++w) {
                    wave_off[r][w] = acc;
                    acc += wave_cnt[r][w];
                }
            s_total = acc;
        }
        __syncthreads();
        const uint32_t total = s_total;
        if (wave == 0) {
            uint64_t prefix = 0;
            if (tile == 0) {
                if (lane == 0) st_agent(&status[0], kFlagIncl | total);
            } else {
                if (lane == 0) st_agent(&status[tile], kFlagAgg | total);
                prefix = lookback(status, tile, total, errp);
                if (lane == 0) st_agent(&status[tile], kFlagIncl | (prefix + total));
            }
            if (lane == 0) {
                s_prefix = prefix;
                if (tile == n_tiles - 1) *total_out = prefix + total;
            }
        }
        __syncthreads();
        const uint64_t prefix = s_prefix;
#pragma unroll
        for (int r = 0; r < kJR; ++r) {
            if (!cnt[r]) continue;
            const uint32_t prow = (uint32_t)(row0 + (int64_t)r * kBlock);
            uint64_t pos = prefix + wave_off[r][wave] + excl[r];
            if (UNIQUE) {
                if (pos < cap) {
                    out_probe[pos] = prow;
                    out_build[pos] = first[r];
                }
            } else {
                table_probe(t, kv[r], [&](uint32_t p) {
                    if (pos < cap) {
                        out_probe[pos] = prow;
                        out_build[pos] = p;
                    }
                    ++pos;
                });
            }
        }
        __syncthreads();
    }
}

// total matches (duplicate build keys: sizes the output before the probe pass)
__global__ void k_join_count(ColRef key, int64_t n, HashTable t, unsigned long long *total) {
    uint64_t c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (col_valid(key, i)) c += (uint64_t)table_probe(t, load_i64(key, i), [](uint32_t) {});
    c = wave_sum_u64(c);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(total, (unsigned long long)c);
}

int join_indices(qeh_ctx *ctx, const qeh_column &probe_key, const BuiltTable &bt, DevBuf *probe_idx,
                 DevBuf *build_idx, int64_t *out_rows) {
    const int64_t n = probe_key.length;
    const ColRef kr = make_colref(probe_key);
    uint64_t cap = (uint64_t)n;
    if (!bt.t.unique && n > 0) {
        void *scr = nullptr;
        QEH_TRY(scratch_zeroed(ctx, 64, &scr));
        {
            KernelTimer kt(ctx, "join_count");
            hipLaunchKernelGGL(k_join_count, dim3(grid_for(ctx, n, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream, kr, n, bt.t,
                               (unsigned long long *)scr);
        }
        QEH_HIP(hipGetLastError());
        QEH_TRY(read_small(ctx, &cap, scr, 8));
    }
    QEH_TRY(probe_idx->alloc(ctx, std::max<uint64_t>(cap, 1) * 4));
    QEH_TRY(build_idx->alloc(ctx, std::max<uint64_t>(cap, 1) * 4));
    const int64_t n_tiles = (n + kJTile - 1) / kJTile;
    uint64_t total = 0;
    if (n_tiles > 0) {
        void *scr = nullptr;
        QEH_TRY(scratch_zeroed(ctx, 64 + (size_t)n_tiles * 8, &scr));
        unsigned long long *ticket = (unsigned long long *)scr;
        uint32_t *err = (uint32_t *)((char *)scr + 8);
        uint64_t *tot = (uint64_t *)((char *)scr + 16);
        uint64_t *status = (uint64_t *)((char *)scr + 64);
        const int grid = grid_for(ctx, n, kJTile, 4);
        {
            KernelTimer kt(ctx, "join_probe");
            if (bt.t.unique)
                hipLaunchKernelGGL(k_join_probe<true>, dim3(grid), dim3(kBlock), 0, ctx->stream, kr, n, n_tiles, bt.t, status,
                                   ticket, probe_idx->as<uint32_t>(), build_idx->as<uint32_t>(), cap, err, tot);
            else
                hipLaunchKernelGGL(k_join_probe<false>, dim3(grid), dim3(kBlock), 0, ctx->stream, kr, n, n_tiles, bt.t, status,
                                   ticket, probe_idx->as<uint32_t>(), build_idx->as<uint32_t>(), cap, err, tot);
        }
        QEH_HIP(hipGetLastError());
        uint64_t hdr[3];
        QEH_TRY(read_small(ctx, hdr, scr, 24));
        QEH_TRY(kernel_error_status((uint32_t)hdr[1], "hash join"));
        total = hdr[2];
        if (total > cap) return fail(QEH_E_INTERNAL, "hash join: match count changed between passes");
    }
    *out_rows = (int64_t)total;
    return QEH_OK;
}

}  // namespace qeh

using namespace qeh;

extern "C" int qeh_hash_join_inner(qeh_ctx *ctx, const qeh_column *probe_key, const qeh_column *probe_cols,
                                   int n_probe_cols, const qeh_column *build_key, const qeh_column *build_cols,
                                   int n_build_cols, qeh_column *out_probe, qeh_column *out_build, int64_t *out_rows) {
    if (!ctx || !probe_key || !build_key || !out_rows) return fail(QEH_E_INVALID, "qeh_hash_join_inner: bad argument");
    *out_rows = 0;
    DeviceGuard dg(ctx->device);
    QEH_TRY(check_column(*probe_key, "probe key"));
    if (probe_key->dtype != QEH_DT_INT64 && probe_key->dtype != QEH_DT_INT32)
        return fail(QEH_E_UNSUPPORTED, "hash join keys must be Int32/Int64 on the device");
    for (int i = 0; i < n_probe_cols; ++i)
        if (probe_cols[i].length != probe_key->length) return fail(QEH_E_INVALID, "probe columns have different lengths");
    for (int i = 0; i < n_build_cols; ++i)
        if (build_cols[i].length != build_key->length) return fail(QEH_E_INVALID, "build columns have different lengths");
    BuiltTable bt;
    QEH_TRY(build_join_table(ctx, *build_key, nullptr, (uint64_t)std::max<int64_t>(build_key->length - 1, 0), &bt));
    DevBuf pidx, bidx;
    int64_t m = 0;
    QEH_TRY(join_indices(ctx, *probe_key, bt, &pidx, &bidx, &m));
    int made_p = 0, made_b = 0;
    int s = QEH_OK;
    for (int i = 0; i < n_probe_cols && s == QEH_OK; ++i) {
        KernelTimer kt(ctx, "join_gather");
        s = gather_column(ctx, probe_cols[i], pidx.as<uint32_t>(), m, &out_probe[i]);
        if (s == QEH_OK) ++made_p;
    }
    for (int i = 0; i < n_build_cols && s == QEH_OK; ++i) {
        KernelTimer kt(ctx, "join_gather");
        s = gather_column(ctx, build_cols[i], bidx.as<uint32_t>(), m, &out_build[i]);
        if (s == QEH_OK) ++made_b;
    }
    if (s == QEH_OK) {
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) s = fail(QEH_E_HIP, std::string("join: ") + hipGetErrorString(e));
    }
    if (s != QEH_OK) {
        for (int i = 0; i < made_p; ++i) qeh_column_release(ctx, &out_probe[i]);
        for (int i = 0; i < made_b; ++i) qeh_column_release(ctx, &out_build[i]);
        return s;
    }
    *out_rows = m;
    return QEH_OK;
}
