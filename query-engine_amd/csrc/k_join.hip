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
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <string>
#include <vector>

#include "expr_device.h"
#include "lookback.h"
#include "ops.h"

namespace qeh {

constexpr int kJR = 8;
constexpr int kJTile = kBlock * kJR;

// OUTER: a probe row without a match (NULL key included) still emits one pair (row, kNullRow);
// `matched` (FULL joins) gets a 1 at every build row that matched.
template <bool UNIQUE, bool OUTER>
__global__ __launch_bounds__(kBlock) void k_join_probe(ColRef key, int64_t n, int64_t n_tiles, HashTable t,
                                                       uint64_t *__restrict__ status, unsigned long long *__restrict__ ticket,
                                                       uint32_t *__restrict__ out_probe, uint32_t *__restrict__ out_build,
                                                       uint64_t cap, uint32_t *__restrict__ errp,
                                                       uint64_t *__restrict__ total_out, uint8_t *__restrict__ matched) {
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
            if (OUTER && cnt[r] == 0 && row0 + (int64_t)r * kBlock < n) {
                cnt[r] = 1;
                first[r] = kNullRow;
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
            if (UNIQUE || (OUTER && first[r] == kNullRow)) {
                if (pos < cap) {
                    out_probe[pos] = prow;
                    out_build[pos] = first[r];
                }
                if (OUTER && matched && first[r] != kNullRow) matched[first[r]] = 1;
            } else {
                table_probe(t, kv[r], [&](uint32_t p) {
                    if (pos < cap) {
                        out_probe[pos] = prow;
                        out_build[pos] = p;
                    }
                    if (OUTER && matched) matched[p] = 1;
                    ++pos;
                });
            }
        }
        __syncthreads();
    }
}

// total matches (duplicate build keys: sizes the output before the probe pass)
template <bool OUTER>
__global__ void k_join_count(ColRef key, int64_t n, HashTable t, unsigned long long *total) {
    uint64_t c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t m = col_valid(key, i) ? (uint64_t)table_probe(t, load_i64(key, i), [](uint32_t) {}) : 0;
        c += (OUTER && m == 0) ? 1 : m;
    }
    c = wave_sum_u64(c);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(total, (unsigned long long)c);
}

// ---- fused materialising probe (unique DIRECT build, non-null 8-byte columns) ----------
// The build side's payload columns are embedded in a key-offset-indexed record
// array (one random 8*NB-byte read per match instead of table -> row -> column)
// and key presence in a bitmap that stays L2-resident.  One pass per probe
// tile: 16-byte loads of key + probe payloads, presence test, record loads,
// ballot ranks, decoupled look-back for the output offset, then every output
// column leaves through LDS as one contiguous, coalesced run.
constexpr int kMatMaxP = 3, kMatMaxB = 3;
constexpr int kMPairs = 4, kMR = 2 * kMPairs, kMTile = kBlock * kMR;
typedef long long v2i64j __attribute__((ext_vector_type(2)));

struct MatIn {
    const int64_t *key;
    const int64_t *pcol[kMatMaxP];
    int64_t *pout[kMatMaxP];
    int64_t *bout[kMatMaxB];
    const int64_t *rec;        // [range][NB]
    const uint32_t *present;   // bit per key offset
    int64_t kmin, kmax;
    int64_t n;
};

// stride = nb, or nb + 1 with a zeroed matched-flag word after the build columns (FULL joins)
__global__ void k_embed_build(ColRef key, int64_t n, int64_t kmin, const int64_t *b0, const int64_t *b1,
                              const int64_t *b2, int nb, int64_t *__restrict__ rec, uint32_t *__restrict__ present,
                              int stride) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!col_valid(key, i)) continue;
        const uint64_t off = (uint64_t)load_i64(key, i) - (uint64_t)kmin;
        atomicOr(&present[off >> 5], 1u << (off & 31));
        rec[off * stride] = b0[i];
        if (nb > 1) rec[off * stride + 1] = b1[i];
        if (nb > 2) rec[off * stride + 2] = b2[i];
        if (stride > nb) rec[off * stride + nb] = 0;
    }
}

__device__ __forceinline__ v2i64j ld_pair(const int64_t *p, int64_t row, int64_t n) {
    if (row + 1 < n) return __builtin_nontemporal_load((const v2i64j *)(p + row));
    v2i64j v = {0, 0};
    if (row < n) v[0] = p[row];
    return v;
}

template <int NP, int NB>
__global__ __launch_bounds__(kBlock) void k_join_mat(MatIn in, int64_t n_tiles, uint64_t *__restrict__ status,
                                                     unsigned long long *__restrict__ ticket, uint32_t *__restrict__ errp,
                                                     uint64_t *__restrict__ total_out) {
    constexpr int W = kBlock / 64;
    __shared__ int64_t stage[kMTile];
    __shared__ uint32_t cnt[W][kMPairs], offs[W][kMPairs];
    __shared__ int64_t s_tile;
    __shared__ uint64_t s_prefix;
    __shared__ uint32_t s_total;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (;;) {
        if (threadIdx.x == 0) s_tile = (int64_t)atomicAdd(ticket, 1ull);
        __syncthreads();
        const int64_t tile = s_tile;
        if (tile >= n_tiles) break;
        const int64_t base = tile * kMTile + (int64_t)wave * (64 * kMR) + 2 * lane;
        v2i64j key[kMPairs], pv[NP > 0 ? NP : 1][kMPairs];
#pragma unroll
        for (int j = 0; j < kMPairs; ++j) key[j] = ld_pair(in.key, base + j * 128, in.n);
#pragma unroll
        for (int c = 0; c < NP; ++c)
#pragma unroll
            for (int j = 0; j < kMPairs; ++j) pv[c][j] = ld_pair(in.pcol[c], base + j * 128, in.n);
        uint32_t hit = 0;
        uint64_t off[kMR];
#pragma unroll
        for (int r = 0; r < kMR; ++r) {
            const int64_t row = base + (r >> 1) * 128 + (r & 1);
            const int64_t k = key[r >> 1][r & 1];
            off[r] = (uint64_t)k - (uint64_t)in.kmin;
            if (row < in.n && k >= in.kmin && k <= in.kmax && ((in.present[off[r] >> 5] >> (off[r] & 31)) & 1))
                hit |= 1u << r;
        }
        int64_t bv[NB][kMR];
#pragma unroll
        for (int r = 0; r < kMR; ++r)
#pragma unroll
            for (int c = 0; c < NB; ++c) bv[c][r] = ((hit >> r) & 1) ? in.rec[off[r] * NB + c] : 0;
        // ranks in tile order (wave, pair j, lane, element)
        uint32_t rank[kMR];
#pragma unroll
        for (int j = 0; j < kMPairs; ++j) {
            const uint64_t m0 = __ballot((hit >> (2 * j)) & 1), m1 = __ballot((hit >> (2 * j + 1)) & 1);
            const uint32_t below = mbcnt(m0) + mbcnt(m1);
            rank[2 * j] = below;
            rank[2 * j + 1] = below + ((hit >> (2 * j)) & 1);
            if (lane == 0) cnt[wave][j] = (uint32_t)(popc64(m0) + popc64(m1));
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            for (int w = 0; w < W; ++w)
                for (int j = 0; j < kMPairs; ++j) {
                    offs[w][j] = acc;
                    acc += cnt[w][j];
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
        // every output column: scatter into LDS by local rank, then one coalesced run
        // (columns expanded at compile time so the register arrays stay in VGPRs)
        auto emit = [&](auto cc) {
            constexpr int c = decltype(cc)::value;
            if constexpr (c < NP + NB) {
#pragma unroll
                for (int r = 0; r < kMR; ++r) {
                    if (!((hit >> r) & 1)) continue;
                    int64_t v;
                    if constexpr (c < NP) v = pv[c][r >> 1][r & 1];
                    else v = bv[c - NP][r];
                    stage[offs[wave][r >> 1] + rank[r]] = v;
                }
                __syncthreads();
                int64_t *dst;
                if constexpr (c < NP) dst = in.pout[c] + prefix;
                else dst = in.bout[c - NP] + prefix;
                for (uint32_t i = threadIdx.x; i < total; i += kBlock) __builtin_nontemporal_store(stage[i], &dst[i]);
                __syncthreads();
            }
        };
        emit(std::integral_constant<int, 0>{});
        emit(std::integral_constant<int, 1>{});
        emit(std::integral_constant<int, 2>{});
        emit(std::integral_constant<int, 3>{});
        emit(std::integral_constant<int, 4>{});
        emit(std::integral_constant<int, 5>{});
    }
}

int join_indices(qeh_ctx *ctx, const qeh_column &probe_key, const BuiltTable &bt, DevBuf *probe_idx,
                 DevBuf *build_idx, int64_t *out_rows, bool outer, uint8_t *matched, int64_t reserve) {
    const int64_t n = probe_key.length;
    const ColRef kr = make_colref(probe_key);
    uint64_t cap = (uint64_t)n;
    if (!bt.t.unique && n > 0) {
        void *scr = nullptr;
        QEH_TRY(scratch_zeroed(ctx, 64, &scr));
        {
            KernelTimer kt(ctx, "join_count");
            if (outer)
                hipLaunchKernelGGL(k_join_count<true>, dim3(grid_for(ctx, n, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream, kr,
                                   n, bt.t, (unsigned long long *)scr);
            else
                hipLaunchKernelGGL(k_join_count<false>, dim3(grid_for(ctx, n, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream,
                                   kr, n, bt.t, (unsigned long long *)scr);
        }
        QEH_HIP(hipGetLastError());
        QEH_TRY(read_small(ctx, &cap, scr, 8));
    }
    if (cap + (uint64_t)reserve >= (uint64_t)kNullRow)
        return fail(QEH_E_UNSUPPORTED, "join output beyond 2^32 - 1 rows");
    QEH_TRY(probe_idx->alloc(ctx, std::max<uint64_t>(cap + reserve, 1) * 4));
    QEH_TRY(build_idx->alloc(ctx, std::max<uint64_t>(cap + reserve, 1) * 4));
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
#define QEH_JP(U, O)                                                                                             \
    hipLaunchKernelGGL((k_join_probe<U, O>), dim3(grid), dim3(kBlock), 0, ctx->stream, kr, n, n_tiles, bt.t, status, \
                       ticket, probe_idx->as<uint32_t>(), build_idx->as<uint32_t>(), cap, err, tot, matched)
            if (bt.t.unique) {
                if (outer) QEH_JP(true, true);
                else QEH_JP(true, false);
            } else {
                if (outer) QEH_JP(false, true);
                else QEH_JP(false, false);
            }
#undef QEH_JP
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

// ---- outer joins over a unique build key: one output row per probe row, in probe order ----
// bidx[i] = build row matching probe row i, or kNullRow (no match / NULL key); FULL also flags
// the matched build rows.  No compaction: the output position of probe row i is i.
__global__ void k_outer_lookup(ColRef key, int64_t n, HashTable t, uint32_t *__restrict__ bidx,
                               uint8_t *__restrict__ matched) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t p = kNullRow;
        if (col_valid(key, i)) table_probe(t, load_i64(key, i), [&](uint32_t q) { p = q; });
        bidx[i] = p;
        if (matched && p != kNullRow) matched[p] = 1;
    }
}

// Unique DIRECT build with <= 3 non-null 8-byte build columns, embedded by key offset
// (k_embed_build): one presence-bit test (the bitmap stays L2-resident) and one record read per
// probe row, outputs written in probe order with their validity words from one ballot per wave.
struct OuterEmbedOut {
    int64_t *bout[kMatMaxB];
    uint64_t *bvalid[kMatMaxB];
};

template <int NB>
__global__ __launch_bounds__(kBlock) void k_outer_embed(ColRef key, int64_t n, const int64_t *__restrict__ rec,
                                                        const uint32_t *__restrict__ present, int64_t kmin, int64_t kmax,
                                                        OuterEmbedOut out) {
    constexpr int U = 4;  // 64-row groups per wave in flight
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (kBlock / 64);
    for (int64_t g0 = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * U; g0 * 64 < n; g0 += nw * U) {
        uint64_t off[U];
        bool hit[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = (g0 + u) * 64 + lane;
            const bool valid = i < n && col_valid(key, i);
            const int64_t k = valid ? load_i64(key, i) : 0;
            const bool in = valid && k >= kmin && k <= kmax;
            off[u] = in ? (uint64_t)k - (uint64_t)kmin : 0;
            hit[u] = in && ((present[off[u] >> 5] >> (off[u] & 31)) & 1u);
        }
        int64_t v[U][NB];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int b = 0; b < NB; ++b) v[u][b] = hit[u] ? rec[off[u] * NB + b] : 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = (g0 + u) * 64 + lane;
            const uint64_t mask = __ballot(hit[u]);
            if (i < n)
#pragma unroll
                for (int b = 0; b < NB; ++b) out.bout[b][i] = v[u][b];
            if (lane == 0 && (g0 + u) * 64 < n)
#pragma unroll
                for (int b = 0; b < NB; ++b) out.bvalid[b][g0 + u] = mask;
        }
    }
}

// FULL over a unique DIRECT build (build columns embedded as for LEFT, probe columns non-null 8-byte):
// one pass writes every output column of the probe rows in probe order -- the probe columns copied
// beside the key read, the build columns from the embedded records (NULL when unmatched) -- and
// flags each matched key in its record (a plain store when the record read shows it clear); the build rows no probe row
// matched are then appended in build-row order (k_full_tail_*).  Replaces the lookup + index arrays +
// one null-aware gather per output column.
struct FullEmbedOut {
    const int64_t *pcol[kMatMaxP];
    int64_t *pout[kMatMaxP];
    uint64_t *pvalid[kMatMaxP];
    int64_t *bout[kMatMaxB];
    uint64_t *bvalid[kMatMaxB];
    int32_t np;
};

template <int NB, int NP>
__global__ __launch_bounds__(kBlock) void k_full_embed(ColRef key, int64_t n, int64_t *__restrict__ rec,
                                                       const uint32_t *__restrict__ present, int64_t kmin, int64_t kmax,
                                                       FullEmbedOut out) {
    constexpr int S = NB + 1;  // record stride: the values, then the matched flag
    constexpr int U = 4;  // 64-row groups per wave in flight
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (kBlock / 64);
    for (int64_t g0 = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * U; g0 * 64 < n; g0 += nw * U) {
        uint64_t off[U];
        bool hit[U];
        int64_t pv[U][NP > 0 ? NP : 1];  // the probe columns' values, loaded beside the keys
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = (g0 + u) * 64 + lane;
#pragma unroll
            for (int p = 0; p < NP; ++p) pv[u][p] = i < n ? __builtin_nontemporal_load(out.pcol[p] + i) : 0;
            const bool valid = i < n && col_valid(key, i);
            const int64_t k = valid ? load_i64(key, i) : 0;
            const bool in = valid && k >= kmin && k <= kmax;
            off[u] = in ? (uint64_t)k - (uint64_t)kmin : 0;
            hit[u] = in && ((present[off[u] >> 5] >> (off[u] & 31)) & 1u);
        }
        int64_t v[U][S];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int b = 0; b < S; ++b) v[u][b] = hit[u] ? rec[off[u] * S + b] : 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = (g0 + u) * 64 + lane;
            const uint64_t mask = __ballot(hit[u]), rows = __ballot(i < n);
            if (i < n) {
#pragma unroll
                for (int b = 0; b < NB; ++b) __builtin_nontemporal_store(v[u][b], out.bout[b] + i);
#pragma unroll
                for (int p = 0; p < NP; ++p) __builtin_nontemporal_store(pv[u][p], out.pout[p] + i);
                if (hit[u] && v[u][NB] == 0) rec[off[u] * S + NB] = 1;  // (idempotent: a race stores it twice)
            }
            if (lane == 0 && (g0 + u) * 64 < n) {
#pragma unroll
                for (int b = 0; b < NB; ++b) out.bvalid[b][g0 + u] = mask;
#pragma unroll
                for (int p = 0; p < NP; ++p) out.pvalid[p][g0 + u] = rows;
            }
        }
    }
}

// One Int64 build column whose values span < 2^31 - 1: 4-B records by key offset, (value - vmin) + 1 in
// the low 31 bits (0 = no build row: no presence bitmap) and FULL's matched flag in bit 31 -- a quarter of
// the 8-B records' footprint (plus the bitmap), so more of the random record reads hit an XCD's L2.
// (R = uint16_t when the values span < 2^15 - 1: 2-B records, flag in bit 15)
template <typename R>
__global__ void k_embed_build32(ColRef key, int64_t n, int64_t kmin, const int64_t *__restrict__ b0, int64_t vmin,
                                R *__restrict__ rec) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!col_valid(key, i)) continue;
        rec[(uint64_t)load_i64(key, i) - (uint64_t)kmin] = (R)((uint64_t)(b0[i] - vmin) + 1u);
    }
}

template <bool FULL, int NP, typename R>
__global__ __launch_bounds__(kBlock) void k_outer_embed32(ColRef key, int64_t n, R *__restrict__ rec, int64_t kmin,
                                                          int64_t kmax, int64_t vmin, FullEmbedOut out) {
    constexpr uint32_t FLAG = 1u << (8 * sizeof(R) - 1), VAL = FLAG - 1u;
    constexpr int U = 4;
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (kBlock / 64);
    for (int64_t g0 = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * U; g0 * 64 < n; g0 += nw * U) {
        uint64_t off[U];
        uint32_t r[U];
        int64_t pv[U][NP > 0 ? NP : 1];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = (g0 + u) * 64 + lane;
#pragma unroll
            for (int p = 0; p < NP; ++p) pv[u][p] = i < n ? __builtin_nontemporal_load(out.pcol[p] + i) : 0;
            const bool valid = i < n && col_valid(key, i);
            const int64_t k = valid ? load_i64(key, i) : 0;
            const bool in = valid && k >= kmin && k <= kmax;
            off[u] = in ? (uint64_t)k - (uint64_t)kmin : 0;
            r[u] = in ? (uint32_t)rec[off[u]] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = (g0 + u) * 64 + lane;
            const bool hit = (r[u] & VAL) != 0;
            const uint64_t mask = __ballot(hit), rows = __ballot(i < n);
            if (i < n) {
                __builtin_nontemporal_store(hit ? vmin + (int64_t)(r[u] & VAL) - 1 : (int64_t)0, out.bout[0] + i);
#pragma unroll
                for (int p = 0; p < NP; ++p) __builtin_nontemporal_store(pv[u][p], out.pout[p] + i);
                if (FULL && hit && !(r[u] & FLAG)) rec[off[u]] = (R)(r[u] | FLAG);  // (idempotent)
            }
            if (lane == 0 && (g0 + u) * 64 < n) {
                out.bvalid[0][g0 + u] = mask;
#pragma unroll
                for (int p = 0; p < NP; ++p) out.pvalid[p][g0 + u] = rows;
            }
        }
    }
}

// build rows with no matching probe row (a NULL key never matches), per block of kUmRows rows
constexpr int kFtRows = kBlock * 8;
// stride 0 / -1: 4-B / 2-B records (k_embed_build32, flag in the top bit); else 8-B records of `stride`
// words, flag last
__device__ __forceinline__ bool full_unmatched(const ColRef &bkey, int64_t j, int64_t kmin, const int64_t *rec, int stride) {
    if (!col_valid(bkey, j)) return true;
    const uint64_t off = (uint64_t)load_i64(bkey, j) - (uint64_t)kmin;
    if (stride == 0) return (((const uint32_t *)rec)[off] >> 31) == 0;
    if (stride < 0) return (((const uint16_t *)rec)[off] >> 15) == 0;
    return rec[off * stride + stride - 1] == 0;
}
// (the flag of every build row also goes to um[] -- one byte, in order -- for the emit pass)
__global__ void k_full_tail_count(ColRef bkey, int64_t nb, int64_t kmin, const int64_t *__restrict__ rec, int stride,
                                  uint8_t *__restrict__ um, uint32_t *__restrict__ counts) {
    const int64_t base = (int64_t)blockIdx.x * kFtRows;
    uint32_t c = 0;
    for (int r = threadIdx.x; r < kFtRows; r += kBlock) {
        const int64_t j = base + r;
        if (j < nb) {
            const bool u = full_unmatched(bkey, j, kmin, rec, stride);
            um[j] = u ? 1 : 0;
            c += u ? 1u : 0u;
        }
    }
    c = (uint32_t)wave_sum_u64(c);
    __shared__ uint32_t part[kBlock / 64];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += part[w];
        counts[blockIdx.x] = t;
    }
}

// the unmatched build rows written at n + their rank, in build-row order: build columns (valid), probe
// columns NULL (their validity words are zero from the allocation)
__global__ void k_full_tail_emit(const uint8_t *__restrict__ um, int64_t nb, const uint64_t *__restrict__ base_of,
                                 int64_t n, FullEmbedOut out,
                                 const int64_t *b0, const int64_t *b1, const int64_t *b2, int nbc) {
    __shared__ uint32_t wcnt[kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * kFtRows;
    uint64_t pos = (uint64_t)n + base_of[blockIdx.x];
    const int64_t *bc[3] = {b0, b1, b2};
    for (int step = 0; step < kFtRows; step += kBlock) {
        const int64_t j = base + step + threadIdx.x;
        const bool u = j < nb && um[j];
        const uint64_t bal = __ballot(u);
        if (lane == 0) wcnt[wave] = (uint32_t)popc64(bal);
        __syncthreads();
        uint32_t before = 0, total = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            before += w < wave ? wcnt[w] : 0;
            total += wcnt[w];
        }
        if (u) {
            const uint64_t o = pos + before + mbcnt(bal);
            for (int b = 0; b < nbc; ++b) {
                out.bout[b][o] = bc[b][j];
                atomicOr((unsigned long long *)&out.bvalid[b][o >> 6], 1ull << (o & 63));
            }
            for (int p = 0; p < out.np; ++p) out.pout[p][o] = 0;
        }
        pos += total;
        __syncthreads();
    }
}

__global__ void k_iota_then_null(uint32_t *__restrict__ out, int64_t n, int64_t m) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = i < n ? (uint32_t)i : kNullRow;
}

// ---- FULL join: build rows no probe row matched, appended in build-row order ------------
constexpr int kUmRows = kBlock * 8;

__global__ void k_unmatched_count(const uint8_t *__restrict__ matched, int64_t n, uint32_t *__restrict__ counts) {
    const int64_t base = (int64_t)blockIdx.x * kUmRows;
    uint32_t c = 0;
    for (int r = threadIdx.x; r < kUmRows; r += kBlock) c += (base + r < n && !matched[base + r]) ? 1u : 0u;
    c = (uint32_t)wave_sum_u64(c);
    __shared__ uint32_t part[kBlock / 64];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += part[w];
        counts[blockIdx.x] = t;
    }
}

// one block per kUmRows rows; rows leave in order (ballot ranks per 256-row step)
__global__ void k_unmatched_emit(const uint8_t *__restrict__ matched, int64_t n, const uint64_t *__restrict__ base_of,
                                 uint64_t out0, uint32_t *__restrict__ out_probe, uint32_t *__restrict__ out_build) {
    __shared__ uint32_t wcnt[kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * kUmRows;
    uint64_t pos = out0 + base_of[blockIdx.x];
    for (int step = 0; step < kUmRows; step += kBlock) {
        const int64_t row = base + step + threadIdx.x;
        const bool um = row < n && !matched[row];
        const uint64_t b = __ballot(um);
        if (lane == 0) wcnt[wave] = (uint32_t)popc64(b);
        __syncthreads();
        uint32_t before = 0, total = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            before += w < wave ? wcnt[w] : 0;
            total += wcnt[w];
        }
        if (um) {
            const uint64_t o = pos + before + mbcnt(b);
            out_probe[o] = kNullRow;
            out_build[o] = (uint32_t)row;
        }
        pos += total;
        __syncthreads();
    }
}

static bool mat_col_ok(const qeh_column &c) {
    return (c.dtype == QEH_DT_INT64 || c.dtype == QEH_DT_FLOAT64) && (!c.validity || c.null_count == 0) &&
           (((uintptr_t)((const int64_t *)c.values + c.offset)) & 15) == 0;
}

constexpr int kNotEligible = -1;

// Fused path of qeh_hash_join_inner; kNotEligible when the shapes do not fit.
static int join_materialise_fused(qeh_ctx *ctx, const qeh_column &probe_key, const qeh_column *probe_cols, int np,
                                  const qeh_column &build_key, const qeh_column *build_cols, int nb, const BuiltTable &bt,
                                  qeh_column *out_probe, qeh_column *out_build, int64_t *out_rows) {
    if (std::getenv("QEH_NO_FUSED_JOIN")) return kNotEligible;
    if (!bt.t.unique || bt.t.kind != TK_DIRECT || np > kMatMaxP || nb < 1 || nb > kMatMaxB) return kNotEligible;
    if (!mat_col_ok(probe_key)) return kNotEligible;
    for (int i = 0; i < np; ++i)
        if (!mat_col_ok(probe_cols[i])) return kNotEligible;
    for (int i = 0; i < nb; ++i)
        if (!mat_col_ok(build_cols[i])) return kNotEligible;
    const uint64_t range = bt.t.range;
    if (range > (1ull << 31)) return kNotEligible;
    const int64_t n = probe_key.length, nbuild = build_key.length;
    DevBuf rec, present;
    QEH_TRY(rec.alloc(ctx, std::max<uint64_t>(range * nb, 1) * 8));
    QEH_TRY(present.alloc(ctx, ((range + 31) / 32 + 1) * 4));
    QEH_HIP(hipMemsetAsync(present.p, 0, ((range + 31) / 32 + 1) * 4, ctx->stream));
    auto cptr = [](const qeh_column &c) { return (const int64_t *)c.values + c.offset; };
    if (nbuild > 0) {
        KernelTimer kt(ctx, "join_build");
        hipLaunchKernelGGL(k_embed_build, dim3(grid_for(ctx, nbuild, kBlock * 4, 8)), dim3(kBlock), 0, ctx->stream,
                           make_colref(build_key), nbuild, bt.t.kmin, cptr(build_cols[0]),
                           nb > 1 ? cptr(build_cols[1]) : nullptr, nb > 2 ? cptr(build_cols[2]) : nullptr, nb,
                           rec.as<int64_t>(), present.as<uint32_t>(), nb);
        QEH_HIP(hipGetLastError());
    }
    // outputs sized for every probe row (a unique build emits at most one row per probe row)
    int made_p = 0, made_b = 0;
    auto cleanup = [&]() {
        for (int i = 0; i < made_p; ++i) qeh_column_release(ctx, &out_probe[i]);
        for (int i = 0; i < made_b; ++i) qeh_column_release(ctx, &out_build[i]);
    };
    int s = QEH_OK;
    for (int i = 0; i < np && s == QEH_OK; ++i)
        if ((s = alloc_column(ctx, probe_cols[i].dtype, n, false, &out_probe[i])) == QEH_OK) ++made_p;
    for (int i = 0; i < nb && s == QEH_OK; ++i)
        if ((s = alloc_column(ctx, build_cols[i].dtype, n, false, &out_build[i])) == QEH_OK) ++made_b;
    if (s != QEH_OK) {
        cleanup();
        return s;
    }
    uint64_t total = 0;
    const int64_t n_tiles = (n + kMTile - 1) / kMTile;
    if (n_tiles > 0) {
        void *scr = nullptr;
        s = scratch_zeroed(ctx, 64 + (size_t)n_tiles * 8, &scr);
        if (s != QEH_OK) {
            cleanup();
            return s;
        }
        MatIn in{};
        in.key = cptr(probe_key);
        for (int i = 0; i < np; ++i) {
            in.pcol[i] = cptr(probe_cols[i]);
            in.pout[i] = (int64_t *)out_probe[i].values;
        }
        for (int i = 0; i < nb; ++i) in.bout[i] = (int64_t *)out_build[i].values;
        in.rec = rec.as<int64_t>();
        in.present = present.as<uint32_t>();
        in.kmin = bt.t.kmin;
        in.kmax = bt.t.kmax;
        in.n = n;
        unsigned long long *ticket = (unsigned long long *)scr;
        uint32_t *err = (uint32_t *)((char *)scr + 8);
        uint64_t *tot = (uint64_t *)((char *)scr + 16);
        uint64_t *status = (uint64_t *)((char *)scr + 64);
        const int grid = grid_for(ctx, n, kMTile, 4);
        {
            KernelTimer kt(ctx, "join_probe");
#define QEH_MAT(NPV, NBV) \
    hipLaunchKernelGGL((k_join_mat<NPV, NBV>), dim3(grid), dim3(kBlock), 0, ctx->stream, in, n_tiles, status, ticket, err, tot)
#define QEH_MAT_B(NPV)                     \
    if (nb == 1) QEH_MAT(NPV, 1);          \
    else if (nb == 2) QEH_MAT(NPV, 2);     \
    else QEH_MAT(NPV, 3);
            if (np == 0) { QEH_MAT_B(0) } else if (np == 1) { QEH_MAT_B(1) } else if (np == 2) { QEH_MAT_B(2) } else { QEH_MAT_B(3) }
#undef QEH_MAT_B
#undef QEH_MAT
        }
        uint64_t hdr[3];
        s = hipGetLastError() == hipSuccess ? read_small(ctx, hdr, scr, 24) : fail(QEH_E_HIP, "join: probe launch failed");
        if (s == QEH_OK) s = kernel_error_status((uint32_t)hdr[1], "hash join");
        if (s != QEH_OK) {
            cleanup();
            return s;
        }
        total = hdr[2];
    }
    for (int i = 0; i < np; ++i) out_probe[i].length = (int64_t)total;
    for (int i = 0; i < nb; ++i) out_build[i].length = (int64_t)total;
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
    if (n_probe_cols == 1 && n_build_cols == 1) {  // BASELINE config 3 shape: LDS-slice pipeline
        const int r = slice_join_materialise(ctx, *probe_key, probe_cols[0], *build_key, build_cols[0], out_probe, out_build,
                                             out_rows);
        if (r != kSliceJoinNotEligible) return r;
    }
    BuiltTable bt;
    QEH_TRY(build_join_table(ctx, *build_key, nullptr, (uint64_t)std::max<int64_t>(build_key->length - 1, 0), &bt));
    {
        const int r = join_materialise_fused(ctx, *probe_key, probe_cols, n_probe_cols, *build_key, build_cols, n_build_cols,
                                             bt, out_probe, out_build, out_rows);
        if (r != kNotEligible) return r;
    }
    DevBuf pidx, bidx;
    int64_t m = 0;
    QEH_TRY(join_indices(ctx, *probe_key, bt, &pidx, &bidx, &m, false, nullptr, 0));
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

// one Int64 build column without NULLs whose values span < 2^31 - 1 (4-B records)
// Returns the record width (0: not compact, 4, or 2 when the values span < 2^15 - 1).
static int compact_records_ok(qeh_ctx *ctx, const qeh_column *bcols, int nbc, int64_t *vmin) {
    if (nbc != 1 || bcols[0].dtype != QEH_DT_INT64 || std::getenv("QEH_NO_COMPACT_RECORDS")) return 0;
    int64_t mn, mx, cnt;
    if (column_minmax(ctx, bcols[0], &mn, &mx, &cnt) != QEH_OK || cnt != bcols[0].length) return 0;
    if (cnt == 0 || (uint64_t)mx - (uint64_t)mn >= 0x7FFFFFFEull) return 0;
    *vmin = mn;
    return (uint64_t)mx - (uint64_t)mn < 0x7FFEull ? 2 : 4;
}

// One narrow Int64 build column embedded as 2-B / 4-B records straight from the build rows, the key's
// uniqueness read off the filled records (a repeated key leaves fewer non-zero records than keys) --
// instead of a DIRECT join table built only to learn that.  built = false: take the general path.
struct PreRecords {
    DevBuf rec;
    int rw = 0;
    int64_t vmin = 0;
    bool built = false;
};
static bool prebuild_records(qeh_ctx *ctx, const qeh_column &bk, const qeh_column *bcols, int nbc, BuiltTable *bt,
                             PreRecords *pr) {
    if (nbc != 1 || !mat_col_ok(bcols[0])) return false;
    int64_t vmin = 0;
    const int rw = compact_records_ok(ctx, bcols, nbc, &vmin);
    if (!rw) return false;
    int64_t mn, mx, cnt;
    if (column_minmax(ctx, bk, &mn, &mx, &cnt) != QEH_OK || cnt <= 0) return false;
    const uint64_t range = (uint64_t)mx - (uint64_t)mn + 1ull;
    // the DIRECT rule build_join_table applies (row-id payloads), and the embed path's range bound
    if (range == 0 || range > (1ull << 31) || !direct_table_ok(range, (uint64_t)cnt, (uint64_t)std::max<int64_t>(bk.length - 1, 0)))
        return false;
    if (pr->rec.alloc(ctx, range * rw) != QEH_OK || hipMemsetAsync(pr->rec.p, 0, range * rw, ctx->stream) != hipSuccess)
        return false;
    {
        KernelTimer kt(ctx, "join_build");
        const int grid = grid_for(ctx, bk.length, kBlock * 4, 8);
        const int64_t *b0 = (const int64_t *)bcols[0].values + bcols[0].offset;
        if (rw == 4)
            hipLaunchKernelGGL(k_embed_build32<uint32_t>, dim3(grid), dim3(kBlock), 0, ctx->stream, make_colref(bk),
                               bk.length, mn, b0, vmin, pr->rec.as<uint32_t>());
        else
            hipLaunchKernelGGL(k_embed_build32<uint16_t>, dim3(grid), dim3(kBlock), 0, ctx->stream, make_colref(bk),
                               bk.length, mn, b0, vmin, pr->rec.as<uint16_t>());
    }
    uint64_t filled = 0;
    if (hipGetLastError() != hipSuccess || count_nonzero_entries(ctx, pr->rec.p, range, rw, &filled) != QEH_OK ||
        filled != (uint64_t)cnt) {
        pr->rec.reset();
        return false;
    }
    bt->t = HashTable{};
    bt->t.kind = TK_DIRECT;
    bt->t.kmin = mn;
    bt->t.kmax = mx;
    bt->t.range = range;
    bt->t.unique = 1;
    bt->n_inserted = cnt;
    pr->rw = rw;
    pr->vmin = vmin;
    pr->built = true;
    return true;
}

// FULL over a unique DIRECT build: k_full_embed for the probe rows, then the unmatched build rows
// appended (k_full_tail_count / scan / k_full_tail_emit).  Output columns are allocated for every probe
// and build row and hold the m rows that result.
static int full_join_embed(qeh_ctx *ctx, const qeh_column &pk, const qeh_column &bk, const BuiltTable &bt,
                           const qeh_column *pcols, int npc, const qeh_column *bcols, int nbc, qeh_column *pout,
                           qeh_column *bout, int64_t *out_rows, PreRecords *pre) {
    const uint64_t range = bt.t.range;
    const int64_t n = pk.length, nbuild = bk.length, cap = n + nbuild;
    auto cptr = [](const qeh_column &c) { return (const int64_t *)c.values + c.offset; };
    // records of nbc build values + a matched flag word: a probe hit reads its record anyway, so it sets the
    // flag only when it reads it clear -- about one store per matched key instead of one per matching row
    // (one Int64 build column of a narrow range: 4-B records, k_embed_build32)
    DevBuf own_rec, present;
    int64_t vmin = pre->built ? pre->vmin : 0;
    const int rw = pre->built ? pre->rw : compact_records_ok(ctx, bcols, nbc, &vmin);
    const bool r32 = rw != 0;
    const int stride = rw == 4 ? 0 : rw == 2 ? -1 : nbc + 1;
    DevBuf &rec = pre->built ? pre->rec : own_rec;
    if (pre->built) {
    } else if (r32) {
        QEH_TRY(rec.alloc(ctx, std::max<uint64_t>(range, 1) * rw));
        QEH_HIP(hipMemsetAsync(rec.p, 0, std::max<uint64_t>(range, 1) * rw, ctx->stream));
    } else {
        QEH_TRY(rec.alloc(ctx, std::max<uint64_t>(range * stride, 1) * 8));
        QEH_TRY(present.alloc(ctx, ((range + 31) / 32 + 1) * 4));
        QEH_HIP(hipMemsetAsync(present.p, 0, ((range + 31) / 32 + 1) * 4, ctx->stream));
    }
    if (nbuild > 0 && !pre->built) {
        KernelTimer kt(ctx, "join_build");
        if (rw == 4)
            hipLaunchKernelGGL(k_embed_build32<uint32_t>, dim3(grid_for(ctx, nbuild, kBlock * 4, 8)), dim3(kBlock), 0,
                               ctx->stream, make_colref(bk), nbuild, bt.t.kmin, cptr(bcols[0]), vmin, rec.as<uint32_t>());
        else if (rw == 2)
            hipLaunchKernelGGL(k_embed_build32<uint16_t>, dim3(grid_for(ctx, nbuild, kBlock * 4, 8)), dim3(kBlock), 0,
                               ctx->stream, make_colref(bk), nbuild, bt.t.kmin, cptr(bcols[0]), vmin, rec.as<uint16_t>());
        else
            hipLaunchKernelGGL(k_embed_build, dim3(grid_for(ctx, nbuild, kBlock * 4, 8)), dim3(kBlock), 0, ctx->stream,
                               make_colref(bk), nbuild, bt.t.kmin, cptr(bcols[0]), nbc > 1 ? cptr(bcols[1]) : nullptr,
                               nbc > 2 ? cptr(bcols[2]) : nullptr, nbc, rec.as<int64_t>(), present.as<uint32_t>(), stride);
    }
    int made_p = 0, made_b = 0, s = QEH_OK;
    FullEmbedOut eo{};
    eo.np = npc;
    for (int i = 0; i < npc && s == QEH_OK; ++i) {
        s = alloc_column(ctx, pcols[i].dtype, cap, true, &pout[i]);
        if (s != QEH_OK) break;
        ++made_p;
        eo.pcol[i] = cptr(pcols[i]);
        eo.pout[i] = (int64_t *)pout[i].values;
        eo.pvalid[i] = (uint64_t *)pout[i].validity;
        s = hipMemsetAsync(pout[i].validity, 0, (size_t)((cap + 63) / 64) * 8, ctx->stream) == hipSuccess
                ? QEH_OK : fail(QEH_E_HIP, "outer join: memset");
    }
    for (int i = 0; i < nbc && s == QEH_OK; ++i) {
        s = alloc_column(ctx, bcols[i].dtype, cap, true, &bout[i]);
        if (s != QEH_OK) break;
        ++made_b;
        eo.bout[i] = (int64_t *)bout[i].values;
        eo.bvalid[i] = (uint64_t *)bout[i].validity;
        s = hipMemsetAsync(bout[i].validity, 0, (size_t)((cap + 63) / 64) * 8, ctx->stream) == hipSuccess
                ? QEH_OK : fail(QEH_E_HIP, "outer join: memset");
    }
    uint64_t extra = 0;
    bool rw_done = false;  // the slice probe ran (k_outer_slice.hip)
    if (s == QEH_OK && n > 0) {
        KernelTimer kt(ctx, "join_probe");
        const int grid = grid_for(ctx, (n + 255) / 256, kBlock / 64, 8);
        auto go = [&](auto nbv) {
            constexpr int NB = decltype(nbv)::value;
            auto k = npc == 0 ? k_full_embed<NB, 0> : npc == 1 ? k_full_embed<NB, 1> : npc == 2 ? k_full_embed<NB, 2>
                                                                                         : k_full_embed<NB, 3>;
            hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, ctx->stream, make_colref(pk), n, rec.as<int64_t>(),
                               present.as<uint32_t>(), bt.t.kmin, bt.t.kmax, eo);
        };
        int st = kOuterSliceNotEligible;
        if (r32)
            st = outer_slice_probe(ctx, pk, rec.p, rw, bt.t.kmin, range, vmin, true, npc, eo.pcol, eo.pout, eo.pvalid,
                                   eo.bout[0], eo.bvalid[0]);
        if (st != kOuterSliceNotEligible) {
            s = st;
            rw_done = true;
        }
        auto go32 = [&](auto rt) {
            typedef decltype(rt) R;
            auto k = npc == 0 ? k_outer_embed32<true, 0, R> : npc == 1 ? k_outer_embed32<true, 1, R>
                   : npc == 2 ? k_outer_embed32<true, 2, R> : k_outer_embed32<true, 3, R>;
            hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, ctx->stream, make_colref(pk), n, rec.as<R>(), bt.t.kmin,
                               bt.t.kmax, vmin, eo);
        };
        if (rw_done) {
        } else if (rw == 4) go32(uint32_t{});
        else if (rw == 2) go32(uint16_t{});
        else if (nbc == 1) go(std::integral_constant<int, 1>{});
        else if (nbc == 2) go(std::integral_constant<int, 2>{});
        else go(std::integral_constant<int, 3>{});
        if (hipGetLastError() != hipSuccess) s = fail(QEH_E_HIP, "outer join: kernel launch failed");
    }
    if (s == QEH_OK && nbuild > 0) {
        KernelTimer kt(ctx, "join_gather");
        const int64_t nblk = (nbuild + kFtRows - 1) / kFtRows;
        DevBuf counts, bases, um;
        s = counts.alloc(ctx, (size_t)nblk * 4);
        if (s == QEH_OK) s = bases.alloc(ctx, (size_t)nblk * 8);
        if (s == QEH_OK) s = um.alloc(ctx, (size_t)nbuild);
        if (s == QEH_OK) {
            hipLaunchKernelGGL(k_full_tail_count, dim3((unsigned)nblk), dim3(kBlock), 0, ctx->stream, make_colref(bk), nbuild,
                               bt.t.kmin, rec.as<int64_t>(), stride, um.as<uint8_t>(), counts.as<uint32_t>());
            s = exclusive_scan_u32(ctx, counts.as<uint32_t>(), bases.as<uint64_t>(), nblk, &extra);
        }
        if (s == QEH_OK) {
            hipLaunchKernelGGL(k_full_tail_emit, dim3((unsigned)nblk), dim3(kBlock), 0, ctx->stream, um.as<uint8_t>(), nbuild,
                               bases.as<uint64_t>(), n, eo, cptr(bcols[0]),
                               nbc > 1 ? cptr(bcols[1]) : nullptr, nbc > 2 ? cptr(bcols[2]) : nullptr, nbc);
            if (hipGetLastError() != hipSuccess) s = fail(QEH_E_HIP, "outer join: kernel launch failed");
        }
    }
    if (s == QEH_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) s = fail(QEH_E_HIP, "outer join: kernel failed");
    if (s != QEH_OK) {
        for (int i = 0; i < made_p; ++i) qeh_column_release(ctx, &pout[i]);
        for (int i = 0; i < made_b; ++i) qeh_column_release(ctx, &bout[i]);
        return s;
    }
    const int64_t m = n + (int64_t)extra;
    for (int i = 0; i < npc; ++i) pout[i].length = m;
    for (int i = 0; i < nbc; ++i) bout[i].length = m;
    *out_rows = m;
    return QEH_OK;
}

// LEFT / RIGHT / FULL equi-join (include/qeh.h).  The preserved side probes (LEFT,
// FULL: left; RIGHT: right) a table built over the other side; unmatched probe rows emit
// (row, kNullRow), and FULL appends the build rows no probe row matched as (kNullRow, row).  The
// filler side's columns come out NULL through the null-aware gather.
extern "C" int qeh_hash_join_outer(qeh_ctx *ctx, int join_type, const qeh_column *left_key, const qeh_column *left_cols,
                                   int n_left_cols, const qeh_column *right_key, const qeh_column *right_cols,
                                   int n_right_cols, qeh_column *out_left, qeh_column *out_right, int64_t *out_rows) {
    if (!ctx || !left_key || !right_key || !out_rows || (n_left_cols > 0 && (!left_cols || !out_left)) ||
        (n_right_cols > 0 && (!right_cols || !out_right)))
        return fail(QEH_E_INVALID, "qeh_hash_join_outer: bad argument");
    *out_rows = 0;
    if (join_type == 0)
        return qeh_hash_join_inner(ctx, left_key, left_cols, n_left_cols, right_key, right_cols, n_right_cols, out_left,
                                   out_right, out_rows);
    if (join_type < 1 || join_type > 3) return fail(QEH_E_INVALID, "outer join type must be LEFT (1), RIGHT (2) or FULL (3)");
    DeviceGuard dg(ctx->device);
    QEH_TRY(check_column(*left_key, "left key"));
    QEH_TRY(check_column(*right_key, "right key"));
    for (const qeh_column *k : {left_key, right_key})
        if (k->dtype != QEH_DT_INT64 && k->dtype != QEH_DT_INT32)
            return fail(QEH_E_UNSUPPORTED, "hash join keys must be Int32/Int64 on the device");
    for (int i = 0; i < n_left_cols; ++i)
        if (left_cols[i].length != left_key->length) return fail(QEH_E_INVALID, "left columns have different lengths");
    for (int i = 0; i < n_right_cols; ++i)
        if (right_cols[i].length != right_key->length) return fail(QEH_E_INVALID, "right columns have different lengths");
    const bool right_outer = join_type == 2, full = join_type == 3;
    const qeh_column &pk = right_outer ? *right_key : *left_key;
    const qeh_column &bk = right_outer ? *left_key : *right_key;
    if (pk.length >= (int64_t)kNullRow || bk.length >= (int64_t)kNullRow)
        return fail(QEH_E_UNSUPPORTED, "join inputs beyond 2^32 - 1 rows");
    const qeh_column *bcols = right_outer ? left_cols : right_cols;
    const qeh_column *pcols = right_outer ? right_cols : left_cols;
    const int nbc = right_outer ? n_left_cols : n_right_cols, npc = right_outer ? n_right_cols : n_left_cols;
    BuiltTable bt;
    PreRecords pre;
    bool want_pre = !std::getenv("QEH_OUTER_COMPACT") && !std::getenv("QEH_NO_FUSED_JOIN") && nbc == 1 &&
                    !std::getenv("QEH_NO_PREBUILD") && forced_table_kind() < 0;
    if (full) {
        want_pre = want_pre && npc <= kMatMaxP;
        for (int i = 0; want_pre && i < npc; ++i) want_pre = mat_col_ok(pcols[i]);
    }
    if (!(want_pre && prebuild_records(ctx, bk, bcols, nbc, &bt, &pre)))
        QEH_TRY(build_join_table(ctx, bk, nullptr, (uint64_t)std::max<int64_t>(bk.length - 1, 0), &bt));
    DevBuf matched, pidx, bidx;
    if (full) {
        QEH_TRY(matched.alloc(ctx, (size_t)std::max<int64_t>(bk.length, 1)));
        QEH_HIP(hipMemsetAsync(matched.p, 0, (size_t)std::max<int64_t>(bk.length, 1), ctx->stream));
    }
    int64_t m = 0;
    // unique build keys: every probe row yields exactly one row, at its own position
    const bool in_place = bt.t.unique && !std::getenv("QEH_OUTER_COMPACT");
    qeh_column *bout = right_outer ? out_left : out_right;
    qeh_column *pout = right_outer ? out_right : out_left;
    bool embed = in_place && bt.t.kind == TK_DIRECT && nbc >= 1 && nbc <= kMatMaxB && bt.t.range <= (1ull << 31) &&
                 !std::getenv("QEH_NO_FUSED_JOIN");
    for (int i = 0; embed && i < nbc; ++i) embed = mat_col_ok(bcols[i]);
    // FULL: the probe columns are copied by the same pass (8-byte, non-null, at most kMatMaxP)
    if (full) {
        embed = embed && npc <= kMatMaxP;
        for (int i = 0; embed && i < npc; ++i) embed = mat_col_ok(pcols[i]);
    }
    if (embed && full) return full_join_embed(ctx, pk, bk, bt, pcols, npc, bcols, nbc, pout, bout, out_rows, &pre);
    if (embed) {
        // LEFT/RIGHT over a unique DIRECT build: build columns embedded by key offset, one fused
        // probe writes them in probe order; the preserved side's columns are returned as views of
        // the inputs (owned = 0, a RecordBatch column clone)
        const uint64_t range = bt.t.range;
        const int64_t n = pk.length, nbuild = bk.length;
        DevBuf own_rec, present;
        int64_t vmin = pre.built ? pre.vmin : 0;
        const int rw = pre.built ? pre.rw : compact_records_ok(ctx, bcols, nbc, &vmin);
        const bool r32 = rw != 0;
        DevBuf &rec = pre.built ? pre.rec : own_rec;
        auto cptr = [](const qeh_column &c) { return (const int64_t *)c.values + c.offset; };
        if (pre.built) {
        } else if (r32) {
            QEH_TRY(rec.alloc(ctx, std::max<uint64_t>(range, 1) * rw));
            QEH_HIP(hipMemsetAsync(rec.p, 0, std::max<uint64_t>(range, 1) * rw, ctx->stream));
        } else {
            QEH_TRY(rec.alloc(ctx, std::max<uint64_t>(range * nbc, 1) * 8));
            QEH_TRY(present.alloc(ctx, ((range + 31) / 32 + 1) * 4));
            QEH_HIP(hipMemsetAsync(present.p, 0, ((range + 31) / 32 + 1) * 4, ctx->stream));
        }
        if (nbuild > 0 && !pre.built) {
            KernelTimer kt(ctx, "join_build");
            if (rw == 4)
                hipLaunchKernelGGL(k_embed_build32<uint32_t>, dim3(grid_for(ctx, nbuild, kBlock * 4, 8)), dim3(kBlock), 0,
                                   ctx->stream, make_colref(bk), nbuild, bt.t.kmin, cptr(bcols[0]), vmin, rec.as<uint32_t>());
            else if (rw == 2)
                hipLaunchKernelGGL(k_embed_build32<uint16_t>, dim3(grid_for(ctx, nbuild, kBlock * 4, 8)), dim3(kBlock), 0,
                                   ctx->stream, make_colref(bk), nbuild, bt.t.kmin, cptr(bcols[0]), vmin, rec.as<uint16_t>());
            else
                hipLaunchKernelGGL(k_embed_build, dim3(grid_for(ctx, nbuild, kBlock * 4, 8)), dim3(kBlock), 0, ctx->stream,
                                   make_colref(bk), nbuild, bt.t.kmin, cptr(bcols[0]), nbc > 1 ? cptr(bcols[1]) : nullptr,
                                   nbc > 2 ? cptr(bcols[2]) : nullptr, nbc, rec.as<int64_t>(), present.as<uint32_t>(), nbc);
        }
        int made = 0, s = QEH_OK;
        OuterEmbedOut eo{};
        for (int i = 0; i < nbc && s == QEH_OK; ++i) {
            s = alloc_column(ctx, bcols[i].dtype, n, true, &bout[i]);
            if (s == QEH_OK) {
                ++made;
                eo.bout[i] = (int64_t *)bout[i].values;
                eo.bvalid[i] = (uint64_t *)bout[i].validity;
            }
        }
        if (s == QEH_OK && n > 0) {
            KernelTimer kt(ctx, "join_probe");
            const int grid = grid_for(ctx, (n + 255) / 256, kBlock / 64, 8);
            const int st = r32 ? outer_slice_probe(ctx, pk, rec.p, rw, bt.t.kmin, range, vmin, false, 0, nullptr, nullptr,
                                                   nullptr, eo.bout[0], eo.bvalid[0])
                               : kOuterSliceNotEligible;
            if (st != kOuterSliceNotEligible) {
                s = st;
            } else if (r32) {
                FullEmbedOut fo{};
                fo.bout[0] = eo.bout[0];
                fo.bvalid[0] = eo.bvalid[0];
                if (rw == 4)
                    hipLaunchKernelGGL((k_outer_embed32<false, 0, uint32_t>), dim3(grid), dim3(kBlock), 0, ctx->stream,
                                       make_colref(pk), n, rec.as<uint32_t>(), bt.t.kmin, bt.t.kmax, vmin, fo);
                else
                    hipLaunchKernelGGL((k_outer_embed32<false, 0, uint16_t>), dim3(grid), dim3(kBlock), 0, ctx->stream,
                                       make_colref(pk), n, rec.as<uint16_t>(), bt.t.kmin, bt.t.kmax, vmin, fo);
            } else if (nbc == 1)
                hipLaunchKernelGGL(k_outer_embed<1>, dim3(grid), dim3(kBlock), 0, ctx->stream, make_colref(pk), n,
                                   rec.as<int64_t>(), present.as<uint32_t>(), bt.t.kmin, bt.t.kmax, eo);
            else if (nbc == 2)
                hipLaunchKernelGGL(k_outer_embed<2>, dim3(grid), dim3(kBlock), 0, ctx->stream, make_colref(pk), n,
                                   rec.as<int64_t>(), present.as<uint32_t>(), bt.t.kmin, bt.t.kmax, eo);
            else
                hipLaunchKernelGGL(k_outer_embed<3>, dim3(grid), dim3(kBlock), 0, ctx->stream, make_colref(pk), n,
                                   rec.as<int64_t>(), present.as<uint32_t>(), bt.t.kmin, bt.t.kmax, eo);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) s = fail(QEH_E_HIP, std::string("outer join: ") + hipGetErrorString(e));
        }
        if (s == QEH_OK) {
            hipError_t e = hipStreamSynchronize(ctx->stream);
            if (e != hipSuccess) s = fail(QEH_E_HIP, std::string("outer join: ") + hipGetErrorString(e));
        }
        if (s != QEH_OK) {
            for (int i = 0; i < made; ++i) qeh_column_release(ctx, &bout[i]);
            return s;
        }
        for (int i = 0; i < npc; ++i) {
            pout[i] = pcols[i];
            pout[i].owned = 0;
        }
        *out_rows = n;
        return QEH_OK;
    }
    if (in_place) {
        const int64_t n = pk.length;
        QEH_TRY(bidx.alloc(ctx, (size_t)std::max<int64_t>(n + (full ? bk.length : 0), 1) * 4));
        if (n > 0) {
            KernelTimer kt(ctx, "join_probe");
            hipLaunchKernelGGL(k_outer_lookup, dim3(grid_for(ctx, n, kBlock * 4, 8)), dim3(kBlock), 0, ctx->stream,
                               make_colref(pk), n, bt.t, bidx.as<uint32_t>(), full ? matched.as<uint8_t>() : nullptr);
        }
        QEH_HIP(hipGetLastError());
        m = n;
    } else {
        QEH_TRY(join_indices(ctx, pk, bt, &pidx, &bidx, &m, true, full ? matched.as<uint8_t>() : nullptr,
                             full ? bk.length : 0));
    }
    if (full && in_place) {  // probe side of FULL: rows 0..n-1 in place, the appended rows NULL
        QEH_TRY(pidx.alloc(ctx, (size_t)std::max<int64_t>(m + bk.length, 1) * 4));
        if (m + bk.length > 0)
            hipLaunchKernelGGL(k_iota_then_null, dim3(grid_for(ctx, m + bk.length, kBlock * 4, 8)), dim3(kBlock), 0,
                               ctx->stream, pidx.as<uint32_t>(), m, m + bk.length);
    }
    if (full && bk.length > 0) {
        const int64_t nb = (bk.length + kUmRows - 1) / kUmRows;
        DevBuf counts, bases;
        QEH_TRY(counts.alloc(ctx, (size_t)nb * 4));
        QEH_TRY(bases.alloc(ctx, (size_t)nb * 8));
        hipLaunchKernelGGL(k_unmatched_count, dim3((unsigned)nb), dim3(kBlock), 0, ctx->stream, matched.as<uint8_t>(),
                           bk.length, counts.as<uint32_t>());
        uint64_t extra = 0;
        QEH_TRY(exclusive_scan_u32(ctx, counts.as<uint32_t>(), bases.as<uint64_t>(), nb, &extra));
        hipLaunchKernelGGL(k_unmatched_emit, dim3((unsigned)nb), dim3(kBlock), 0, ctx->stream, matched.as<uint8_t>(),
                           bk.length, bases.as<uint64_t>(), (uint64_t)m, pidx.as<uint32_t>(), bidx.as<uint32_t>());
        QEH_HIP(hipGetLastError());
        m += (int64_t)extra;
    }
    const bool probe_copy = in_place && !full;  // probe columns leave unchanged: one normalising copy each
    // probe side: NULL only for FULL's appended rows; build side: NULL for unmatched probe rows
    const uint32_t *lidx = right_outer ? bidx.as<uint32_t>() : pidx.as<uint32_t>();
    const uint32_t *ridx = right_outer ? pidx.as<uint32_t>() : bidx.as<uint32_t>();
    const bool lnull = right_outer || full, rnull = !right_outer || full;
    int made_l = 0, made_r = 0, s = QEH_OK;
    auto out_col = [&](const qeh_column &src, const uint32_t *idx, bool nullable, bool probe_side, qeh_column *dst) {
        KernelTimer kt(ctx, "join_gather");
        if (probe_side && probe_copy) {
            const qeh_column *one = &src;
            return concat_columns(ctx, &one, 1, dst);
        }
        return gather_column(ctx, src, idx, m, dst, nullable);
    };
    for (int i = 0; i < n_left_cols && s == QEH_OK; ++i) {
        s = out_col(left_cols[i], lidx, lnull, !right_outer, &out_left[i]);
        if (s == QEH_OK) ++made_l;
    }
    for (int i = 0; i < n_right_cols && s == QEH_OK; ++i) {
        s = out_col(right_cols[i], ridx, rnull, right_outer, &out_right[i]);
        if (s == QEH_OK) ++made_r;
    }
    if (s == QEH_OK) {
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) s = fail(QEH_E_HIP, std::string("outer join: ") + hipGetErrorString(e));
    }
    if (s != QEH_OK) {
        for (int i = 0; i < made_l; ++i) qeh_column_release(ctx, &out_left[i]);
        for (int i = 0; i < made_r; ++i) qeh_column_release(ctx, &out_right[i]);
        return s;
    }
    *out_rows = m;
    return QEH_OK;
}
