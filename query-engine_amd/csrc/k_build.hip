// Build side of HashJoinExec and group-id assignment (HBM hash tables).
//
// Reference: the join operators are stubs (executor.rs:363-381 emits the
// Cartesian product and ignores `on`); the intended semantics
// are an INNER equi-join where NULL keys never match.  This file builds the
// table over the right (build) input; probing lives with the consumers
// (k_join.hip, k_pipeline.hip).
#include <algorithm>
#include <cstdlib>
#include <string>

#include "device_common.h"
#include "grouptable.h"
#include "ops.h"

namespace qeh {

static constexpr uint32_t kEmpty32 = 0xFFFFFFFFu;

// ---- key min/max over valid rows -------------------------------------------------
__device__ __forceinline__ void key_minmax_body(const ColRef &key, int64_t n, MinMax *out);

// Several columns in one launch (blockIdx.y = column): each workgroup writes its partial to
// part[column * gridDim.x + workgroup] and k_minmax_final reduces them -- same-address atomics from
// every workgroup serialise at ~12 ns each (MI355X_MICROARCH.md, fanin), 74 us for 2 x 1024
// workgroups against the 20 us the two 1e7-row build columns take to read.
constexpr int kMinMaxCols = 4;
struct MinMaxJob {
    ColRef c[kMinMaxCols];
    int64_t n[kMinMaxCols];
};
__global__ __launch_bounds__(kBlock) void k_key_minmax_n(MinMaxJob j, MinMax *part) {
    key_minmax_body(j.c[blockIdx.y], j.n[blockIdx.y], part + (int64_t)blockIdx.y * gridDim.x + blockIdx.x);
}

// blockIdx.x = column: reduce its nb partials into out[column]
__global__ __launch_bounds__(kBlock) void k_minmax_final(const MinMax *__restrict__ part, int nb, MinMax *__restrict__ out) {
    __shared__ int64_t smn[kBlock / 64], smx[kBlock / 64];
    __shared__ uint64_t scnt[kBlock / 64];
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    uint64_t cnt = 0;
    for (int i = threadIdx.x; i < nb; i += kBlock) {
        const MinMax q = part[(int64_t)blockIdx.x * nb + i];
        mn = q.mn < mn ? q.mn : mn;
        mx = q.mx > mx ? q.mx : mx;
        cnt += q.cnt;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const int64_t a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64);
        const uint64_t c = __shfl_xor(cnt, d, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
        cnt += c;
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) smn[w] = mn, smx[w] = mx, scnt[w] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < kBlock / 64; ++i) {
            mn = smn[i] < mn ? smn[i] : mn;
            mx = smx[i] > mx ? smx[i] : mx;
            cnt += scnt[i];
        }
        out[blockIdx.x] = MinMax{mn, mx, cnt, 0u};
    }
}

// One workgroup's (min, max, valid count) over its share of the rows, stored at *out.
__device__ __forceinline__ void key_minmax_body(const ColRef &key, int64_t n, MinMax *out) {
    __shared__ int64_t smn[kBlock / 64], smx[kBlock / 64];
    __shared__ uint64_t scnt[kBlock / 64];
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    uint64_t cnt = 0;
    if (key.validity == nullptr && key.dtype == QEH_DT_INT64 && ((uintptr_t)key.values & 15) == 0) {
        // no nulls: non-temporal 16-B loads, eight in flight per thread, counted once
        typedef long long v2 __attribute__((ext_vector_type(2)));
        const v2 *kv = (const v2 *)key.values;
        const int64_t pairs = n / 2, stride = (int64_t)gridDim.x * blockDim.x;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < pairs; i += 8 * stride) {
            v2 q[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)  // pad with pair i
                q[u] = __builtin_nontemporal_load(kv + (i + u * stride < pairs ? i + u * stride : i));
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t a = q[u].x, b = q[u].y;
                mn = a < mn ? a : mn;
                mx = a > mx ? a : mx;
                mn = b < mn ? b : mn;
                mx = b > mx ? b : mx;
            }
        }
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
            const int64_t k = ((const int64_t *)key.values)[n - 1];
            mn = k < mn ? k : mn;
            mx = k > mx ? k : mx;
        }
        cnt = (blockIdx.x == 0 && threadIdx.x == 0) ? (uint64_t)n : 0;
    } else {
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
            if (!col_valid(key, i)) continue;
            int64_t k = load_i64(key, i);
            mn = k < mn ? k : mn;
            mx = k > mx ? k : mx;
            ++cnt;
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        int64_t a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64);
        uint64_t c = __shfl_xor(cnt, d, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
        cnt += c;
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) smn[w] = mn, smx[w] = mx, scnt[w] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < kBlock / 64; ++i) {
            mn = smn[i] < mn ? smn[i] : mn;
            mx = smx[i] > mx ? smx[i] : mx;
            cnt += scnt[i];
        }
        *out = MinMax{mn, mx, cnt, 0u};
    }
}


// ---- inserts -------------------------------------------------------------------------
__device__ __forceinline__ uint32_t payload_of(const RowPayload &rp, int64_t row) {
    if (rp.ids) return rp.ids[row];
    if (rp.values) return (uint32_t)((uint64_t)rp.values[row] - (uint64_t)rp.bias);
    if (rp.slot) return (uint32_t)rp.dense[rp.slot[row]];
    return (uint32_t)row;
}

// DIRECT inserts: entry = payload + 1 at key - kmin, plain stores (any writer
// of a duplicated key wins).  Duplicates are found afterwards by counting the
// non-empty entries: fewer than valid build rows <=> some key repeats (the
// table is then rebuilt hashed).  No returning atomics on the build path.
__global__ void k_insert_direct(ColRef key, int64_t n, RowPayload rp, HashTable t) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!col_valid(key, i)) continue;
        t.payload[(uint64_t)load_i64(key, i) - (uint64_t)t.kmin] = payload_of(rp, i) + 1u;
    }
}

__global__ void k_insert_direct16(ColRef key, int64_t n, RowPayload rp, HashTable t) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!col_valid(key, i)) continue;
        t.payload16[(uint64_t)load_i64(key, i) - (uint64_t)t.kmin] = (uint16_t)(payload_of(rp, i) + 1u);
    }
}

// The same insert with the table split into 8 key ranges, range q written only by workgroups
// b with b % 8 == q -- consecutive workgroup ids go to different XCDs, so each XCD's scattered
// 2-B stores stay in its own L2 slice of the table (20 MB table / 8 < 4 MB L2) and leave as
// whole lines, instead of every XCD dirtying partial lines all over the table.  Every
// workgroup reads all keys (8 reads of an 80 MB key column, mostly Infinity-Cache hits).
__global__ void k_insert_direct16_xcd(ColRef key, int64_t n, RowPayload rp, HashTable t) {
    const uint32_t part = blockIdx.x & 7u;
    const int64_t nb = gridDim.x >> 3;
    const uint64_t span = (t.range + 7) >> 3;
    for (int64_t i = (int64_t)(blockIdx.x >> 3) * blockDim.x + threadIdx.x; i < n; i += nb * blockDim.x) {
        if (!col_valid(key, i)) continue;
        const uint64_t o = (uint64_t)load_i64(key, i) - (uint64_t)t.kmin;
        if (o / span != part) continue;
        t.payload16[o] = (uint16_t)(payload_of(rp, i) + 1u);
    }
}

// The XCD-split insert in two steps, each key read once: k_xcd_lists appends every build row's
// (key offset << 16 | payload + 1) to the list of its table range q = offset / span (one LDS rank per
// row, one global cursor reservation per range per workgroup, ~1 K-entry contiguous runs per
// range); k_insert_xcd_lists then has the workgroups of XCD q (b % 8 == q) drain list q, so range q
// of the table is written only through XCD q's L2.  Lists hold up to n entries each (keys may all
// fall into one range).
constexpr int kXcdRows = 8;  // rows per thread in k_xcd_lists
__global__ __launch_bounds__(kBlock) void k_xcd_lists(ColRef key, int64_t n, RowPayload rp, int64_t kmin, uint64_t span,
                                                    uint64_t *__restrict__ lists, int64_t cap,
                                                    unsigned long long *__restrict__ cursor) {
    __shared__ uint32_t cnt[8];
    __shared__ unsigned long long base[8];
    for (int64_t t0 = (int64_t)blockIdx.x * kBlock * kXcdRows; t0 < n; t0 += (int64_t)gridDim.x * kBlock * kXcdRows) {
        if (threadIdx.x < 8) cnt[threadIdx.x] = 0u;
        __syncthreads();
        uint64_t e[kXcdRows];
        uint32_t q[kXcdRows], rk[kXcdRows];
#pragma unroll
        for (int r = 0; r < kXcdRows; ++r) {
            const int64_t i = t0 + (int64_t)r * kBlock + threadIdx.x;
            q[r] = 8u;
            e[r] = 0ull;
            rk[r] = 0u;
            if (i < n && col_valid(key, i)) {
                const uint64_t o = (uint64_t)load_i64(key, i) - (uint64_t)kmin;
                q[r] = (uint32_t)(o / span);
                e[r] = (o << 16) | (uint64_t)(uint16_t)(payload_of(rp, i) + 1u);
                rk[r] = atomicAdd(&cnt[q[r]], 1u);
            }
        }
        __syncthreads();
        if (threadIdx.x < 8)
            base[threadIdx.x] = cnt[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], (unsigned long long)cnt[threadIdx.x]) : 0ull;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kXcdRows; ++r)
            if (q[r] < 8u) lists[(int64_t)q[r] * cap + (int64_t)base[q[r]] + rk[r]] = e[r];
        __syncthreads();
    }
}

__global__ __launch_bounds__(kBlock) void k_insert_xcd_lists(const uint64_t *__restrict__ lists, int64_t cap,
                                                           const unsigned long long *__restrict__ cursor, HashTable t) {
    const uint32_t q = blockIdx.x & 7u;
    const int64_t nb = gridDim.x >> 3, m = (int64_t)cursor[q];
    const uint64_t *l = lists + (int64_t)q * cap;
    for (int64_t i = (int64_t)(blockIdx.x >> 3) * blockDim.x + threadIdx.x; i < m; i += nb * blockDim.x) {
        const uint64_t e = __builtin_nontemporal_load(l + i);
        t.payload16[e >> 16] = (uint16_t)(e & 0xFFFFu);
    }
}

// Non-zero entries of a table of `n` words of `bytes` bytes (2 or 4), summed into *out.
// max_entry > 0 (u16 tables only): entries above it are not counted and are cleared in place, so a
// probe of the table afterwards reads them as misses -- a summed table of the distributed table form
// holds world x (G + 1) where a build key sits on two ranks, and the probe kernels index group states
// with entry - 1 unchecked (the caller's count < rows then sends the query to the general path).
__global__ __launch_bounds__(kBlock) void k_count_nonzero(void *__restrict__ table, uint64_t n, int bytes,
                                                          unsigned long long *out, uint32_t max_entry = 0) {
    __shared__ uint64_t part[kBlock / 64];
    uint64_t c = 0;
    const uint64_t words = bytes == 2 ? n / 8 : n / 4;  // 16-B chunks
    uint4 *v = (uint4 *)table;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 q = v[i];
        uint32_t w[4] = {q.x, q.y, q.z, q.w};
        bool cleared = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (bytes == 2) {
                uint32_t lo = w[j] & 0xFFFFu, hi = w[j] >> 16;
                if (max_entry && lo > max_entry) lo = 0, cleared = true;
                if (max_entry && hi > max_entry) hi = 0, cleared = true;
                c += (lo != 0u) + (hi != 0u);
                w[j] = lo | (hi << 16);
            } else {
                c += w[j] != 0u;
            }
        }
        if (cleared) v[i] = uint4{w[0], w[1], w[2], w[3]};
    }
    if (blockIdx.x == 0) {  // ragged tail
        const uint64_t done = bytes == 2 ? words * 8 : words * 4;
        for (uint64_t i = done + threadIdx.x; i < n; i += blockDim.x) {
            if (bytes == 2) {
                uint16_t *e = (uint16_t *)table + i;
                if (max_entry && *e > max_entry) *e = 0;
                c += *e != 0;
            } else {
                c += ((const uint32_t *)table)[i] != 0u;
            }
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int i = 0; i < kBlock / 64; ++i) t += part[i];
        if (t) atomicAdd(out, (unsigned long long)t);
    }
}

__global__ void k_insert_packed(ColRef key, int64_t n, RowPayload row_payload, HashTable t, uint32_t *dup) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!col_valid(key, i)) continue;
        int64_t k = load_i64(key, i);
        uint64_t kp = (uint64_t)k - (uint64_t)t.kmin + 1ull;
        uint64_t e = (kp << t.pbits) | (uint64_t)payload_of(row_payload, i);
        uint64_t h = hash64((uint64_t)k) & t.mask;
        bool d = false;
        for (uint64_t probe = 0; probe <= t.mask; ++probe) {
            unsigned long long old = atomicCAS((unsigned long long *)&t.slots[h], 0ull, (unsigned long long)e);
            if (old == 0ull) break;
            if ((old >> t.pbits) == kp) d = true;
            h = (h + 1) & t.mask;
        }
        if (d) *dup = 1u;
    }
}

// WIDE: claim a slot by CAS on its payload word (0 = empty), then store the key.  Probes run
// only after the build kernel has finished, so a claimed slot's key is always visible to them.
__global__ void k_insert_wide(ColRef key, int64_t n, RowPayload row_payload, HashTable t) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!col_valid(key, i)) continue;
        int64_t k = load_i64(key, i);
        const unsigned long long e = (unsigned long long)payload_of(row_payload, i) + 1ull;
        uint64_t h = hash64((uint64_t)k) & t.mask;
        for (uint64_t probe = 0; probe <= t.mask; ++probe) {
            if (atomicCAS((unsigned long long *)&t.slots[2 * h + 1], 0ull, e) == 0ull) {
                t.slots[2 * h] = (uint64_t)k;
                break;
            }
            h = (h + 1) & t.mask;
        }
    }
}

// BUCKET: one returning atomic on the bucket's count word claims slot s; a full bucket sends the key on
// to the next one (the count keeps rising there, which tells probes to follow).  Payload halves and the
// count share bytes of one word: byte-granular stores beside a 4-B atomic on the other bytes.
__global__ void k_insert_bucket(ColRef key, int64_t n, RowPayload row_payload, HashTable t) {
    const int S = bucket_slots(t.pbits);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!col_valid(key, i)) continue;
        const int64_t k = load_i64(key, i);
        const uint32_t e = payload_of(row_payload, i) + 1u;
        uint64_t b = bucket_home(t, (uint64_t)k);
        for (uint64_t step = 0; step < t.nbkt; ++step) {
            uint64_t *line = t.slots + b * 8;
            const uint32_t s = atomicAdd((uint32_t *)(line + 7) + 1, 1u);
            if (s < (uint32_t)S) {
                line[s] = (uint64_t)k;
                if (t.pbits == 16) ((uint16_t *)(line + S))[s] = (uint16_t)e;
                else ((uint32_t *)(line + S))[s] = e;
                break;
            }
            b = b + 1 == t.nbkt ? 0 : b + 1;
        }
    }
}

// Duplicate detection for WIDE / BUCKET tables (separate launch: all slots are final).
__global__ void k_wide_dups(ColRef key, int64_t n, HashTable t, uint32_t *dup) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!col_valid(key, i)) continue;
        int64_t k = load_i64(key, i);
        int c = table_probe(t, k, [](uint32_t) {});
        if (c > 1) *dup = 1u;
    }
}

// Broadcast join in table form (qeh_direct_group_table_insert): this rank's shard into the shared
// DIRECT u16 table, entry = group slot + 1; out-of-range keys / group keys and NULL group keys flag
// `bad` and are not written (NULL join keys never match and are skipped).
__global__ void k_direct_group_insert(ColRef key, ColRef gkey, int64_t n, int64_t kmin, uint64_t range, int64_t gmin,
                                      uint16_t *__restrict__ table, uint32_t *__restrict__ bad) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!col_valid(key, i)) continue;
        const uint64_t o = (uint64_t)load_i64(key, i) - (uint64_t)kmin;
        const uint64_t g = (uint64_t)load_i64(gkey, i) - (uint64_t)gmin;
        if (o >= range || !col_valid(gkey, i) || g >= 0xFFFEull) {
            *bad = 1u;
            continue;
        }
        table[o] = (uint16_t)(g + 1u);
    }
}

static int direct_group_table_insert(qeh_ctx *ctx, const qeh_column *build_key, const qeh_column *group_key, int64_t key_min,
                                     uint64_t key_range, int64_t group_min, uint16_t *table, bool check);

extern "C" int qeh_direct_group_table_insert(qeh_ctx *ctx, const qeh_column *build_key, const qeh_column *group_key,
                                             int64_t key_min, uint64_t key_range, int64_t group_min, uint16_t *table) {
    return direct_group_table_insert(ctx, build_key, group_key, key_min, key_range, group_min, table, true);
}

extern "C" int qeh_direct_group_table_insert_async(qeh_ctx *ctx, const qeh_column *build_key, const qeh_column *group_key,
                                                   int64_t key_min, uint64_t key_range, int64_t group_min, uint16_t *table) {
    return direct_group_table_insert(ctx, build_key, group_key, key_min, key_range, group_min, table, false);
}

static int direct_group_table_insert(qeh_ctx *ctx, const qeh_column *build_key, const qeh_column *group_key, int64_t key_min,
                                     uint64_t key_range, int64_t group_min, uint16_t *table, bool check) {
    if (!ctx || !build_key || !group_key || !table || key_range == 0)
        return fail(QEH_E_INVALID, "qeh_direct_group_table_insert: bad argument");
    if (build_key->length != group_key->length) return fail(QEH_E_INVALID, "build columns have different lengths");
    for (const qeh_column *c : {build_key, group_key}) {
        QEH_TRY(check_column(*c, "table build column"));
        if (c->dtype != QEH_DT_INT64 && c->dtype != QEH_DT_INT32)
            return fail(QEH_E_UNSUPPORTED, "table build columns must be Int32 / Int64");
    }
    DeviceGuard dg(ctx->device);
    const int64_t n = build_key->length;
    DevBuf bad;
    QEH_TRY(bad.alloc(ctx, 8));
    // the async form never reads the flag: no memset, whose blit kernel queued beside a running phase A
    // waited for its CUs (0.63 ms) and held the insert behind it
    if (check) QEH_HIP(hipMemsetAsync(bad.p, 0, 8, ctx->stream));
    if (n > 0) {
        KernelTimer kt(ctx, "join_build");
        hipLaunchKernelGGL(k_direct_group_insert, dim3(grid_for(ctx, n, kBlock * 4, 8)), dim3(kBlock), 0, ctx->stream,
                           make_colref(*build_key), make_colref(*group_key), n, key_min, key_range, group_min, table,
                           bad.as<uint32_t>());
        QEH_HIP(hipGetLastError());
    }
    if (!check) {  // rows outside the range are skipped: the caller's non-empty count shows them
        // (the flag buffer is freed to the pool in stream order)
        return QEH_OK;
    }
    uint32_t b = 0;
    QEH_TRY(read_small(ctx, &b, bad.p, 4));
    if (b) return fail(QEH_E_INVALID, "qeh_direct_group_table_insert: key or group key outside the given range (or NULL group key)");
    return QEH_OK;
}

extern "C" int qeh_columns_minmax(qeh_ctx *ctx, const qeh_column *cols, int n_cols, int64_t *out) {
    if (!ctx || !cols || !out || n_cols < 1) return fail(QEH_E_INVALID, "qeh_columns_minmax: bad argument");
    for (int i = 0; i < n_cols; ++i) {
        QEH_TRY(check_column(cols[i], "min/max column"));
        if (cols[i].dtype != QEH_DT_INT64 && cols[i].dtype != QEH_DT_INT32)
            return fail(QEH_E_UNSUPPORTED, "qeh_columns_minmax: Int32 / Int64 columns");
    }
    DeviceGuard dg(ctx->device);
    std::vector<int64_t> mn(n_cols), mx(n_cols), cnt(n_cols);
    QEH_TRY(columns_minmax(ctx, cols, n_cols, mn.data(), mx.data(), cnt.data()));
    for (int i = 0; i < n_cols; ++i) out[3 * i] = mn[i], out[3 * i + 1] = mx[i], out[3 * i + 2] = cnt[i];
    return QEH_OK;
}

struct StatsExtra {
    int64_t v[16];
    int32_t n;
};
__global__ void k_bcast_stats(const MinMax *__restrict__ mm, int64_t rows, StatsExtra ex, int64_t *__restrict__ out) {
    const int t = threadIdx.x;
    if (t == 0) {
        out[0] = rows;
        out[1] = rows ? mm[0].mn : INT64_MAX;
        out[2] = rows ? mm[0].mx : INT64_MIN;
        out[3] = rows ? mm[1].mn : INT64_MAX;
        out[4] = rows ? mm[1].mx : INT64_MIN;
    }
    if (t < ex.n) out[5 + t] = ex.v[t];
}

extern "C" int qeh_broadcast_stats(qeh_ctx *ctx, const qeh_column *build_key, const qeh_column *group_key,
                                   const int64_t *extra, int n_extra, int64_t *dev_out) {
    if (!ctx || !build_key || !group_key || !dev_out || n_extra < 0 || n_extra > 16 || (n_extra > 0 && !extra))
        return fail(QEH_E_INVALID, "qeh_broadcast_stats: bad argument");
    const qeh_column both[2] = {*build_key, *group_key};
    for (int i = 0; i < 2; ++i) {
        QEH_TRY(check_column(both[i], "broadcast stats column"));
        if (both[i].dtype != QEH_DT_INT64 && both[i].dtype != QEH_DT_INT32)
            return fail(QEH_E_UNSUPPORTED, "qeh_broadcast_stats: Int32 / Int64 columns");
    }
    if (build_key->length != group_key->length) return fail(QEH_E_INVALID, "qeh_broadcast_stats: columns have different lengths");
    DeviceGuard dg(ctx->device);
    DevBuf mm;  // stream-ordered reuse: read by k_bcast_stats before any later allocation's kernels
    QEH_TRY(mm.alloc(ctx, sizeof(MinMax) * 2 + 16));
    if (build_key->length > 0) QEH_TRY(columns_minmax_launch(ctx, both, 2, mm.as<MinMax>()));
    StatsExtra ex{};
    ex.n = n_extra;
    for (int i = 0; i < n_extra; ++i) ex.v[i] = extra[i];
    hipLaunchKernelGGL(k_bcast_stats, dim3(1), dim3(64), 0, ctx->stream, mm.as<MinMax>(), build_key->length, ex, dev_out);
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

// Non-zero entries of a device table of n entries of `bytes` (2 or 4) bytes (one synchronous read).
int count_nonzero_entries(qeh_ctx *ctx, const void *table, uint64_t n, int bytes, uint64_t *out) {
    *out = 0;
    if (n == 0) return QEH_OK;
    if (bytes != 2 && bytes != 4) return fail(QEH_E_INVALID, "count_nonzero_entries: entry width");
    DevBuf c;
    QEH_TRY(c.alloc(ctx, 8));
    QEH_HIP(hipMemsetAsync(c.p, 0, 8, ctx->stream));
    const int gc = grid_for(ctx, (int64_t)(n * bytes / 16 + 1), kBlock * 4, 1);
    hipLaunchKernelGGL(k_count_nonzero, dim3(gc), dim3(kBlock), 0, ctx->stream, (void *)table, n, bytes,
                       c.as<unsigned long long>(), 0u);
    QEH_HIP(hipGetLastError());
    unsigned long long v = 0;
    QEH_TRY(read_small(ctx, &v, c.p, 8));
    *out = (uint64_t)v;
    return QEH_OK;
}

extern "C" int qeh_u16_count_nonzero(qeh_ctx *ctx, const uint16_t *table, uint64_t n, int64_t *out) {
    if (!ctx || !out || (n > 0 && !table)) return fail(QEH_E_INVALID, "qeh_u16_count_nonzero: bad argument");
    DeviceGuard dg(ctx->device);
    *out = 0;
    if (n == 0) return QEH_OK;
    DevBuf c;
    QEH_TRY(c.alloc(ctx, 8));
    QEH_HIP(hipMemsetAsync(c.p, 0, 8, ctx->stream));
    const int gc = grid_for(ctx, (int64_t)(n / 8 + 1), kBlock * 4, 1);
    hipLaunchKernelGGL(k_count_nonzero, dim3(gc), dim3(kBlock), 0, ctx->stream, (void *)table, n, 2,
                       c.as<unsigned long long>(), 0u);
    QEH_HIP(hipGetLastError());
    unsigned long long v = 0;
    QEH_TRY(read_small(ctx, &v, c.p, 8));
    *out = (int64_t)v;
    return QEH_OK;
}

extern "C" int qeh_u16_count_nonzero_dev(qeh_ctx *ctx, const uint16_t *table, uint64_t n, uint64_t *dev_out) {
    if (!ctx || !dev_out || (n > 0 && !table)) return fail(QEH_E_INVALID, "qeh_u16_count_nonzero_dev: bad argument");
    DeviceGuard dg(ctx->device);
    QEH_HIP(hipMemsetAsync(dev_out, 0, 8, ctx->stream));
    if (n == 0) return QEH_OK;
    const int gc = grid_for(ctx, (int64_t)(n / 8 + 1), kBlock * 4, 1);
    hipLaunchKernelGGL(k_count_nonzero, dim3(gc), dim3(kBlock), 0, ctx->stream, (void *)table, n, 2,
                       (unsigned long long *)dev_out, 0u);
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

extern "C" int qeh_u16_table_check_dev(qeh_ctx *ctx, uint16_t *table, uint64_t n, uint32_t max_entry, uint64_t *dev_out) {
    if (!ctx || !dev_out || (n > 0 && !table) || max_entry == 0 || max_entry > 0xFFFFu)
        return fail(QEH_E_INVALID, "qeh_u16_table_check_dev: bad argument");
    DeviceGuard dg(ctx->device);
    QEH_HIP(hipMemsetAsync(dev_out, 0, 8, ctx->stream));
    if (n == 0) return QEH_OK;
    const int gc = grid_for(ctx, (int64_t)(n / 8 + 1), kBlock * 4, 1);
    hipLaunchKernelGGL(k_count_nonzero, dim3(gc), dim3(kBlock), 0, ctx->stream, (void *)table, n, 2,
                       (unsigned long long *)dev_out, max_entry);
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

int column_minmax(qeh_ctx *ctx, const qeh_column &col, int64_t *mn, int64_t *mx, int64_t *valid) {
    return columns_minmax(ctx, &col, 1, mn, mx, valid);
}

static bool memo_get(qeh_ctx *ctx, const qeh_column &c, int64_t *mn, int64_t *mx, int64_t *cnt) {
    if (!ctx->mm_memo_on) return false;
    for (int i = 0; i < ctx->mm_memo_n; ++i) {
        const auto &e = ctx->mm_memo[i];
        if (e.values == c.values && e.validity == c.validity && e.offset == c.offset && e.length == c.length &&
            e.dtype == c.dtype) {
            *mn = e.mn, *mx = e.mx, *cnt = e.cnt;
            return true;
        }
    }
    return false;
}

static void memo_put(qeh_ctx *ctx, const qeh_column &c, int64_t mn, int64_t mx, int64_t cnt) {
    const int cap = (int)(sizeof(ctx->mm_memo) / sizeof(ctx->mm_memo[0]));
    if (!ctx->mm_memo_on || ctx->mm_memo_n >= cap) return;
    ctx->mm_memo[ctx->mm_memo_n++] = {c.values, c.validity, c.offset, c.length, c.dtype, mn, mx, cnt};
}

int columns_minmax_launch(qeh_ctx *ctx, const qeh_column *cols, int n, MinMax *dev_out) {
    // one partial-reduction launch per group of up to four columns (blockIdx.y = column), then one
    // final reduction per group; four workgroups per CU on long columns (64 KB of loads in flight
    // per CU), one per CU below 2^26 rows
    const int cus = ctx->props.multiProcessorCount;
    DevBuf part;  // stream-ordered pool: reusable once the kernels below have run
    QEH_TRY(part.alloc(ctx, sizeof(MinMax) * (size_t)kMinMaxCols * cus * 4));
    for (int i0 = 0; i0 < n; i0 += kMinMaxCols) {
        MinMaxJob j{};
        int64_t longest = 0;
        const int nc = std::min(kMinMaxCols, n - i0);
        for (int q = 0; q < nc; ++q) {
            j.c[q] = make_colref(cols[i0 + q]);
            j.n[q] = cols[i0 + q].length;
            longest = std::max<int64_t>(longest, cols[i0 + q].length);
        }
        const int nb = grid_for(ctx, std::max<int64_t>(longest, 1), kBlock * 8, longest >= ((int64_t)1 << 26) ? 4 : 1);
        hipLaunchKernelGGL(k_key_minmax_n, dim3(nb, nc), dim3(kBlock), 0, ctx->stream, j, part.as<MinMax>());
        hipLaunchKernelGGL(k_minmax_final, dim3(nc), dim3(kBlock), 0, ctx->stream, part.as<MinMax>(), nb, dev_out + i0);
    }
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

// The partial min / max of up to kMinMaxCols columns only (part[column * nb + workgroup], nb workgroups
// per column): for callers that reduce the partials in a kernel of their own.
int columns_minmax_partials(qeh_ctx *ctx, const qeh_column *cols, int n, MinMax *part, int *nb_out) {
    if (n < 1 || n > kMinMaxCols) return fail(QEH_E_INVALID, "columns_minmax_partials: 1..4 columns");
    MinMaxJob j{};
    int64_t longest = 0;
    for (int q = 0; q < n; ++q) {
        j.c[q] = make_colref(cols[q]);
        j.n[q] = cols[q].length;
        longest = std::max<int64_t>(longest, cols[q].length);
    }
    const int nb = grid_for(ctx, std::max<int64_t>(longest, 1), kBlock * 8, longest >= ((int64_t)1 << 26) ? 4 : 1);
    hipLaunchKernelGGL(k_key_minmax_n, dim3(nb, n), dim3(kBlock), 0, ctx->stream, j, part);
    QEH_HIP(hipGetLastError());
    *nb_out = nb;
    return QEH_OK;
}
int minmax_partials_max_blocks(qeh_ctx *ctx) { return ctx->props.multiProcessorCount * 4; }

int columns_minmax_collect(qeh_ctx *ctx, const qeh_column *cols, int n, const MinMax *dev_out, int64_t *mn, int64_t *mx,
                           int64_t *valid) {
    std::vector<MinMax> hm((size_t)n);
    QEH_TRY(read_small(ctx, hm.data(), dev_out, sizeof(MinMax) * (size_t)n));
    for (int i = 0; i < n; ++i) {
        mn[i] = hm[i].mn;
        mx[i] = hm[i].mx;
        valid[i] = (int64_t)hm[i].cnt;
        memo_put(ctx, cols[i], mn[i], mx[i], valid[i]);
    }
    return QEH_OK;
}

// several columns, one synchronous read for all of them (none when every range is memoised)
int columns_minmax(qeh_ctx *ctx, const qeh_column *cols, int n, int64_t *mn, int64_t *mx, int64_t *valid) {
    if (n <= 0) return QEH_OK;
    bool all = true;
    for (int i = 0; i < n && all; ++i) all = memo_get(ctx, cols[i], &mn[i], &mx[i], &valid[i]);
    if (all) return QEH_OK;
    DevBuf mm;
    QEH_TRY(mm.alloc(ctx, sizeof(MinMax) * (size_t)n + 16));
    QEH_TRY(columns_minmax_launch(ctx, cols, n, mm.as<MinMax>()));
    return columns_minmax_collect(ctx, cols, n, mm.as<MinMax>(), mn, mx, valid);
}

static uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

static int bits_for(uint64_t v) {  // bits to represent values 0..v
    int b = 1;
    while (b < 64 && (v >> b) != 0) ++b;
    return b;
}

// BUCKET payload width for a build's largest payload: 16 or 32 bits, 0 = too wide (QEH_NO_BUCKET=1: never)
static int bucket_pbits(uint64_t payload_max) {
    if (std::getenv("QEH_NO_BUCKET")) return 0;
    return payload_max < 0xFFFFull ? 16 : payload_max < 0xFFFFFFFFull ? 32 : 0;
}

int build_join_table(qeh_ctx *ctx, const qeh_column &key, const RowPayload &row_payload, uint64_t payload_max,
                     BuiltTable *out, int force_kind) {
    QEH_TRY(check_column(key, "join key"));
    if (key.dtype != QEH_DT_INT64 && key.dtype != QEH_DT_INT32)
        return fail(QEH_E_UNSUPPORTED, "hash join keys must be Int32/Int64 on the device");
    const int64_t n = key.length;
    ColRef kr = make_colref(key);
    MinMax hm{};
    {
        int64_t mn, mx, cnt;
        QEH_TRY(columns_minmax(ctx, &key, 1, &mn, &mx, &cnt));
        hm.mn = mn, hm.mx = mx, hm.cnt = (uint64_t)cnt;
    }

    HashTable &t = out->t;
    t = HashTable{};
    out->n_inserted = (int64_t)hm.cnt;
    if (hm.cnt == 0) {  // nothing can match: empty DIRECT table with an impossible range
        t.kind = TK_DIRECT;
        t.kmin = 1;
        t.kmax = 0;
        t.unique = 1;
        return QEH_OK;
    }
    t.kmin = hm.mn;
    t.kmax = hm.mx;
    const uint64_t range = (uint64_t)hm.mx - (uint64_t)hm.mn + 1ull;  // may wrap to 0 for the full int64 range
    const uint64_t nv = hm.cnt;
    int kind = force_kind >= 0 ? force_kind : forced_table_kind();
    const bool direct_ok = direct_table_ok(range, nv, payload_max);
    const int pbits = bits_for(payload_max);
    const int kbits = range == 0 ? 64 : bits_for(range);  // key part holds 1..range
    const bool packed_ok = kbits + pbits <= 64;
    if (kind == TK_DIRECT && !direct_ok) kind = -1;
    if (kind == TK_PACKED && !packed_ok) kind = -1;
    if (kind < 0) kind = direct_ok ? TK_DIRECT : (packed_ok ? TK_PACKED : bucket_pbits(payload_max) ? TK_BUCKET : TK_WIDE);
    if (kind == TK_BUCKET && !bucket_pbits(payload_max)) kind = TK_WIDE;

    DevBuf flag;
    QEH_TRY(flag.alloc(ctx, 8));
    QEH_HIP(hipMemsetAsync(flag.p, 0, 8, ctx->stream));
    const int grid = grid_for(ctx, n, kBlock * 4, 8);
    uint32_t dup = 0;

    if (kind == TK_DIRECT) {
        t.kind = TK_DIRECT;
        t.range = range;
        // entries fit 16 bits: half the table's cache footprint, built in place
        const bool narrow = payload_max < 0xFFFFull && !std::getenv("QEH_NO_U16");
        unsigned long long *nz = (unsigned long long *)flag.p;
        {
            KernelTimer kt(ctx, "join_build");
            const int gc = grid_for(ctx, (int64_t)(range / 8 + 1), kBlock * 4, 1);  // one partial sum per CU
            if (narrow) {
                QEH_TRY(out->payload16.alloc(ctx, range * 2 + 16));
                t.payload16 = out->payload16.as<uint16_t>();
                QEH_HIP(hipMemsetAsync(t.payload16, 0, range * 2 + 16, ctx->stream));
                // XCD-split insert for tables past one L2 when the build runs under a long phase A:
                // alone it is slower (every workgroup reads all keys: 0.75 vs 0.52 ms for 1e7
                // rows), beside 1e9 probe rows it disturbs phase A less (6.65-6.76 vs 6.85 ms per
                // metric step, same box).  QEH_INSERT_XCD=0/1 overrides.
                // QEH_INSERT_XCD=1 (default for the XCD split): every XCD's workgroups read all keys
                // and keep their range's (8 key reads); 2: keys partitioned into per-range lists once
                // (k_xcd_lists), each list drained by one XCD
                // (measured: the list version cuts phase A's interference, 6.67 vs 6.82 ms of kernel
                // time, but its two dependent kernels finish after phase A: 7.2 vs 7.0 ms per step)
                int xcd = range * 2 >= (4ull << 20) && ctx->build_beside_rows >= 32 * n ? 1 : 0;
                if (const char *e = std::getenv("QEH_INSERT_XCD")) xcd = std::atoi(e);
                // the eight lists are sized for every row each (64 B per build row): opt-in only, and
                // capped at 2^24 build rows (1 GB of lists) so it cannot crowd a large probe's memory
                DevBuf lists, cursor;
                if (xcd == 2 && (n > ((int64_t)1 << 24) || lists.alloc(ctx, (size_t)n * 8 * 8) != QEH_OK ||
                                 cursor.alloc(ctx, 64) != QEH_OK))
                    xcd = 1;
                if (xcd == 2) {
                    const uint64_t span = (range + 7) >> 3;
                    QEH_HIP(hipMemsetAsync(cursor.p, 0, 64, ctx->stream));
                    hipLaunchKernelGGL(k_xcd_lists, dim3(grid_for(ctx, n, kBlock * kXcdRows, 4)), dim3(kBlock), 0,
                                       ctx->stream, kr, n, row_payload, t.kmin, span, lists.as<uint64_t>(), n,
                                       cursor.as<unsigned long long>());
                    hipLaunchKernelGGL(k_insert_xcd_lists, dim3(grid_for(ctx, n / 8 + 1, kBlock * 4, 4) * 8), dim3(kBlock),
                                       0, ctx->stream, lists.as<uint64_t>(), n, cursor.as<unsigned long long>(), t);
                } else if (xcd)
                    hipLaunchKernelGGL(k_insert_direct16_xcd, dim3(grid_for(ctx, n, kBlock * 4, 8) * 8), dim3(kBlock), 0,
                                       ctx->stream, kr, n, row_payload, t);
                else
                    hipLaunchKernelGGL(k_insert_direct16, dim3(grid), dim3(kBlock), 0, ctx->stream, kr, n, row_payload, t);
                hipLaunchKernelGGL(k_count_nonzero, dim3(gc), dim3(kBlock), 0, ctx->stream, (void *)t.payload16, range, 2,
                                   nz, 0u);
            } else {
                QEH_TRY(out->payload.alloc(ctx, range * 4 + 16));
                t.payload = out->payload.as<uint32_t>();
                QEH_HIP(hipMemsetAsync(t.payload, 0, range * 4 + 16, ctx->stream));
                hipLaunchKernelGGL(k_insert_direct, dim3(grid), dim3(kBlock), 0, ctx->stream, kr, n, row_payload, t);
                hipLaunchKernelGGL(k_count_nonzero, dim3(gc), dim3(kBlock), 0, ctx->stream, (void *)t.payload, range, 4,
                                   nz, 0u);
            }
        }
        QEH_HIP(hipGetLastError());
        unsigned long long filled = 0;
        QEH_TRY(read_small(ctx, &filled, flag.p, 8));
        if (filled == (unsigned long long)hm.cnt) {
            t.unique = 1;
            return QEH_OK;
        }
        t.payload16 = nullptr;
        t.payload = nullptr;
        out->payload16.reset();
        // duplicate build keys: a perfect-hash slot holds one row; rebuild hashed
        out->payload.reset();
        QEH_HIP(hipMemsetAsync(flag.p, 0, 8, ctx->stream));
        kind = packed_ok ? TK_PACKED : bucket_pbits(payload_max) ? TK_BUCKET : TK_WIDE;
        if (force_kind == TK_DIRECT) force_kind = -1;
    }

    if (kind == TK_BUCKET) {
        t.kind = TK_BUCKET;
        t.pbits = bucket_pbits(payload_max);
        t.nbkt = std::max<uint64_t>(64, (nv * 10 + 6 * bucket_slots(t.pbits) - 1) / (6 * bucket_slots(t.pbits)));  // 60 % load
        QEH_TRY(out->slots.alloc(ctx, t.nbkt * 64));
        t.slots = out->slots.as<uint64_t>();
        {
            KernelTimer kt(ctx, "join_build");
            QEH_HIP(hipMemsetAsync(t.slots, 0, t.nbkt * 64, ctx->stream));
            hipLaunchKernelGGL(k_insert_bucket, dim3(grid), dim3(kBlock), 0, ctx->stream, kr, n, row_payload, t);
            t.unique = 0;
            hipLaunchKernelGGL(k_wide_dups, dim3(grid), dim3(kBlock), 0, ctx->stream, kr, n, t, flag.as<uint32_t>());
        }
        QEH_HIP(hipGetLastError());
        QEH_TRY(read_small(ctx, &dup, flag.p, 4));
        if (!dup) {
            t.unique = 1;
            return QEH_OK;
        }
        // repeated build keys: the WIDE layout (multi-match probing over 16-B slots)
        out->slots.reset();
        t.slots = nullptr;
        QEH_HIP(hipMemsetAsync(flag.p, 0, 8, ctx->stream));
        kind = TK_WIDE;
    }

    const uint64_t cap = std::max<uint64_t>(1024, next_pow2((nv * 5 + 2) / 3));
    t.mask = cap - 1;
    if (kind == TK_PACKED) {
        t.kind = TK_PACKED;
        t.pbits = pbits;
        QEH_TRY(out->slots.alloc(ctx, cap * 8));
        t.slots = out->slots.as<uint64_t>();
        {
            KernelTimer kt(ctx, "join_build");
            QEH_HIP(hipMemsetAsync(t.slots, 0, cap * 8, ctx->stream));
            hipLaunchKernelGGL(k_insert_packed, dim3(grid), dim3(kBlock), 0, ctx->stream, kr, n, row_payload, t,
                               flag.as<uint32_t>());
        }
        QEH_HIP(hipGetLastError());
        QEH_TRY(read_small(ctx, &dup, flag.p, 4));
        t.unique = dup ? 0 : 1;
        return QEH_OK;
    }
    t.kind = TK_WIDE;
    QEH_TRY(out->slots.alloc(ctx, cap * 16));
    t.slots = out->slots.as<uint64_t>();
    {
        KernelTimer kt(ctx, "join_build");
        QEH_HIP(hipMemsetAsync(t.slots, 0, cap * 16, ctx->stream));
        hipLaunchKernelGGL(k_insert_wide, dim3(grid), dim3(kBlock), 0, ctx->stream, kr, n, row_payload, t);
        t.unique = 0;
        hipLaunchKernelGGL(k_wide_dups, dim3(grid), dim3(kBlock), 0, ctx->stream, kr, n, t, flag.as<uint32_t>());
    }
    QEH_HIP(hipGetLastError());
    QEH_TRY(read_small(ctx, &dup, flag.p, 4));
    t.unique = dup ? 0 : 1;
    return QEH_OK;
}

// ---- group ids over key tuples ------------------------------------------------------
// Insert every row's key tuple; slot_of_row[i] = its slot.  A row that probes
// more than kGroupMaxProbe slots flags overflow and the host retries with an
// 8x table; once flagged, the remaining rows stop early.
constexpr uint64_t kGroupMaxProbe = 64;

__global__ void k_group_insert(KeyCols keys, int64_t n, uint32_t *__restrict__ slots, uint64_t mask,
                               uint32_t *__restrict__ slot_of_row, uint32_t *overflow) {
    int iter = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if ((++iter & 7) == 0 && __hip_atomic_load(overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
        uint64_t h = tuple_hash(keys, i) & mask;
        uint64_t probe = 0;
        for (; probe <= mask && probe < kGroupMaxProbe; ++probe) {
            // read first: few groups x many rows would otherwise serialise on
            // atomics to the same words; a stale EMPTY just falls into the CAS
            uint32_t old = __hip_atomic_load(&slots[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old == kEmpty32) old = atomicCAS(&slots[h], kEmpty32, (uint32_t)i);
            if (old == kEmpty32 || tuple_eq(keys, old, i)) break;
            h = (h + 1) & mask;
        }
        if (probe > mask || probe >= kGroupMaxProbe) {
            *overflow = 1u;
            return;
        }
        if (slot_of_row) slot_of_row[i] = (uint32_t)h;
    }
}

__global__ void k_slot_occupied(const uint32_t *__restrict__ slots, uint64_t cap, uint32_t *__restrict__ occ) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)cap; i += (int64_t)gridDim.x * blockDim.x)
        occ[i] = slots[i] != kEmpty32;
}

__global__ void k_dense_rep(const uint32_t *__restrict__ slots, uint64_t cap, const uint64_t *__restrict__ dense,
                            uint32_t *__restrict__ rep_row) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)cap; i += (int64_t)gridDim.x * blockDim.x)
        if (slots[i] != kEmpty32) rep_row[dense[i]] = slots[i];
}

__global__ void k_row_gid(const uint32_t *__restrict__ slot_of_row, int64_t n, const uint64_t *__restrict__ dense,
                          uint32_t *__restrict__ gid) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        gid[i] = (uint32_t)dense[slot_of_row[i]];
}

// DIRECT group table (one non-null integer key of bounded range): slot =
// key - kmin, slots[slot] = any row carrying the key (plain stores).
__global__ void k_group_direct(ColRef key, int64_t n, int64_t kmin, uint32_t *__restrict__ slots,
                               uint32_t *__restrict__ slot_of_row) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)((uint64_t)load_i64(key, i) - (uint64_t)kmin);
        slots[s] = (uint32_t)i;
        slot_of_row[i] = s;
    }
}

// Small key ranges: the slots live in LDS per workgroup and each workgroup publishes only the
// slots it filled.  Plain global stores from every row to a few hundred lines serialise on those
// lines (90 us for 1e7 rows into 1024 slots; a winner per slot is all the table needs).
constexpr uint32_t kGroupDirectLds = 16384;  // slots (64 KB of LDS)

__global__ __launch_bounds__(kBlock) void k_group_direct_lds(ColRef key, int64_t n, int64_t kmin, uint32_t range,
                                                             uint32_t *__restrict__ slots, uint32_t *__restrict__ slot_of_row) {
    extern __shared__ uint32_t ls[];
    for (uint32_t i = threadIdx.x; i < range; i += blockDim.x) ls[i] = 0xFFFFFFFFu;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)((uint64_t)load_i64(key, i) - (uint64_t)kmin);
        ls[s] = (uint32_t)i;
        slot_of_row[i] = s;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < range; i += blockDim.x)
        if (ls[i] != 0xFFFFFFFFu) slots[i] = ls[i];
}

static int group_table_finish(qeh_ctx *ctx, GroupTable *out);

int build_group_table(qeh_ctx *ctx, const qeh_column *keys, int n_keys, int64_t n_rows, GroupTable *out,
                      uint32_t *slot_of_row, bool allow_direct) {
    if (n_keys < 1 || n_keys > kMaxGroupKeys)
        return fail(QEH_E_UNSUPPORTED, "1..4 group keys supported on the device");
    KeyCols &kc = out->keys;
    kc = KeyCols{};
    kc.n = n_keys;
    for (int i = 0; i < n_keys; ++i) {
        QEH_TRY(check_column(keys[i], "group key"));
        if (keys[i].dtype == QEH_DT_UTF8) return fail(QEH_E_UNSUPPORTED, "Utf8 group keys are not supported on the device");
        if (keys[i].length != n_rows) return fail(QEH_E_INVALID, "group key length mismatch");
        kc.c[i] = make_colref(keys[i]);
    }
    out->direct = false;
    if (allow_direct && slot_of_row && n_keys == 1 && n_rows > 0 && kc.c[0].validity == nullptr &&
        (kc.c[0].dtype == QEH_DT_INT64 || kc.c[0].dtype == QEH_DT_INT32) && !std::getenv("QEH_NO_DIRECT_GROUPS")) {
        MinMax hm{};
        {
            int64_t mn, mx, cnt;
            QEH_TRY(columns_minmax(ctx, &keys[0], 1, &mn, &mx, &cnt));
            hm.mn = mn, hm.mx = mx, hm.cnt = (uint64_t)cnt;
        }
        const uint64_t range = (uint64_t)hm.mx - (uint64_t)hm.mn + 1ull;
        if (range != 0 && range <= std::max<uint64_t>(4 * (uint64_t)n_rows, 65536) && range < (1ull << 31)) {
            out->direct = true;
            out->kmin = hm.mn;
            out->cap = range;
            QEH_TRY(out->slots.alloc(ctx, range * 4));
            QEH_HIP(hipMemsetAsync(out->slots.p, 0xFF, range * 4, ctx->stream));
            {
                KernelTimer kt(ctx, "group_insert");
                if (range <= kGroupDirectLds && !std::getenv("QEH_NO_GROUP_LDS"))
                    hipLaunchKernelGGL(k_group_direct_lds, dim3(grid_for(ctx, n_rows, kBlock * 16, 1)), dim3(kBlock),
                                       range * 4, ctx->stream, kc.c[0], n_rows, hm.mn, (uint32_t)range,
                                       out->slots.as<uint32_t>(), slot_of_row);
                else
                    hipLaunchKernelGGL(k_group_direct, dim3(grid_for(ctx, n_rows, kBlock * 4, 8)), dim3(kBlock), 0,
                                       ctx->stream, kc.c[0], n_rows, hm.mn, out->slots.as<uint32_t>(), slot_of_row);
            }
            QEH_HIP(hipGetLastError());
            return group_table_finish(ctx, out);
        }
    }
    // capacity: start at 16 Ki slots (L2-resident; the common few-groups case)
    // bounded by 2x the rows, grown 8x whenever a probe sequence overflows
    uint64_t cap = std::max<uint64_t>(1024, std::min<uint64_t>(16384, next_pow2((uint64_t)std::max<int64_t>(n_rows, 1) * 2)));
    DevBuf flag;
    QEH_TRY(flag.alloc(ctx, 8));
    for (;;) {
        QEH_TRY(out->slots.alloc(ctx, cap * 4));
        QEH_HIP(hipMemsetAsync(out->slots.p, 0xFF, cap * 4, ctx->stream));
        QEH_HIP(hipMemsetAsync(flag.p, 0, 8, ctx->stream));
        if (n_rows > 0) {
            KernelTimer kt(ctx, "group_insert");
            hipLaunchKernelGGL(k_group_insert, dim3(grid_for(ctx, n_rows, kBlock * 4, 8)), dim3(kBlock), 0, ctx->stream, kc,
                               n_rows, out->slots.as<uint32_t>(), cap - 1, slot_of_row, flag.as<uint32_t>());
        }
        QEH_HIP(hipGetLastError());
        uint32_t ovf = 0;
        QEH_TRY(read_small(ctx, &ovf, flag.p, 4));
        if (!ovf) break;
        if (cap >= (1ull << 33)) return fail(QEH_E_OOM, "group table overflow");
        cap <<= 3;
    }
    out->cap = cap;
    return group_table_finish(ctx, out);
}

// Dense ids 0..G-1 in slot order and a representative row per group.
// Small tables: occupancy, exclusive scan, dense ids, representative rows and the group count in
// one workgroup.  Under the prelaunched phase A the separate single-workgroup scan kernel
// (k_scan_top) was held for the whole of phase A, and the build behind it with it.
constexpr int kSmallFinishPer = 16;
constexpr uint64_t kSmallFinish = (uint64_t)kBlock * kSmallFinishPer;

__global__ __launch_bounds__(kBlock) void k_group_finish_small(const uint32_t *__restrict__ slots, uint64_t cap,
                                                               uint64_t *__restrict__ dense, uint32_t *__restrict__ rep_row,
                                                               uint64_t *__restrict__ total) {
    __shared__ uint32_t wsum[kBlock / 64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t s[kSmallFinishPer], cnt = 0;
#pragma unroll
    for (int j = 0; j < kSmallFinishPer; ++j) {
        const uint64_t i = (uint64_t)t * kSmallFinishPer + j;
        s[j] = i < cap ? slots[i] : kEmpty32;
        cnt += s[j] != kEmpty32;
    }
    uint32_t incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 64);
        if (lane >= d) incl += o;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int q = 0; q < w; ++q) base += wsum[q];
    uint32_t ex = base + incl - cnt;
#pragma unroll
    for (int j = 0; j < kSmallFinishPer; ++j) {
        const uint64_t i = (uint64_t)t * kSmallFinishPer + j;
        if (i >= cap) break;
        dense[i] = ex;
        if (s[j] != kEmpty32) rep_row[ex++] = s[j];
    }
    if (t == kBlock - 1) {
        uint32_t g = 0;
        for (int q = 0; q < kBlock / 64; ++q) g += wsum[q];
        *total = g;
    }
}

static int group_table_finish(qeh_ctx *ctx, GroupTable *out) {
    const uint64_t cap = out->cap;
    if (cap <= kSmallFinish && !std::getenv("QEH_NO_SMALL_FINISH")) {
        QEH_TRY(out->dense.alloc(ctx, cap * 8));
        QEH_TRY(out->rep_row.alloc(ctx, std::max<uint64_t>(cap, 1) * 4));
        DevBuf tot;
        QEH_TRY(tot.alloc(ctx, 16));
        hipLaunchKernelGGL(k_group_finish_small, dim3(1), dim3(kBlock), 0, ctx->stream, out->slots.as<uint32_t>(), cap,
                           out->dense.as<uint64_t>(), out->rep_row.as<uint32_t>(), tot.as<uint64_t>());
        QEH_HIP(hipGetLastError());
        uint64_t G = 0;
        QEH_TRY(read_small(ctx, &G, tot.p, 8));
        out->groups = (int64_t)G;
        return QEH_OK;
    }
    DevBuf occ;
    QEH_TRY(occ.alloc(ctx, cap * 4));
    QEH_TRY(out->dense.alloc(ctx, cap * 8));
    const int g2 = grid_for(ctx, (int64_t)cap, kBlock * 4, 8);
    hipLaunchKernelGGL(k_slot_occupied, dim3(g2), dim3(kBlock), 0, ctx->stream, out->slots.as<uint32_t>(), cap,
                       occ.as<uint32_t>());
    uint64_t G = 0;
    QEH_TRY(exclusive_scan_u32(ctx, occ.as<uint32_t>(), out->dense.as<uint64_t>(), (int64_t)cap, &G));
    out->groups = (int64_t)G;
    QEH_TRY(out->rep_row.alloc(ctx, std::max<uint64_t>(G, 1) * 4));
    hipLaunchKernelGGL(k_dense_rep, dim3(g2), dim3(kBlock), 0, ctx->stream, out->slots.as<uint32_t>(), cap,
                       out->dense.as<uint64_t>(), out->rep_row.as<uint32_t>());
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

int group_slots_of_rows(qeh_ctx *ctx, const qeh_column *keys, int n_keys, int64_t n_rows, GroupTable *table,
                        DevBuf *slot_of_row) {
    QEH_TRY(slot_of_row->alloc(ctx, (size_t)std::max<int64_t>(n_rows, 1) * 4));
    return build_group_table(ctx, keys, n_keys, n_rows, table, slot_of_row->as<uint32_t>(), true);
}

int assign_group_ids(qeh_ctx *ctx, const qeh_column *keys, int n_keys, int64_t n_rows, GroupTable *table,
                     DevBuf *gid_of_row) {
    DevBuf slot_of_row;
    QEH_TRY(group_slots_of_rows(ctx, keys, n_keys, n_rows, table, &slot_of_row));
    QEH_TRY(gid_of_row->alloc(ctx, (size_t)std::max<int64_t>(n_rows, 1) * 4));
    if (n_rows > 0)
        hipLaunchKernelGGL(k_row_gid, dim3(grid_for(ctx, n_rows, kBlock * 4, 8)), dim3(kBlock), 0, ctx->stream,
                           slot_of_row.as<uint32_t>(), n_rows, table->dense.as<uint64_t>(), gid_of_row->as<uint32_t>());
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

}  // namespace qeh
