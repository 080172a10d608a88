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
struct MinMax {
    int64_t mn, mx;
    uint64_t cnt;
    uint32_t bad;  // unsupported key type seen
};

__global__ void k_key_minmax(ColRef key, int64_t n, MinMax *out) {
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    uint64_t cnt = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!col_valid(key, i)) continue;
        int64_t k = load_i64(key, i);
        mn = k < mn ? k : mn;
        mx = k > mx ? k : mx;
        ++cnt;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        int64_t a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64);
        uint64_t c = __shfl_xor(cnt, d, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
        cnt += c;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin((long long *)&out->mn, (long long)mn);
        atomicMax((long long *)&out->mx, (long long)mx);
        atomicAdd((unsigned long long *)&out->cnt, (unsigned long long)cnt);
    }
}

__global__ void k_minmax_init(MinMax *m) {
    m->mn = INT64_MAX;
    m->mx = INT64_MIN;
    m->cnt = 0;
    m->bad = 0;
}

// ---- inserts -------------------------------------------------------------------------
__device__ __forceinline__ uint32_t payload_of(const uint32_t *row_payload, int64_t row) {
    return row_payload ? row_payload[row] : (uint32_t)row;
}

__global__ void k_insert_direct(ColRef key, int64_t n, const uint32_t *row_payload, HashTable t, uint32_t *dup) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!col_valid(key, i)) continue;
        int64_t k = load_i64(key, i);
        uint32_t e = payload_of(row_payload, i) + 1u;
        uint32_t old = atomicCAS(&t.payload[(uint64_t)k - (uint64_t)t.kmin], 0u, e);
        if (old != 0u) *dup = 1u;
    }
}

__global__ void k_insert_packed(ColRef key, int64_t n, const uint32_t *row_payload, HashTable t, uint32_t *dup) {
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

__global__ void k_insert_wide(ColRef key, int64_t n, const uint32_t *row_payload, HashTable t) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!col_valid(key, i)) continue;
        int64_t k = load_i64(key, i);
        uint64_t h = hash64((uint64_t)k) & t.mask;
        for (uint64_t probe = 0; probe <= t.mask; ++probe) {
            if (atomicCAS(&t.state[h], 0u, 1u) == 0u) {
                t.slots[h] = (uint64_t)k;
                t.payload[h] = payload_of(row_payload, i);
                break;
            }
            h = (h + 1) & t.mask;
        }
    }
}

__global__ void k_narrow_direct(const uint32_t *__restrict__ in, uint64_t n, uint16_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (uint16_t)in[i];
}

// Duplicate detection for WIDE tables (separate launch: all slots are final).
__global__ void k_wide_dups(ColRef key, int64_t n, HashTable t, uint32_t *dup) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!col_valid(key, i)) continue;
        int64_t k = load_i64(key, i);
        int c = table_probe(t, k, [](uint32_t) {});
        if (c > 1) *dup = 1u;
    }
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

int build_join_table(qeh_ctx *ctx, const qeh_column &key, const uint32_t *row_payload, uint64_t payload_max,
                     BuiltTable *out, int force_kind) {
    QEH_TRY(check_column(key, "join key"));
    if (key.dtype != QEH_DT_INT64 && key.dtype != QEH_DT_INT32)
        return fail(QEH_E_UNSUPPORTED, "hash join keys must be Int32/Int64 on the device");
    const int64_t n = key.length;
    ColRef kr = make_colref(key);
    DevBuf mm;
    QEH_TRY(mm.alloc(ctx, sizeof(MinMax) + 16));
    MinMax hm{};
    {
        KernelTimer kt(ctx, "join_build");
        hipLaunchKernelGGL(k_minmax_init, dim3(1), dim3(1), 0, ctx->stream, mm.as<MinMax>());
        if (n > 0)
            hipLaunchKernelGGL(k_key_minmax, dim3(grid_for(ctx, n, kBlock * 16, 4)), dim3(kBlock), 0, ctx->stream, kr, n,
                               mm.as<MinMax>());
    }
    QEH_HIP(hipGetLastError());
    QEH_TRY(read_small(ctx, &hm, mm.p, sizeof(MinMax)));

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
    const bool direct_ok = range != 0 && range <= 4 * nv + 1024 && range < (1ull << 32) && payload_max < 0xFFFFFFFEull;
    const int pbits = bits_for(payload_max);
    const int kbits = range == 0 ? 64 : bits_for(range);  // key part holds 1..range
    const bool packed_ok = kbits + pbits <= 64;
    if (kind == TK_DIRECT && !direct_ok) kind = -1;
    if (kind == TK_PACKED && !packed_ok) kind = -1;
    if (kind < 0) kind = direct_ok ? TK_DIRECT : (packed_ok ? TK_PACKED : TK_WIDE);

    DevBuf flag;
    QEH_TRY(flag.alloc(ctx, 8));
    QEH_HIP(hipMemsetAsync(flag.p, 0, 8, ctx->stream));
    const int grid = grid_for(ctx, n, kBlock * 4, 8);
    uint32_t dup = 0;

    if (kind == TK_DIRECT) {
        t.kind = TK_DIRECT;
        t.range = range;
        QEH_TRY(out->payload.alloc(ctx, range * 4));
        t.payload = out->payload.as<uint32_t>();
        {
            KernelTimer kt(ctx, "join_build");
            QEH_HIP(hipMemsetAsync(t.payload, 0, range * 4, ctx->stream));
            hipLaunchKernelGGL(k_insert_direct, dim3(grid), dim3(kBlock), 0, ctx->stream, kr, n, row_payload, t,
                               flag.as<uint32_t>());
        }
        QEH_HIP(hipGetLastError());
        QEH_TRY(read_small(ctx, &dup, flag.p, 4));
        if (!dup) {
            t.unique = 1;
            if (payload_max < 0xFFFFull && !std::getenv("QEH_NO_U16")) {  // entries fit 16 bits: halve the table's cache footprint
                QEH_TRY(out->payload16.alloc(ctx, range * 2));
                {
                    KernelTimer kt(ctx, "join_build");
                    hipLaunchKernelGGL(k_narrow_direct, dim3(grid_for(ctx, (int64_t)range, kBlock * 8, 8)), dim3(kBlock), 0,
                                       ctx->stream, t.payload, range, out->payload16.as<uint16_t>());
                }
                QEH_HIP(hipGetLastError());
                t.payload16 = out->payload16.as<uint16_t>();
                t.payload = nullptr;
                out->payload.reset();
            }
            return QEH_OK;
        }
        // duplicate build keys: a perfect-hash slot holds one row; rebuild hashed
        out->payload.reset();
        QEH_HIP(hipMemsetAsync(flag.p, 0, 8, ctx->stream));
        kind = packed_ok ? TK_PACKED : TK_WIDE;
        if (force_kind == TK_DIRECT) force_kind = -1;
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
    QEH_TRY(out->slots.alloc(ctx, cap * 8));
    QEH_TRY(out->payload.alloc(ctx, cap * 4));
    QEH_TRY(out->state.alloc(ctx, cap * 4));
    t.slots = out->slots.as<uint64_t>();
    t.payload = out->payload.as<uint32_t>();
    t.state = out->state.as<uint32_t>();
    {
        KernelTimer kt(ctx, "join_build");
        QEH_HIP(hipMemsetAsync(t.state, 0, cap * 4, ctx->stream));
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
__global__ void k_group_insert(KeyCols keys, int64_t n, uint32_t *__restrict__ slots, uint64_t mask,
                               uint32_t *__restrict__ slot_of_row, uint32_t *overflow) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t h = tuple_hash(keys, i) & mask;
        uint64_t probe = 0;
        for (; probe <= mask; ++probe) {
            // read first: few groups x many rows would otherwise serialise on
            // atomics to the same words; a stale EMPTY just falls into the CAS
            uint32_t old = __hip_atomic_load(&slots[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old == kEmpty32) old = atomicCAS(&slots[h], kEmpty32, (uint32_t)i);
            if (old == kEmpty32 || tuple_eq(keys, old, i)) break;
            h = (h + 1) & mask;
        }
        if (probe > mask) *overflow = 1u;
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

int build_group_table(qeh_ctx *ctx, const qeh_column *keys, int n_keys, int64_t n_rows, GroupTable *out,
                      uint32_t *slot_of_row) {
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
    // capacity: 2x the row bound capped at 2^21 slots, grown 4x on overflow
    uint64_t cap = std::max<uint64_t>(1024, next_pow2((uint64_t)std::min<int64_t>(n_rows, 1 << 20) * 2));
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
        cap <<= 2;
    }
    out->cap = cap;
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

int assign_group_ids(qeh_ctx *ctx, const qeh_column *keys, int n_keys, int64_t n_rows, GroupTable *table,
                     DevBuf *gid_of_row) {
    DevBuf slot_of_row;
    QEH_TRY(slot_of_row.alloc(ctx, (size_t)std::max<int64_t>(n_rows, 1) * 4));
    QEH_TRY(build_group_table(ctx, keys, n_keys, n_rows, table, slot_of_row.as<uint32_t>()));
    QEH_TRY(gid_of_row->alloc(ctx, (size_t)std::max<int64_t>(n_rows, 1) * 4));
    if (n_rows > 0)
        hipLaunchKernelGGL(k_row_gid, dim3(grid_for(ctx, n_rows, kBlock * 4, 8)), dim3(kBlock), 0, ctx->stream,
                           slot_of_row.as<uint32_t>(), n_rows, table->dense.as<uint64_t>(), gid_of_row->as<uint32_t>());
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

}  // namespace qeh
