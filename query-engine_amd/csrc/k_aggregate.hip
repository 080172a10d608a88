// HashAggregateExec and the fused Filter -> HashJoin -> HashAggregate pipeline.
//
// Reference: execute_aggregate (crates/query-executor/src/executor.rs:157-190)
// computes global aggregates by concatenating every batch of the argument and
// calling evaluate_aggregate (operators.rs:745-848); GROUP BY returns no rows
// (:189).  The intended grouped semantics are SURVEY.md §8.0: one row per
// distinct key tuple, NULL keys form one group, key columns then aggregates.
//
// Device design: each row resolves a dense group id (0 for a global
// aggregate, a read-only group-table probe for GROUP BY, a join-table probe
// whose payload IS the group id for the fused pipeline), then updates 64-bit
// state words with LDS atomics (per-workgroup partials, flushed once per
// workgroup with global atomics) or directly with global atomics when the
// states do not fit the LDS budget.  A finalize pass compacts non-empty
// groups and converts states to the reference's result types.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <memory>
#include <type_traits>

#include "agg.h"
#include "expr_device.h"
#include "fast_tile.h"
#include "ops.h"

namespace qeh {

constexpr int kAggR = 4;                           // rows per lane
constexpr int kAggTile = kBlock * kAggR;           // rows per workgroup iteration
constexpr size_t kLdsStateBudget = 48 * 1024;      // bytes of LDS state per workgroup
constexpr int kFastTile = kBlock * kFastR;         // 2048 rows per fast-path workgroup iteration

enum GidMode { GM_ZERO = 0, GM_JOIN = 1, GM_GROUP = 2, GM_LDSHASH = 3 };
enum PredMode { PM_NONE = 0, PM_TERMS = 1, PM_PROG = 2 };

constexpr int64_t kEmptyKey = INT64_MIN;
struct GTable {                  // GM_LDSHASH: HBM table of group keys (EMPTY = INT64_MIN)
    int64_t *keys;
    uint64_t mask;               // capacity - 1; states index gcap = NULL group, gcap+1 = key INT64_MIN
    uint32_t *overflow;
};

struct GidSource {
    HashTable jt;            // GM_JOIN
    int32_t key_col;         // GM_JOIN: probe key column in the ColSet
    int32_t _pad;
    KeyCols gk;              // GM_GROUP: key columns (absolute ColRefs)
    const uint32_t *gslots;  // GM_GROUP
    uint64_t gmask;
    const uint64_t *gdense;
    GTable gt;               // GM_LDSHASH
    int32_t lcap;            // GM_LDSHASH: LDS slots per workgroup
    int32_t _pad2;
};

// Global states are kept in specs.shards copies ([shard][slot][G]); workgroup b
// merges into copy b % shards, so thousands of workgroups do not all hit the
// same few KB with atomics.  k_states_reduce folds the copies into copy 0.
__device__ __forceinline__ uint64_t *shard_states(uint64_t *all, const AggSpecs &specs, int64_t G) {
    return all + (uint64_t)(blockIdx.x % (unsigned)specs.shards) * (uint64_t)specs.n_slots * (uint64_t)G;
}

template <int GM, int PM, bool LDS>
__global__ __launch_bounds__(kBlock) void k_agg_rows(ColSet cols, int64_t n, PredTerms terms, DevProgram prog,
                                                     GidSource src, AggSpecs specs, int64_t G,
                                                     uint64_t *__restrict__ gstates_all, uint32_t *__restrict__ errp) {
    uint64_t *__restrict__ gstates = shard_states(gstates_all, specs, G);
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    uint64_t *st = LDS ? lds : gstates;
    const int64_t stride_slot = G;
    if (LDS) {
        const int64_t words = (int64_t)specs.n_slots * G;
        for (int64_t i = threadIdx.x; i < words; i += blockDim.x) lds[i] = 0;
        __syncthreads();
        for (int a = 0; a < specs.n; ++a) {
            const AggSpec sp = specs.a[a];
            if (sp.kind == AK_MIN || sp.kind == AK_MAX)
                for (int64_t g = threadIdx.x; g < G; g += blockDim.x)
                    lds[(int64_t)sp.val_slot * stride_slot + g] = (uint64_t)agg_init_value(sp.kind);
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t err = 0;
    const int64_t ntiles = (n + kAggTile - 1) / kAggTile;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t row0 = tile * kAggTile + (int64_t)wave * 64 * kAggR + lane;
        uint32_t sel;
        if (PM == PM_TERMS) {
            sel = eval_terms<kAggR>(terms, cols, row0, 64, n);
        } else if (PM == PM_PROG) {
            ExprRegs<kAggR> X;
            run_program<kAggR>(prog, cols, row0, 64, n, X, err);
            sel = program_true_mask<kAggR>(X);
        } else {
            sel = 0;
#pragma unroll
            for (int r = 0; r < kAggR; ++r)
                if (row0 + r * 64 < n) sel |= 1u << r;
        }
        int64_t kv[kAggR];
        uint32_t kvalid = 0;
        if (GM == GM_JOIN) load_rows<kAggR>(cols.c[src.key_col], row0, 64, n, kv, kvalid);
#pragma unroll
        for (int r = 0; r < kAggR; ++r) {
            if (!((sel >> r) & 1)) continue;
            const int64_t row = row0 + r * 64;
            auto apply = [&](uint32_t g) {
                atomicAdd((unsigned long long *)&st[g], 1ull);
                for (int a = 0; a < specs.n; ++a) {
                    const AggSpec sp = specs.a[a];
                    const ColRef &c = cols.c[sp.col];
                    if (!col_valid(c, row)) continue;
                    if (sp.cnt_slot) atomicAdd((unsigned long long *)&st[(int64_t)sp.cnt_slot * stride_slot + g], 1ull);
                    if (sp.kind != AK_COUNT) {
                        int64_t x = agg_input(sp.kind, sp.in_type, load_i64(c, row));
                        agg_apply<LDS>(sp.kind, &st[(int64_t)sp.val_slot * stride_slot + g], x);
                    }
                }
            };
            if (GM == GM_ZERO) {
                apply(0u);
            } else if (GM == GM_JOIN) {
                if ((kvalid >> r) & 1) table_probe(src.jt, kv[r], apply);
            } else {
                uint64_t s = group_find(src.gk, row, src.gslots, src.gmask);
                apply((uint32_t)src.gdense[s]);
            }
        }
    }
    if (err) atomicOr(errp, err);
    if (LDS) {
        __syncthreads();
        for (int64_t g = threadIdx.x; g < G; g += blockDim.x) {
            uint64_t rows = lds[g];
            if (!rows) continue;
            atomicAdd((unsigned long long *)&gstates[g], (unsigned long long)rows);
            for (int a = 0; a < specs.n; ++a) {
                const AggSpec sp = specs.a[a];
                if (sp.cnt_slot) {
                    uint64_t c = lds[(int64_t)sp.cnt_slot * stride_slot + g];
                    if (c) atomicAdd((unsigned long long *)&gstates[(int64_t)sp.cnt_slot * stride_slot + g], (unsigned long long)c);
                }
                if (sp.kind != AK_COUNT)
                    agg_merge_global(sp.kind, &gstates[(int64_t)sp.val_slot * stride_slot + g],
                                     lds[(int64_t)sp.val_slot * stride_slot + g]);
            }
        }
    }
}

// ---- fast fused probe: no-null 8-byte columns, unique join table (any layout) ----------
// Each lane owns 8 rows as four 16-byte pairs (every load instruction of a
// wave reads 1 KiB contiguous); all column loads of a tile are issued before
// the predicate is evaluated, all table probes before any LDS update, so a
// wave keeps 4 * (1 + terms + agg columns) HBM loads and 8 probes in flight.
__device__ __forceinline__ bool probe_unique(const HashTable &t, int64_t key, uint32_t &gid) {
    if (key < t.kmin || key > t.kmax) return false;
    if (t.kind == TK_DIRECT) {
        const uint64_t i = (uint64_t)key - (uint64_t)t.kmin;
        uint32_t e = t.payload16 ? (uint32_t)t.payload16[i] : t.payload[i];
        gid = e - 1u;
        return e != 0;
    }
    if (t.kind == TK_BUCKET) {
        const int S = bucket_slots(t.pbits);
        uint64_t b = bucket_home(t, (uint64_t)key);
        for (uint64_t step = 0; step < t.nbkt; ++step) {
            uint64_t w[8];
            bucket_load(t, b, w);
            const uint32_t cnt = (uint32_t)(w[7] >> 32);
            // every slot compared with constant register indices (a runtime slot index into w
            // costs a chain of selects per access), the payload picked the same way
            uint32_t hit = 0;
#pragma unroll
            for (int s = 0; s < 6; ++s) hit |= (s < S && s < (int)cnt && (int64_t)w[s] == key) ? 1u << s : 0u;
            if (hit) {
                const int s0 = __builtin_ctz(hit);
                uint32_t pl = 0;
#pragma unroll
                for (int s = 0; s < 6; ++s)
                    if (s == s0) pl = bucket_payload(w, s, t.pbits);
                gid = pl - 1u;
                return true;
            }
            if (cnt <= (uint32_t)S) return false;
            b = b + 1 == t.nbkt ? 0 : b + 1;
        }
        return false;
    }
    uint64_t h = hash64((uint64_t)key) & t.mask;
    if (t.kind == TK_WIDE) {
        for (uint64_t i = 0; i <= t.mask; ++i) {
            const v2u64 e = wide_slot(t, h);
            if (e[1] == 0) return false;
            if ((int64_t)e[0] == key) {
                gid = (uint32_t)(e[1] - 1ull);
                return true;
            }
            h = (h + 1) & t.mask;
        }
        return false;
    }
    const uint64_t want = (uint64_t)key - (uint64_t)t.kmin + 1ull;
    for (uint64_t i = 0; i <= t.mask; ++i) {
        uint64_t e = t.slots[h];
        if (e == 0) return false;
        if ((e >> t.pbits) == want) {
            gid = (uint32_t)(e & ((1ull << t.pbits) - 1ull));
            return true;
        }
        h = (h + 1) & t.mask;
    }
    return false;
}

// Apply one tile's rows (mask m, LDS state slot per row) to LDS states laid
// out [value slot][stride] with row counts in slot 0.  Aggregate kinds are
// uniform, so the switch sits outside the row loop and each aggregate's LDS
// atomics for the tile's rows issue back to back.
template <int NTERMS, int NACOL, bool NT>
__device__ __forceinline__ void lds_apply_rows(uint64_t *lds, int64_t stride, const AggSpecs &specs, const FastIn &in,
                                               const FastTile<NTERMS, NACOL, NT> &ft, uint32_t m, const int *slot) {
#pragma unroll
    for (int r = 0; r < kFastR; ++r)
        if ((m >> r) & 1) atomicAdd((unsigned long long *)&lds[slot[r]], 1ull);
    for (int a = 0; a < specs.n; ++a) {
        const AggSpec sp = specs.a[a];
        uint64_t *st = lds + (int64_t)sp.val_slot * stride;
        const int cs = in.agg_colslot[a];
        switch (sp.kind) {
            case AK_SUM_F:
#pragma unroll
                for (int r = 0; r < kFastR; ++r)
                    if ((m >> r) & 1) atomicAdd((double *)&st[slot[r]], as_f64(ft.a(cs, r)));
                break;
            case AK_SUM_I:
#pragma unroll
                for (int r = 0; r < kFastR; ++r)
                    if ((m >> r) & 1) atomicAdd((unsigned long long *)&st[slot[r]], (unsigned long long)ft.a(cs, r));
                break;
            case AK_MIN:
            case AK_MAX:
#pragma unroll
                for (int r = 0; r < kFastR; ++r)
                    if ((m >> r) & 1) agg_apply<true>(sp.kind, &st[slot[r]], agg_input(sp.kind, sp.in_type, ft.a(cs, r)));
                break;
            default: break;  // COUNT of a no-null column = the row count
        }
    }
}

template <int NTERMS, int NACOL, bool NT>
__global__ __launch_bounds__(kBlock) void k_join_agg_fast(FastIn in, PredTerms terms, AggSpecs specs, HashTable t,
                                                          int64_t G, int64_t n_tiles, uint64_t *__restrict__ gstates_all) {
    uint64_t *__restrict__ gstates = shard_states(gstates_all, specs, G);
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    {
        const int64_t words = (int64_t)specs.n_slots * G;
        for (int64_t i = threadIdx.x; i < words; i += blockDim.x) lds[i] = 0;
        __syncthreads();
        for (int a = 0; a < specs.n; ++a) {
            const AggSpec sp = specs.a[a];
            if (sp.kind == AK_MIN || sp.kind == AK_MAX)
                for (int64_t g = threadIdx.x; g < G; g += blockDim.x) lds[(int64_t)sp.val_slot * G + g] = (uint64_t)agg_init_value(sp.kind);
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int64_t base = tile * kFastTile + (int64_t)wave * (64 * kFastR) + 2 * lane;
        FastTile<NTERMS, NACOL, NT> ft;
        ft.load(in, terms, base);
        const uint32_t sel = ft.sel;
        uint32_t gid[kFastR];
        int slot[kFastR];
        uint32_t hit = 0;
#pragma unroll
        for (int r = 0; r < kFastR; ++r) {
            gid[r] = 0;
            if ((sel >> r) & 1)
                if (probe_unique(t, ft.k(r), gid[r])) hit |= 1u << r;
            slot[r] = (int)gid[r];
        }
        lds_apply_rows(lds, G, specs, in, ft, hit, slot);
    }
    __syncthreads();
    for (int64_t g = threadIdx.x; g < G; g += blockDim.x) {
        uint64_t rows = lds[g];
        if (!rows) continue;
        atomicAdd((unsigned long long *)&gstates[g], (unsigned long long)rows);
        for (int a = 0; a < specs.n; ++a) {
            const AggSpec sp = specs.a[a];
            if (sp.kind != AK_COUNT)
                agg_merge_global(sp.kind, &gstates[(int64_t)sp.val_slot * G + g], lds[(int64_t)sp.val_slot * G + g]);
        }
    }
}

// ---- bucket-range partitioned probe (BUCKET tables: sparse 64-bit keys; opt-in, see try_bucket_parts) --
// A BUCKET table of 1e7 sparse keys is 178 MB: the single fused pass (k_join_agg_fast) reads one 64-B
// bucket line per selected probe row from the Infinity Cache.  Here the probe rows are first split by
// the high bits of the key's hash -- the home bucket is monotone in the hash, so each of the 64
// partitions owns a contiguous 1/64 of the table (2.8 MB at 1e7 keys) -- and each partition is then
// probed by the workgroups of one XCD together, so its part of the table stays in that XCD's 4 MB L2.
//   P1 k_bp_part: FastTile loads + predicate; the selected rows' (key, aggregate input) are staged in
//      LDS by partition and appended to the workgroup's open 256-item chunk per partition (chunks from
//      one global counter, tagged with their partition; runs of ~32 rows per partition per tile).
//   P2 k_bp_probe: XCD x (blockIdx % 8) takes partitions x, x + 8, ...; its workgroups split each
//      partition's chunk list (chunk_lists), probe the table (L2 hits) and aggregate in LDS states.
// HBM bytes per probe row: 24 read (x, k, v) + 16 written and read back per selected row; the table
// once per partition.  A key stored past its partition's last bucket (linear probing by buckets) is
// still found: the probe reads the real table.
constexpr int kBpBlock = 512;
constexpr int kBpWaves = kBpBlock / 64;
constexpr int kBpTile = kBpBlock * kFastR;  // 4096 probe rows per P1 iteration
constexpr int kBpPBits = 6;
constexpr int kBpP = 1 << kBpPBits;         // partitions
constexpr int kBpChunk = 256;

// LDS-only workgroup barrier: the next tile's loads stay in flight across it
__device__ __forceinline__ void bp_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int NTERMS, int NACOL, bool NT>
__global__ __launch_bounds__(kBpBlock) void k_bp_part(FastIn in, PredTerms terms, int64_t n, int acs,
                                                      uint64_t *__restrict__ okey, uint64_t *__restrict__ oval,
                                                      uint16_t *__restrict__ tag, uint16_t *__restrict__ ccnt,
                                                      uint32_t *__restrict__ nchunk) {
    __shared__ uint32_t pc[kBpP], tstart[kBpP], fillp[kBpP], curc[kBpP], cbase[kBpP];
    __shared__ uint64_t skey[kBpTile];
    __shared__ uint64_t sval[NACOL > 0 ? kBpTile : 1];
    __shared__ uint32_t sdst[kBpTile];
    __shared__ uint32_t tot_s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < kBpP) pc[tid] = 0, fillp[tid] = kBpChunk, curc[tid] = 0;  // fill 256: no open chunk
    __syncthreads();
    const int64_t n_tiles = (n + kBpTile - 1) / kBpTile;
    const int64_t woff = (int64_t)wave * (64 * kFastR) + 2 * lane;
    // the next tile's loads are issued before this tile's LDS phases (full tiles; the ragged last tile
    // is loaded on its own)
    FastTile<NTERMS, NACOL, NT> nx;
    if ((int64_t)blockIdx.x < n_tiles && ((int64_t)blockIdx.x + 1) * kBpTile <= n) nx.issue(in, (int64_t)blockIdx.x * kBpTile + woff);
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int64_t base = tile * kBpTile + woff;
        FastTile<NTERMS, NACOL, NT> ft;
        if ((tile + 1) * kBpTile <= n) {
            ft = nx;
            ft.eval(in, terms);
            const int64_t t2 = tile + gridDim.x;
            if (t2 < n_tiles && (t2 + 1) * kBpTile <= n) nx.issue(in, t2 * kBpTile + woff);
        } else {
            ft.issue_tail(in, base, n);
            ft.eval(in, terms);
            ft.sel &= FastTile<NTERMS, NACOL, NT>::tail_mask(base, n);
        }
        uint32_t part[kFastR], rk[kFastR];
#pragma unroll
        for (int r = 0; r < kFastR; ++r) {
            part[r] = (uint32_t)(hash64((uint64_t)ft.k(r)) >> (64 - kBpPBits));
            rk[r] = ((ft.sel >> r) & 1u) ? atomicAdd(&pc[part[r]], 1u) : 0u;
        }
        bp_barrier();
        if (tid < kBpP) {  // wave 0: the tile's starts, and the chunks each partition opens
            const uint32_t c = pc[tid];
            const uint32_t incl = wave_incl_scan(c);
            tstart[tid] = incl - c;
            if (tid == kBpP - 1) tot_s = incl;
            const uint32_t room = kBpChunk - fillp[tid];
            const uint32_t spill = c > room ? c - room : 0u;
            const uint32_t nnew = (spill + kBpChunk - 1) / kBpChunk;
            uint32_t b = 0;
            if (nnew) {
                b = atomicAdd(nchunk, nnew);
                for (uint32_t i = 0; i < nnew; ++i) tag[b + i] = (uint16_t)tid, ccnt[b + i] = (uint16_t)kBpChunk;
            }
            cbase[tid] = b;
        }
        bp_barrier();
#pragma unroll
        for (int r = 0; r < kFastR; ++r) {
            if (!((ft.sel >> r) & 1u)) continue;
            const uint32_t p = part[r], f = fillp[p], room = kBpChunk - f;
            uint32_t dst;
            if (rk[r] < room) {
                dst = curc[p] * kBpChunk + f + rk[r];
            } else {
                const uint32_t q = rk[r] - room;
                dst = (cbase[p] + q / kBpChunk) * kBpChunk + q % kBpChunk;
            }
            const uint32_t st = tstart[p] + rk[r];
            skey[st] = (uint64_t)ft.k(r);
            if (NACOL > 0) sval[st] = (uint64_t)ft.a(acs, r);
            sdst[st] = dst;
        }
        bp_barrier();
        const uint32_t tot = tot_s;
        for (uint32_t i = tid; i < tot; i += kBpBlock) {
            const uint32_t d = sdst[i];
            okey[d] = skey[i];
            if (NACOL > 0) oval[d] = sval[i];
        }
        if (tid < kBpP) {
            const uint32_t c = pc[tid], f = fillp[tid], room = kBpChunk - f;
            if (c <= room) {
                fillp[tid] = f + c;
            } else {
                const uint32_t q = c - room;
                curc[tid] = cbase[tid] + (q - 1) / kBpChunk;
                fillp[tid] = (q - 1) % kBpChunk + 1;
            }
            pc[tid] = 0;
        }
        bp_barrier();
    }
    if (tid < kBpP && fillp[tid] < kBpChunk) ccnt[curc[tid]] = (uint16_t)fillp[tid];
}

template <int NACOL>
__global__ __launch_bounds__(kBpBlock) void k_bp_probe(AggSpecs specs, FastIn in, HashTable t, int64_t G,
                                                       const uint32_t *__restrict__ sbase, const uint32_t *__restrict__ list,
                                                       const uint64_t *__restrict__ ikey, const uint64_t *__restrict__ ival,
                                                       uint64_t *__restrict__ gstates_all) {
    uint64_t *__restrict__ gstates = shard_states(gstates_all, specs, G);
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    {
        const int64_t words = (int64_t)specs.n_slots * G;
        for (int64_t i = threadIdx.x; i < words; i += blockDim.x) lds[i] = 0;
        __syncthreads();
        for (int a = 0; a < specs.n; ++a) {
            const AggSpec sp = specs.a[a];
            if (sp.kind == AK_MIN || sp.kind == AK_MAX)
                for (int64_t g = threadIdx.x; g < G; g += blockDim.x) lds[(int64_t)sp.val_slot * G + g] = (uint64_t)agg_init_value(sp.kind);
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = blockIdx.x & 7;
    const uint32_t wi = blockIdx.x >> 3, nwg = gridDim.x >> 3;
    constexpr int U = 2;  // chunks per wave in flight (8 probes per lane)
    for (int p = x; p < kBpP; p += 8) {
        const uint32_t lo = sbase[p], hi = sbase[p + 1];
        const uint32_t stride = nwg * kBpWaves * U;
        uint32_t ent[U];  // this iteration's list entries (the next ones are read while it probes)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t e = lo + (wi * kBpWaves + wave) * U + u;
            ent[u] = e < hi ? list[e] : 0xFFFFFFFFu;
        }
        for (uint32_t e0 = lo + (wi * kBpWaves + wave) * U; e0 < hi; e0 += stride) {
            int64_t key[U][4], val[U][4];
            uint32_t cn[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                cn[u] = ent[u] == 0xFFFFFFFFu ? 0u : (ent[u] >> 24) + 1u;
                const uint64_t at = (uint64_t)(ent[u] & 0xFFFFFFu) * kBpChunk + lane * 4;
                if (cn[u]) {
                    const v2i64 k0 = __builtin_nontemporal_load((const v2i64 *)(ikey + at));
                    const v2i64 k1 = __builtin_nontemporal_load((const v2i64 *)(ikey + at + 2));
                    key[u][0] = k0[0], key[u][1] = k0[1], key[u][2] = k1[0], key[u][3] = k1[1];
                    if (NACOL > 0) {
                        const v2i64 v0 = __builtin_nontemporal_load((const v2i64 *)(ival + at));
                        const v2i64 v1 = __builtin_nontemporal_load((const v2i64 *)(ival + at + 2));
                        val[u][0] = v0[0], val[u][1] = v0[1], val[u][2] = v1[0], val[u][3] = v1[1];
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t e = e0 + stride + u;
                ent[u] = e < hi ? list[e] : 0xFFFFFFFFu;
            }
            uint32_t gid[U][4];
            uint32_t hit = 0;
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    gid[u][q] = 0;
                    if ((uint32_t)(lane * 4 + q) < cn[u] && probe_unique(t, key[u][q], gid[u][q])) hit |= 1u << (u * 4 + q);
                }
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if ((hit >> (u * 4 + q)) & 1u) atomicAdd((unsigned long long *)&lds[gid[u][q]], 1ull);
            for (int a = 0; a < specs.n; ++a) {
                const AggSpec sp = specs.a[a];
                if (sp.kind == AK_COUNT || in.agg_colslot[a] < 0) continue;
                uint64_t *st = lds + (int64_t)sp.val_slot * G;
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if ((hit >> (u * 4 + q)) & 1u) {
                            const int64_t v = NACOL > 0 ? val[u][q] : 0;
                            if (sp.kind == AK_SUM_F) atomicAdd((double *)&st[gid[u][q]], as_f64(v));
                            else if (sp.kind == AK_SUM_I) atomicAdd((unsigned long long *)&st[gid[u][q]], (unsigned long long)v);
                            else agg_apply<true>(sp.kind, &st[gid[u][q]], agg_input(sp.kind, sp.in_type, v));
                        }
            }
        }
    }
    __syncthreads();
    for (int64_t g = threadIdx.x; g < G; g += blockDim.x) {
        uint64_t rows = lds[g];
        if (!rows) continue;
        atomicAdd((unsigned long long *)&gstates[g], (unsigned long long)rows);
        for (int a = 0; a < specs.n; ++a) {
            const AggSpec sp = specs.a[a];
            if (sp.kind != AK_COUNT)
                agg_merge_global(sp.kind, &gstates[(int64_t)sp.val_slot * G + g], lds[(int64_t)sp.val_slot * G + g]);
        }
    }
}

// ---- LDS-slice partitioned probe (direct u16 tables larger than L2) ----------------
// A single fused pass pays one L2 miss (a 64-B Infinity-Cache request) per
// probe once the table outgrows an XCD's 4 MiB L2; at the BASELINE shape
// (1e7-key u16 table = 20 MB) that doubles the pass.  This path splits the
// table into slices of 2^16 entries (128 KB, one CU's LDS) and runs:
//   phase A (k_slice_partition): stream the probe columns once, filter, rank
//     each selected row by slice in LDS, stage the tile sorted by slice, and
//     append each slice's (16-bit key offset, aggregate input) items to the
//     workgroup's own region for that slice in whole 32-item chunks (64 B of
//     keys + 256 B of values per chunk: whole-sector HBM writes).  The < 32
//     items left over per slice are carried in LDS into the next tile.
//   phase B (k_slice_probe): a workgroup loads one slice into LDS and drains
//     that slice's regions with LDS lookups and LDS aggregate states.
// HBM bytes per selected row: 2 + 8*NACOL written and read back; lookups
// cost LDS cycles only.
constexpr int kSliceBits = 16;
constexpr int kSliceKeys = 1 << kSliceBits;
constexpr int kSliceMaxF = 160;                  // slices: key range <= 160 * 65536
constexpr int kSliceBlock = 1024;                // one workgroup per CU in both phases
constexpr int kSliceTile = kSliceBlock * kFastR;  // 8192 probe rows per phase-A iteration
constexpr int kSliceChunk = 32;                  // items per flushed chunk
constexpr int kMaxSliceGrid = 512;               // phase-A workgroups / build regions (items form) phase B walks
constexpr int kSliceStateWords = 3584;           // phase-B LDS aggregate states (n_slots * G)
// Group-range slices (G too large for LDS states): phase A looks the group id up and partitions
// by gid >> kGidSliceBits; phase B aggregates one range of 2^kGidSliceBits groups in LDS.
constexpr int kGidSliceBits = 12;
constexpr int kGidStateWords = 16384;            // n_slots * 2^kGidSliceBits <= this (128 KB)

// Workgroup barrier ordering LDS only: the next tile's global loads stay in
// flight across it (__syncthreads also drains vmcnt).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct SliceRegions {
    uint16_t *key;        // [grid][F][cap] key - kmin - slice * 2^16
    int64_t *val;         // [grid][F][cap] aggregate input (NACOL >= 1)
    int64_t *val2;        // [grid][F][cap] second aggregate input (NACOL == 2)
    uint32_t *count;      // [grid][F]
    uint32_t *overflow;   // set when a region fills up (skewed probe keys)
    uint64_t cap;         // items per region, multiple of kSliceChunk
    int32_t F;            // slices
    // exact layout (materialising join): region (workgroup r, slice b) starts at
    // rbase[b * grid + r] (slice-major, no gaps) instead of (r * F + b) * cap
    const uint64_t *rbase;
    // partitioned layout (the shuffle join's items form, pw > 0 ranks). Phase A: region (w, b) is number
    // part_region(b, w), slice-major with the slices of one destination rank (b % pw) together -- rank q's
    // regions are one contiguous block. Phase B: the packed regions received from pw ranks, local slice
    // j (global slice j * pw + prank) region (q, w) numbered (q * S + j) * pgrid + w, at rbase[number].
    int32_t pw;
    int32_t prank;
    int32_t pgrid;
    // phase B of the partitioned layout: this rank's own regions (source prank) read in place from phase
    // A's layout (region number * ocap) instead of from the packed receive buffers
    const uint16_t *okey;
    const int64_t *oval;
    uint64_t ocap;
};
// the partitioned layout's slices per rank and a region's number (phase A, pw > 0)
__host__ __device__ __forceinline__ int part_slices(int F, int pw) { return (F + pw - 1) / pw; }
__host__ __device__ __forceinline__ uint64_t part_region(int b, int w, int F, int pw, int grid) {
    return ((uint64_t)(b % pw) * part_slices(F, pw) + (uint64_t)(b / pw)) * grid + w;
}


// Phase A's shape when it is planned on the device (the prelaunch ahead of the build reads the build
// key's range from device memory instead of waiting for the host: no host round trip between the
// min/max kernels and phase A).  plan_slices is the one rule, evaluated on the device by
// k_slice_plan and on the host to adopt the result; regions are allocated for the worst case and
// the plan's cap divides them among grid x F regions.
struct SlicePlan {
    int64_t kmin;
    uint64_t range;
    uint64_t cap;
    int32_t F;
    int32_t ok;
    int64_t src[6];  // the build ranges it was planned from: key min, max, count, group key min, max, count
};
struct SlicePlanIn {
    uint64_t min_bytes;    // smallest table (bytes) worth the two-phase pipeline
    uint64_t alloc_items;  // items allocated for all regions together
    int32_t grid;
    int32_t n_slots;
    int32_t sparse_ok;     // direct_table_ok's sparse rule enabled
    int32_t chunk;         // items per flushed chunk (regions are whole chunks); 0 = kSliceChunk
    int32_t world;         // > 1: the partitioned layout's regions (F rounded up to a multiple of world)
};
__host__ __device__ inline SlicePlan plan_slices(const SlicePlanIn &pi, int64_t kmn, int64_t kmx, int64_t kcnt, int64_t gmn,
                                                 int64_t gmx, int64_t gcnt) {
    SlicePlan p{};
    p.src[0] = kmn, p.src[1] = kmx, p.src[2] = kcnt, p.src[3] = gmn, p.src[4] = gmx, p.src[5] = gcnt;
    if (kcnt <= 0) return p;
    // the group count is at most the group key's range (+ the NULL group)
    const uint64_t gr = gcnt ? (uint64_t)gmx - (uint64_t)gmn + 1ull : 0;
    const int64_t g_bound = (gr == 0 || gr > (1ull << 20)) ? -1 : (int64_t)gr + 1;
    if (g_bound <= 0 || g_bound >= 0xFFFF || (int64_t)pi.n_slots * g_bound > kSliceStateWords) return p;
    const uint64_t range = (uint64_t)kmx - (uint64_t)kmn + 1ull;
    // the DIRECT rule of build_join_table, and the slice path's own limits
    if (!direct_table_ok_with(range, (uint64_t)kcnt, (uint64_t)g_bound, pi.sparse_ok != 0)) return p;
    if (range * 2 < pi.min_bytes) return p;
    const uint64_t F = (range + kSliceKeys - 1) >> kSliceBits;
    if (F == 0 || F > (uint64_t)kSliceMaxF) return p;
    p.kmin = kmn;
    p.range = range;
    p.F = (int32_t)F;
    const uint64_t ch = pi.chunk > 0 ? (uint64_t)pi.chunk : (uint64_t)kSliceChunk;
    const uint64_t Fr = pi.world > 1 ? (F + pi.world - 1) / pi.world * pi.world : F;  // regions' slices
    p.cap = pi.alloc_items / ((uint64_t)pi.grid * Fr) / ch * ch;
    p.ok = p.cap >= ch;
    return p;
}
// mm[0] = build key, mm[1] = group key ranges
__global__ void k_slice_plan(const MinMax *__restrict__ mm, SlicePlanIn pi, SlicePlan *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0)
        *out = plan_slices(pi, mm[0].mn, mm[0].mx, (int64_t)mm[0].cnt, mm[1].mn, mm[1].mx, (int64_t)mm[1].cnt);
}
// The job-wide ranges from the gathered rows of qeh_broadcast_stats ([rows, key min, max, group key
// min, max, has-bitmap, ...] per rank): min / max over the ranks with rows, counts = all rows; no
// plan when any shard has a bitmap (the counts would not be the non-null counts).
__global__ void k_slice_plan_stats(const int64_t *__restrict__ M, int world, int row_len, SlicePlanIn pi, SlicePlan *out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int64_t tot = 0, kmn = INT64_MAX, kmx = INT64_MIN, gmn = INT64_MAX, gmx = INT64_MIN, bitmap = 0;
    for (int r = 0; r < world; ++r) {
        const int64_t *m = M + (int64_t)r * row_len;
        bitmap |= m[5];
        if (m[0] <= 0) continue;
        tot += m[0];
        kmn = m[1] < kmn ? m[1] : kmn, kmx = m[2] > kmx ? m[2] : kmx;
        gmn = m[3] < gmn ? m[3] : gmn, gmx = m[4] > gmx ? m[4] : gmx;
    }
    SlicePlan p = plan_slices(pi, kmn, kmx, tot, gmn, gmx, tot);
    if (bitmap || kmn > kmx || gmn > gmx) p.ok = 0;
    *out = p;
}

// The fused pipeline's plan (qeh_join_filter_aggregate with one bounded integer group key): the slice
// shape of the build key's range plus the group key's range -- the join table's entries are group
// slots (g - gmin + 1) instead of dense group ids, so the build needs no group table first.
struct FusedPlan {
    SlicePlan sp;      // sp.ok: every condition of the fused pipeline holds
    int64_t gmin;      // group slot s <-> group key gmin + s
    int64_t ngroups;   // gmax - gmin + 1
    uint64_t dcap;     // build rows per (phase-A workgroup, slice) region, a multiple of 4
};
// Phase A's prologue in the fused pipeline: the build rows grouped by slice into per-(workgroup,
// slice) regions (items = key offset << 16 | group slot + 1), and the output group keys.
struct FusedPro {
    const int64_t *dk;     // build key (Int64, no NULLs)
    ColRef dg;             // group key (Int64 / Int32, no NULLs)
    int64_t nd;
    uint32_t *ditems;      // [grid][F][dcap]
    uint32_t *dcount;      // [grid][F]
    uint32_t *status;      // [1]: a region overflowed (probe or build rows)
    void *gkeys;           // output group keys: gmin + i for i < G (Int32 when as32)
    uint32_t *rep;         // i (the finalize's representative rows)
    int64_t G;
    int32_t as32;
    const FusedPlan *plan;
};
// Phase B's view of the build rows (DIM): slice b's rows are items[(r * F + b) * dcap ..] for every
// phase-A workgroup r, count[r * F + b] of them.
struct DimSlices {
    const uint32_t *items;
    const uint32_t *count;
    uint32_t *dup;     // set when two build rows share a key
    const FusedPlan *plan;
    // the items form of the distributed broadcast join: the build rows come grouped by slice from the
    // ranks instead of from phase A's prologue -- nreg > 0 regions (every rank's build spans), region r's
    // items at items + r * rstride, with o = offs + r * 2 * (kSliceMaxF + 1): slice b's o[S + 1 + b] items
    // at o[b] (a multiple of 4)
    int32_t nreg;
    int32_t _pad;
    uint64_t rstride;
    const uint32_t *offs;
};

// One whole chunk of phase A's flush, planned by the slice's owner thread while the tile is staged:
// item x of the chunk (x < CH) comes from the carried items (c_key/c_v[coff + x]) when x < clim, else
// from the staged tile (st_key/st_v[soff + x]); it lands at absolute item g + x when lo <= x < hi
// (items below lo are placeholders ahead of an exact-layout region, items from hi on overflow it).
struct __attribute__((aligned(16))) SliceChunk {
    uint64_t g;
    int32_t soff;
    uint32_t pk;  // slice (8 bits; its carries start at slice * CH) | clim << 8 | lo << 15 | hi << 22 (7 bits each)
};

// MODE 0: slices of the join key's offset (k - kmin) >> kSliceBits, items = 16-bit key offsets.
// MODE 1: the group id is looked up here (any unique table layout) and rows are partitioned by
// gid >> kGidSliceBits, items = gid & (2^kGidSliceBits - 1); `range` = number of groups.
//
// Three barriers per tile, software-pipelined: tile t's whole chunks are flushed at the top of
// iteration t+1 while its loads are still arriving (no barrier after the flush: a wave that finishes
// early goes on to rank its rows), and tile t's carries (the < CH items per slice left over) are
// copied by waves 1-15 while wave 0 scans tile t+1's counts.  Counts, carried counts, write
// positions and tile offsets are double-buffered by tile parity.
//   [flush(t-1); eval + rank(t)] B1 [scan(t) | carry(t-1)] B2 [stage(t), plan chunks(t), issue(t+1)] B3
// NACOL = 2 (two aggregate columns, 18-B items) stages half tiles (P = 2 pairs per lane, 4096 rows)
// and flushes 16-item chunks, so staging and carries fit one CU's LDS.
// EARLY (the fused pipeline) may take its own tile and chunk (QEH_EARLY_PAIRS / QEH_EARLY_CHUNK at
// build time): 64-item chunks (128 B of keys + 512 B of values, whole lines) with 4096-row tiles keep
// the carries and the staging in one CU's LDS.
#ifndef QEH_EARLY_PAIRS
#define QEH_EARLY_PAIRS 2
#endif
// 1: tile t-1's flush after tile t's rows are ranked (and, EARLY, tile t+1's loads issued); 0: at the
// top of the iteration, before tile t's loads are waited for (the round-4 order)
#ifndef QEH_SLICE_FLUSH_LATE
#define QEH_SLICE_FLUSH_LATE 1
#endif
#ifndef QEH_EARLY_CHUNK
#define QEH_EARLY_CHUNK 64
#endif
template <int NACOL, bool EARLY = false, int NTH = kSliceBlock>
struct SliceShape {
    static constexpr int P = NACOL > 1 ? 2 : (EARLY ? QEH_EARLY_PAIRS : kFastPairs);
    static constexpr int CH = NACOL > 1 ? 16 : (EARLY ? QEH_EARLY_CHUNK : kSliceChunk);
    static constexpr int TILE = NTH * 2 * P;
};

// Phase A's prologue in the fused pipeline (before the first tile's loads): the output group keys,
// then this workgroup's share of the build rows, each into its slice's region (LDS atomics on dcnt
// give the positions; no order inside a region is needed).  Not inlined: its registers stay out of
// the tile loop's allocation.
template <int NTH>
__device__ __attribute__((noinline)) void fused_prologue(const FusedPro &fp, int F, int64_t kmin, uint32_t *dcnt) {
    const int tid = threadIdx.x;
    const FusedPlan fpl = *fp.plan;
    for (int i = tid; i < F; i += NTH) dcnt[i] = 0;
    for (int64_t i = (int64_t)blockIdx.x * NTH + tid; i < fp.G; i += (int64_t)gridDim.x * NTH) {
        if (fp.as32) ((int32_t *)fp.gkeys)[i] = (int32_t)(fpl.gmin + i);
        else ((int64_t *)fp.gkeys)[i] = fpl.gmin + i;
        fp.rep[i] = (uint32_t)i;
    }
    __syncthreads();
    const int64_t chunk = (fp.nd + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * chunk, hi = lo + chunk < fp.nd ? lo + chunk : fp.nd;
    uint32_t *dreg = fp.ditems + (uint64_t)blockIdx.x * F * fpl.dcap;
    bool dovf = false;
    constexpr int DR = 8;
    for (int64_t i0 = lo + tid; i0 < hi; i0 += DR * NTH) {
        int64_t kk[DR], gg[DR];
#pragma unroll
        for (int q = 0; q < DR; ++q) {
            const int64_t i = i0 + (int64_t)q * NTH;
            kk[q] = i < hi ? fp.dk[i] : kmin;
            gg[q] = i < hi ? load_i64(fp.dg, i) : 0;
        }
#pragma unroll
        for (int q = 0; q < DR; ++q) {
            if (i0 + (int64_t)q * NTH >= hi) continue;
            const uint64_t o = (uint64_t)kk[q] - (uint64_t)kmin;
            const uint32_t b = (uint32_t)(o >> kSliceBits);
            const uint32_t r = atomicAdd(&dcnt[b], 1u);
            if (r < fpl.dcap)
                dreg[(uint64_t)b * fpl.dcap + r] =
                    ((uint32_t)(o & (kSliceKeys - 1)) << 16) | ((uint32_t)((uint64_t)gg[q] - (uint64_t)fpl.gmin) + 1u);
            else
                dovf = true;
        }
    }
    __syncthreads();
    if (fp.dcount)  // (the items form: no build rows here)
        for (int i = tid; i < F; i += NTH) {
            fp.dcount[(uint64_t)blockIdx.x * F + i] = dcnt[i] < fpl.dcap ? dcnt[i] : (uint32_t)fpl.dcap;
            dovf |= dcnt[i] > fpl.dcap;
        }
    if (dovf) fp.status[1] = 1u;
}

// Diagnostic build only (-DQEH_PA_STAMPS=1; the default build has no stamp): every wave of the fused
// phase A accumulates the shader-clock cycles of each phase of its tile loop and writes them, with
// its tile count and the s_memtime / s_memrealtime bounds of the loop, to qeh_pa_stamps (plain vector
// stores from lane 0), which qeh_debug_pa_stamps copies out.
#ifndef QEH_PA_STAMPS
#define QEH_PA_STAMPS 0
#endif
#if QEH_PA_STAMPS
constexpr int kPaStampWords = 16;
__device__ uint64_t qeh_pa_stamps[kMaxSliceGrid * 16 * kPaStampWords];
#define PA_STAMP(i)                                          \
    do {                                                     \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();    \
        pa_acc[i] += t_ - pa_prev;                           \
        pa_prev = t_;                                        \
    } while (0)
#else
#define PA_STAMP(i) \
    do {            \
    } while (0)
#endif

// EARLY: the next tile's loads are issued right after this tile's rows are ranked (its registers are
// free from then on), so they stay in flight across the scan, staging and flush phases; it takes every
// VGPR of the SIMD (nothing else fits beside phase A), so only the fused pipeline, whose build runs
// before phase A, uses it (the prelaunched phase A of the other paths keeps room for the build).
// tail_rows > 0: one more, partial tile of that many rows after the n_tiles full ones (fused pipeline;
// the other paths run their ragged tail through the generic kernel).
template <int NTERMS, int NACOL, bool NT, int MODE = 0, bool EARLY = false, int NTH = kSliceBlock>
__global__ __launch_bounds__(NTH) void k_slice_partition(FastIn in, PredTerms terms, int64_t kmin, uint64_t range,
                                                                 int64_t n_tiles, SliceRegions rg, HashTable t,
                                                                 const SlicePlan *__restrict__ dplan = nullptr,
                                                                 int64_t tail_rows = 0, FusedPro fp = FusedPro{}) {
    using Shape = SliceShape<NACOL, EARLY, NTH>;
    constexpr int P = Shape::P, R = 2 * P, TILE = Shape::TILE, CH = Shape::CH;
    constexpr int MAXF = kSliceMaxF;
    if (dplan) {  // planned on the device: the shape comes from the build key's range in memory
        const SlicePlan pl = *dplan;
        if (!pl.ok) return;  // not the slice path: the host discards this launch
        kmin = pl.kmin, range = pl.range;
        rg.F = pl.F, rg.cap = pl.cap;
    }
    constexpr int SB = MODE ? kGidSliceBits : kSliceBits;
    constexpr int VC = NACOL;               // staged value columns
    constexpr int VS = VC > 0 ? VC : 1;
    __shared__ uint32_t cntb[2][MAXF], cnb[2][MAXF], posb[2][MAXF], lofsb[2][MAXF], mpre[MAXF], hd[MAXF];
    __shared__ uint64_t abase[MAXF];  // region start, aligned down to a whole chunk (exact layout)
    __shared__ uint32_t s_chunks;
    __shared__ SliceChunk cdesc[TILE / CH + MAXF];
    __shared__ uint16_t st_key[TILE];
    __shared__ int64_t st_v[VS][VC ? TILE : 1];
    __shared__ uint16_t c_key[MAXF * CH];
    __shared__ int64_t c_v[VS][VC ? MAXF * CH : 1];
    __shared__ uint8_t st_b[EARLY ? TILE : 1];  // EARLY: slice of each staged item (the per-item carry)
    int64_t *const vout[2] = {rg.val, rg.val2};
    const int F = rg.F;
    const uint64_t cap = rg.cap;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t region0 = (uint64_t)blockIdx.x * F;
    for (int i = tid; i < MAXF; i += NTH) {
        cntb[0][i] = 0, cntb[1][i] = 0, posb[0][i] = 0, hd[i] = 0, abase[i] = 0;
        if (i < F) {
            // exact layout: regions start anywhere; chunks stay aligned to absolute multiples
            // of CH items by starting each region h = start % CH placeholder items early (never
            // written) -- whole 64-B key / 256-B value chunks, as with the capacity layout
            const uint64_t st = rg.rbase ? rg.rbase[(uint64_t)i * gridDim.x + blockIdx.x]
                                : rg.pw ? part_region(i, blockIdx.x, F, rg.pw, gridDim.x) * cap
                                        : (region0 + i) * cap;
            hd[i] = (uint32_t)(st % CH);
            abase[i] = st - hd[i];
        }
        cnb[0][i] = hd[i];
    }
    __syncthreads();
    bool ovf = false;
    // tile t-1's whole chunks (descriptors, staged items and the carries from before it): two
    // consecutive items per lane, one chunk per quarter-wave (items sit at absolute multiples of
    // CH, so even positions are 4-B / 16-B aligned)
    auto flush = [&](uint32_t M) {
        const uint32_t xl = (tid & (CH / 2 - 1)) * 2;
        for (uint32_t c = tid / (CH / 2); c < M; c += NTH / (CH / 2)) {
            const SliceChunk d = cdesc[c];
            const uint32_t coff = (d.pk & 255u) * CH, clim = (d.pk >> 8) & 127u, lo = (d.pk >> 15) & 127u,
                           hi = (d.pk >> 22) & 127u;
            uint16_t kv[2];
            int64_t vv[VS][2] = {};
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const uint32_t x = xl + q;
                if (x < clim) {
                    kv[q] = c_key[coff + x];
#pragma unroll
                    for (int u = 0; u < VC; ++u) vv[u][q] = c_v[u][coff + x];
                } else {
                    kv[q] = st_key[d.soff + (int32_t)x];
#pragma unroll
                    for (int u = 0; u < VC; ++u) vv[u][q] = st_v[u][d.soff + (int32_t)x];
                }
            }
            const uint64_t o = d.g + xl;
            if (lo == 0 && hi == (uint32_t)CH) {
                // the fused pipeline's phase B reads each item once: non-temporal, so no dirty key lines
                // are left for phase B to drain (0.98 -> 0.79 ms); the other consumers re-read the items
                // through L2 (the key-window aggregate, the materialising join) and keep them cached
                const uint32_t kw = (uint32_t)kv[0] | ((uint32_t)kv[1] << 16);
                if constexpr (EARLY) __builtin_nontemporal_store(kw, (uint32_t *)(rg.key + o));
                else *(uint32_t *)(rg.key + o) = kw;
#pragma unroll
                for (int u = 0; u < VC; ++u) {
                    v2i64 w;
                    w[0] = vv[u][0], w[1] = vv[u][1];
                    __builtin_nontemporal_store(w, (v2i64 *)(vout[u] + o));
                }
            } else {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    if (xl + q < lo || xl + q >= hi) continue;
                    rg.key[o + q] = kv[q];
#pragma unroll
                    for (int u = 0; u < VC; ++u) __builtin_nontemporal_store(vv[u][q], vout[u] + o + q);
                }
            }
        }
    };
    // carries after tile t-1 from the carries before it (cn_o), its counts (cnt_o) and offsets
    // (lofs_o): appended when no whole chunk left, else the tile's last T % CH items
    auto carry = [&](const uint32_t *cn_o, const uint32_t *cnt_o, const uint32_t *lofs_o, int p0, int stride) {
        if constexpr (EARLY) {
            // one pass over the staged items (the tile's selected rows) instead of every (slice, slot):
            // item j of slice b's segment is carried when no whole chunk was left (appended after the
            // cb carried before) or when it is among the segment's last T % CH items
            const uint32_t total = lofs_o[F - 1] + cnt_o[F - 1];
            for (uint32_t si = (uint32_t)p0; si < total; si += (uint32_t)stride) {
                const int b = st_b[si];
                const uint32_t cb = cn_o[b], nb = cnt_o[b], T = cb + nb, L = T % CH, j = si - lofs_o[b];
                int dst = -1;
                if (T < CH) dst = (int)(cb + j);
                else if (j >= nb - L) dst = (int)(j - (nb - L));
                if (dst >= 0) {
                    c_key[b * CH + dst] = st_key[si];
#pragma unroll
                    for (int u = 0; u < VC; ++u) c_v[u][b * CH + dst] = st_v[u][si];
                }
            }
            return;
        }
        for (int p = p0; p < F * CH; p += stride) {
            const int b = p / CH, kx = p % CH;
            const uint32_t cb = cn_o[b], nb = cnt_o[b], T = cb + nb, L = T % CH;
            int src = -1;
            if (T < CH) {
                if (kx >= (int)cb && kx < (int)T) src = (int)(lofs_o[b] + kx - cb);  // append
            } else if (kx < (int)L) {
                src = (int)(lofs_o[b] + nb - L + kx);  // the tile's last L items
            }
            if (src >= 0) {
                c_key[b * CH + kx] = st_key[src];
#pragma unroll
                for (int u = 0; u < VC; ++u) c_v[u][b * CH + kx] = st_v[u][src];
            }
        }
    };
    FastTile<NTERMS, NACOL, NT, P> ft;
    int64_t tile = blockIdx.x;
    int par = 0;
    uint32_t m_prev = 0;
    bool have_prev = false;
    // the partial last tile only in the fused pipeline (EARLY): the other paths keep their registers
    const int64_t n_all = n_tiles + (EARLY && tail_rows > 0 ? 1 : 0), lim = n_tiles * TILE + tail_rows;
    auto issue_tile = [&](int64_t tl) {
        const int64_t b = tl * TILE + (int64_t)wave * (64 * R) + 2 * lane;
        if (!EARLY || tl < n_tiles) ft.issue(in, b);
        else ft.issue_tail(in, b, lim);
    };
    if constexpr (EARLY) {
        __shared__ uint32_t dcnt[MAXF];
        fused_prologue<NTH>(fp, F, kmin, dcnt);
    }
    if (tile < n_all) issue_tile(tile);
#if QEH_PA_STAMPS
    uint64_t pa_acc[10] = {};
    const uint64_t pa_t0 = __builtin_amdgcn_s_memtime(), pa_r0 = __builtin_amdgcn_s_memrealtime();
    uint64_t pa_prev = pa_t0;
#endif
    for (; tile < n_all; tile += gridDim.x) {
        uint32_t *cnt = cntb[par], *cn = cnb[par], *pos = posb[par], *lofs = lofsb[par];
        const int pq = par ^ 1;
        if (!QEH_SLICE_FLUSH_LATE && have_prev) flush(m_prev);
#if QEH_PA_STAMPS
        PA_STAMP(9);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tile's loads (and older stores)
        PA_STAMP(0);
#endif
        ft.eval(in, terms);
        uint32_t sel = ft.sel, off[R], rk[R];
        if (EARLY && tile >= n_tiles) sel &= decltype(ft)::tail_mask(tile * TILE + (int64_t)wave * (64 * R) + 2 * lane, lim);
        if constexpr (MODE == 1) {
            // all probes first (independent loads in flight), then the LDS ranks
#pragma unroll
            for (int r = 0; r < R; ++r) {
                off[r] = 0;
                if (((sel >> r) & 1) && !probe_unique(t, ft.k(r), off[r])) sel &= ~(1u << r);
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                rk[r] = 0;
                if ((sel >> r) & 1) rk[r] = atomicAdd(&cnt[off[r] >> SB], 1u);
            }
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint64_t o = (uint64_t)ft.k(r) - (uint64_t)kmin;  // out of range -> huge, dropped
                off[r] = (uint32_t)o;
                rk[r] = 0;
                if (((sel >> r) & 1) && o < range) rk[r] = atomicAdd(&cnt[(uint32_t)o >> kSliceBits], 1u);
                else sel &= ~(1u << r);
            }
        }
        int64_t vcur[VS][R];
#pragma unroll
        for (int u = 0; u < VS; ++u)
#pragma unroll
            for (int r = 0; r < R; ++r) vcur[u][r] = VC ? ft.a(u, r) : 0;
        PA_STAMP(1);
        if (EARLY && tile + gridDim.x < n_all) issue_tile(tile + gridDim.x);
        // tile t-1's chunks go out after this tile's loads were waited for (and the next tile's
        // issued): flushed at the top of the iteration, the stores sat in front of the loop head's
        // s_waitcnt vmcnt(0) -- vmcnt counts stores too, so every tile waited for its own flush's
        // write round trip before it could evaluate its rows
        if (QEH_SLICE_FLUSH_LATE && have_prev) flush(m_prev);
        PA_STAMP(2);
        lds_barrier();  // B1: counts complete, tile t-1 flushed
        PA_STAMP(3);
        if (wave == 0) {
            // three consecutive slices per lane: exclusive scans of the staged
            // counts (tile offsets) and of the whole chunks each slice flushes
            uint32_t n3[3], m3[3], ns = 0, ms = 0;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int b = lane * 3 + q;
                n3[q] = b < F ? cnt[b] : 0u;
                m3[q] = b < F ? (cn[b] + n3[q]) / CH : 0u;
                ns += n3[q];
                ms += m3[q];
            }
            uint32_t ni = ns, mi = ms;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t a = __shfl_up(ni, d, 64), c = __shfl_up(mi, d, 64);
                if (lane >= d) ni += a, mi += c;
            }
            uint32_t no = ni - ns, mo = mi - ms;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int b = lane * 3 + q;
                if (b < MAXF) lofs[b] = no, mpre[b] = mo;
                no += n3[q];
                mo += m3[q];
            }
            if (lane == 63) s_chunks = mi;
        } else if (have_prev) {
            carry(cnb[pq], cntb[pq], lofsb[pq], tid - 64, NTH - 64);
        }
        PA_STAMP(4);
        lds_barrier();  // B2: offsets ready, carries hold everything before tile t
        PA_STAMP(5);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!((sel >> r) & 1)) continue;
            const uint32_t s = lofs[off[r] >> SB] + rk[r];
            st_key[s] = (uint16_t)(off[r] & ((1u << SB) - 1u));
            if constexpr (EARLY) st_b[s] = (uint8_t)(off[r] >> SB);
#pragma unroll
            for (int u = 0; u < VC; ++u) st_v[u][s] = vcur[u][r];
        }
        if (tid < F) {
            // plan this slice's whole chunks; the next tile's state (its copies were last read by
            // tile t-1's flush and carry, before B2)
            const uint32_t cb = cn[tid], T = cb + cnt[tid], m = T / CH, m0 = mpre[tid];
            const uint32_t lo0 = lofs[tid];
            const uint64_t p0 = pos[tid], h = hd[tid], gb = abase[tid] + p0;
            for (uint32_t j = 0; j < m; ++j) {
                const uint64_t ds = p0 + (uint64_t)j * CH;  // region item of the chunk's first slot
                const uint32_t lo = h > ds ? (uint32_t)std::min<uint64_t>(h - ds, CH) : 0u;
                const uint32_t hi = cap > ds ? (uint32_t)std::min<uint64_t>(cap - ds, CH) : 0u;
                if (hi < (uint32_t)CH) ovf = true;
                const uint32_t clim = j == 0 ? cb : 0u;
                SliceChunk d;
                d.g = gb + (uint64_t)j * CH;
                d.soff = (int32_t)lo0 + (int32_t)(j * CH) - (int32_t)cb;
                d.pk = (uint32_t)tid | (clim << 8) | (lo << 15) | (hi << 22);
                cdesc[m0 + j] = d;
            }
            posb[pq][tid] = (uint32_t)(p0 + (uint64_t)m * CH);
            cnb[pq][tid] = T % CH;
            cntb[pq][tid] = 0;
        }
        if (!EARLY && tile + gridDim.x < n_all) issue_tile(tile + gridDim.x);
        PA_STAMP(6);
        lds_barrier();  // B3: staged, chunks planned
        PA_STAMP(7);
        m_prev = s_chunks;
        have_prev = true;
        par = pq;
#if QEH_PA_STAMPS
        pa_acc[8] += 1;
#endif
    }
#if QEH_PA_STAMPS
    if (EARLY && lane == 0) {
        uint64_t *o = qeh_pa_stamps + ((uint64_t)blockIdx.x * (NTH / 64) + wave) * kPaStampWords;
        for (int i = 0; i < 10; ++i) o[i] = pa_acc[i];
        o[10] = __builtin_amdgcn_s_memtime() - pa_t0;
        o[11] = __builtin_amdgcn_s_memrealtime() - pa_r0;
    }
#endif
    if (have_prev) {
        flush(m_prev);
        lds_barrier();
        const int pq = par ^ 1;  // the last tile's buffers
        carry(cnb[pq], cntb[pq], lofsb[pq], tid, NTH);
        lds_barrier();
    }
    const uint32_t *cn = cnb[par], *pos = posb[par];
    for (int p = tid; p < F * CH; p += NTH) {  // partial last chunks
        const int b = p / CH, kx = p % CH;
        if (kx >= (int)cn[b]) continue;
        const uint64_t dst = (uint64_t)pos[b] + kx;
        if (dst < hd[b]) continue;
        if (dst < cap) {
            const uint64_t o = abase[b] + dst;
            rg.key[o] = c_key[b * CH + kx];
#pragma unroll
            for (int u = 0; u < VC; ++u) vout[u][o] = c_v[u][b * CH + kx];
        } else {
            ovf = true;
        }
    }
    if (ovf) *rg.overflow = 1u;
    for (int b = tid; b < F; b += NTH) {
        const uint64_t n = (uint64_t)pos[b] + cn[b];
        rg.count[rg.pw ? part_region(b, blockIdx.x, F, rg.pw, gridDim.x) : region0 + b] =
            (uint32_t)((n < cap ? n : cap) - hd[b]);
    }
}

// Phase B.  Region slots are enumerated slice-major (slot = b * nreg + r);
// workgroup w drains the contiguous slot range [w*T/grid, (w+1)*T/grid), so it
// loads at most a few slices, and its waves take the range's regions in turn.
// Merge LDS states laid out [slot][stride] (row counts as u32 in slot 0's words) into the global
// states for groups g0 + [0, ng).
__device__ __forceinline__ void slice_states_flush(const uint64_t *lst, int64_t stride, int64_t g0, int64_t ng,
                                                   const AggSpecs &specs, int64_t G, uint64_t *__restrict__ gstates) {
    const uint32_t *lcnt = (const uint32_t *)lst;
    for (int64_t i = threadIdx.x; i < ng; i += blockDim.x) {
        const uint64_t rows = lcnt[i];
        if (!rows) continue;
        const int64_t g = g0 + i;
        atomicAdd((unsigned long long *)&gstates[g], (unsigned long long)rows);
        for (int a = 0; a < specs.n; ++a) {
            const AggSpec sp = specs.a[a];
            if (sp.kind != AK_COUNT)
                agg_merge_global(sp.kind, &gstates[(int64_t)sp.val_slot * G + g], lst[(int64_t)sp.val_slot * stride + i]);
        }
    }
}

__device__ __forceinline__ void slice_states_init(uint64_t *lst, int64_t stride, const AggSpecs &specs) {
    const int64_t words = (int64_t)specs.n_slots * stride;
    for (int64_t i = threadIdx.x; i < words; i += blockDim.x) lst[i] = 0;
    __syncthreads();
    for (int a = 0; a < specs.n; ++a) {
        const AggSpec sp = specs.a[a];
        if (sp.kind == AK_MIN || sp.kind == AK_MAX)
            for (int64_t g = threadIdx.x; g < stride; g += blockDim.x)
                lst[(int64_t)sp.val_slot * stride + g] = (uint64_t)agg_init_value(sp.kind);
    }
}

// IDENT = false: items are key offsets looked up in an LDS slice of the u16 table; states for all
// G groups stay in LDS.  IDENT = true (group-range slices): items are group ids within the slice's
// range of 2^kGidSliceBits groups, whose states live in LDS while the workgroup drains that slice
// and are merged into the global states when it moves on.
// PF: the next 512 items of a region are loaded while this chunk is looked up and aggregated.
// PV: items loaded two per lane (a 4-B key pair and a 16-B value pair per load; 128 items per wave
// load instead of 64) -- half the load instructions for the same bytes.
// DIM (fused pipeline): there is no join table in memory; slice b's entries are built in LDS from the
// build rows phase A's prologue grouped by slice (entry = group slot + 1 at the key offset), with a
// duplicate build key flagged in *dim.dup, and the shape (F, cap) comes from the device plan.
template <int NACOL, bool IDENT = false, bool PF = false, bool PV = false, bool DIM = false>
__global__ __launch_bounds__(kSliceBlock) void k_slice_probe(SliceRegions rg, int nreg, int splits, HashTable t, FastIn in,
                                                             AggSpecs specs, int64_t G, uint64_t *__restrict__ gstates_all,
                                                             DimSlices dim = DimSlices{}) {
    constexpr int VC = NACOL > 0 ? 1 : 0;
    __shared__ __attribute__((aligned(16))) uint16_t tslice[IDENT ? 8 : kSliceKeys];
    __shared__ uint64_t lst[IDENT ? kGidStateWords : kSliceStateWords];
    __shared__ uint32_t rcnt[DIM ? kMaxSliceGrid : 1];  // DIM: the build-row counts of the slice's regions
    __shared__ uint32_t rbase[DIM ? kMaxSliceGrid : 1];  // DIM: where they start (items, < 2^32)
    uint32_t *lcnt = (uint32_t *)lst;
    uint64_t dcap = 0;
    int Fg = 0;  // DIM: the plan's slices (the partitioned layout's local slices are fewer)
    if constexpr (DIM) {
        const FusedPlan pl = *dim.plan;
        if (!pl.sp.ok) return;
        Fg = pl.sp.F;
        rg.F = rg.pw ? part_slices(pl.sp.F, rg.pw) : pl.sp.F, rg.cap = pl.sp.cap;
        dcap = pl.dcap;
    }
    uint64_t *__restrict__ gstates = shard_states(gstates_all, specs, G);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int W = kSliceBlock / 64;
    const int64_t stride = IDENT ? (1 << kGidSliceBits) : G;  // LDS state words per slot
    slice_states_init(lst, stride, specs);
    const int F = rg.F;
    const int64_t T = (int64_t)F * nreg;
    // splits == 0: one contiguous slot range per workgroup; else units of
    // nreg/splits regions of one slice dealt round-robin
    const int64_t units = splits ? (int64_t)F * splits : (int64_t)gridDim.x;
    int cur_b = -1;
    for (int64_t u = blockIdx.x; u < units; u += gridDim.x) {
    int64_t s0, s1;
    if (splits) {
        const int64_t ub = u / splits, sp = u % splits;
        s0 = ub * nreg + sp * nreg / splits;
        s1 = ub * nreg + (sp + 1) * nreg / splits;
    } else {
        s0 = u * T / gridDim.x;
        s1 = (u + 1) * T / gridDim.x;
    }
    for (int64_t sb = s0; sb < s1;) {
        const int b = (int)(sb / nreg);
        const int64_t se = std::min<int64_t>(s1, (int64_t)(b + 1) * nreg);
        __syncthreads();
        if (IDENT && b != cur_b) {
            if (cur_b >= 0) {
                const int64_t g0 = (int64_t)cur_b << kGidSliceBits;
                slice_states_flush(lst, stride, g0, std::min<int64_t>(stride, G - g0), specs, G, gstates);
                __syncthreads();
                slice_states_init(lst, stride, specs);
            }
            cur_b = b;
        }
        if (DIM && b != cur_b) {
            cur_b = b;
            uint32_t *tw = (uint32_t *)tslice;
            for (int i = tid; i < kSliceKeys / 2; i += kSliceBlock) tw[i] = 0u;
            // build-row regions of the slice: one per phase-A workgroup, or (items form) one per rank
            const int dn = dim.nreg ? dim.nreg : nreg;
            const int bg = rg.pw ? b * rg.pw + rg.prank : b;  // the slice's number in the plan
            for (int r = tid; r < dn; r += kSliceBlock) {
                if (bg >= Fg) {
                    rcnt[r] = 0u, rbase[r] = 0u;  // (a local slice past the plan's last: no rows)
                } else if (dim.nreg) {
                    const uint32_t *o = dim.offs + (uint64_t)r * 2 * (kSliceMaxF + 1);
                    rcnt[r] = o[kSliceMaxF + 1 + bg];
                    rbase[r] = (uint32_t)((uint64_t)r * dim.rstride + o[bg]);
                } else {
                    rcnt[r] = dim.count[(uint64_t)r * F + b];
                    rbase[r] = (uint32_t)(((uint64_t)r * F + b) * dcap);
                }
            }
            __syncthreads();
            // slice b's build rows: every wave takes 8 regions at a time, lane j their items 4j..4j+3
            uint32_t dup = 0;
            for (int r0 = wave * 8; r0 < dn; r0 += W * 8) {
                v4u32 w[8];
                uint32_t cq[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int r = r0 + q;
                    cq[q] = r < dn ? rcnt[r] : 0u;
                    w[q] = (uint32_t)lane * 4 < cq[q] ? *(const v4u32 *)(dim.items + (uint64_t)rbase[r] + lane * 4)
                                                      : v4u32{0u, 0u, 0u, 0u};
                }
#pragma unroll
                for (int q = 0; q < 8; ++q)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        if ((uint32_t)lane * 4 + e >= cq[q]) break;  // past the region's rows
                        const uint32_t it = w[q][e];
                        const uint32_t off = it >> 16, sh = (off & 1u) * 16u;
                        dup |= (atomicOr(&tw[off >> 1], (it & 0xFFFFu) << sh) >> sh) & 0xFFFFu;
                    }
                // regions with more than 256 rows (build keys crowded into one slice)
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int r = r0 + q;
                    const uint32_t c = r < dn ? rcnt[r] : 0u;
                    for (uint32_t i = 256 + (uint32_t)lane * 4; i < c; i += 256) {
                        const v4u32 x = *(const v4u32 *)(dim.items + (uint64_t)rbase[r] + i);
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            if (i + e >= c) break;
                            const uint32_t off = x[e] >> 16, sh = (off & 1u) * 16u;
                            dup |= (atomicOr(&tw[off >> 1], (x[e] & 0xFFFFu) << sh) >> sh) & 0xFFFFu;
                        }
                    }
                }
            }
            if (dup) *dim.dup = 1u;
        } else if (!DIM && !IDENT && b != cur_b) {
            cur_b = b;
            const uint64_t k0 = (uint64_t)b << kSliceBits;
            const uint64_t nk = t.range - k0 < (uint64_t)kSliceKeys ? t.range - k0 : (uint64_t)kSliceKeys;
            for (int i = tid * 8; i < kSliceKeys; i += kSliceBlock * 8) {
                v4u32 w = {0u, 0u, 0u, 0u};
                if ((uint64_t)i + 8 <= nk) {
                    w = *(const v4u32 *)(t.payload16 + k0 + i);
                } else {
                    for (int q = 0; q < 8; ++q)
                        if ((uint64_t)(i + q) < nk) w[q >> 1] |= (uint32_t)t.payload16[k0 + i + q] << ((q & 1) * 16);
                }
                *(v4u32 *)&tslice[i] = w;
            }
        }
        __syncthreads();
        for (int64_t s = sb + wave; s < se; s += W) {
            uint64_t reg, rb;
            const uint16_t *kbase = rg.key;
            const int64_t *vbase = rg.val;
            if (rg.pw) {  // packed regions received from the ranks: (source q, workgroup w) of local slice b
                const int64_t r = s - (int64_t)b * nreg, q = r / rg.pgrid;
                reg = ((uint64_t)q * F + b) * rg.pgrid + (uint64_t)(r - q * rg.pgrid);
                if (rg.okey && q == rg.prank) {  // (this rank's own regions, in phase A's layout)
                    kbase = rg.okey, vbase = rg.oval;
                    rb = reg * rg.ocap;
                } else {
                    rb = rg.rbase[reg];
                }
            } else {
                reg = (uint64_t)(s - (int64_t)b * nreg) * F + b;
                rb = reg * rg.cap;
            }
            const uint32_t n_r = rg.count[reg];
            const uint16_t *kp = kbase + rb;
            const int64_t *vp = VC ? vbase + rb : nullptr;
            const int64_t *vp2 = NACOL > 1 ? rg.val2 + rb : nullptr;
            uint32_t en[8];
            int64_t vn[8], vn2[NACOL > 1 ? 8 : 1];
            // item of register j (the masks below use the same map)
            auto item = [&](uint32_t i0, int j) -> uint32_t {
                return PV ? i0 + (uint32_t)(j >> 1) * 128 + 2 * lane + (uint32_t)(j & 1) : i0 + (uint32_t)j * 64 + lane;
            };
            auto ld = [&](uint32_t i0) {
                if constexpr (PV) {
                    // pairs start at even items; a pair past the count reads inside the region buffer
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t i = item(i0, 2 * j);
                        const uint32_t ii = i < n_r ? i : 0u;
                        const uint32_t kk = __builtin_nontemporal_load((const uint32_t *)(kp + ii));
                        en[2 * j] = kk & 0xFFFFu, en[2 * j + 1] = kk >> 16;
                        if (VC) {
                            const v2i64 w = __builtin_nontemporal_load((const v2i64 *)(vp + ii));
                            vn[2 * j] = w[0], vn[2 * j + 1] = w[1];
                        } else {
                            vn[2 * j] = vn[2 * j + 1] = 0;
                        }
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const uint32_t i = item(i0, j);
                        const uint32_t ii = i < n_r ? i : 0u;
                        en[j] = __builtin_nontemporal_load(kp + ii);
                        vn[j] = VC ? __builtin_nontemporal_load(vp + ii) : 0;
                        if constexpr (NACOL > 1) vn2[j] = __builtin_nontemporal_load(vp2 + ii);
                    }
                }
            };
            if (PF && n_r) ld(0);
            for (uint32_t i0 = 0; i0 < n_r; i0 += 64 * 8) {
                uint32_t e[8];
                int64_t v[8], v2[NACOL > 1 ? 8 : 1];
                if (!PF) ld(i0);
#pragma unroll
                for (int j = 0; j < 8; ++j) e[j] = en[j], v[j] = vn[j];
                if constexpr (NACOL > 1) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) v2[j] = vn2[j];
                }
                if (PF && i0 + 64 * 8 < n_r) ld(i0 + 64 * 8);
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    e[j] = (item(i0, j) < n_r) ? (IDENT ? e[j] + 1u : (uint32_t)tslice[e[j]]) : 0u;

                // aggregate kinds are uniform: switch once per aggregate, then
                // issue the 8 items' LDS atomics back to back
#pragma unroll
                for (int j = 0; j < 8; ++j)  // row counts as u32 in slot 0's words (< 2^32 rows per workgroup)
                    if (e[j]) atomicAdd(lcnt + (e[j] - 1u), 1u);
                for (int a = 0; a < specs.n; ++a) {
                    const AggSpec sp = specs.a[a];
                    uint64_t *st = lst + (int64_t)sp.val_slot * stride - 1;  // indexed by entry = gid + 1
                    const bool second = NACOL > 1 && in.agg_colslot[a] == 1;  // uniform
                    auto val = [&](int j) -> int64_t {
                        if constexpr (NACOL > 1) return second ? v2[j] : v[j];
                        return v[j];
                    };
                    switch (sp.kind) {
                        case AK_SUM_F:
#pragma unroll
                            for (int j = 0; j < 8; ++j)
                                if (e[j]) atomicAdd((double *)&st[e[j]], as_f64(val(j)));
                            break;
                        case AK_SUM_I:
#pragma unroll
                            for (int j = 0; j < 8; ++j)
                                if (e[j]) atomicAdd((unsigned long long *)&st[e[j]], (unsigned long long)val(j));
                            break;
                        case AK_MIN:
                        case AK_MAX:
#pragma unroll
                            for (int j = 0; j < 8; ++j)
                                if (e[j]) agg_apply<true>(sp.kind, &st[e[j]], agg_input(sp.kind, sp.in_type, val(j)));
                            break;
                        default: break;  // COUNT: the row count slot
                    }
                }
            }
        }
        sb = se;
    }
    }
    __syncthreads();
    if (IDENT) {
        if (cur_b >= 0) {
            const int64_t g0 = (int64_t)cur_b << kGidSliceBits;
            slice_states_flush(lst, stride, g0, std::min<int64_t>(stride, G - g0), specs, G, gstates);
        }
    } else {
        slice_states_flush(lst, stride, 0, G, specs, G, gstates);
    }
}

// Phase B of the key-window pipeline (group states too large for LDS, join key range within the slice
// shape): the group is a function of the join key, so rows are aggregated per KEY first and each key's
// partial state is merged into its group's global states once -- 1e7 merges instead of one global
// atomic per row and aggregate, and no group-id gather in phase A (try_gid_slices' MODE 1 read a
// 40-MB table at random: 11.8 of the 12.6 ms of the 2^17-group query).
// Per-key states of a whole 2^16-key slice do not fit LDS, so a slice is split into nw windows of ws
// keys (ws * (4 + 8 * value slots) bytes of LDS: a u32 row count and the value slots per key), one per
// workgroup of a group of nw workgroups that all read the slice's items and keep those of their
// window.  The group's workgroups sit on one XCD (workgroup x runs on XCD x % 8) and walk the regions
// in the same order, so each item line comes from HBM once and from that XCD's L2 the other nw - 1
// times (r04 counters: 39.5M HBM read requests = the items once, 82 % L2 hits): the L2 -> CU traffic
// is what bounds the kernel, hence the compact states and the fewest windows that fit.
// Work units: slices [0, full) whole, then each remaining slice split into `tparts` parts of its
// regions, so the last round of units is short instead of leaving most groups idle (two groups holding
// partials of one key each merge theirs: the merges are memory-side atomics, ~0.5 ms per 1e7 keys, so
// only the tail is split).  gridDim.x = 8 * (groups per XCD) * nw.
// C16: u16 row counts (two per LDS dword, returned atomics catch a count passing 65535 and flag the
// regions' overflow word, so the host falls back): SUM + COUNT fit 4 windows of 16384 keys, COUNT alone
// one window per slice.
constexpr int kKeyAggWords = 20480;  // LDS words of k_slice_keyagg's states (163840 B, all of a CU's LDS)
template <int NACOL, bool C16 = false>
__global__ __launch_bounds__(kSliceBlock) void k_slice_keyagg(SliceRegions rg, int nreg, HashTable t, AggSpecs specs,
                                                              int64_t G, uint64_t *__restrict__ gstates_all, int nw, int ws,
                                                              int full, int tparts) {
    __shared__ uint64_t lbuf[kKeyAggWords];
    uint32_t *lcnt = (uint32_t *)lbuf;  // [ws] row counts (C16: [ws / 2] dwords of two)
    uint64_t *lval = lbuf + (C16 ? ((uint32_t)ws + 3u) / 4u : ((uint32_t)ws + 1u) / 2u);  // [slot - 1][ws] value slots
    bool ovf = false;
    uint64_t *__restrict__ gstates = shard_states(gstates_all, specs, G);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int W = kSliceBlock / 64;
    const int gpx = (int)gridDim.x / 8 / nw;  // groups per XCD
    const int xcd = (int)blockIdx.x & 7, x = (int)blockIdx.x >> 3;
    const int grp = xcd * gpx + x / nw, ngrp = 8 * gpx;
    const uint32_t lo = (uint32_t)(x % nw) * (uint32_t)ws;  // this workgroup's keys: [lo, lo + ws) of the slice
    auto init = [&]() {
        for (int i = tid; i < (C16 ? (ws + 1) / 2 : ws); i += kSliceBlock) lcnt[i] = 0u;
        for (int a = 0; a < specs.n; ++a) {
            const AggSpec sp = specs.a[a];
            if (sp.kind == AK_COUNT) continue;
            const uint64_t v0 = (uint64_t)agg_init_value(sp.kind);
            for (int i = tid; i < ws; i += kSliceBlock) lval[(int64_t)(sp.val_slot - 1) * ws + i] = v0;
        }
    };
    init();
    const int units = full + (rg.F - full) * tparts;
    for (int u = grp; u < units; u += ngrp) {
        const int tu = u - full;
        const int b = tu < 0 ? u : full + tu / tparts, parts = tu < 0 ? 1 : tparts, part = tu < 0 ? 0 : tu % tparts;
        const int r0 = part * nreg / parts, r1 = (part + 1) * nreg / parts;
        __syncthreads();
        for (int r = r0 + wave; r < r1; r += W) {
            const uint64_t reg = (uint64_t)r * rg.F + b;
            const uint32_t n_r = rg.count[reg];
            const uint16_t *kp = rg.key + reg * rg.cap;
            const int64_t *vp = NACOL ? rg.val + reg * rg.cap : nullptr;
            for (uint32_t i0 = 0; i0 < n_r; i0 += 64 * 8) {
                uint32_t e[8];
                int64_t v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t i = i0 + (uint32_t)j * 64 + lane;
                    const uint32_t ii = i < n_r ? i : 0u;
                    const uint32_t k = (uint32_t)kp[ii] - lo;  // below the window -> huge
                    v[j] = NACOL ? vp[ii] : 0;
                    e[j] = (i < n_r && k < (uint32_t)ws) ? k + 1u : 0u;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (!e[j]) continue;
                    if constexpr (C16) {
                        const uint32_t sh = ((e[j] - 1u) & 1u) * 16u;
                        const uint32_t old = atomicAdd(lcnt + ((e[j] - 1u) >> 1), 1u << sh);
                        ovf |= ((old >> sh) & 0xFFFFu) == 0xFFFFu;  // this add carried into the neighbour
                    } else {
                        atomicAdd(lcnt + (e[j] - 1u), 1u);
                    }
                }
                for (int a = 0; a < specs.n; ++a) {
                    const AggSpec sp = specs.a[a];
                    if (sp.kind == AK_COUNT) continue;  // the row count
                    uint64_t *st = lval + (int64_t)(sp.val_slot - 1) * ws - 1;  // indexed by entry = key + 1
                    switch (sp.kind) {
                        case AK_SUM_F:
#pragma unroll
                            for (int j = 0; j < 8; ++j)
                                if (e[j]) atomicAdd((double *)&st[e[j]], as_f64(v[j]));
                            break;
                        case AK_SUM_I:
#pragma unroll
                            for (int j = 0; j < 8; ++j)
                                if (e[j]) atomicAdd((unsigned long long *)&st[e[j]], (unsigned long long)v[j]);
                            break;
                        default:  // MIN / MAX
#pragma unroll
                            for (int j = 0; j < 8; ++j)
                                if (e[j]) agg_apply<true>(sp.kind, &st[e[j]], agg_input(sp.kind, sp.in_type, v[j]));
                            break;
                    }
                }
            }
        }
        __syncthreads();
        // the window's keys with rows: their group from the join table, one merge per key
        const uint64_t k0 = ((uint64_t)b << kSliceBits) + lo;
        for (int i = tid; i < ws; i += kSliceBlock) {
            const uint64_t rows = C16 ? (lcnt[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu : lcnt[i];
            if (!rows || k0 + i >= t.range) continue;
            const uint32_t ent = t.payload16 ? (uint32_t)t.payload16[k0 + i] : t.payload[k0 + i];
            if (!ent) continue;  // no build row with this key
            const int64_t g = (int64_t)ent - 1;
            atomicAdd((unsigned long long *)&gstates[g], (unsigned long long)rows);
            for (int a = 0; a < specs.n; ++a) {
                const AggSpec sp = specs.a[a];
                if (sp.kind != AK_COUNT)
                    agg_merge_global(sp.kind, &gstates[(int64_t)sp.val_slot * G + g], lval[(int64_t)(sp.val_slot - 1) * ws + i]);
            }
        }
        __syncthreads();
        init();
    }
    if (C16 && ovf) *rg.overflow = 1u;
}

// ---- fused pipeline: the plan -----------------------------------------------------------------
// The build rows (key, group key) take the probe rows' route: phase A's prologue groups them by slice
// (4-B items), and phase B builds each slice's entries in LDS from them instead of loading a join table
// from HBM.  No table is written, there are no scattered 2-B stores (the XCD-split insert read every
// key 8 times, 1.2 GB per query), and nothing of the build runs beside phase A.
// mm[0] = build key, mm[1] = group key ranges; nd = build rows (no NULLs allowed); dim_items = the
// build-row region buffer's size in items; st = the status words (zeroed here, [5] = the verdict).
// One launch ahead of phase A: workgroup 0 reduces the build key / group key partial min / max
// (part[c * nb + w], c = 0 key, 1 group key) and writes the plan and the zeroed status words; every
// workgroup initialises its share of the aggregate states.
__global__ __launch_bounds__(1024) void k_fused_plan(const MinMax *__restrict__ part, int nb, SlicePlanIn pi, int64_t g_cap,
                                                     int64_t nd, uint64_t dim_items, FusedPlan *out, uint32_t *__restrict__ st,
                                                     uint64_t *__restrict__ states, int64_t G, AggSpecs specs) {
    const int64_t words = (int64_t)specs.shards * specs.n_slots * G;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t slot = (i / G) % specs.n_slots;
        uint64_t v = 0;
        for (int a = 0; a < specs.n; ++a)
            if (specs.a[a].val_slot == slot) v = (uint64_t)agg_init_value(specs.a[a].kind);
        states[i] = v;
    }
    if (blockIdx.x != 0) return;
    __shared__ MinMax sm[2][16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int c = 0; c < 2; ++c) {
        int64_t mn = INT64_MAX, mx = INT64_MIN;
        uint64_t cnt = 0;
        uint32_t bad = 0;
        for (int i = threadIdx.x; i < nb; i += blockDim.x) {
            const MinMax q = part[(int64_t)c * nb + i];
            mn = q.mn < mn ? q.mn : mn;
            mx = q.mx > mx ? q.mx : mx;
            cnt += q.cnt;
            bad |= q.bad;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const int64_t a = __shfl_xor(mn, d, 64), b2 = __shfl_xor(mx, d, 64);
            const uint64_t cc = __shfl_xor(cnt, d, 64);
            const uint32_t bb = __shfl_xor(bad, d, 64);
            mn = a < mn ? a : mn;
            mx = b2 > mx ? b2 : mx;
            cnt += cc;
            bad |= bb;
        }
        if (lane == 0) sm[c][wave] = MinMax{mn, mx, cnt, bad};
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    MinMax mm[2];
    for (int c = 0; c < 2; ++c) {
        mm[c] = sm[c][0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
            const MinMax q = sm[c][w];
            mm[c].mn = q.mn < mm[c].mn ? q.mn : mm[c].mn;
            mm[c].mx = q.mx > mm[c].mx ? q.mx : mm[c].mx;
            mm[c].cnt += q.cnt;
            mm[c].bad |= q.bad;
        }
    }
    FusedPlan p{};
    p.sp = plan_slices(pi, mm[0].mn, mm[0].mx, (int64_t)mm[0].cnt, mm[1].mn, mm[1].mx, (int64_t)mm[1].cnt);
    const bool full = (int64_t)mm[0].cnt == nd && (int64_t)mm[1].cnt == nd && !mm[0].bad && !mm[1].bad;
    p.gmin = mm[1].mn;
    p.ngroups = full ? (int64_t)((uint64_t)mm[1].mx - (uint64_t)mm[1].mn + 1ull) : 0;
    p.dcap = p.sp.F > 0 ? dim_items / ((uint64_t)pi.grid * p.sp.F) / 4 * 4 : 0;
    p.sp.ok = p.sp.ok && full && p.ngroups >= 1 && p.ngroups <= g_cap && p.ngroups < 0xFFFF && p.dcap >= 4;
    *out = p;
    for (int i = 0; i < 8; ++i) st[i] = 0u;
    st[5] = p.sp.ok ? 1u : 0u;
}

// ---- LDS-slice materialising INNER join (BASELINE config 3) -----------------------------
// Same phase A as the aggregate (k_slice_partition: items = 16-bit key offset +
// the probe payload).  Phase B writes the joined rows: the build payload is
// stored in the u16 table as (a - amin) + 1, so a slice in LDS answers both
// "matches?" and "with which value?".  Rows leave in slice order (the join's
// row order is not part of its contract); each wave reserves
// its matches with one atomic per 512 items and writes them contiguously.
// write the wave's matches of one 8-items-per-lane step at out[*base ...]
// (j-major, lanes in order within j: contiguous stores), advancing *base
__device__ __forceinline__ void emit_matches(const uint32_t *e, const int64_t *v, const bool *live, int64_t amin,
                                             uint64_t *base, int64_t *__restrict__ out_v, int64_t *__restrict__ out_a) {
    uint64_t b = *base;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const bool m = live[j] && e[j] != 0u;
        const uint64_t mask = __ballot(m);
        if (m) {
            const uint64_t pos = b + mbcnt(mask);
            out_v[pos] = v[j];
            out_a[pos] = (int64_t)(e[j] - 1u) + amin;
        }
        b += popc64(mask);
    }
    *base = b;
}

__device__ __forceinline__ void load_slice(uint16_t *tslice, const HashTable &t, int b, int tid) {
    const uint64_t k0 = (uint64_t)b << kSliceBits;
    const uint64_t nk = t.range - k0 < (uint64_t)kSliceKeys ? t.range - k0 : (uint64_t)kSliceKeys;
    for (int i = tid * 8; i < kSliceKeys; i += kSliceBlock * 8) {
        v4u32 w = {0u, 0u, 0u, 0u};
        if ((uint64_t)i + 8 <= nk) {
            w = *(const v4u32 *)(t.payload16 + k0 + i);
        } else {
            for (int q = 0; q < 8; ++q)
                if ((uint64_t)(i + q) < nk) w[q >> 1] |= (uint32_t)t.payload16[k0 + i + q] << ((q & 1) * 16);
        }
        *(v4u32 *)&tslice[i] = w;
    }
}

// Phase B of the join in two passes, no atomics: EMIT = false counts each
// region's matches (keys only) into counts[slot]; after an exclusive scan of
// those (slot order), EMIT = true writes each region's matches from its base.
template <bool EMIT>
__global__ __launch_bounds__(kSliceBlock) void k_slice_join_b(SliceRegions rg, int nreg, HashTable t, int64_t amin,
                                                              uint32_t *__restrict__ counts, const uint64_t *__restrict__ bases,
                                                              int64_t *__restrict__ out_v, int64_t *__restrict__ out_a) {
    __shared__ __attribute__((aligned(16))) uint16_t tslice[kSliceKeys];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int W = kSliceBlock / 64;
    const int F = rg.F;
    const int64_t T = (int64_t)F * nreg;
    const int64_t s0 = (int64_t)blockIdx.x * T / gridDim.x, s1 = (int64_t)(blockIdx.x + 1) * T / gridDim.x;
    for (int64_t sb = s0; sb < s1;) {
        const int b = (int)(sb / nreg);
        const int64_t se = std::min<int64_t>(s1, (int64_t)(b + 1) * nreg);
        __syncthreads();
        load_slice(tslice, t, b, tid);
        __syncthreads();
        for (int64_t s = sb + wave; s < se; s += W) {
            const uint64_t reg = (uint64_t)(s - (int64_t)b * nreg) * F + b;
            const uint32_t n_r = rg.count[reg];
            const uint64_t rb = rg.rbase ? rg.rbase[s] : reg * rg.cap;
            const uint16_t *kp = rg.key + rb;
            const int64_t *vp = rg.val + rb;
            uint64_t base = EMIT ? bases[s] : 0;
            uint32_t matches = 0;
            for (uint32_t i0 = 0; i0 < n_r; i0 += 64 * 8) {
                uint32_t e[8];
                int64_t v[8];
                bool live[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t i = i0 + j * 64 + lane;
                    live[j] = i < n_r;
                    const uint32_t ii = live[j] ? i : 0u;
                    e[j] = __builtin_nontemporal_load(kp + ii);
                    v[j] = EMIT ? __builtin_nontemporal_load(vp + ii) : 0;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) e[j] = live[j] ? (uint32_t)tslice[e[j]] : 0u;
                if (EMIT) {
                    emit_matches(e, v, live, amin, &base, out_v, out_a);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) matches += (uint32_t)popc64(__ballot(live[j] && e[j] != 0u));
                }
            }
            if (!EMIT && lane == 0) counts[s] = matches;
        }
        sb = se;
    }
}

// Exact region sizes for phase A of the materialising join: the same tile ->
// workgroup assignment as k_slice_partition, keys only (16-B loads), per-wave
// LDS counters; counts[b * grid + wg] (slice-major slots).
__global__ __launch_bounds__(kSliceBlock) void k_slice_count(const int64_t *__restrict__ key, int64_t kmin, uint64_t range,
                                                             int64_t n_tiles, int F, uint32_t *__restrict__ counts) {
    constexpr int W = kSliceBlock / 64;
    __shared__ uint32_t cnt[W][kSliceMaxF];
    const int tid = threadIdx.x, wave = tid >> 6;
    for (int i = tid; i < W * kSliceMaxF; i += kSliceBlock) (&cnt[0][0])[i] = 0;
    __syncthreads();
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int64_t base = tile * kSliceTile;
        v2i64 kk[kSliceTile / (2 * kSliceBlock)];
#pragma unroll
        for (int q = 0; q < kSliceTile / (2 * kSliceBlock); ++q)
            kk[q] = __builtin_nontemporal_load((const v2i64 *)(key + base + 2 * ((int64_t)q * kSliceBlock + tid)));
#pragma unroll
        for (int q = 0; q < kSliceTile / (2 * kSliceBlock); ++q)
#pragma unroll
            for (int x = 0; x < 2; ++x) {
                const uint64_t o = (uint64_t)kk[q][x] - (uint64_t)kmin;
                if (o < range) atomicAdd(&cnt[wave][(uint32_t)(o >> kSliceBits)], 1u);
            }
    }
    __syncthreads();
    for (int b = tid; b < F; b += kSliceBlock) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) c += cnt[w][b];
        counts[(uint64_t)b * gridDim.x + blockIdx.x] = c;
    }
}

// Phase B of the exact-layout join: the probe payload already sits at its
// output position (phase A wrote it into the output column), so each item only
// needs the build payload written beside it: read the 16-bit key offset, look
// it up in the LDS slice, store a.  Items without a match are counted (a
// non-zero count sends the host to the compacting two-pass emit).
__global__ __launch_bounds__(kSliceBlock) void k_slice_join_inplace(SliceRegions rg, int nreg, HashTable t, int64_t amin,
                                                                    int64_t *__restrict__ out_a,
                                                                    unsigned long long *__restrict__ misses) {
    __shared__ __attribute__((aligned(16))) uint16_t tslice[kSliceKeys];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int W = kSliceBlock / 64;
    const int F = rg.F;
    const int64_t T = (int64_t)F * nreg;
    const int64_t s0 = (int64_t)blockIdx.x * T / gridDim.x, s1 = (int64_t)(blockIdx.x + 1) * T / gridDim.x;
    uint32_t miss = 0;
    for (int64_t sb = s0; sb < s1;) {
        const int b = (int)(sb / nreg);
        const int64_t se = std::min<int64_t>(s1, (int64_t)(b + 1) * nreg);
        __syncthreads();
        load_slice(tslice, t, b, tid);
        __syncthreads();
        for (int64_t s = sb + wave; s < se; s += W) {
            const uint64_t reg = (uint64_t)(s - (int64_t)b * nreg) * F + b;
            const uint32_t n_r = rg.count[reg];
            const uint64_t rb = rg.rbase[s];
            const uint16_t *kp = rg.key + rb;
            int64_t *ap = out_a + rb;
            // the next 1024 keys are loaded before this batch's lookups and stores
            uint32_t e[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t i = j * 64 + lane;
                e[j] = __builtin_nontemporal_load(kp + (i < n_r ? i : 0u));
            }
            for (uint32_t i0 = 0; i0 < n_r; i0 += 64 * 16) {
                uint32_t en[16];
                const uint32_t i1 = i0 + 64 * 16;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const uint32_t i = i1 + j * 64 + lane;
                    en[j] = __builtin_nontemporal_load(kp + (i < n_r ? i : 0u));
                }
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const uint32_t i = i0 + j * 64 + lane;
                    if (i < n_r) {
                        const uint32_t x = tslice[e[j]];
                        miss += x == 0u;
                        __builtin_nontemporal_store((int64_t)(x - 1u) + amin, ap + i);
                    }
                }
#pragma unroll
                for (int j = 0; j < 16; ++j) e[j] = en[j];
            }
        }
        sb = se;
    }
    const uint64_t m = wave_sum_u64(miss);
    if (lane == 0 && m) atomicAdd(misses, (unsigned long long)m);
}

// ragged tail (< one 8192-row tile): probe the u16 table directly and append
// after the regions' rows (a few waves: one atomic each per 512 rows)
__global__ __launch_bounds__(kBlock) void k_slice_join_tail(const int64_t *__restrict__ key, const int64_t *__restrict__ val,
                                                            int64_t n, HashTable t, int64_t amin, int64_t *__restrict__ out_v,
                                                            int64_t *__restrict__ out_a, unsigned long long *counter) {
    const int lane = threadIdx.x & 63;
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x * 8 + (threadIdx.x & ~63) * 8; i0 < n;
         i0 += (int64_t)gridDim.x * blockDim.x * 8) {
        uint32_t e[8];
        int64_t v[8];
        bool live[8];
        uint32_t total = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int64_t i = i0 + j * 64 + lane;
            live[j] = i < n;
            e[j] = 0u;
            v[j] = 0;
            if (live[j]) {
                const uint64_t o = (uint64_t)key[i] - (uint64_t)t.kmin;
                if (o < t.range) e[j] = t.payload16[o];
                v[j] = val[i];
            }
            total += (uint32_t)popc64(__ballot(live[j] && e[j] != 0u));
        }
        unsigned long long b = 0;
        if (lane == 0 && total) b = atomicAdd(counter, (unsigned long long)total);
        uint64_t base = __shfl(b, 0, 64);
        emit_matches(e, v, live, amin, &base, out_v, out_a);
    }
}

// ---- single-pass GROUP BY on one key: LDS hash table per workgroup ----------------------
// Each workgroup aggregates its rows into an LDS open-addressing table keyed by
// the key's 64-bit payload (ints sign-extended, floats as bits); rows whose key
// does not find a slot within a few probes go straight to the HBM table.  At
// the end the workgroup merges its occupied slots into the HBM table with
// global atomics: one global update per (workgroup, group), not per row.
__device__ __forceinline__ int64_t gt_slot(const GTable &g, int64_t key) {
    uint64_t h = hash64((uint64_t)key) & g.mask;
    for (uint64_t p = 0; p <= g.mask; ++p) {
        const long long cur = __hip_atomic_load((long long *)&g.keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == key) return (int64_t)h;
        if (cur == kEmptyKey) {
            const unsigned long long old =
                atomicCAS((unsigned long long *)&g.keys[h], (unsigned long long)kEmptyKey, (unsigned long long)key);
            if ((long long)old == kEmptyKey || (long long)old == key) return (int64_t)h;
        }
        if (p > 4096) break;  // a healthy table never probes this far: report overflow, host regrows
        h = (h + 1) & g.mask;
    }
    *g.overflow = 1u;
    return -1;
}

template <int PM>
__global__ __launch_bounds__(kBlock) void k_groupby_lds(ColSet cols, int64_t n, PredTerms terms, DevProgram prog,
                                                        int key_col, GidSource src, AggSpecs specs, int64_t G,
                                                        uint64_t *__restrict__ gstates_all, uint32_t *__restrict__ errp) {
    uint64_t *__restrict__ gstates = shard_states(gstates_all, specs, G);
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const int lcap = src.lcap;
    int64_t *lkeys = (int64_t *)lds;
    uint64_t *lst = lds + lcap;  // [n_slots][lcap]
    for (int i = threadIdx.x; i < lcap; i += blockDim.x) lkeys[i] = kEmptyKey;
    for (int64_t i = threadIdx.x; i < (int64_t)specs.n_slots * lcap; i += blockDim.x) lst[i] = 0;
    __syncthreads();
    for (int a = 0; a < specs.n; ++a) {
        const AggSpec sp = specs.a[a];
        if (sp.kind == AK_MIN || sp.kind == AK_MAX)
            for (int i = threadIdx.x; i < lcap; i += blockDim.x) lst[(int64_t)sp.val_slot * lcap + i] = (uint64_t)agg_init_value(sp.kind);
    }
    __syncthreads();
    const int64_t gcap = (int64_t)src.gt.mask + 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t err = 0;
    const int64_t ntiles = (n + kAggTile - 1) / kAggTile;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t row0 = tile * kAggTile + (int64_t)wave * 64 * kAggR + lane;
        uint32_t sel;
        if (PM == PM_TERMS) {
            sel = eval_terms<kAggR>(terms, cols, row0, 64, n);
        } else if (PM == PM_PROG) {
            ExprRegs<kAggR> X;
            run_program<kAggR>(prog, cols, row0, 64, n, X, err);
            sel = program_true_mask<kAggR>(X);
        } else {
            sel = 0;
#pragma unroll
            for (int r = 0; r < kAggR; ++r)
                if (row0 + r * 64 < n) sel |= 1u << r;
        }
        int64_t kv[kAggR];
        uint32_t kvalid;
        load_rows<kAggR>(cols.c[key_col], row0, 64, n, kv, kvalid);
#pragma unroll
        for (int r = 0; r < kAggR; ++r) {
            if (!((sel >> r) & 1)) continue;
            const int64_t row = row0 + r * 64;
            const int64_t key = kv[r];
            uint64_t *st;
            int64_t stride, idx;
            bool local = false;
            int lslot = -1;
            if (((kvalid >> r) & 1) && key != kEmptyKey) {
                int h = (int)(hash64((uint64_t)key) & (uint64_t)(lcap - 1));
                for (int p = 0; p < 32; ++p) {
                    const int64_t cur = lkeys[h];
                    if (cur == key) { lslot = h; break; }
                    if (cur == kEmptyKey) {
                        const unsigned long long old = atomicCAS((unsigned long long *)&lkeys[h],
                                                                 (unsigned long long)kEmptyKey, (unsigned long long)key);
                        if ((long long)old == kEmptyKey || (long long)old == key) { lslot = h; break; }
                    }
                    h = (h + 1) & (lcap - 1);
                }
            }
            if (lslot >= 0) {
                local = true;
                st = lst;
                stride = lcap;
                idx = lslot;
            } else {
                st = gstates;
                stride = G;
                if (!((kvalid >> r) & 1)) idx = gcap;            // the NULL group
                else if (key == kEmptyKey) idx = gcap + 1;       // the key that doubles as EMPTY
                else idx = gt_slot(src.gt, key);
                if (idx < 0) continue;                            // overflow flagged; host regrows and reruns
            }
            atomicAdd((unsigned long long *)&st[idx], 1ull);
            for (int a = 0; a < specs.n; ++a) {
                const AggSpec sp = specs.a[a];
                const ColRef &c = cols.c[sp.col];
                if (!col_valid(c, row)) continue;
                if (sp.cnt_slot) atomicAdd((unsigned long long *)&st[(int64_t)sp.cnt_slot * stride + idx], 1ull);
                if (sp.kind != AK_COUNT) {
                    const int64_t x = agg_input(sp.kind, sp.in_type, load_i64(c, row));
                    if (local) agg_apply<true>(sp.kind, &st[(int64_t)sp.val_slot * stride + idx], x);
                    else agg_apply<false>(sp.kind, &st[(int64_t)sp.val_slot * stride + idx], x);
                }
            }
        }
    }
    if (err) atomicOr(errp, err);
    __syncthreads();
    for (int i = threadIdx.x; i < lcap; i += blockDim.x) {
        const int64_t key = lkeys[i];
        if (key == kEmptyKey) continue;
        const int64_t g = gt_slot(src.gt, key);
        if (g < 0) continue;
        atomicAdd((unsigned long long *)&gstates[g], (unsigned long long)lst[i]);
        for (int a = 0; a < specs.n; ++a) {
            const AggSpec sp = specs.a[a];
            if (sp.cnt_slot) {
                const uint64_t c = lst[(int64_t)sp.cnt_slot * lcap + i];
                if (c) atomicAdd((unsigned long long *)&gstates[(int64_t)sp.cnt_slot * G + g], (unsigned long long)c);
            }
            if (sp.kind != AK_COUNT)
                agg_merge_global(sp.kind, &gstates[(int64_t)sp.val_slot * G + g], lst[(int64_t)sp.val_slot * lcap + i]);
        }
    }
}

// cheap multiplicative hash for the per-workgroup LDS table (the HBM table keeps hash64)
__device__ __forceinline__ uint32_t lds_hash(int64_t key) {
    const uint32_t x = (uint32_t)key ^ (uint32_t)((uint64_t)key >> 32);
    return (x * 0x9E3779B1u) ^ ((x * 0x9E3779B1u) >> 15);
}

// Fast single-key GROUP BY: the FastTile loads of k_join_agg_fast with the
// group slot found in a per-workgroup LDS hash of keys (linear probing, CAS
// insert); keys that do not fit the LDS table (or INT64_MIN, the empty
// marker) update the HBM table's states directly with global atomics.
template <int NTERMS, int NACOL, bool NT, int BLOCK = kBlock>
__global__ __launch_bounds__(BLOCK) void k_group_agg_fast(FastIn in, PredTerms terms, AggSpecs specs, GTable gt,
                                                           int lcap, int64_t G, int64_t n_tiles,
                                                           uint64_t *__restrict__ gstates_all) {
    uint64_t *__restrict__ gstates = shard_states(gstates_all, specs, G);
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    int64_t *lkeys = (int64_t *)lds;
    uint64_t *lst = lds + lcap;  // [n_slots][lcap]
    for (int i = threadIdx.x; i < lcap; i += blockDim.x) lkeys[i] = kEmptyKey;
    for (int64_t i = threadIdx.x; i < (int64_t)specs.n_slots * lcap; i += blockDim.x) lst[i] = 0;
    __syncthreads();
    for (int a = 0; a < specs.n; ++a) {
        const AggSpec sp = specs.a[a];
        if (sp.kind == AK_MIN || sp.kind == AK_MAX)
            for (int i = threadIdx.x; i < lcap; i += blockDim.x) lst[(int64_t)sp.val_slot * lcap + i] = (uint64_t)agg_init_value(sp.kind);
    }
    __syncthreads();
    const int64_t gcap = (int64_t)gt.mask + 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int64_t base = tile * (BLOCK * kFastR) + (int64_t)wave * (64 * kFastR) + 2 * lane;
        FastTile<NTERMS, NACOL, NT> ft;
        ft.load(in, terms, base);
        const uint32_t sel = ft.sel;
        // first probe of all rows at once (a warm table answers nearly every row
        // there), then the rest of the probe sequence for the few that need it
        int slot[kFastR], h0[kFastR];
        int64_t first[kFastR];
#pragma unroll
        for (int r = 0; r < kFastR; ++r) {
            h0[r] = (int)(lds_hash(ft.k(r)) & (uint32_t)(lcap - 1));
            first[r] = lkeys[h0[r]];
        }
#pragma unroll
        for (int r = 0; r < kFastR; ++r) {
            const int64_t key = ft.k(r);
            slot[r] = (first[r] == key && key != kEmptyKey) ? h0[r] : -1;
            if (slot[r] >= 0 || !((sel >> r) & 1) || key == kEmptyKey) continue;
            int h = h0[r];
            for (int p = 0; p < 32; ++p) {
                const int64_t cur = lkeys[h];
                if (cur == key) { slot[r] = h; break; }
                if (cur == kEmptyKey) {
                    const unsigned long long old = atomicCAS((unsigned long long *)&lkeys[h], (unsigned long long)kEmptyKey,
                                                             (unsigned long long)key);
                    if ((long long)old == kEmptyKey || (long long)old == key) { slot[r] = h; break; }
                }
                h = (h + 1) & (lcap - 1);
            }
        }
        uint32_t in_lds = 0;
#pragma unroll
        for (int r = 0; r < kFastR; ++r) in_lds |= (((sel >> r) & 1) && slot[r] >= 0) ? 1u << r : 0u;
        lds_apply_rows(lst, lcap, specs, in, ft, in_lds, slot);
#pragma unroll
        for (int r = 0; r < kFastR; ++r) {
            if (!((sel >> r) & 1)) continue;
            if (slot[r] < 0) {
                const int64_t key = ft.k(r);
                const int64_t g = key == kEmptyKey ? gcap + 1 : gt_slot(gt, key);
                if (g < 0) continue;  // overflow flagged; host regrows and reruns
                atomicAdd((unsigned long long *)&gstates[g], 1ull);
                for (int a = 0; a < specs.n; ++a) {
                    const AggSpec sp = specs.a[a];
                    if (sp.kind == AK_COUNT) continue;
                    agg_apply<false>(sp.kind, &gstates[(int64_t)sp.val_slot * G + g],
                                     agg_input(sp.kind, sp.in_type, ft.a(in.agg_colslot[a], r)));
                }
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < lcap; i += blockDim.x) {
        const int64_t key = lkeys[i];
        if (key == kEmptyKey) continue;
        const int64_t g = gt_slot(gt, key);
        if (g < 0) continue;
        atomicAdd((unsigned long long *)&gstates[g], (unsigned long long)lst[i]);
        for (int a = 0; a < specs.n; ++a) {
            const AggSpec sp = specs.a[a];
            if (sp.kind != AK_COUNT)
                agg_merge_global(sp.kind, &gstates[(int64_t)sp.val_slot * G + g], lst[(int64_t)sp.val_slot * lcap + i]);
        }
    }
}

__global__ void k_fill_i64(int64_t *p, int64_t n, int64_t v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

__global__ void k_iota(uint32_t *p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)i;
}

__global__ void k_states_init(uint64_t *states, int64_t G, AggSpecs specs) {
    const int64_t words = (int64_t)specs.shards * specs.n_slots * G;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t slot = (i / G) % specs.n_slots;
        uint64_t v = 0;
        for (int a = 0; a < specs.n; ++a)
            if (specs.a[a].val_slot == slot) v = (uint64_t)agg_init_value(specs.a[a].kind);
        states[i] = v;
    }
}

// Fold the shard copies into copy 0 (same merge as agg_merge_global, no atomics).
__global__ void k_states_reduce(uint64_t *states, int64_t G, AggSpecs specs) {
    const int64_t words = (int64_t)specs.n_slots * G;
    const int64_t stride = words;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t slot = i / G;
        int kind = -1;  // counts
        for (int a = 0; a < specs.n; ++a)
            if (specs.a[a].val_slot == slot) kind = specs.a[a].kind;
        uint64_t acc = states[i];
        for (int sh = 1; sh < specs.shards; ++sh) {
            const uint64_t v = states[i + sh * stride];
            switch (kind) {
                case AK_SUM_F: acc = __builtin_bit_cast(uint64_t, as_f64(acc) + as_f64(v)); break;
                case AK_MIN: acc = (int64_t)v < (int64_t)acc ? v : acc; break;
                case AK_MAX: acc = (int64_t)v > (int64_t)acc ? v : acc; break;
                default: acc += v; break;  // counts, wrapping int sums
            }
        }
        states[i] = acc;
    }
}

// Small group tables (G <= kCompactSmallG): fold the shard copies, flag the non-empty groups and
// scan the flags in one workgroup -- one launch where the general path takes five (reduce,
// flags, three scan kernels), ~4-5 us per dependent launch on the query's critical path.
// pos[g] = non-empty groups before g; the count lands in total (the status words).
// Shard fold of small state tables by many workgroups (one word per thread, sixteen shard loads in
// flight): states written by device-scope atomics live beyond the XCD L2s, so a single workgroup
// folding 1024 groups x 64 shards waited ~40 us on load round trips (round-3 step trace).
__global__ __launch_bounds__(256) void k_states_fold(uint64_t *__restrict__ states, int64_t Gs, AggSpecs specs) {
    const int64_t words = (int64_t)specs.n_slots * Gs;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= words) return;
    const int64_t slot = i / Gs;
    int kind = -1;  // counts
    for (int a = 0; a < specs.n; ++a)
        if (specs.a[a].val_slot == slot) kind = specs.a[a].kind;
    uint64_t acc = states[i];
    constexpr int B = 16;
    for (int sh0 = 1; sh0 < specs.shards; sh0 += B) {
        uint64_t v[B];
#pragma unroll
        for (int q = 0; q < B; ++q) v[q] = sh0 + q < specs.shards ? states[i + (sh0 + q) * words] : 0ull;
#pragma unroll
        for (int q = 0; q < B; ++q) {
            if (sh0 + q >= specs.shards) break;
            switch (kind) {
                case AK_SUM_F: acc = __builtin_bit_cast(uint64_t, as_f64(acc) + as_f64(v[q])); break;
                case AK_MIN: acc = (int64_t)v[q] < (int64_t)acc ? v[q] : acc; break;
                case AK_MAX: acc = (int64_t)v[q] > (int64_t)acc ? v[q] : acc; break;
                default: acc += v[q]; break;  // counts, wrapping int sums
            }
        }
    }
    states[i] = acc;
}

// lanes[0][g] = rows of group g, lanes[1 + j][g] = aggregate j's partial (COUNT or float SUM; the
// caller checked the kinds), every shard copy folded in: one thread per lane entry, 16 shard loads
// in flight
// status (the no-wait form): lanes[(1 + n) * G] = 1 when the operator's error or overflow word is set,
// so the caller's all-reduce of the lanes carries every rank's flag.
// fused: the fused pipeline's status words -- a duplicate build key (status[4]) or a declined plan
// (!status[5]) also set the status lane.
__global__ __launch_bounds__(256) void k_states_lanes(const uint64_t *__restrict__ states, int64_t Gs, int64_t G,
                                                      AggSpecs specs, double *__restrict__ lanes,
                                                      const uint32_t *__restrict__ status, int fused = 0) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e == 0 && status)
        lanes[(int64_t)(1 + specs.n) * G] =
            (status[0] | status[1] | (fused ? (status[4] | (status[5] ? 0u : 1u)) : 0u)) ? 1.0 : 0.0;
    if (e >= (int64_t)(1 + specs.n) * G) return;
    const int j = (int)(e / G) - 1;  // -1: the row-count lane
    const int64_t g = e % G;
    const bool fsum = j >= 0 && specs.a[j].kind == AK_SUM_F;
    const int slot = j < 0 ? 0 : (fsum ? specs.a[j].val_slot : specs.a[j].cnt_slot);
    const int64_t words = (int64_t)specs.n_slots * Gs;
    const uint64_t *p = states + (int64_t)slot * Gs + g;
    constexpr int B = 16;
    double fv = 0.0;
    uint64_t uv = 0;
    for (int q0 = 0; q0 < specs.shards; q0 += B) {
        uint64_t v[B];
#pragma unroll
        for (int q = 0; q < B; ++q) v[q] = q0 + q < specs.shards ? p[(int64_t)(q0 + q) * words] : 0ull;
#pragma unroll
        for (int q = 0; q < B; ++q) {
            if (q0 + q >= specs.shards) break;
            if (fsum) fv += as_f64((int64_t)v[q]);
            else uv += v[q];
        }
    }
    lanes[e] = fsum ? fv : (double)uv;
}

constexpr int kCompactSmallG = 16384;
__global__ __launch_bounds__(1024) void k_states_compact_small(uint64_t *__restrict__ states, int64_t Gs, int64_t G,
                                                              AggSpecs specs, uint64_t *__restrict__ pos,
                                                              uint64_t *__restrict__ total) {
    __shared__ uint32_t wsum[16];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (specs.shards > 1) {
        const int64_t words = (int64_t)specs.n_slots * Gs;
        for (int64_t i = t; i < words; i += 1024) {
            const int64_t slot = i / Gs;
            int kind = -1;  // counts
            for (int a = 0; a < specs.n; ++a)
                if (specs.a[a].val_slot == slot) kind = specs.a[a].kind;
            uint64_t acc = states[i];
            // sixteen shard loads in flight: one workgroup folds ~1 MB for 1024 groups x 64 shards,
            // so it is bound by load round trips (four in flight: 32 us per query, profiles/r02)
            constexpr int B = 16;
            for (int sh0 = 1; sh0 < specs.shards; sh0 += B) {
                uint64_t v[B];
#pragma unroll
                for (int q = 0; q < B; ++q) v[q] = sh0 + q < specs.shards ? states[i + (sh0 + q) * words] : 0ull;
#pragma unroll
                for (int q = 0; q < B; ++q) {
                    if (sh0 + q >= specs.shards) break;
                    switch (kind) {
                        case AK_SUM_F: acc = __builtin_bit_cast(uint64_t, as_f64(acc) + as_f64(v[q])); break;
                        case AK_MIN: acc = (int64_t)v[q] < (int64_t)acc ? v[q] : acc; break;
                        case AK_MAX: acc = (int64_t)v[q] > (int64_t)acc ? v[q] : acc; break;
                        default: acc += v[q]; break;  // counts, wrapping int sums
                    }
                }
            }
            states[i] = acc;
        }
        __syncthreads();  // the row counts (slot 0) are folded before they are flagged
    }
    // thread t owns groups [t * per, (t + 1) * per)
    const int64_t per = (G + 1023) / 1024, g0 = (int64_t)t * per, g1 = g0 + per < G ? g0 + per : G;
    uint32_t c = 0;
    for (int64_t g = g0; g < g1; ++g) c += states[g] != 0;
    const uint32_t incl = wave_incl_scan(c);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t base = incl - c, all = 0;
    for (int w = 0; w < 16; ++w) {
        base += w < wave ? wsum[w] : 0u;
        all += wsum[w];
    }
    for (int64_t g = g0; g < g1; ++g) {
        pos[g] = base;
        base += states[g] != 0;
    }
    if (t == 0) *total = all;
}

// ---- finalize ------------------------------------------------------------------------
__global__ void k_group_nonempty(const uint64_t *states, int64_t G, uint32_t *flags) {
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (int64_t)gridDim.x * blockDim.x)
        flags[g] = states[g] != 0;
}

struct OutCol {
    void *values;
    uint32_t *validity;  // nullptr when never null
    int32_t dtype;
    int32_t _pad;
};
struct OutCols {
    OutCol c[kMaxGroupKeys + kMaxAggs];
};

__device__ __forceinline__ void write_value(const OutCol &o, int64_t p, int64_t payload, bool valid) {
    if (o.validity && valid) atomicOr(&o.validity[p >> 5], 1u << (p & 31));
    switch (o.dtype) {
        case QEH_DT_BOOL:
            if (payload & 1) atomicOr(&((uint32_t *)o.values)[p >> 5], 1u << (p & 31));
            break;
        case QEH_DT_INT32: ((int32_t *)o.values)[p] = (int32_t)payload; break;
        case QEH_DT_FLOAT32: ((float *)o.values)[p] = (float)as_f64(payload); break;
        default: ((int64_t *)o.values)[p] = payload; break;  // INT64, FLOAT64 bits
    }
}

__global__ void k_finalize(const uint64_t *__restrict__ states, int64_t G, const uint64_t *__restrict__ pos,
                           KeyCols keys, const uint32_t *__restrict__ rep_row, AggSpecs specs, OutCols outs) {
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t rows = states[g];
        int64_t p;
        if (pos) {
            if (!rows) continue;
            p = (int64_t)pos[g];
        } else {
            p = g;
        }
        for (int k = 0; k < keys.n; ++k) {
            const int64_t r = rep_row[g];
            write_value(outs.c[k], p, load_i64(keys.c[k], r), col_valid(keys.c[k], r));
        }
        for (int a = 0; a < specs.n; ++a) {
            const AggSpec sp = specs.a[a];
            const uint64_t cnt = sp.cnt_slot ? states[(int64_t)sp.cnt_slot * G + g] : rows;
            const int64_t v = sp.kind == AK_COUNT ? 0 : (int64_t)states[(int64_t)sp.val_slot * G + g];
            const OutCol &o = outs.c[keys.n + a];
            const bool i32 = sp.in_type == QEH_DT_INT32;
            const bool flt = sp.in_type == QEH_DT_FLOAT32 || sp.in_type == QEH_DT_FLOAT64;
            switch (sp.func) {
                case QEH_AGG_COUNT: write_value(o, p, (int64_t)cnt, true); break;
                case QEH_AGG_SUM:
                    // Int32 sums wrap at 32 bits before widening (compute::sum(Int32Array) as i64)
                    write_value(o, p, i32 ? (int64_t)(int32_t)v : v, cnt != 0);
                    break;
                case QEH_AGG_AVG: {
                    double s = flt ? as_f64(v) : (double)(i32 ? (int64_t)(int32_t)v : v);
                    write_value(o, p, f64_bits(cnt ? s / (double)cnt : 0.0), cnt != 0);
                    break;
                }
                default: {  // MIN / MAX keep the input type
                    int64_t out = flt ? f64_bits(f64_from_order_key(v)) : v;
                    write_value(o, p, out, cnt != 0);
                    break;
                }
            }
        }
    }
}

// After phase B (shard copies folded): one workgroup compacts the non-empty group slots, writes the
// output keys, aggregates and validity words (zeroed here first) and the group count (*total).
__global__ __launch_bounds__(1024) void k_fused_finish(const uint64_t *__restrict__ states, int64_t G, KeyCols keys,
                                                       const uint32_t *__restrict__ rep, AggSpecs specs, OutCols outs,
                                                       uint64_t *__restrict__ total) {
    __shared__ uint32_t pos[kSliceStateWords];
    __shared__ uint32_t vbits[kMaxGroupKeys + kMaxAggs][kSliceStateWords / 32];  // validity, built in LDS
    __shared__ uint32_t wsum[16];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int nout = keys.n + specs.n;
    const int64_t vwords = (G + 31) / 32;
    for (int c = 0; c < nout; ++c)
        for (int64_t w = t; w < vwords; w += blockDim.x) vbits[c][w] = 0u;
    const int64_t per = (G + 1023) / 1024, g0 = (int64_t)t * per, g1 = g0 + per < G ? g0 + per : G;
    uint32_t c = 0;
    for (int64_t g = g0; g < g1; ++g) c += states[g] != 0;
    const uint32_t incl = wave_incl_scan(c);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t base = incl - c, all = 0;
    for (int w = 0; w < 16; ++w) {
        base += w < wave ? wsum[w] : 0u;
        all += wsum[w];
    }
    for (int64_t g = g0; g < g1; ++g) {
        pos[g] = base;
        base += states[g] != 0;
    }
    if (t == 0) *total = all;
    __syncthreads();  // validity bits zeroed, positions known
    // values by plain stores, validity bits in LDS (written out once below)
    auto put = [&](int c, int64_t p, int64_t payload, bool valid) {
        OutCol o = outs.c[c];
        if (o.validity && valid) atomicOr(&vbits[c][p >> 5], 1u << (p & 31));
        o.validity = nullptr;
        write_value(o, p, payload, true);
    };
    for (int64_t g = t; g < G; g += blockDim.x) {
        const uint64_t rows = states[g];
        if (!rows) continue;
        const int64_t p = pos[g];
        for (int k = 0; k < keys.n; ++k) {
            const int64_t r = rep[g];
            put(k, p, load_i64(keys.c[k], r), col_valid(keys.c[k], r));
        }
        for (int a = 0; a < specs.n; ++a) {
            const AggSpec sp = specs.a[a];
            const uint64_t cnt = sp.cnt_slot ? states[(int64_t)sp.cnt_slot * G + g] : rows;
            const int64_t v = sp.kind == AK_COUNT ? 0 : (int64_t)states[(int64_t)sp.val_slot * G + g];
            const int o = keys.n + a;
            const bool i32 = sp.in_type == QEH_DT_INT32;
            const bool flt = sp.in_type == QEH_DT_FLOAT32 || sp.in_type == QEH_DT_FLOAT64;
            switch (sp.func) {
                case QEH_AGG_COUNT: put(o, p, (int64_t)cnt, true); break;
                case QEH_AGG_SUM: put(o, p, i32 ? (int64_t)(int32_t)v : v, cnt != 0); break;
                case QEH_AGG_AVG: {
                    double sm = flt ? as_f64(v) : (double)(i32 ? (int64_t)(int32_t)v : v);
                    put(o, p, f64_bits(cnt ? sm / (double)cnt : 0.0), cnt != 0);
                    break;
                }
                default: put(o, p, flt ? f64_bits(f64_from_order_key(v)) : v, cnt != 0); break;
            }
        }
    }
    __syncthreads();
    for (int c = 0; c < nout; ++c)
        if (outs.c[c].validity)
            for (int64_t w = t; w < vwords; w += blockDim.x) outs.c[c].validity[w] = vbits[c][w];
}

// ---- host helpers ----------------------------------------------------------------------
static int agg_output_type(int func, int in_type) {
    switch (func) {
        case QEH_AGG_COUNT: return QEH_DT_INT64;
        case QEH_AGG_SUM: return (in_type == QEH_DT_FLOAT32 || in_type == QEH_DT_FLOAT64) ? QEH_DT_FLOAT64 : QEH_DT_INT64;
        case QEH_AGG_AVG: return QEH_DT_FLOAT64;
        default: return in_type;
    }
}

// `cols` are the kernel's columns; aggs[i].column indexes `agg_cols[]`, which
// maps to ColSet indexes through `colset_index`.
static int plan_aggs(const qeh_agg *aggs, int n_aggs, const qeh_column *inputs, int n_inputs,
                     const int *colset_index, AggSpecs *out) {
    if (n_aggs > kMaxAggs) return fail(QEH_E_UNSUPPORTED, "too many aggregates for one device operator (max 8)");
    std::memset(out, 0, sizeof(*out));
    out->n = n_aggs;
    out->shards = 1;
    int slot = 1;
    for (int i = 0; i < n_aggs; ++i) {
        const qeh_agg &a = aggs[i];
        if (a.column < 0 || a.column >= n_inputs) return fail(QEH_E_INVALID, "aggregate input index out of range");
        const qeh_column &c = inputs[a.column];
        int t = c.dtype;
        AggSpec &s = out->a[i];
        s.func = a.func;
        s.col = colset_index[a.column];
        s.in_type = t;
        const bool numeric = t == QEH_DT_INT32 || t == QEH_DT_INT64 || t == QEH_DT_FLOAT32 || t == QEH_DT_FLOAT64;
        const bool flt = t == QEH_DT_FLOAT32 || t == QEH_DT_FLOAT64;
        switch (a.func) {
            case QEH_AGG_COUNT: s.kind = AK_COUNT; break;
            case QEH_AGG_SUM:
                if (!numeric) return fail(QEH_E_TYPE, "Unsupported type for SUM");
                s.kind = flt ? AK_SUM_F : AK_SUM_I;
                break;
            case QEH_AGG_AVG:
                if (!numeric) return fail(QEH_E_TYPE, "Unsupported type for AVG");
                s.kind = flt ? AK_SUM_F : AK_SUM_I;
                break;
            case QEH_AGG_MIN:
                if (!numeric) return fail(QEH_E_TYPE, "Unsupported type for MIN");
                s.kind = AK_MIN;
                break;
            case QEH_AGG_MAX:
                if (!numeric) return fail(QEH_E_TYPE, "Unsupported type for MAX");
                s.kind = AK_MAX;
                break;
            default: return fail(QEH_E_INVALID, "unknown aggregate function");
        }
        s.val_slot = s.kind == AK_COUNT ? -1 : slot++;
        const bool has_nulls = c.validity != nullptr && c.null_count != 0;
        s.cnt_slot = has_nulls ? slot++ : 0;
    }
    out->n_slots = slot;
    return QEH_OK;
}

struct PredPlan {
    int mode = PM_NONE;
    PredTerms terms{};
    DevProgram prog{};
};

static int plan_predicate(const qeh_expr *pred, const int32_t *dtypes, int n_cols, PredPlan *pp) {
    pp->mode = PM_NONE;
    if (!pred || pred->n_nodes == 0) return QEH_OK;
    QEH_TRY(compile_expr(pred, dtypes, n_cols, &pp->prog));
    if (pp->prog.result_type != QEH_DT_BOOL)
        return fail(QEH_E_TYPE, "Filter predicate must return boolean");
    pp->mode = lower_to_terms(pred, dtypes, n_cols, &pp->terms) ? PM_TERMS : PM_PROG;
    return QEH_OK;
}

template <int GM>
static void launch_agg_rows(qeh_ctx *ctx, int pm, bool lds, int grid, size_t shmem, const ColSet &cols, int64_t n,
                            const PredPlan &pp, const GidSource &src, const AggSpecs &specs, int64_t G,
                            uint64_t *states, uint32_t *err) {
#define QEH_LAUNCH(PMV, LDSV)                                                                                  \
    hipLaunchKernelGGL((k_agg_rows<GM, PMV, LDSV>), dim3(grid), dim3(kBlock), shmem, ctx->stream, cols, n, pp.terms, \
                       pp.prog, src, specs, G, states, err)
    if (pm == PM_NONE) { if (lds) QEH_LAUNCH(PM_NONE, true); else QEH_LAUNCH(PM_NONE, false); }
    else if (pm == PM_TERMS) { if (lds) QEH_LAUNCH(PM_TERMS, true); else QEH_LAUNCH(PM_TERMS, false); }
    else { if (lds) QEH_LAUNCH(PM_PROG, true); else QEH_LAUNCH(PM_PROG, false); }
#undef QEH_LAUNCH
}

static ColRef advance(ColRef c, int64_t rows) {
    size_t es = dtype_size(c.dtype);
    if (c.dtype != QEH_DT_BOOL && es) c.values = (const char *)c.values + (size_t)rows * es;
    c.vbit0 += rows;
    return c;
}

static bool fast_col_ok(const ColRef &c) {
    return (c.dtype == QEH_DT_INT64 || c.dtype == QEH_DT_FLOAT64) && c.validity == nullptr &&
           ((uintptr_t)c.values & 15) == 0;
}

static int fast_nt_mode() {
    static int m = -1;
    if (m < 0) {
        const char *e = std::getenv("QEH_NT_LOADS");  // non-temporal fact-column loads (default on: -4%)
        m = (e && e[0] == '0') ? 0 : 1;
    }
    return m;
}

// The fused probe's fast path: returns true when it launched (full tiles by
// k_join_agg_fast, the ragged tail by the generic kernel).
// Eligibility of the specialised probe kernels; fills the kernel's view.
// `key_col`: the column read as FastIn::key (join probe key or group key).
static bool fast_cols_eligible(const ColSet &cols, const PredPlan &pp, int key_col, const AggSpecs &specs,
                               FastIn *inp, int *nterms_out, int *nacol_out) {
    if (pp.mode == PM_PROG || (pp.mode == PM_TERMS && pp.terms.n > 2)) return false;
    if (!fast_col_ok(cols.c[key_col])) return false;
    FastIn &in = *inp;
    in = FastIn{};
    in.key = (const int64_t *)cols.c[key_col].values;
    const int nterms = pp.mode == PM_TERMS ? pp.terms.n : 0;
    for (int i = 0; i < nterms; ++i) {
        const ColRef &c = cols.c[pp.terms.t[i].col];
        if (!fast_col_ok(c)) return false;
        in.term[i] = (const int64_t *)c.values;
        in.term_dt[i] = c.dtype;
    }
    int nacol = 0;
    int acol_idx[2] = {-1, -1};
    for (int a = 0; a < specs.n; ++a) {
        const AggSpec &sp = specs.a[a];
        if (sp.cnt_slot != 0) return false;
        in.agg_colslot[a] = -1;
        if (sp.kind == AK_COUNT) continue;
        int slot = -1;
        for (int c = 0; c < nacol; ++c)
            if (acol_idx[c] == sp.col) slot = c;
        if (slot < 0) {
            if (nacol == 2) return false;
            if (!fast_col_ok(cols.c[sp.col])) return false;
            acol_idx[nacol] = sp.col;
            in.acol[nacol] = (const int64_t *)cols.c[sp.col].values;
            slot = nacol++;
        }
        in.agg_colslot[a] = slot;
    }
    *nterms_out = nterms;
    *nacol_out = nacol;
    return true;
}

static bool fast_eligible(const ColSet &cols, const PredPlan &pp, const GidSource &src, const AggSpecs &specs,
                          FastIn *inp, int *nterms_out, int *nacol_out) {
    if (!src.jt.unique) return false;
    if (cols.c[src.key_col].dtype != QEH_DT_INT64) return false;
    return fast_cols_eligible(cols, pp, src.key_col, specs, inp, nterms_out, nacol_out);
}

static void launch_tail(qeh_ctx *ctx, const ColSet &cols, int64_t n, int64_t done, const PredPlan &pp,
                        const GidSource &src, const AggSpecs &specs, int64_t G, uint64_t *states, uint32_t *err,
                        size_t lds_bytes) {
    if (done >= n) return;
    ColSet tail = cols;
    for (int i = 0; i < cols.n; ++i) tail.c[i] = advance(cols.c[i], done);
    // a few workgroups (each merges its LDS partials into the global states): one took 70 us
    // for the 6464 rows past the last full tile of a 1.25e8-row shard
    const int grid = (int)std::min<int64_t>(16, (n - done + kAggTile - 1) / kAggTile);
    launch_agg_rows<GM_JOIN>(ctx, pp.mode, true, std::max(grid, 1), lds_bytes, tail, n - done, pp, src, specs, G, states,
                             err);
}

static uint64_t table_bytes(const HashTable &t);

// The bucket-range partitioned probe (k_bp_part + chunk_lists + k_bp_probe) for a BUCKET table past
// the Infinity Cache's comfortable share; false when it does not apply (nothing launched).
static bool try_bucket_parts(qeh_ctx *ctx, const FastIn &in, const PredPlan &pp, int nterms, int nacol,
                             const AggSpecs &specs, const HashTable &t, int64_t G, int64_t n, uint64_t *states,
                             size_t lds_bytes) {
    // opt-in (QEH_BUCKET_PARTS=1): measured slower than the single pass at the sparse metric shape
    // (P1 7.5-7.9 ms + P2 8.9 ms against 13.2 ms; profiles/r06/bucket_parts.txt) -- the probes hit the
    // XCD's L2 (4.7e8 TCC hits, 1.1e8 misses) and still run at the single pass's ~56 G probes/s
    if (t.kind != TK_BUCKET || nacol > 1 || !std::getenv("QEH_BUCKET_PARTS")) return false;
    if (lds_bytes > 64 * 1024) return false;
    const int cus = ctx->props.multiProcessorCount;
    const int64_t n_tiles = (n + kBpTile - 1) / kBpTile;
    const int grid1 = (int)std::max<int64_t>(1, std::min<int64_t>(2 * (int64_t)cus, n_tiles));
    const uint64_t max_chunks = (uint64_t)(n + kBpChunk - 1) / kBpChunk + (uint64_t)grid1 * kBpP;
    if (max_chunks >= (1ull << 24)) return false;
    DevBuf keys, vals, tags, cnts, lists, ctr;
    if (keys.alloc(ctx, max_chunks * kBpChunk * 8) != QEH_OK || (nacol && vals.alloc(ctx, max_chunks * kBpChunk * 8) != QEH_OK) ||
        tags.alloc(ctx, max_chunks * 2) != QEH_OK || cnts.alloc(ctx, max_chunks * 2) != QEH_OK ||
        lists.alloc(ctx, max_chunks * 4 + (kBpP + 1) * 4 + chunk_lists_work_words(kBpP) * 4) != QEH_OK ||
        ctr.alloc(ctx, 4) != QEH_OK)
        return false;
    if (hipMemsetAsync(tags.p, 0xFF, max_chunks * 2, ctx->stream) != hipSuccess ||
        hipMemsetAsync(ctr.p, 0, 4, ctx->stream) != hipSuccess)
        return false;
    const int acs = nacol ? 0 : -1;
    KernelTimer kt(ctx, "bucket_parts");
    const bool nt = fast_nt_mode() == 1;
#define QEH_BP(NTV, NAV, NTB)                                                                                            \
    hipLaunchKernelGGL((k_bp_part<NTV, NAV, NTB>), dim3(grid1), dim3(kBpBlock), 0, ctx->stream, in, pp.terms, n, acs,   \
                       keys.as<uint64_t>(), vals.as<uint64_t>(), tags.as<uint16_t>(), cnts.as<uint16_t>(), ctr.as<uint32_t>())
#define QEH_BP_NA(NTV, NTB)                  \
    if (nacol == 0) QEH_BP(NTV, 0, NTB);     \
    else QEH_BP(NTV, 1, NTB);
#define QEH_BP_NT(NTB)                           \
    if (nterms == 0) { QEH_BP_NA(0, NTB) }       \
    else if (nterms == 1) { QEH_BP_NA(1, NTB) }  \
    else { QEH_BP_NA(2, NTB) }
    if (nt) { QEH_BP_NT(true) } else { QEH_BP_NT(false) }
#undef QEH_BP_NT
#undef QEH_BP_NA
#undef QEH_BP
    uint32_t *sbase = lists.as<uint32_t>() + max_chunks;
    if (chunk_lists(ctx, tags.as<uint16_t>(), cnts.as<uint16_t>(), max_chunks, kBpP, sbase, lists.as<uint32_t>(),
                    sbase + kBpP + 1) != QEH_OK)
        return false;
    const int grid2 = std::max(8, (2 * cus + 7) / 8 * 8);  // a multiple of 8: every XCD the same count
    if (nacol)
        hipLaunchKernelGGL(k_bp_probe<1>, dim3(grid2), dim3(kBpBlock), lds_bytes, ctx->stream, specs, in, t, G, sbase,
                           lists.as<uint32_t>(), keys.as<uint64_t>(), vals.as<uint64_t>(), states);
    else
        hipLaunchKernelGGL(k_bp_probe<0>, dim3(grid2), dim3(kBpBlock), lds_bytes, ctx->stream, specs, in, t, G, sbase,
                           lists.as<uint32_t>(), keys.as<uint64_t>(), vals.as<uint64_t>(), states);
    // the pool buffers above must outlive the kernels
    return hipStreamSynchronize(ctx->stream) == hipSuccess;
}

static bool try_fast_join(qeh_ctx *ctx, const ColSet &cols, int64_t n, const PredPlan &pp, const GidSource &src,
                          const AggSpecs &specs, int64_t G, uint64_t *states, uint32_t *err, size_t lds_bytes,
                          int per_cu) {
    if (std::getenv("QEH_NO_FAST")) return false;
    FastIn in;
    int nterms, nacol;
    if (!fast_eligible(cols, pp, src, specs, &in, &nterms, &nacol)) return false;
    if (try_bucket_parts(ctx, in, pp, nterms, nacol, specs, src.jt, G, n, states, lds_bytes)) return true;
    const int64_t n_tiles = n / kFastTile;
    if (n_tiles > 0) {
        const int grid = grid_for(ctx, n_tiles * kFastTile, kFastTile, per_cu);
        const bool nt = fast_nt_mode() == 1;
#define QEH_FAST(NTV, NAV, NTB)                                                                                    \
    hipLaunchKernelGGL((k_join_agg_fast<NTV, NAV, NTB>), dim3(grid), dim3(kBlock), lds_bytes, ctx->stream, in, pp.terms, \
                       specs, src.jt, G, n_tiles, states)
#define QEH_FAST_NA(NTV, NTB)                       \
    if (nacol == 0) QEH_FAST(NTV, 0, NTB);          \
    else if (nacol == 1) QEH_FAST(NTV, 1, NTB);     \
    else QEH_FAST(NTV, 2, NTB);
#define QEH_FAST_NT(NTB)                            \
    if (nterms == 0) { QEH_FAST_NA(0, NTB) }        \
    else if (nterms == 1) { QEH_FAST_NA(1, NTB) }   \
    else { QEH_FAST_NA(2, NTB) }
        if (nt) { QEH_FAST_NT(true) } else { QEH_FAST_NT(false) }
#undef QEH_FAST_NT
#undef QEH_FAST_NA
#undef QEH_FAST
    }
    launch_tail(ctx, cols, n, n_tiles * kFastTile, pp, src, specs, G, states, err, lds_bytes);
    return true;
}

static uint64_t table_bytes(const HashTable &t) {
    if (t.kind == TK_DIRECT) return t.range * (t.payload16 ? 2 : 4);
    if (t.kind == TK_PACKED) return (t.mask + 1) * 8;
    if (t.kind == TK_BUCKET) return t.nbkt * 64;
    return (t.mask + 1) * 16;
}

// Phase A does not need the join table — only its key range — so the fused join-aggregate
// launches it on the context's second queue right after the build key's min/max, and the
// build (group table, join table) runs on the main queue underneath it.  try_slice_join then
// only waits for it before phase B.  When the finished table turns out not to fit the slice
// path (duplicate keys, wide payloads), the prelaunched work is discarded.
struct SlicePre {
    bool launched = false;
    int64_t kmin = 0;
    uint64_t range = 0;
    int grid = 0;
    int64_t n_tiles = 0;
    DevBuf kbuf, vbuf, cbuf, planbuf, vbuf2;
    SliceRegions rg{};
    hipEvent_t done = nullptr;
    bool dev_planned = false;  // launched from a plan in device memory, not yet read back (resolve_dev_plan)
    hipEvent_t plan_copied = nullptr;  // the plan's copy into ctx->pinned_plan (queued ahead of phase A)
    ~SlicePre() {
        if (done) {  // the buffers below must outlive the kernel
            (void)hipEventSynchronize(done);
            (void)hipEventDestroy(done);
        }
        if (plan_copied) {
            (void)hipEventSynchronize(plan_copied);
            (void)hipEventDestroy(plan_copied);
        }
    }
};

// Build-side ranges phase A is planned from: build key min / max / non-null count and the
// group key's (one integer group key).
struct BuildRanges {
    int64_t mn[2], mx[2], cnt[2];
    bool operator==(const BuildRanges &o) const {
        return std::memcmp(mn, o.mn, sizeof mn) == 0 && std::memcmp(mx, o.mx, sizeof mx) == 0 &&
               std::memcmp(cnt, o.cnt, sizeof cnt) == 0;
    }
};

// Phase A launched by qeh_join_filter_aggregate_prelaunch, waiting on the context for the call it
// belongs to: the same probe columns, key, predicate and aggregates (compared by identity / by
// value).  Phase A stages the aggregate input column it was planned with, so a call with other
// aggregates (COUNT vs SUM(v), SUM over another column) must not adopt it.
struct PendingSlice {
    SlicePre pre;
    std::vector<const void *> vals;
    std::vector<int64_t> offs, lens;
    std::vector<int32_t> dtypes;
    int key_idx = -1;
    std::vector<uint8_t> pred;  // the predicate's serialised form (empty = none)
    std::vector<int32_t> agg_fc;  // (func, column) of every aggregate
    BuildRanges br{};
    static std::vector<uint8_t> serialise(const qeh_expr *e);
    static std::vector<int32_t> agg_list(const qeh_agg *aggs, int n_aggs) {
        std::vector<int32_t> v;
        for (int i = 0; i < n_aggs; ++i) v.push_back(aggs[i].func), v.push_back(aggs[i].column);
        return v;
    }
    bool matches(const qeh_column *cols, int n_cols, int key, const qeh_expr *predicate, const qeh_agg *aggs,
                 int n_aggs) const {
        if (n_cols != (int)vals.size() || key != key_idx) return false;
        for (int i = 0; i < n_cols; ++i)
            if (cols[i].values != vals[i] || cols[i].offset != offs[i] || cols[i].length != lens[i] ||
                cols[i].dtype != dtypes[i])
                return false;
        return agg_list(aggs, n_aggs) == agg_fc && serialise(predicate) == pred;
    }
    void take(SlicePre *dst) {
        dst->launched = pre.launched;
        dst->kmin = pre.kmin;
        dst->range = pre.range;
        dst->grid = pre.grid;
        dst->n_tiles = pre.n_tiles;
        std::swap(dst->kbuf.p, pre.kbuf.p), std::swap(dst->kbuf.n, pre.kbuf.n), std::swap(dst->kbuf.ctx, pre.kbuf.ctx);
        std::swap(dst->vbuf.p, pre.vbuf.p), std::swap(dst->vbuf.n, pre.vbuf.n), std::swap(dst->vbuf.ctx, pre.vbuf.ctx);
        std::swap(dst->cbuf.p, pre.cbuf.p), std::swap(dst->cbuf.n, pre.cbuf.n), std::swap(dst->cbuf.ctx, pre.cbuf.ctx);
        std::swap(dst->planbuf.p, pre.planbuf.p), std::swap(dst->planbuf.n, pre.planbuf.n),
            std::swap(dst->planbuf.ctx, pre.planbuf.ctx);
        std::swap(dst->vbuf2.p, pre.vbuf2.p), std::swap(dst->vbuf2.n, pre.vbuf2.n), std::swap(dst->vbuf2.ctx, pre.vbuf2.ctx);
        dst->rg = pre.rg;
        dst->dev_planned = pre.dev_planned;
        std::swap(dst->done, pre.done);
        pre.launched = false;
    }
};

std::vector<uint8_t> PendingSlice::serialise(const qeh_expr *e) {
    std::vector<uint8_t> b;
    if (!e || !e->nodes || e->n_nodes <= 0) return b;
    b.resize((size_t)e->n_nodes * sizeof(qeh_expr_node));
    std::memcpy(b.data(), e->nodes, b.size());
    return b;
}

// regions sized for every row selected with keys uniform over the slices, +25 %
static bool slice_regions(qeh_ctx *ctx, int64_t n_tiles, int grid, uint64_t F, int nacol, DevBuf *kbuf, DevBuf *vbuf,
                          DevBuf *cbuf, SliceRegions *rg, hipStream_t stream, int64_t tile_rows = kSliceTile,
                          DevBuf *vbuf2 = nullptr) {
    const int64_t tiles_per_wg = (n_tiles + grid - 1) / grid;
    uint64_t cap = (uint64_t)((double)tiles_per_wg * tile_rows / (double)F * 1.25) + 256;
    cap = (cap + kSliceChunk - 1) / kSliceChunk * kSliceChunk;
    const uint64_t nreg = (uint64_t)grid * F;
    if (kbuf->alloc(ctx, nreg * cap * 2 + 64) != QEH_OK) return false;
    if (nacol && vbuf->alloc(ctx, nreg * cap * 8 + 64) != QEH_OK) return false;
    if (nacol > 1 && (!vbuf2 || vbuf2->alloc(ctx, nreg * cap * 8 + 64) != QEH_OK)) return false;
    if (cbuf->alloc(ctx, nreg * 4 + 64) != QEH_OK) return false;
    *rg = SliceRegions{};
    rg->key = kbuf->as<uint16_t>();
    rg->val = nacol ? vbuf->as<int64_t>() : nullptr;
    rg->val2 = nacol > 1 ? vbuf2->as<int64_t>() : nullptr;
    rg->count = cbuf->as<uint32_t>();
    rg->overflow = rg->count + nreg;
    rg->cap = cap;
    rg->F = (int32_t)F;
    return hipMemsetAsync(rg->overflow, 0, 4, stream) == hipSuccess;
}

// gid_table != nullptr: MODE 1 (group-range slices, `range` = groups)
static void launch_slice_partition(qeh_ctx *ctx, const FastIn &in, const PredPlan &pp, int nterms, int nacol, int64_t kmin,
                                   uint64_t range, int64_t n_tiles, int grid, const SliceRegions &rg_in, hipStream_t stream,
                                   const HashTable *gid_table = nullptr, const SlicePlan *dplan = nullptr) {
    const bool nt = fast_nt_mode() == 1;
    SliceRegions rg = rg_in;
    KernelTimer kta(ctx, "slice_partition", stream);
    const HashTable t = gid_table ? *gid_table : HashTable{};
#define QEH_SA(NTV, NAV, NTB)                                                                                        \
    if (gid_table)                                                                                                   \
        hipLaunchKernelGGL((k_slice_partition<NTV, NAV, NTB, 1>), dim3(grid), dim3(kSliceBlock), 0, stream, in,     \
                           pp.terms, kmin, range, n_tiles, rg, t, nullptr);                                          \
    else                                                                                                             \
        hipLaunchKernelGGL((k_slice_partition<NTV, NAV, NTB>), dim3(grid), dim3(kSliceBlock), 0, stream, in,        \
                           pp.terms, kmin, range, n_tiles, rg, t, dplan)
#define QEH_SA_NA(NTV, NTB)                    \
    if (nacol == 0) { QEH_SA(NTV, 0, NTB); }   \
    else if (nacol == 1) { QEH_SA(NTV, 1, NTB); } \
    else { QEH_SA(NTV, 2, NTB); }
#define QEH_SA_NT(NTB)                         \
    if (nterms == 0) { QEH_SA_NA(0, NTB) }     \
    else if (nterms == 1) { QEH_SA_NA(1, NTB) } \
    else { QEH_SA_NA(2, NTB) }
    if (nt) { QEH_SA_NT(true) } else { QEH_SA_NT(false) }
#undef QEH_SA_NT
#undef QEH_SA_NA
#undef QEH_SA
}

// Tiles per chunk of the chunked slice pipeline (QEH_SLICE_CHUNK_TILES; 0 = one pass).
static int64_t slice_chunk_tiles() {
    const char *e = std::getenv("QEH_SLICE_CHUNK_TILES");
    return e ? std::strtoll(e, nullptr, 10) : 0;
}

static int slice_prelaunch_ranges(qeh_ctx *ctx, const ColSet &cols, int64_t n, const PredPlan &pp, const AggSpecs &specs,
                                  int key_col, const BuildRanges &br, SlicePre *pre);

// Phase A launched from a plan in device memory: regions for the worst case, `launch_plan` queues the
// plan kernel on the main queue (into pre->planbuf), phase A follows on the second queue.  Returns
// whether it launched (*launched); pre->launched stays false until the plan is known on the host.
template <class LaunchPlan>
static int slice_launch_dev(qeh_ctx *ctx, const ColSet &cols, int64_t n, const PredPlan &pp, const AggSpecs &specs,
                            int key_col, SlicePlanIn *pi, SlicePre *pre, LaunchPlan launch_plan, bool *launched) {
    *launched = false;
    FastIn in;
    int nterms, nacol;
    if (!fast_cols_eligible(cols, pp, key_col, specs, &in, &nterms, &nacol) || nacol > 2 ||
        (nacol == 2 && std::getenv("QEH_NO_SLICE_AGG2")))
        return QEH_OK;
    const int64_t tile_rows = nacol == 2 ? (int64_t)SliceShape<2>::TILE : (int64_t)kSliceTile;
    const int64_t n_tiles = n / tile_rows;
    hipStream_t side = n_tiles ? aux_stream(ctx) : nullptr;
    if (!side) return QEH_OK;
    *pi = SlicePlanIn{};
    pi->min_bytes = 6ull << 20;
    if (const char *e = std::getenv("QEH_SLICE_MIN_BYTES")) pi->min_bytes = std::strtoull(e, nullptr, 10);
    pi->grid = (int)std::min<int64_t>(ctx->props.multiProcessorCount, n_tiles);
    pi->n_slots = specs.n_slots;
    pi->sparse_ok = direct_sparse_allowed() ? 1 : 0;
    const uint64_t tiles_per_wg = (uint64_t)((n_tiles + pi->grid - 1) / pi->grid);
    // every row selected, keys uniform over the slices, +25 % (and per-region slack for the largest F)
    pi->alloc_items = tiles_per_wg * pi->grid * (uint64_t)tile_rows * 5 / 4 + (uint64_t)pi->grid * kSliceMaxF * 288;
    const uint64_t nreg_max = (uint64_t)pi->grid * kSliceMaxF;
    if (pre->kbuf.alloc(ctx, pi->alloc_items * 2 + 64) != QEH_OK ||
        (nacol && pre->vbuf.alloc(ctx, pi->alloc_items * 8 + 64) != QEH_OK) ||
        (nacol > 1 && pre->vbuf2.alloc(ctx, pi->alloc_items * 8 + 64) != QEH_OK) ||
        pre->cbuf.alloc(ctx, nreg_max * 4 + 64) != QEH_OK || pre->planbuf.alloc(ctx, sizeof(SlicePlan)) != QEH_OK)
        return QEH_OK;
    hipEvent_t ready = nullptr;
    if (hipEventCreateWithFlags(&ready, hipEventDisableTiming) != hipSuccess) return QEH_OK;
    if (hipEventCreateWithFlags(&pre->done, hipEventDisableTiming) != hipSuccess) {
        pre->done = nullptr;
        (void)hipEventDestroy(ready);
        return QEH_OK;
    }
    SliceRegions &rg = pre->rg;
    rg = SliceRegions{};
    rg.key = pre->kbuf.as<uint16_t>();
    rg.val = nacol ? pre->vbuf.as<int64_t>() : nullptr;
    rg.val2 = nacol > 1 ? pre->vbuf2.as<int64_t>() : nullptr;
    rg.count = pre->cbuf.as<uint32_t>();
    rg.overflow = rg.count + nreg_max;
    QEH_HIP(hipMemsetAsync(rg.overflow, 0, 4, ctx->stream));
    launch_plan(*pi, pre->planbuf.as<SlicePlan>());
    // the plan's host copy goes ahead of phase A: a copy queued behind it would wait for phase A's
    // workgroups to leave the CUs, and with it the host that reads the plan
    if (!ctx->pinned_plan && hipHostMalloc(&ctx->pinned_plan, sizeof(SlicePlan), hipHostMallocDefault) != hipSuccess)
        ctx->pinned_plan = nullptr;
    if (ctx->pinned_plan && hipEventCreateWithFlags(&pre->plan_copied, hipEventDisableTiming) == hipSuccess) {
        if (hipMemcpyAsync(ctx->pinned_plan, pre->planbuf.p, sizeof(SlicePlan), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
            hipEventRecord(pre->plan_copied, ctx->stream) != hipSuccess) {
            (void)hipEventDestroy(pre->plan_copied);
            pre->plan_copied = nullptr;
        }
    }
    (void)hipEventRecord(ready, ctx->stream);  // inputs, the plan and the overflow reset
    (void)hipStreamWaitEvent(side, ready, 0);
    launch_slice_partition(ctx, in, pp, nterms, nacol, 0, 0, n_tiles, pi->grid, rg, side, nullptr,
                           pre->planbuf.as<SlicePlan>());
    (void)hipEventRecord(pre->done, side);
    (void)hipEventDestroy(ready);
    if (hipGetLastError() != hipSuccess) return fail(QEH_E_HIP, "slice prelaunch failed");
    pre->dev_planned = true;
    pre->grid = pi->grid;
    pre->n_tiles = n_tiles;
    *launched = true;
    return QEH_OK;
}

// A device-planned launch whose plan is `pl`: adopted (launched, shape set) when it planned the slice
// path; else phase A returned at once and its worst-case regions are released now.
static void settle_dev_plan(qeh_ctx *ctx, SlicePre *pre, const SlicePlan &pl) {
    pre->dev_planned = false;
    if (!pl.ok) {
        // the launch returned at once: its timing record is not a phase A
        for (auto it = ctx->timing_pending.rbegin(); it != ctx->timing_pending.rend(); ++it)
            if (it->name == "slice_partition") {
                it->name = "slice_partition_declined";
                break;
            }
        (void)hipEventSynchronize(pre->done);
        (void)hipEventDestroy(pre->done);
        pre->done = nullptr;
        pre->kbuf.reset(), pre->vbuf.reset(), pre->cbuf.reset(), pre->planbuf.reset(), pre->vbuf2.reset();
        return;
    }
    pre->rg.F = pl.F;
    pre->rg.cap = pl.cap;
    pre->launched = true;
    pre->kmin = pl.kmin;
    pre->range = pl.range;
}

// The plan of a device-planned launch read back (one small read; the plan kernel ran long before).
static int resolve_dev_plan(qeh_ctx *ctx, SlicePre *pre, BuildRanges *br) {
    SlicePlan pl{};
    if (pre->plan_copied) {  // copied ahead of phase A: wait for that copy only
        QEH_HIP(hipEventSynchronize(pre->plan_copied));
        (void)hipEventDestroy(pre->plan_copied);
        pre->plan_copied = nullptr;
        std::memcpy(&pl, ctx->pinned_plan, sizeof pl);
    } else {
        QEH_TRY(read_small(ctx, &pl, pre->planbuf.p, sizeof pl));
    }
    for (int q = 0; q < 2; ++q) br->mn[q] = pl.src[3 * q], br->mx[q] = pl.src[3 * q + 1], br->cnt[q] = pl.src[3 * q + 2];
    settle_dev_plan(ctx, pre, pl);
    return QEH_OK;
}

// Launch phase A ahead of the build when the slice path is predictable from the build key's
// range alone (and the group count is known to stay small).  Not launching is never an error.
// The ranges' min/max kernels, the plan (k_slice_plan) and phase A are queued back to back -- phase A
// reads its shape from device memory -- and the host reads the ranges back while phase A runs; it
// adopts the launch when its own evaluation of the same plan says the slice path applies (phase A
// returned at once otherwise).
static int slice_prelaunch(qeh_ctx *ctx, const ColSet &cols, int64_t n, const PredPlan &pp, const AggSpecs &specs,
                           int key_col, const qeh_column &build_key, const qeh_column &group_key, SlicePre *pre) {
    if (std::getenv("QEH_NO_SLICES") || std::getenv("QEH_NO_OVERLAP") || slice_chunk_tiles() > 0) return QEH_OK;
    if (cols.c[key_col].dtype != QEH_DT_INT64 || build_key.dtype != QEH_DT_INT64) return QEH_OK;
    if (group_key.dtype != QEH_DT_INT64 && group_key.dtype != QEH_DT_INT32) return QEH_OK;
    if (n / SliceShape<2>::TILE == 0) return QEH_OK;
    const qeh_column both[2] = {build_key, group_key};
    if (std::getenv("QEH_HOST_PLAN")) {  // the ranges read back before phase A is launched
        BuildRanges br;
        QEH_TRY(columns_minmax(ctx, both, 2, br.mn, br.mx, br.cnt));
        return slice_prelaunch_ranges(ctx, cols, n, pp, specs, key_col, br, pre);
    }
    DevBuf mm;
    QEH_TRY(mm.alloc(ctx, sizeof(MinMax) * 2 + 16));
    QEH_TRY(columns_minmax_launch(ctx, both, 2, mm.as<MinMax>()));
    SlicePlanIn pi;
    bool launched = false;
    QEH_TRY(slice_launch_dev(
        ctx, cols, n, pp, specs, key_col, &pi, pre,
        [&](const SlicePlanIn &p, SlicePlan *out) {
            hipLaunchKernelGGL(k_slice_plan, dim3(1), dim3(64), 0, ctx->stream, mm.as<MinMax>(), p, out);
        },
        &launched));
    BuildRanges br;  // read while phase A runs (and memoised for the build)
    QEH_TRY(columns_minmax_collect(ctx, both, 2, mm.as<MinMax>(), br.mn, br.mx, br.cnt));
    if (launched) settle_dev_plan(ctx, pre, plan_slices(pi, br.mn[0], br.mx[0], br.cnt[0], br.mn[1], br.mx[1], br.cnt[1]));
    return QEH_OK;
}

static int slice_prelaunch_ranges(qeh_ctx *ctx, const ColSet &cols, int64_t n, const PredPlan &pp, const AggSpecs &specs,
                                  int key_col, const BuildRanges &br, SlicePre *pre) {
    if (std::getenv("QEH_NO_SLICES") || std::getenv("QEH_NO_OVERLAP") || slice_chunk_tiles() > 0) return QEH_OK;
    if (cols.c[key_col].dtype != QEH_DT_INT64) return QEH_OK;
    FastIn in;
    int nterms, nacol;
    if (!fast_cols_eligible(cols, pp, key_col, specs, &in, &nterms, &nacol) || nacol > 1) return QEH_OK;
    const int64_t n_tiles = n / kSliceTile;
    if (n_tiles == 0) return QEH_OK;
    const int64_t *mns = br.mn, *mxs = br.mx, *cnts = br.cnt;
    const int64_t mn = mns[0], mx = mxs[0], cnt = cnts[0];
    if (cnt == 0) return QEH_OK;
    const uint64_t gr = cnts[1] ? (uint64_t)mxs[1] - (uint64_t)mns[1] + 1ull : 0;
    const int64_t g_bound = (gr == 0 || gr > (1ull << 20)) ? -1 : (int64_t)gr + 1;
    if (g_bound <= 0 || g_bound >= 0xFFFF || (int64_t)specs.n_slots * g_bound > kSliceStateWords) return QEH_OK;
    const uint64_t range = (uint64_t)mx - (uint64_t)mn + 1ull;
    // the DIRECT rule of build_join_table, and the slice path's own limits
    if (!direct_table_ok(range, (uint64_t)cnt, (uint64_t)g_bound)) return QEH_OK;
    uint64_t min_bytes = 6ull << 20;
    if (const char *e = std::getenv("QEH_SLICE_MIN_BYTES")) min_bytes = std::strtoull(e, nullptr, 10);
    if (range * 2 < min_bytes) return QEH_OK;
    const uint64_t F = (range + kSliceKeys - 1) >> kSliceBits;
    if (F == 0 || F > (uint64_t)kSliceMaxF) return QEH_OK;
    // optionally leave CUs to the build on the main queue (QEH_SLICE_RESERVE_CUS): with one
    // phase-A workgroup on every CU the build's kernels wait for phase A to drain, but phase A
    // loses more on fewer CUs than the build costs afterwards
    int reserve = 0;
    if (const char *e = std::getenv("QEH_SLICE_RESERVE_CUS")) reserve = std::atoi(e);
    reserve = std::max(0, std::min(reserve, ctx->props.multiProcessorCount / 2));
    const int grid = (int)std::min<int64_t>(ctx->props.multiProcessorCount - reserve, n_tiles);
    hipStream_t side = aux_stream(ctx);
    if (!side) return QEH_OK;
    if (!slice_regions(ctx, n_tiles, grid, F, nacol, &pre->kbuf, &pre->vbuf, &pre->cbuf, &pre->rg, ctx->stream))
        return QEH_OK;
    hipEvent_t ready;
    if (hipEventCreateWithFlags(&ready, hipEventDisableTiming) != hipSuccess) return QEH_OK;
    if (hipEventCreateWithFlags(&pre->done, hipEventDisableTiming) != hipSuccess) {
        (void)hipEventDestroy(ready);
        pre->done = nullptr;
        return QEH_OK;
    }
    (void)hipEventRecord(ready, ctx->stream);  // inputs and the region buffers' reset are on the main queue
    (void)hipStreamWaitEvent(side, ready, 0);
    launch_slice_partition(ctx, in, pp, nterms, nacol, mn, range, n_tiles, grid, pre->rg, side);
    (void)hipEventRecord(pre->done, side);
    (void)hipEventDestroy(ready);
    if (hipGetLastError() != hipSuccess) return fail(QEH_E_HIP, "slice prelaunch failed");
    pre->launched = true;
    pre->kmin = mn;
    pre->range = range;
    pre->grid = grid;
    pre->n_tiles = n_tiles;
    return QEH_OK;
}

static bool slice_probe_prefetch() {
    static const int v = [] {
        const char *e = std::getenv("QEH_SLICE_B_PREFETCH");
        return e ? std::atoi(e) : 1;
    }();
    return v != 0;
}

static void launch_slice_probe(qeh_ctx *ctx, const SliceRegions &rg, int nreg, const HashTable &t, const FastIn &in,
                               const AggSpecs &specs, int64_t G, uint64_t *states, int nacol) {
    KernelTimer ktb(ctx, "slice_probe");
    const int gridB = ctx->props.multiProcessorCount;
    const bool pf = slice_probe_prefetch();
    static const bool pv = std::getenv("QEH_SLICE_B_PAIRS") && std::atoi(std::getenv("QEH_SLICE_B_PAIRS")) == 1;
#define QEH_SB(NAV, PFV)                                                                                           \
    do {                                                                                                           \
        if (pv)                                                                                                    \
            hipLaunchKernelGGL((k_slice_probe<NAV, false, PFV, true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream, rg, \
                               nreg, 0, t, in, specs, G, states);                                            \
        else                                                                                                       \
            hipLaunchKernelGGL((k_slice_probe<NAV, false, PFV>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream, rg, nreg, \
                               0, t, in, specs, G, states);                                                  \
    } while (0)
    if (nacol == 0) {
        if (pf) QEH_SB(0, true);
        else QEH_SB(0, false);
    } else {
        if (pf) QEH_SB(1, true);
        else QEH_SB(1, false);
    }
#undef QEH_SB
}

// LDS-slice partitioned probe (k_slice_partition + k_slice_probe) for unique
// direct u16 tables past an XCD's L2.  Returns 1 when it ran; 0 when not
// eligible, or when a region overflowed (probe keys skewed onto few slices),
// in which case the states are re-initialised for the single pass.
// ovf_copy != nullptr: the overflow flag is copied there (stream-ordered) and 2 returned instead of
// reading it here; the caller reads it with its other results and re-runs on overflow.
static int try_slice_join(qeh_ctx *ctx, const ColSet &cols, int64_t n, const PredPlan &pp, const GidSource &src,
                          const AggSpecs &specs, int64_t G, uint64_t *states, uint32_t *err, size_t lds_bytes,
                          SlicePre *pre, uint32_t *ovf_copy = nullptr) {
    if (std::getenv("QEH_NO_SLICES")) return 0;
    FastIn in;
    int nterms, nacol;
    if (!fast_eligible(cols, pp, src, specs, &in, &nterms, &nacol)) return 0;
    const HashTable &t = src.jt;
    if (t.kind != TK_DIRECT || !t.payload16 || nacol > 2 || (nacol == 2 && std::getenv("QEH_NO_SLICE_AGG2"))) return 0;
    if ((int64_t)specs.n_slots * G > kSliceStateWords) return 0;
    const uint64_t F = (t.range + kSliceKeys - 1) >> kSliceBits;
    if (F == 0 || F > (uint64_t)kSliceMaxF) return 0;
    // below ~1.5 L2s the single pass's lookups mostly hit L2 and it wins
    uint64_t min_bytes = 6ull << 20;
    if (const char *e = std::getenv("QEH_SLICE_MIN_BYTES")) min_bytes = std::strtoull(e, nullptr, 10);
    if (table_bytes(t) < min_bytes) return 0;
    // two aggregate columns: half tiles (SliceShape<2>)
    const int64_t tile_rows = nacol == 2 ? (int64_t)SliceShape<2>::TILE : (int64_t)kSliceTile;
    const int64_t n_tiles = n / tile_rows;
    if (n_tiles == 0) return 0;
    int grid = (int)std::min<int64_t>(ctx->props.multiProcessorCount, n_tiles);
    bool tail_done = false;
    hipEvent_t tail_ev = nullptr;
    DevBuf kbuf, vbuf, cbuf, vbuf2;
    SliceRegions rg{};
    if (pre && pre->launched && pre->kmin == t.kmin && pre->range == t.range && pre->n_tiles == n_tiles) {
        grid = pre->grid;  // phase A's workgroups = regions per slice
        rg = pre->rg;  // phase A already ran on the second queue, under the build
        // The ragged tail (rows past the last full tile, one workgroup) runs on the second queue
        // right after phase A, once the build it reads is done: launched beside phase A it sat on
        // one CU for the whole of phase A (profiles/r02: 4.9 ms resident) and slowed that CU's
        // phase-A workgroup, the one the static tile split waits for.  QEH_TAIL_BESIDE=1: old order.
        // Phase B waits for phase A only; the tail runs on the second queue beside phase B (both
        // merge into the global states with atomics) and the main queue waits for it after phase B.
        if (std::getenv("QEH_TAIL_BESIDE")) {
            launch_tail(ctx, cols, n, n_tiles * tile_rows, pp, src, specs, G, states, err, lds_bytes);
        } else if (n > n_tiles * tile_rows) {
            hipStream_t side = aux_stream(ctx), main = ctx->stream;
            hipEvent_t built;
            if (hipEventCreateWithFlags(&built, hipEventDisableTiming) != hipSuccess) return 0;
            if (hipEventCreateWithFlags(&tail_ev, hipEventDisableTiming) != hipSuccess) {
                (void)hipEventDestroy(built);
                tail_ev = nullptr;
                return 0;
            }
            (void)hipEventRecord(built, main);
            (void)hipStreamWaitEvent(side, built, 0);
            (void)hipEventDestroy(built);
            ctx->stream = side;
            launch_tail(ctx, cols, n, n_tiles * tile_rows, pp, src, specs, G, states, err, lds_bytes);
            ctx->stream = main;
            (void)hipEventRecord(tail_ev, side);
        }
        tail_done = true;
        if (hipStreamWaitEvent(ctx->stream, pre->done, 0) != hipSuccess) return 0;
    } else {
        const int64_t chunk = slice_chunk_tiles();
        if (chunk > 0 && chunk < n_tiles && nacol < 2) {
            // chunked pipeline: phase A and phase B alternate over chunks of `chunk` tiles; each
            // chunk's exchange (plain stores) is read back by its phase B from the Infinity Cache
            const int gridc = (int)std::min<int64_t>(ctx->props.multiProcessorCount, chunk);
            if (!slice_regions(ctx, chunk, gridc, F, nacol, &kbuf, &vbuf, &cbuf, &rg, ctx->stream)) return 0;
            for (int64_t t0 = 0; t0 < n_tiles; t0 += chunk) {
                const int64_t nt = std::min<int64_t>(chunk, n_tiles - t0);
                FastIn ic = in;
                const int64_t r0 = t0 * kSliceTile;
                ic.key += r0;
                for (int q = 0; q < 2; ++q) {
                    if (ic.term[q]) ic.term[q] += r0;
                    if (ic.acol[q]) ic.acol[q] += r0;
                }
                const int g = (int)std::min<int64_t>(gridc, nt);
                launch_slice_partition(ctx, ic, pp, nterms, nacol, t.kmin, t.range, nt, g, rg, ctx->stream);
                launch_slice_probe(ctx, rg, g, t, ic, specs, G, states, nacol);
            }
            if (hipGetLastError() != hipSuccess) return 0;
            launch_tail(ctx, cols, n, n_tiles * tile_rows, pp, src, specs, G, states, err, lds_bytes);
            uint32_t of = 0;
            if (read_small(ctx, &of, rg.overflow, 4) != QEH_OK) return 0;
            if (of) {
                hipLaunchKernelGGL(k_states_init, dim3(grid_for(ctx, specs.shards * specs.n_slots * G, kBlock * 4, 8)),
                                   dim3(kBlock), 0, ctx->stream, states, G, specs);
                return 0;
            }
            return 1;
        }
        if (!slice_regions(ctx, n_tiles, grid, F, nacol, &kbuf, &vbuf, &cbuf, &rg, ctx->stream, tile_rows, &vbuf2)) return 0;
        launch_slice_partition(ctx, in, pp, nterms, nacol, t.kmin, t.range, n_tiles, grid, rg, ctx->stream);
    }
    {
        KernelTimer ktb(ctx, "slice_probe");
        const int gridB = ctx->props.multiProcessorCount;
        int splits = 0;
        if (const char *e = std::getenv("QEH_SLICE_SPLITS")) splits = std::atoi(e);
        const bool pf = slice_probe_prefetch();
        static const bool pv = std::getenv("QEH_SLICE_B_PAIRS") && std::atoi(std::getenv("QEH_SLICE_B_PAIRS")) == 1;
#define QEH_SB(NAV, PFV)                                                                                              \
    do {                                                                                                              \
        if (pv)                                                                                                       \
            hipLaunchKernelGGL((k_slice_probe<NAV, false, PFV, true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream, rg, \
                               grid, splits, t, in, specs, G, states);                                          \
        else                                                                                                          \
            hipLaunchKernelGGL((k_slice_probe<NAV, false, PFV>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream, rg, grid, \
                               splits, t, in, specs, G, states);                                                \
    } while (0)
        if (nacol == 0) {
            if (pf) QEH_SB(0, true);
            else QEH_SB(0, false);
        } else if (nacol == 1) {
            if (pf) QEH_SB(1, true);
            else QEH_SB(1, false);
        } else {
            if (pf) QEH_SB(2, true);
            else QEH_SB(2, false);
        }
#undef QEH_SB
    }
    if (tail_ev) {  // the tail beside phase B: the states are complete once it is done too
        (void)hipStreamWaitEvent(ctx->stream, tail_ev, 0);
        (void)hipEventDestroy(tail_ev);
    }
    if (hipGetLastError() != hipSuccess) return 0;
    if (!tail_done) launch_tail(ctx, cols, n, n_tiles * tile_rows, pp, src, specs, G, states, err, lds_bytes);
    if (ovf_copy) {
        if (hipMemcpyAsync(ovf_copy, rg.overflow, 4, hipMemcpyDeviceToDevice, ctx->stream) != hipSuccess) return -1;
        return 2;
    }
    uint32_t of = 0;
    if (read_small(ctx, &of, rg.overflow, 4) != QEH_OK) return 0;
    if (of) {
        hipLaunchKernelGGL(k_states_init, dim3(grid_for(ctx, specs.shards * specs.n_slots * G, kBlock * 4, 8)), dim3(kBlock), 0,
                           ctx->stream, states, G, specs);
        return 0;
    }
    return 1;
}

// Key-window slices (k_slice_keyagg) for joins whose group states do not fit LDS but whose build key
// range fits the slice shape (a direct table, entries of any width): phase A as for the LDS-state
// pipeline, phase B aggregates per join key.  Returns 1 when it ran; 0 when not eligible or a region
// overflowed, with the states re-initialised.
static int try_key_slices(qeh_ctx *ctx, const ColSet &cols, int64_t n, const PredPlan &pp, const GidSource &src,
                          const AggSpecs &specs, int64_t G, uint64_t *states, uint32_t *err) {
    if (std::getenv("QEH_NO_SLICES") || std::getenv("QEH_NO_KEY_SLICES")) return 0;
    FastIn in;
    int nterms, nacol;
    if (!fast_eligible(cols, pp, src, specs, &in, &nterms, &nacol) || nacol > 1) return 0;
    const HashTable &t = src.jt;
    if (t.kind != TK_DIRECT || !t.unique) return 0;
    // windows: the fewest whose per-key states (u32 count + 8 B per value slot) fit the LDS words
    // (u16 counts when they save a window: QEH_KEYAGG_C16=0 keeps u32)
    auto windows = [&](int cb) { return (int)((kSliceKeys + (int64_t)kKeyAggWords * 8 / (cb + 8 * (int64_t)(specs.n_slots - 1)) / 4 * 4 - 1) /
                                              ((int64_t)kKeyAggWords * 8 / (cb + 8 * (int64_t)(specs.n_slots - 1)) / 4 * 4)); };
    const bool c16 = windows(2) < windows(4) && !(std::getenv("QEH_KEYAGG_C16") && std::atoi(std::getenv("QEH_KEYAGG_C16")) == 0);
    const int64_t per_key = (c16 ? 2 : 4) + 8 * (int64_t)(specs.n_slots - 1);
    const int nw = windows(c16 ? 2 : 4);
    const int ws = (int)(((kSliceKeys + nw - 1) / nw + 3) / 4 * 4);
    const int gpx = ctx->props.multiProcessorCount / 8 / nw;  // groups of nw workgroups per XCD
    if (gpx == 0 || (int64_t)ws * per_key > (int64_t)kKeyAggWords * 8) return 0;
    const int gridB = 8 * gpx * nw;
    const uint64_t F = (t.range + kSliceKeys - 1) >> kSliceBits;
    if (F == 0 || F > (uint64_t)kSliceMaxF) return 0;
    uint64_t min_bytes = 6ull << 20;
    if (const char *e = std::getenv("QEH_SLICE_MIN_BYTES")) min_bytes = std::strtoull(e, nullptr, 10);
    if (table_bytes(t) < min_bytes) return 0;
    const int64_t n_tiles = n / kSliceTile;
    if (n_tiles == 0) return 0;
    const int grid = (int)std::min<int64_t>(ctx->props.multiProcessorCount, n_tiles);
    DevBuf kbuf, vbuf, cbuf;
    SliceRegions rg{};
    if (!slice_regions(ctx, n_tiles, grid, F, nacol, &kbuf, &vbuf, &cbuf, &rg, ctx->stream)) return 0;
    launch_slice_partition(ctx, in, pp, nterms, nacol, t.kmin, t.range, n_tiles, grid, rg, ctx->stream);
    {
        KernelTimer ktb(ctx, "slice_keyagg");
        // whole slices for the full rounds of the 8 * gpx groups; the slices left over split so that the
        // last round has about one part per group (QEH_KEYAGG_TAIL=0: whole slices only)
        const int ngrp = 8 * gpx;
        int full = (int)F / ngrp * ngrp, tparts = 1;
        if ((int)F > full) tparts = std::max(1, std::min(grid, ngrp / ((int)F - full)));
        if (const char *e = std::getenv("QEH_KEYAGG_TAIL"))
            if (std::atoi(e) == 0) full = (int)F, tparts = 1;
#define QEH_KA(NAV, C16V)                                                                                            \
    hipLaunchKernelGGL((k_slice_keyagg<NAV, C16V>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream, rg, grid, t, specs, G, \
                       states, nw, ws, full, tparts)
        if (nacol == 0) {
            if (c16) QEH_KA(0, true);
            else QEH_KA(0, false);
        } else {
            if (c16) QEH_KA(1, true);
            else QEH_KA(1, false);
        }
#undef QEH_KA
    }
    const int64_t done = n_tiles * kSliceTile;
    if (done < n) {  // ragged tail: generic kernel, global states
        ColSet tail = cols;
        for (int i = 0; i < cols.n; ++i) tail.c[i] = advance(cols.c[i], done);
        launch_agg_rows<GM_JOIN>(ctx, pp.mode, false, 1, 0, tail, n - done, pp, src, specs, G, states, err);
    }
    if (hipGetLastError() != hipSuccess) return 0;
    uint32_t of = 0;
    if (read_small(ctx, &of, rg.overflow, 4) != QEH_OK) return 0;
    if (of) {
        hipLaunchKernelGGL(k_states_init, dim3(grid_for(ctx, specs.shards * specs.n_slots * G, kBlock * 4, 8)), dim3(kBlock), 0,
                           ctx->stream, states, G, specs);
        return 0;
    }
    return 1;
}

// Group-range slices for joins whose group states do not fit LDS (G > kSliceStateWords /
// n_slots): phase A (MODE 1) looks each selected row's group id up in the join table and
// partitions the rows by gid >> kGidSliceBits; phase B (IDENT) aggregates each range of
// 2^kGidSliceBits groups in LDS.  Replaces one scattered global atomic per row and aggregate
// (the generic kernel) by 10 bytes of exchange per selected row.  Returns 1 when it ran; 0 when
// not eligible or a region overflowed (skewed groups), with the states re-initialised.
static int try_gid_slices(qeh_ctx *ctx, const ColSet &cols, int64_t n, const PredPlan &pp, const GidSource &src,
                          const AggSpecs &specs, int64_t G, uint64_t *states, uint32_t *err) {
    if (std::getenv("QEH_NO_SLICES") || std::getenv("QEH_NO_GID_SLICES")) return 0;
    FastIn in;
    int nterms, nacol;
    if (!fast_eligible(cols, pp, src, specs, &in, &nterms, &nacol) || nacol > 1) return 0;
    if (((int64_t)specs.n_slots << kGidSliceBits) > kGidStateWords) return 0;
    const uint64_t F = ((uint64_t)G + (1u << kGidSliceBits) - 1) >> kGidSliceBits;
    if (F == 0 || F > (uint64_t)kSliceMaxF) return 0;
    const int64_t n_tiles = n / kSliceTile;
    if (n_tiles == 0) return 0;
    const int grid = (int)std::min<int64_t>(ctx->props.multiProcessorCount, n_tiles);
    DevBuf kbuf, vbuf, cbuf;
    SliceRegions rg{};
    if (!slice_regions(ctx, n_tiles, grid, F, nacol, &kbuf, &vbuf, &cbuf, &rg, ctx->stream)) return 0;
    launch_slice_partition(ctx, in, pp, nterms, nacol, 0, (uint64_t)G, n_tiles, grid, rg, ctx->stream, &src.jt);
    {
        KernelTimer ktb(ctx, "slice_probe");
        const int gridB = ctx->props.multiProcessorCount;
        if (nacol == 0)
            hipLaunchKernelGGL((k_slice_probe<0, true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream, rg, grid, 0, src.jt,
                               in, specs, G, states);
        else
            hipLaunchKernelGGL((k_slice_probe<1, true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream, rg, grid, 0, src.jt,
                               in, specs, G, states);
    }
    const int64_t done = n_tiles * kSliceTile;
    if (done < n) {  // ragged tail: generic kernel, global states
        ColSet tail = cols;
        for (int i = 0; i < cols.n; ++i) tail.c[i] = advance(cols.c[i], done);
        launch_agg_rows<GM_JOIN>(ctx, pp.mode, false, 1, 0, tail, n - done, pp, src, specs, G, states, err);
    }
    if (hipGetLastError() != hipSuccess) return 0;
    uint32_t of = 0;
    if (read_small(ctx, &of, rg.overflow, 4) != QEH_OK) return 0;
    if (of) {
        hipLaunchKernelGGL(k_states_init, dim3(grid_for(ctx, specs.shards * specs.n_slots * G, kBlock * 4, 8)), dim3(kBlock), 0,
                           ctx->stream, states, G, specs);
        return 0;
    }
    return 1;
}

int slice_join_materialise(qeh_ctx *ctx, const qeh_column &probe_key, const qeh_column &probe_val,
                           const qeh_column &build_key, const qeh_column &build_val, qeh_column *out_probe,
                           qeh_column *out_build, int64_t *out_rows) {
    if (std::getenv("QEH_NO_SLICES")) return kSliceJoinNotEligible;
    const ColRef pk = make_colref(probe_key), pv = make_colref(probe_val);
    if (probe_key.dtype != QEH_DT_INT64 || !fast_col_ok(pk) || !fast_col_ok(pv)) return kSliceJoinNotEligible;
    if (build_val.dtype != QEH_DT_INT64 || (build_val.validity && build_val.null_count != 0)) return kSliceJoinNotEligible;
    if (build_key.validity && build_key.null_count != 0) return kSliceJoinNotEligible;
    const int64_t n = probe_key.length;
    const int64_t n_tiles = n / kSliceTile;
    if (n_tiles == 0 || build_key.length == 0) return kSliceJoinNotEligible;
    // build payload as a frame-of-reference u16: (a - amin) + 1 in the direct table
    int64_t amin, amax, avalid;
    QEH_TRY(column_minmax(ctx, build_val, &amin, &amax, &avalid));
    if ((uint64_t)amax - (uint64_t)amin >= 0xFFFEull) return kSliceJoinNotEligible;
    BuiltTable bt;
    RowPayload rp;
    rp.values = (const int64_t *)build_val.values + build_val.offset;
    rp.bias = amin;
    QEH_TRY(build_join_table(ctx, build_key, rp, (uint64_t)amax - (uint64_t)amin, &bt));
    const HashTable &t = bt.t;
    if (!t.unique || t.kind != TK_DIRECT || !t.payload16) return kSliceJoinNotEligible;
    const uint64_t F = (t.range + kSliceKeys - 1) >> kSliceBits;
    if (F == 0 || F > (uint64_t)kSliceMaxF) return kSliceJoinNotEligible;
    uint64_t min_bytes = 6ull << 20;
    if (const char *e = std::getenv("QEH_SLICE_MIN_BYTES")) min_bytes = std::strtoull(e, nullptr, 10);
    if (table_bytes(t) < min_bytes) return kSliceJoinNotEligible;

    // Exact region layout: a key-only count pass sizes every (workgroup, slice) region, so
    // phase A writes the probe payload straight into the output column (slice-major, no
    // gaps) and phase B only adds the build payload beside it.  When some probe rows have
    // no match, the two-pass emit compacts the regions into fresh columns instead.
    const int grid = (int)std::min<int64_t>(ctx->props.multiProcessorCount, n_tiles);
    const uint64_t nreg = (uint64_t)grid * F;
    const uint64_t T = nreg;  // region slots, slice-major
    DevBuf kbuf, cbuf, counts, bases;
    QEH_TRY(cbuf.alloc(ctx, nreg * 4 + 64));
    QEH_TRY(counts.alloc(ctx, T * 4 + 16));
    QEH_TRY(bases.alloc(ctx, T * 8 + 16));
    FastIn in{};
    in.key = (const int64_t *)pk.values;
    in.acol[0] = (const int64_t *)pv.values;
    in.agg_colslot[0] = 0;
    uint64_t region_rows = 0;
    {
        KernelTimer kt(ctx, "join_probe");
        hipLaunchKernelGGL(k_slice_count, dim3(grid), dim3(kSliceBlock), 0, ctx->stream, in.key, t.kmin, t.range, n_tiles,
                           (int)F, counts.as<uint32_t>());
        QEH_HIP(hipGetLastError());
    }
    QEH_TRY(exclusive_scan_u32(ctx, counts.as<uint32_t>(), bases.as<uint64_t>(), (int64_t)T, &region_rows));
    QEH_TRY(kbuf.alloc(ctx, region_rows * 2 + 64));
    SliceRegions rg{};
    rg.key = kbuf.as<uint16_t>();
    rg.count = cbuf.as<uint32_t>();
    rg.overflow = rg.count + nreg;                                                                     // 4 B
    unsigned long long *counter = (unsigned long long *)(cbuf.as<char>() + ((nreg * 4 + 15) & ~15ull));  // 8 B
    unsigned long long *misses = counter + 1;                                                          // 8 B
    rg.cap = 1ull << 62;  // exact regions never overflow
    rg.F = (int32_t)F;
    rg.rbase = bases.as<uint64_t>();
    QEH_HIP(hipMemsetAsync(rg.overflow, 0, 4, ctx->stream));
    QEH_HIP(hipMemsetAsync(counter, 0, 16, ctx->stream));
    QEH_TRY(alloc_column(ctx, probe_val.dtype, n, false, out_probe));
    int st = alloc_column(ctx, QEH_DT_INT64, n, false, out_build);
    if (st != QEH_OK) {
        qeh_column_release(ctx, out_probe);
        return st;
    }
    rg.val = (int64_t *)out_probe->values;
    PredTerms none{};
    const bool nt = fast_nt_mode() == 1;
    int64_t *oa = (int64_t *)out_build->values;
    const int gridB = ctx->props.multiProcessorCount;
    {
        KernelTimer kt(ctx, "join_probe");
        if (nt)
            hipLaunchKernelGGL((k_slice_partition<0, 1, true>), dim3(grid), dim3(kSliceBlock), 0, ctx->stream, in, none,
                               t.kmin, t.range, n_tiles, rg, HashTable{}, nullptr);
        else
            hipLaunchKernelGGL((k_slice_partition<0, 1, false>), dim3(grid), dim3(kSliceBlock), 0, ctx->stream, in, none,
                               t.kmin, t.range, n_tiles, rg, HashTable{}, nullptr);
        hipLaunchKernelGGL(k_slice_join_inplace, dim3(gridB), dim3(kSliceBlock), 0, ctx->stream, rg, grid, t, amin, oa,
                           misses);
        if (hipGetLastError() != hipSuccess) st = fail(QEH_E_HIP, "slice join launch failed");
    }
    uint64_t nmiss = 0;
    if (st == QEH_OK) st = read_small(ctx, &nmiss, misses, 8);
    qeh_column cv = *out_probe, ca = *out_build;  // the columns the tail appends to
    if (st == QEH_OK && nmiss != 0) {
        // some probe rows have no match: compact the regions (read from the first output
        // column) into fresh columns with the two-pass emit
        qeh_column cv2{}, ca2{};
        DevBuf counts2, bases2;
        st = alloc_column(ctx, probe_val.dtype, n, false, &cv2);
        if (st == QEH_OK) st = alloc_column(ctx, QEH_DT_INT64, n, false, &ca2);
        if (st == QEH_OK) st = counts2.alloc(ctx, T * 4 + 16);
        if (st == QEH_OK) st = bases2.alloc(ctx, T * 8 + 16);
        if (st == QEH_OK) {
            KernelTimer kt(ctx, "join_probe");
            hipLaunchKernelGGL((k_slice_join_b<false>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream, rg, grid, t, amin,
                               counts2.as<uint32_t>(), nullptr, nullptr, nullptr);
        }
        if (st == QEH_OK) st = exclusive_scan_u32(ctx, counts2.as<uint32_t>(), bases2.as<uint64_t>(), (int64_t)T, &region_rows);
        if (st == QEH_OK) {
            KernelTimer kt(ctx, "join_probe");
            hipLaunchKernelGGL((k_slice_join_b<true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream, rg, grid, t, amin,
                               nullptr, bases2.as<uint64_t>(), (int64_t *)cv2.values, (int64_t *)ca2.values);
            if (hipGetLastError() != hipSuccess) st = fail(QEH_E_HIP, "slice join launch failed");
        }
        if (st == QEH_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) st = fail(QEH_E_HIP, "slice join sync failed");
        if (st == QEH_OK) {
            qeh_column_release(ctx, out_probe);
            qeh_column_release(ctx, out_build);
            *out_probe = cv = cv2;
            *out_build = ca = ca2;
        } else {
            if (cv2.values) qeh_column_release(ctx, &cv2);
            if (ca2.values) qeh_column_release(ctx, &ca2);
        }
    }
    if (st == QEH_OK) {
        KernelTimer kt(ctx, "join_probe");
        const int64_t done = n_tiles * kSliceTile;
        hipLaunchKernelGGL(k_fill_i64, dim3(1), dim3(1), 0, ctx->stream, (int64_t *)counter, (int64_t)1, (int64_t)region_rows);
        if (done < n)
            hipLaunchKernelGGL(k_slice_join_tail, dim3(grid_for(ctx, n - done, kBlock * 8, 2)), dim3(kBlock), 0, ctx->stream,
                               in.key + done, in.acol[0] + done, n - done, t, amin, (int64_t *)cv.values,
                               (int64_t *)ca.values, counter);
        if (hipGetLastError() != hipSuccess) st = fail(QEH_E_HIP, "slice join launch failed");
    }
    uint64_t rows = 0;
    if (st == QEH_OK) st = read_small(ctx, &rows, counter, 8);
    if (st != QEH_OK) {
        qeh_column_release(ctx, out_probe);
        qeh_column_release(ctx, out_build);
        return st;
    }
    out_probe->length = (int64_t)rows;
    out_build->length = (int64_t)rows;
    *out_rows = (int64_t)rows;
    return QEH_OK;
}

// Fast single-key GROUP BY (k_group_agg_fast) over the full tiles, generic
// LDS-hash kernel over the ragged tail.  False when not eligible.
static bool lds_group_fast(qeh_ctx *ctx, const ColSet &cols, int64_t n, const PredPlan &pp, const GidSource &src,
                           const AggSpecs &specs, int64_t G, uint64_t *states, uint32_t *err) {
    if (std::getenv("QEH_NO_FAST")) return false;
    FastIn in;
    int nterms, nacol;
    if (!fast_cols_eligible(cols, pp, src.key_col, specs, &in, &nterms, &nacol)) return false;
    int lcap = 2048;
    while (lcap > 256 && (size_t)(1 + specs.n_slots) * lcap * 8 > 64 * 1024) lcap >>= 1;
    const size_t shm = (size_t)(1 + specs.n_slots) * lcap * 8;
    if (shm > 64 * 1024) return false;
    // big LDS tables leave room for few workgroups per CU: make them 1024 threads
    // wide so a CU still holds 16-32 waves of loads in flight
    const bool wide = shm > 40 * 1024;
    const int block = wide ? 1024 : kBlock;
    const int64_t tile_rows = (int64_t)block * kFastR;
    const int64_t n_tiles = n / tile_rows;
    if (n_tiles > 0) {
        const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(wide ? 2 : 8, (160 * 1024) / shm));
        const int grid = grid_for(ctx, n_tiles * tile_rows, (int)tile_rows, per_cu);
        const bool nt = fast_nt_mode() == 1;
#define QEH_GF(NTV, NAV, NTB)                                                                                            \
    if (wide)                                                                                                            \
        hipLaunchKernelGGL((k_group_agg_fast<NTV, NAV, NTB, 1024>), dim3(grid), dim3(1024), shm, ctx->stream, in,        \
                           pp.terms, specs, src.gt, lcap, G, n_tiles, states);                                          \
    else                                                                                                                 \
        hipLaunchKernelGGL((k_group_agg_fast<NTV, NAV, NTB>), dim3(grid), dim3(kBlock), shm, ctx->stream, in, pp.terms, \
                           specs, src.gt, lcap, G, n_tiles, states)
#define QEH_GF_NA(NTV, NTB)                       \
    if (nacol == 0) QEH_GF(NTV, 0, NTB);          \
    else if (nacol == 1) QEH_GF(NTV, 1, NTB);     \
    else QEH_GF(NTV, 2, NTB);
#define QEH_GF_NT(NTB)                            \
    if (nterms == 0) { QEH_GF_NA(0, NTB) }        \
    else if (nterms == 1) { QEH_GF_NA(1, NTB) }   \
    else { QEH_GF_NA(2, NTB) }
        if (nt) { QEH_GF_NT(true) } else { QEH_GF_NT(false) }
#undef QEH_GF_NT
#undef QEH_GF_NA
#undef QEH_GF
    }
    const int64_t done = n_tiles * tile_rows;
    if (done < n) {
        ColSet tail = cols;
        for (int i = 0; i < cols.n; ++i) tail.c[i] = advance(cols.c[i], done);
        const size_t tshm = (size_t)(1 + specs.n_slots) * src.lcap * 8;
        if (pp.mode == PM_TERMS)
            hipLaunchKernelGGL(k_groupby_lds<PM_TERMS>, dim3(1), dim3(kBlock), tshm, ctx->stream, tail, n - done, pp.terms,
                               pp.prog, src.key_col, src, specs, G, states, err);
        else
            hipLaunchKernelGGL(k_groupby_lds<PM_NONE>, dim3(1), dim3(kBlock), tshm, ctx->stream, tail, n - done, pp.terms,
                               pp.prog, src.key_col, src, specs, G, states, err);
    }
    return true;
}

constexpr int kRetryBigger = 100;  // internal: group table too small

// Run the row-aggregation kernel and finalize into owned output columns.
static int aggregate_rows(qeh_ctx *ctx, int gm, const ColSet &cols, int64_t n, const PredPlan &pp,
                          const GidSource &src, const AggSpecs &specs_in, int64_t G, const KeyCols &out_keys_src,
                          const int32_t *key_dtypes, const uint32_t *rep_row, bool drop_empty, const char *kname,
                          qeh_column *out_keys, qeh_column *out_aggs, int64_t *out_groups, SlicePre *pre = nullptr,
                          double *lanes = nullptr, uint32_t *dev_status = nullptr) {
    DevBuf states, errw;
    const int64_t Gs = std::max<int64_t>(G, 1);
    AggSpecs specs = specs_in;
    specs.shards = 1;  // state copies (shard_states): up to 64 while they stay small
    while (specs.shards < 64 && (size_t)specs.n_slots * Gs * 8 * specs.shards * 2 <= (8u << 20)) specs.shards *= 2;
    if (std::getenv("QEH_NO_SHARDS")) specs.shards = 1;
    QEH_TRY(states.alloc(ctx, (size_t)specs.shards * specs.n_slots * Gs * 8));
    // status words, read back in one go: [0] kernel error bits, [1] slice-region overflow, [2..3] groups
    QEH_TRY(errw.alloc(ctx, 16));
    QEH_HIP(hipMemsetAsync(errw.p, 0, 16, ctx->stream));
    bool ovf_pending = false;
    hipLaunchKernelGGL(k_states_init, dim3(grid_for(ctx, specs.shards * specs.n_slots * Gs, kBlock * 4, 8)), dim3(kBlock), 0,
                       ctx->stream, states.as<uint64_t>(), Gs, specs);
    const size_t lds_bytes = (size_t)specs.n_slots * Gs * 8;
    const bool lds = lds_bytes <= kLdsStateBudget;
    // fused join-aggregate when the LDS-slice pipeline does not run (or overflowed)
    auto join_fallback = [&](int grid, int per_cu) {
        if (!lds && (try_key_slices(ctx, cols, n, pp, src, specs, Gs, states.as<uint64_t>(), errw.as<uint32_t>()) == 1 ||
                     try_gid_slices(ctx, cols, n, pp, src, specs, Gs, states.as<uint64_t>(), errw.as<uint32_t>()) == 1)) {
        } else if (!(lds && try_fast_join(ctx, cols, n, pp, src, specs, Gs, states.as<uint64_t>(), errw.as<uint32_t>(),
                                          lds_bytes, per_cu)))
            launch_agg_rows<GM_JOIN>(ctx, pp.mode, lds, grid, lds ? lds_bytes : 0, cols, n, pp, src, specs, Gs,
                                     states.as<uint64_t>(), errw.as<uint32_t>());
    };
    int per_cu = lds ? (int)std::max<size_t>(1, std::min<size_t>(8, (160 * 1024) / std::max<size_t>(lds_bytes, 1))) : 8;
    per_cu = std::min(per_cu, 8);
    const int grid = grid_for(ctx, n, kAggTile, per_cu);
    if (n > 0 && G > 0) {
        // LDS partials: ~3-6 workgroups per CU; fewer per CU when the state is large (per_cu above)
        KernelTimer kt(ctx, kname);
        if (gm == GM_ZERO) launch_agg_rows<GM_ZERO>(ctx, pp.mode, lds, grid, lds ? lds_bytes : 0, cols, n, pp, src, specs, Gs, states.as<uint64_t>(), errw.as<uint32_t>());
        else if (gm == GM_JOIN) {
            const int sj = lds ? try_slice_join(ctx, cols, n, pp, src, specs, Gs, states.as<uint64_t>(), errw.as<uint32_t>(),
                                                lds_bytes, pre, errw.as<uint32_t>() + 1)
                               : 0;
            if (sj < 0) return fail(QEH_E_HIP, "slice join: overflow flag copy failed");
            ovf_pending = sj == 2;
            if (sj == 0) join_fallback(grid, per_cu);
        }
        else if (gm == GM_LDSHASH && lds_group_fast(ctx, cols, n, pp, src, specs, Gs, states.as<uint64_t>(),
                                                      errw.as<uint32_t>())) {
        }
        else if (gm == GM_LDSHASH) {
            const size_t shm = (size_t)(1 + specs.n_slots) * src.lcap * 8;
            const int pc = (int)std::max<size_t>(1, std::min<size_t>(4, (160 * 1024) / shm));
            const int g2 = grid_for(ctx, n, kAggTile, pc);
            if (pp.mode == PM_TERMS)
                hipLaunchKernelGGL(k_groupby_lds<PM_TERMS>, dim3(g2), dim3(kBlock), shm, ctx->stream, cols, n, pp.terms,
                                   pp.prog, src.key_col, src, specs, Gs, states.as<uint64_t>(), errw.as<uint32_t>());
            else if (pp.mode == PM_PROG)
                hipLaunchKernelGGL(k_groupby_lds<PM_PROG>, dim3(g2), dim3(kBlock), shm, ctx->stream, cols, n, pp.terms,
                                   pp.prog, src.key_col, src, specs, Gs, states.as<uint64_t>(), errw.as<uint32_t>());
            else
                hipLaunchKernelGGL(k_groupby_lds<PM_NONE>, dim3(g2), dim3(kBlock), shm, ctx->stream, cols, n, pp.terms,
                                   pp.prog, src.key_col, src, specs, Gs, states.as<uint64_t>(), errw.as<uint32_t>());
        }
        else launch_agg_rows<GM_GROUP>(ctx, pp.mode, lds, grid, lds ? lds_bytes : 0, cols, n, pp, src, specs, Gs, states.as<uint64_t>(), errw.as<uint32_t>());
    }
    QEH_HIP(hipGetLastError());
    // small tables with empty groups dropped: shards folded, flagged and scanned in compact() below
    const bool small = drop_empty && G > 0 && Gs <= kCompactSmallG;
    auto reduce_shards = [&]() {
        if (specs.shards > 1 && !small)
            hipLaunchKernelGGL(k_states_reduce, dim3(grid_for(ctx, specs.n_slots * Gs, kBlock, 8)), dim3(kBlock), 0,
                               ctx->stream, states.as<uint64_t>(), Gs, specs);
    };
    reduce_shards();
    if (gm == GM_LDSHASH) {  // table overflow: the caller regrows and reruns
        uint32_t of = 0;
        QEH_TRY(read_small(ctx, &of, src.gt.overflow, 4));
        if (of) return kRetryBigger;
    }

    if (lanes) {
        // dense f64 lanes instead of compacted output columns (the distributed final stage sums them
        // over the ranks): one host round trip for the status words, none for outputs
        auto emit = [&](const uint32_t *status) -> int {
            const int64_t ne = std::max<int64_t>((1 + specs.n) * G, 1);
            hipLaunchKernelGGL(k_states_lanes, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, ctx->stream,
                               states.as<uint64_t>(), Gs, G, specs, lanes, status);
            return hipGetLastError() == hipSuccess ? QEH_OK : fail(QEH_E_HIP, "aggregate: lanes launch failed");
        };
        if (dev_status) {  // the caller reads the status later (and recovers from an overflow)
            QEH_TRY(emit(errw.as<uint32_t>()));  // + the status lane
            QEH_HIP(hipMemcpyAsync(dev_status, errw.p, 16, hipMemcpyDeviceToDevice, ctx->stream));
            *out_groups = G;
            return QEH_OK;
        }
        if (G > 0) QEH_TRY(emit(nullptr));
        uint32_t stw[4];
        QEH_TRY(read_small(ctx, stw, errw.p, 16));
        if (ovf_pending && stw[1]) {
            hipLaunchKernelGGL(k_states_init, dim3(grid_for(ctx, specs.shards * specs.n_slots * Gs, kBlock * 4, 8)), dim3(kBlock),
                               0, ctx->stream, states.as<uint64_t>(), Gs, specs);
            QEH_HIP(hipMemsetAsync(errw.p, 0, 16, ctx->stream));
            {
                KernelTimer kt(ctx, kname);
                join_fallback(grid, per_cu);
            }
            QEH_HIP(hipGetLastError());
            if (G > 0) QEH_TRY(emit(nullptr));
            QEH_TRY(read_small(ctx, stw, errw.p, 16));
        }
        QEH_TRY(kernel_error_status(stw[0], "aggregate"));
        *out_groups = G;
        return QEH_OK;
    }

    // compact non-empty groups; the group count lands in the status words
    DevBuf flags, pos;
    uint64_t out_n = (uint64_t)G;
    const uint64_t *posp = nullptr;
    if (drop_empty && G > 0) {
        QEH_TRY(flags.alloc(ctx, Gs * 4));
        QEH_TRY(pos.alloc(ctx, Gs * 8));
        posp = pos.as<uint64_t>();
    }
    auto compact = [&]() -> int {
        if (!posp) return QEH_OK;
        if (small) {
            AggSpecs cs = specs;
            if (specs.shards > 1 && !std::getenv("QEH_FOLD_ONE_WG")) {
                const int64_t words = (int64_t)specs.n_slots * Gs;
                hipLaunchKernelGGL(k_states_fold, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, ctx->stream,
                                   states.as<uint64_t>(), Gs, specs);
                cs.shards = 1;  // folded: the compact kernel only flags and scans
            }
            hipLaunchKernelGGL(k_states_compact_small, dim3(1), dim3(1024), 0, ctx->stream, states.as<uint64_t>(), Gs, G,
                               cs, pos.as<uint64_t>(), (uint64_t *)(errw.as<uint32_t>() + 2));
            return hipGetLastError() == hipSuccess ? QEH_OK : fail(QEH_E_HIP, "aggregate: compact launch failed");
        }
        hipLaunchKernelGGL(k_group_nonempty, dim3(grid_for(ctx, Gs, kBlock, 8)), dim3(kBlock), 0, ctx->stream,
                           states.as<uint64_t>(), Gs, flags.as<uint32_t>());
        return exclusive_scan_u32_dev(ctx, flags.as<uint32_t>(), pos.as<uint64_t>(), G, (uint64_t *)(errw.as<uint32_t>() + 2));
    };
    QEH_TRY(compact());

    OutCols oc{};
    const int nk = out_keys_src.n;
    int made = 0;
    auto cleanup = [&]() {
        for (int i = 0; i < made; ++i) {
            qeh_column *c = i < nk ? &out_keys[i] : &out_aggs[i - nk];
            qeh_column_release(ctx, c);
        }
        made = 0;
    };
    // output columns with room for `rows` groups (their length is set once the count is known)
    auto make_outputs = [&](uint64_t rows) -> int {
        for (int i = 0; i < nk + specs.n; ++i) {
            qeh_column *c = i < nk ? &out_keys[i] : &out_aggs[i - nk];
            int dt;
            bool nullable;
            if (i < nk) {
                dt = key_dtypes[i];
                nullable = out_keys_src.c[i].validity != nullptr;
            } else {
                const AggSpec &sp = specs.a[i - nk];
                dt = agg_output_type(sp.func, sp.in_type);
                nullable = sp.func != QEH_AGG_COUNT;
            }
            int s = alloc_column(ctx, dt, (int64_t)rows, nullable, c);
            if (s != QEH_OK) {
                cleanup();
                return s;
            }
            ++made;
            if (nullable) QEH_HIP(hipMemsetAsync(c->validity, 0, ((rows + 63) / 64) * 8, ctx->stream));
            if (dt == QEH_DT_BOOL) QEH_HIP(hipMemsetAsync(c->values, 0, ((rows + 63) / 64) * 8, ctx->stream));
            oc.c[i].values = c->values;
            oc.c[i].validity = (uint32_t *)c->validity;
            oc.c[i].dtype = dt;
        }
        return QEH_OK;
    };
    auto finalize = [&]() -> int {
        KernelTimer kt(ctx, "aggregate_finalize");
        hipLaunchKernelGGL(k_finalize, dim3(grid_for(ctx, Gs, kBlock, 8)), dim3(kBlock), 0, ctx->stream,
                           states.as<uint64_t>(), Gs, posp, out_keys_src, rep_row, specs, oc);
        return hipGetLastError() == hipSuccess ? QEH_OK : fail(QEH_E_HIP, "aggregate: finalize launch failed");
    };
    uint32_t stw[4];
    // Small group counts: the outputs are allocated for all G groups and finalized before the group
    // count is known (k_finalize writes every non-empty group at its compacted position), so the
    // status words are read once, after the last kernel -- one host round trip per call instead of two.
    const bool early = G > 0 && Gs <= (1 << 20) && !std::getenv("QEH_FINALIZE_LATE");
    if (early) {
        QEH_TRY(make_outputs((uint64_t)Gs));
        int s = finalize();
        if (s == QEH_OK) s = read_small(ctx, stw, errw.p, 16);  // syncs: the finalize has run
        if (s != QEH_OK || (ovf_pending && stw[1]) || stw[0]) cleanup();
        QEH_TRY(s);
    } else {
        QEH_TRY(read_small(ctx, stw, errw.p, 16));  // one host round trip: error bits, overflow, group count
    }
    if (ovf_pending && stw[1]) {
        // a slice region overflowed (probe keys skewed onto few slices): the single fused pass instead
        hipLaunchKernelGGL(k_states_init, dim3(grid_for(ctx, specs.shards * specs.n_slots * Gs, kBlock * 4, 8)), dim3(kBlock),
                           0, ctx->stream, states.as<uint64_t>(), Gs, specs);
        QEH_HIP(hipMemsetAsync(errw.p, 0, 16, ctx->stream));
        {
            KernelTimer kt(ctx, kname);
            join_fallback(grid, per_cu);
        }
        QEH_HIP(hipGetLastError());
        reduce_shards();
        QEH_TRY(compact());
        QEH_TRY(read_small(ctx, stw, errw.p, 16));
    }
    QEH_TRY(kernel_error_status(stw[0], "aggregate"));
    if (posp) out_n = (uint64_t)stw[2] | ((uint64_t)stw[3] << 32);
    if (made == 0) {  // not finalized early (large G, or re-run after an overflow)
        QEH_TRY(make_outputs(out_n));
        if (G > 0 && out_n > 0) {
            const int s = finalize();
            if (s != QEH_OK) cleanup();
            QEH_TRY(s);
        }
        QEH_HIP(hipStreamSynchronize(ctx->stream));
    }
    for (int i = 0; i < nk + specs.n; ++i) {
        qeh_column *c = i < nk ? &out_keys[i] : &out_aggs[i - nk];
        c->length = (int64_t)out_n;
        c->null_count = c->validity ? -1 : 0;
    }
    *out_groups = (int64_t)out_n;
    return QEH_OK;
}

int hash_aggregate_filtered(qeh_ctx *ctx, const qeh_column *keys, int n_keys, const qeh_column *agg_inputs,
                            int n_inputs, const qeh_agg *aggs, int n_aggs, const qeh_column *pred_cols,
                            int n_pred_cols, const qeh_expr *predicate, int64_t input_batches,
                            qeh_column *out_keys, qeh_column *out_aggs, int64_t *out_groups);

// More aggregates than one kernel carries (kMaxAggs): run the operator once per
// chunk of aggregates.  Group order differs between runs (slot races), so every
// chunk's output is put in key order (the radix sort; keys are unique per group)
// and the chunks then line up row for row.
static int aggregate_chunked(qeh_ctx *ctx, const qeh_column *keys, int n_keys, const qeh_column *agg_inputs,
                             int n_inputs, const qeh_agg *aggs, int n_aggs, const qeh_column *pred_cols,
                             int n_pred_cols, const qeh_expr *predicate, int64_t input_batches,
                             qeh_column *out_keys, qeh_column *out_aggs, int64_t *out_groups) {
    std::vector<qeh_column> made;  // everything produced so far, released on error
    auto release_all = [&]() {
        for (auto &c : made) qeh_column_release(ctx, &c);
    };
    std::vector<qeh_column> ck(n_keys);
    std::vector<int8_t> asc(n_keys, 1);
    int64_t groups = -1;
    for (int a0 = 0; a0 < n_aggs; a0 += kMaxAggs) {
        const int na = std::min(kMaxAggs, n_aggs - a0);
        int64_t g = 0;
        int s = hash_aggregate_filtered(ctx, keys, n_keys, agg_inputs, n_inputs, aggs + a0, na, pred_cols,
                                        n_pred_cols, predicate, input_batches, ck.data(), out_aggs + a0, &g);
        if (s != QEH_OK) {
            release_all();
            return s;
        }
        if (groups >= 0 && g != groups) {
            for (int i = 0; i < n_keys; ++i) qeh_column_release(ctx, &ck[i]);
            for (int i = 0; i < na; ++i) qeh_column_release(ctx, &out_aggs[a0 + i]);
            release_all();
            return fail(QEH_E_INTERNAL, "aggregate chunks disagree on the group count");
        }
        groups = g;
        if (n_keys > 0 && g > 1) {
            qeh_column perm{};
            s = qeh_sort_indices(ctx, ck.data(), n_keys, asc.data(), &perm);
            for (int i = 0; s == QEH_OK && i < n_keys + na; ++i) {
                qeh_column *c = i < n_keys ? &ck[i] : &out_aggs[a0 + i - n_keys];
                qeh_column t{};
                s = qeh_take(ctx, c, &perm, &t);
                qeh_column_release(ctx, c);
                *c = t;
            }
            qeh_column_release(ctx, &perm);
            if (s != QEH_OK) {
                for (int i = 0; i < n_keys; ++i) qeh_column_release(ctx, &ck[i]);
                for (int i = 0; i < na; ++i) qeh_column_release(ctx, &out_aggs[a0 + i]);
                release_all();
                return s;
            }
        }
        for (int i = 0; i < n_keys; ++i) {
            if (a0 == 0) out_keys[i] = ck[i], made.push_back(ck[i]);
            else qeh_column_release(ctx, &ck[i]);
        }
        for (int i = 0; i < na; ++i) made.push_back(out_aggs[a0 + i]);
    }
    *out_groups = groups;
    return QEH_OK;
}

// Internal entry shared by qeh_hash_aggregate and the executor's fused
// Aggregate(Filter(..)) path: `cols` = key columns then aggregate inputs.
int hash_aggregate_filtered(qeh_ctx *ctx, const qeh_column *keys, int n_keys, const qeh_column *agg_inputs,
                            int n_inputs, const qeh_agg *aggs, int n_aggs, const qeh_column *pred_cols,
                            int n_pred_cols, const qeh_expr *predicate, int64_t input_batches,
                            qeh_column *out_keys, qeh_column *out_aggs, int64_t *out_groups) {
    if (!out_groups) return fail(QEH_E_INVALID, "qeh_hash_aggregate: out_groups is NULL");
    *out_groups = 0;
    if (n_aggs == 0) return QEH_OK;  // executor.rs:163-165: no aggregates -> no batches
    if (n_aggs > kMaxAggs)
        return aggregate_chunked(ctx, keys, n_keys, agg_inputs, n_inputs, aggs, n_aggs, pred_cols, n_pred_cols,
                                 predicate, input_batches, out_keys, out_aggs, out_groups);
    int64_t n = -1;
    auto take_len = [&](const qeh_column &c) -> int {
        if (n < 0) n = c.length;
        else if (c.length != n) return fail(QEH_E_INVALID, "aggregate columns have different lengths");
        return QEH_OK;
    };
    for (int i = 0; i < n_keys; ++i) QEH_TRY(take_len(keys[i]));
    for (int i = 0; i < n_inputs; ++i) QEH_TRY(take_len(agg_inputs[i]));
    for (int i = 0; i < n_pred_cols; ++i) QEH_TRY(take_len(pred_cols[i]));
    if (n < 0) n = 0;
    // kernel ColSet = predicate columns, then aggregate inputs (keys are read through KeyCols);
    // when the predicate reads the aggregate inputs themselves they are passed once
    const bool shared_cols = pred_cols == agg_inputs && n_pred_cols == n_inputs;
    std::vector<qeh_column> all;
    if (!shared_cols)
        for (int i = 0; i < n_pred_cols; ++i) all.push_back(pred_cols[i]);
    std::vector<int> idx(n_inputs);
    for (int i = 0; i < n_inputs; ++i) {
        idx[i] = (int)all.size();
        all.push_back(agg_inputs[i]);
    }
    ColSet cols;
    QEH_TRY(make_colset(all.data(), (int)all.size(), &cols));
    std::vector<int32_t> dts(all.size());
    for (size_t i = 0; i < all.size(); ++i) dts[i] = all[i].dtype;
    PredPlan pp;
    QEH_TRY(plan_predicate(predicate, dts.data(), n_pred_cols, &pp));
    AggSpecs specs;
    QEH_TRY(plan_aggs(aggs, n_aggs, agg_inputs, n_inputs, idx.data(), &specs));
    DeviceGuard dg(ctx->device);
    GidSource src{};
    std::vector<int32_t> kd(n_keys);
    for (int i = 0; i < n_keys; ++i) kd[i] = keys[i].dtype;
    if (n_keys == 0) {
        if (input_batches == 0) return QEH_OK;  // executor.rs:178-186: no batches -> no row
        KeyCols none{};
        return aggregate_rows(ctx, GM_ZERO, cols, n, pp, src, specs, 1, none, nullptr, nullptr, false,
                              "aggregate_rows", out_keys, out_aggs, out_groups);
    }
    const int kd0 = keys[0].dtype;
    if (n_keys == 1 && kd0 != QEH_DT_UTF8 && !std::getenv("QEH_NO_LDS_GROUPBY")) {
        // single key: one pass, LDS hash table per workgroup, HBM table for the merge
        uint64_t gcap = 1ull << 16;
        while (gcap < (uint64_t)(n / 16) && gcap < (1ull << 22)) gcap <<= 1;
        ColSet cols2;
        std::vector<qeh_column> all2 = all;
        all2.push_back(keys[0]);
        QEH_TRY(make_colset(all2.data(), (int)all2.size(), &cols2));
        for (;;) {
            const int64_t G = (int64_t)gcap + 2;
            DevBuf gkeys, ovf, iota, gvalid;
            QEH_TRY(gkeys.alloc(ctx, (size_t)G * 8));
            QEH_TRY(ovf.alloc(ctx, 8));
            QEH_TRY(iota.alloc(ctx, (size_t)G * 4));
            QEH_TRY(gvalid.alloc(ctx, (size_t)((G + 63) / 64) * 8));
            QEH_HIP(hipMemsetAsync(ovf.p, 0, 8, ctx->stream));
            const int gg = grid_for(ctx, G, kBlock * 8, 8);
            hipLaunchKernelGGL(k_fill_i64, dim3(gg), dim3(kBlock), 0, ctx->stream, gkeys.as<int64_t>(), (int64_t)gcap, kEmptyKey);
            const int64_t tail[2] = {0, kEmptyKey};
            QEH_HIP(hipMemcpyAsync(gkeys.as<int64_t>() + gcap, tail, 16, hipMemcpyHostToDevice, ctx->stream));
            hipLaunchKernelGGL(k_iota, dim3(gg), dim3(kBlock), 0, ctx->stream, iota.as<uint32_t>(), G);
            QEH_HIP(hipMemsetAsync(gvalid.p, 0xFF, (size_t)((G + 63) / 64) * 8, ctx->stream));
            uint8_t nb = 0;  // clear the NULL group's validity bit (bit gcap)
            uint8_t byte = (uint8_t)~(1u << (gcap & 7));
            (void)nb;
            QEH_HIP(hipMemcpyAsync(gvalid.as<uint8_t>() + (gcap >> 3), &byte, 1, hipMemcpyHostToDevice, ctx->stream));
            QEH_HIP(hipStreamSynchronize(ctx->stream));  // host staging above
            GidSource ls{};
            ls.gt.keys = gkeys.as<int64_t>();
            ls.gt.mask = gcap - 1;
            ls.gt.overflow = ovf.as<uint32_t>();
            ls.key_col = (int)all.size();
            int lcap = 2048;
            while (lcap > 256 && (size_t)(1 + specs.n_slots) * lcap * 8 > 64 * 1024) lcap >>= 1;
            ls.lcap = lcap;
            KeyCols kc{};
            kc.n = 1;
            kc.c[0].values = gkeys.p;
            kc.c[0].dtype = QEH_DT_INT64;  // raw 64-bit payloads; written back as the key's dtype
            kc.c[0].validity = gvalid.as<uint8_t>();
            kc.c[0].vbit0 = 0;
            const int s = aggregate_rows(ctx, GM_LDSHASH, cols2, n, pp, ls, specs, G, kc, kd.data(), iota.as<uint32_t>(),
                                         true, "aggregate_rows", out_keys, out_aggs, out_groups);
            if (s != kRetryBigger) {
                if (s == QEH_OK && keys[0].validity == nullptr) {
                    // keys without nulls produce a never-null key column
                }
                return s;
            }
            if (gcap >= (1ull << 30)) return fail(QEH_E_OOM, "group table overflow");
            gcap <<= 4;
        }
    }
    GroupTable gt;
    QEH_TRY(build_group_table(ctx, keys, n_keys, n, &gt, nullptr));
    src.gk = gt.keys;
    src.gslots = gt.slots.as<uint32_t>();
    src.gmask = gt.cap - 1;
    src.gdense = gt.dense.as<uint64_t>();
    return aggregate_rows(ctx, GM_GROUP, cols, n, pp, src, specs, gt.groups, gt.keys, kd.data(),
                          gt.rep_row.as<uint32_t>(), true, "aggregate_rows", out_keys, out_aggs, out_groups);
}

}  // namespace qeh

using namespace qeh;

extern "C" int qeh_hash_aggregate(qeh_ctx *ctx, const qeh_column *keys, int n_keys, const qeh_column *agg_inputs,
                                  int n_inputs, const qeh_agg *aggs, int n_aggs, int64_t input_batches,
                                  qeh_column *out_keys, qeh_column *out_aggs, int64_t *out_groups) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    return hash_aggregate_filtered(ctx, keys, n_keys, agg_inputs, n_inputs, aggs, n_aggs, nullptr, 0, nullptr,
                                   input_batches, out_keys, out_aggs, out_groups);
}

extern "C" int qeh_filter_aggregate(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *predicate,
                                    const int32_t *key_idx, int n_keys, const qeh_agg *aggs, int n_aggs,
                                    int64_t input_batches, qeh_column *out_keys, qeh_column *out_aggs,
                                    int64_t *out_groups) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    if (n_keys > kMaxGroupKeys) return fail(QEH_E_UNSUPPORTED, "1..4 group keys supported on the device");
    std::vector<qeh_column> keys(n_keys);
    for (int i = 0; i < n_keys; ++i) {
        if (key_idx[i] < 0 || key_idx[i] >= n_cols) return fail(QEH_E_INVALID, "group key index out of range");
        keys[i] = cols[key_idx[i]];
    }
    return hash_aggregate_filtered(ctx, keys.data(), n_keys, cols, n_cols, aggs, n_aggs, cols, n_cols, predicate,
                                   input_batches, out_keys, out_aggs, out_groups);
}

// Phase A of the fused join-aggregate ahead of its build side: the caller knows the build key's
// and group key's [min, max, non-null count] (e.g. from a small collective over the shards) while
// the build columns are still in flight (an RCCL all-gather), so phase A streams the probe side
// meanwhile.  The next qeh_join_filter_aggregate adopts it when its probe columns, key and
// predicate are the same and the build columns it gets have exactly these ranges; otherwise the
// work is discarded.  Not launching (shape not eligible) is not an error.
extern "C" int qeh_join_filter_aggregate_prelaunch(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols,
                                                   int probe_key_idx, const qeh_expr *predicate, const qeh_agg *aggs,
                                                   int n_aggs, const int64_t *build_key_range,
                                                   const int64_t *group_key_range) {
    if (!ctx || !probe_cols || n_probe_cols < 1 || !build_key_range || !group_key_range || (n_aggs > 0 && !aggs))
        return fail(QEH_E_INVALID, "qeh_join_filter_aggregate_prelaunch: bad argument");
    if (probe_key_idx < 0 || probe_key_idx >= n_probe_cols) return fail(QEH_E_INVALID, "probe key index out of range");
    DeviceGuard dg(ctx->device);
    ctx->pending_slice.reset();
    if (n_aggs == 0) return QEH_OK;
    const int64_t n = probe_cols[0].length;
    for (int i = 0; i < n_probe_cols; ++i)
        if (probe_cols[i].length != n) return fail(QEH_E_INVALID, "probe columns have different lengths");
    ColSet cols;
    QEH_TRY(make_colset(probe_cols, n_probe_cols, &cols));
    std::vector<int32_t> dts(n_probe_cols);
    std::vector<int> idx(n_probe_cols);
    for (int i = 0; i < n_probe_cols; ++i) {
        dts[i] = probe_cols[i].dtype;
        idx[i] = i;
    }
    PredPlan pp;
    QEH_TRY(plan_predicate(predicate, dts.data(), n_probe_cols, &pp));
    AggSpecs specs;
    QEH_TRY(plan_aggs(aggs, n_aggs, probe_cols, n_probe_cols, idx.data(), &specs));
    auto p = std::make_shared<PendingSlice>();
    for (int q = 0; q < 2; ++q) {
        const int64_t *r = q ? group_key_range : build_key_range;
        p->br.mn[q] = r[0], p->br.mx[q] = r[1], p->br.cnt[q] = r[2];
    }
    QEH_TRY(slice_prelaunch_ranges(ctx, cols, n, pp, specs, probe_key_idx, p->br, &p->pre));
    if (!p->pre.launched) return QEH_OK;
    for (int i = 0; i < n_probe_cols; ++i) {
        p->vals.push_back(probe_cols[i].values);
        p->offs.push_back(probe_cols[i].offset);
        p->lens.push_back(probe_cols[i].length);
        p->dtypes.push_back(probe_cols[i].dtype);
    }
    p->key_idx = probe_key_idx;
    p->pred = PendingSlice::serialise(predicate);
    p->agg_fc = PendingSlice::agg_list(aggs, n_aggs);
    ctx->pending_slice = p;
    return QEH_OK;
}

extern "C" int qeh_join_filter_aggregate_prelaunch_stats(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols,
                                                         int probe_key_idx, const qeh_expr *predicate, const qeh_agg *aggs,
                                                         int n_aggs, const int64_t *stats, int world, int row_len) {
    if (!ctx || !probe_cols || n_probe_cols < 1 || !stats || world < 1 || row_len < 6 || (n_aggs > 0 && !aggs))
        return fail(QEH_E_INVALID, "qeh_join_filter_aggregate_prelaunch_stats: bad argument");
    if (probe_key_idx < 0 || probe_key_idx >= n_probe_cols) return fail(QEH_E_INVALID, "probe key index out of range");
    DeviceGuard dg(ctx->device);
    ctx->pending_slice.reset();
    if (n_aggs == 0 || std::getenv("QEH_NO_SLICES") || std::getenv("QEH_NO_OVERLAP") || slice_chunk_tiles() > 0) return QEH_OK;
    const int64_t n = probe_cols[0].length;
    for (int i = 0; i < n_probe_cols; ++i)
        if (probe_cols[i].length != n) return fail(QEH_E_INVALID, "probe columns have different lengths");
    if (probe_cols[probe_key_idx].dtype != QEH_DT_INT64) return QEH_OK;
    ColSet cols;
    QEH_TRY(make_colset(probe_cols, n_probe_cols, &cols));
    std::vector<int32_t> dts(n_probe_cols);
    std::vector<int> idx(n_probe_cols);
    for (int i = 0; i < n_probe_cols; ++i) {
        dts[i] = probe_cols[i].dtype;
        idx[i] = i;
    }
    PredPlan pp;
    QEH_TRY(plan_predicate(predicate, dts.data(), n_probe_cols, &pp));
    AggSpecs specs;
    QEH_TRY(plan_aggs(aggs, n_aggs, probe_cols, n_probe_cols, idx.data(), &specs));
    auto p = std::make_shared<PendingSlice>();
    SlicePlanIn pi;
    bool launched = false;
    QEH_TRY(slice_launch_dev(
        ctx, cols, n, pp, specs, probe_key_idx, &pi, &p->pre,
        [&](const SlicePlanIn &q, SlicePlan *out) {
            hipLaunchKernelGGL(k_slice_plan_stats, dim3(1), dim3(64), 0, ctx->stream, stats, world, row_len, q, out);
        },
        &launched));
    if (!launched) return QEH_OK;
    for (int i = 0; i < n_probe_cols; ++i) {
        p->vals.push_back(probe_cols[i].values);
        p->offs.push_back(probe_cols[i].offset);
        p->lens.push_back(probe_cols[i].length);
        p->dtypes.push_back(probe_cols[i].dtype);
    }
    p->key_idx = probe_key_idx;
    p->pred = PendingSlice::serialise(predicate);
    p->agg_fc = PendingSlice::agg_list(aggs, n_aggs);
    ctx->pending_slice = p;
    return QEH_OK;
}

// ---- dense partial states of a distributed broadcast join (qeh_dense_states_f64 / _take) ----
struct DenseCols {
    const void *vals[kMaxAggs];
    int32_t dt[kMaxAggs];
    int32_t n;
};

__global__ void k_dense_scatter(ColRef key, int64_t n, DenseCols dc, int64_t kmin, int64_t range,
                                double *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t o = (uint64_t)load_i64(key, i) - (uint64_t)kmin;
        if (o >= (uint64_t)range) continue;
        out[o] = 1.0;
        for (int j = 0; j < dc.n; ++j) {
            double v;
            if (dc.dt[j] == QEH_DT_FLOAT64) v = ((const double *)dc.vals[j])[i];
            else if (dc.dt[j] == QEH_DT_INT32) v = (double)((const int32_t *)dc.vals[j])[i];
            else v = (double)((const int64_t *)dc.vals[j])[i];
            out[(int64_t)(j + 1) * range + (int64_t)o] = v;
        }
    }
}

// one workgroup: the owned slots o = rank + world * q with presence > 0, in key order
__global__ __launch_bounds__(1024) void k_dense_take(const double *__restrict__ in, int64_t kmin, int64_t range, int world,
                                                     int rank, int32_t key_dt, void *__restrict__ okeys, DenseCols oc,
                                                     int64_t *__restrict__ total, int with_status = 0) {
    __shared__ uint32_t wsum[16];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t owned = range > rank ? (range - rank + world - 1) / world : 0;
    const int64_t per = (owned + 1023) / 1024, q0 = (int64_t)t * per, q1 = q0 + per < owned ? q0 + per : owned;
    uint32_t c = 0;
    for (int64_t q = q0; q < q1; ++q) c += in[rank + q * world] > 0.0;
    const uint32_t incl = wave_incl_scan(c);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t base = incl - c, all = 0;
    for (int w = 0; w < 16; ++w) {
        base += w < wave ? wsum[w] : 0u;
        all += wsum[w];
    }
    for (int64_t q = q0; q < q1; ++q) {
        const int64_t o = rank + q * world;
        if (!(in[o] > 0.0)) continue;
        const int64_t key = kmin + o;
        if (key_dt == QEH_DT_INT32) ((int32_t *)okeys)[base] = (int32_t)key;
        else ((int64_t *)okeys)[base] = key;
        for (int j = 0; j < oc.n; ++j) {
            const double v = in[(int64_t)(j + 1) * range + o];
            if (oc.dt[j] == QEH_DT_FLOAT64) ((double *)oc.vals[j])[base] = v;
            else ((int64_t *)oc.vals[j])[base] = (int64_t)v;
        }
        ++base;
    }
    if (t == 0) {
        total[0] = all;
        // the status lane after the (1 + n) * range lanes (the no-wait forms), in the same read
        if (with_status) total[1] = __builtin_bit_cast(int64_t, in[(int64_t)(1 + oc.n) * range]);
    }
}

extern "C" int qeh_dense_states_f64(qeh_ctx *ctx, const qeh_column *keys, const qeh_column *vals, int n_vals,
                                    int64_t key_min, int64_t range, double *out) {
    if (!ctx || !keys || !out || n_vals < 0 || n_vals > kMaxAggs || (n_vals > 0 && !vals) || range <= 0)
        return fail(QEH_E_INVALID, "qeh_dense_states_f64: bad argument");
    QEH_TRY(check_column(*keys, "dense state key"));
    if (keys->dtype != QEH_DT_INT64 && keys->dtype != QEH_DT_INT32) return fail(QEH_E_UNSUPPORTED, "dense state keys must be Int32 / Int64");
    if (keys->validity && keys->null_count != 0) return fail(QEH_E_UNSUPPORTED, "dense state keys must be non-null");
    DenseCols dc{};
    dc.n = n_vals;
    for (int j = 0; j < n_vals; ++j) {
        QEH_TRY(check_column(vals[j], "dense state value"));
        if (vals[j].length != keys->length) return fail(QEH_E_INVALID, "dense state columns have different lengths");
        if ((vals[j].dtype != QEH_DT_INT64 && vals[j].dtype != QEH_DT_FLOAT64 && vals[j].dtype != QEH_DT_INT32) ||
            (vals[j].validity && vals[j].null_count != 0))
            return fail(QEH_E_UNSUPPORTED, "dense state values must be non-null Int32 / Int64 / Float64");
        dc.vals[j] = (const char *)vals[j].values + (size_t)vals[j].offset * dtype_size(vals[j].dtype);
        dc.dt[j] = vals[j].dtype;
    }
    DeviceGuard dg(ctx->device);
    const int64_t n = keys->length;
    if (n > 0)
        hipLaunchKernelGGL(k_dense_scatter, dim3(grid_for(ctx, n, kBlock, 8)), dim3(kBlock), 0, ctx->stream, make_colref(*keys),
                           n, dc, key_min, range, out);
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

static int dense_states_take(qeh_ctx *ctx, const double *in, int n_vals, int64_t key_min, int64_t range, int world,
                             int rank, int32_t key_dtype, const int32_t *out_dtypes, qeh_column *out_keys,
                             qeh_column *out_vals, int64_t *out_groups, double *status) {
    if (!ctx || !in || !out_keys || !out_groups || n_vals < 0 || n_vals > kMaxAggs || (n_vals > 0 && (!out_vals || !out_dtypes)) ||
        range <= 0 || world < 1 || rank < 0 || rank >= world || (key_dtype != QEH_DT_INT64 && key_dtype != QEH_DT_INT32))
        return fail(QEH_E_INVALID, "qeh_dense_states_take: bad argument");
    for (int j = 0; j < n_vals; ++j)
        if (out_dtypes[j] != QEH_DT_INT64 && out_dtypes[j] != QEH_DT_FLOAT64)
            return fail(QEH_E_UNSUPPORTED, "dense state outputs are Int64 / Float64");
    DeviceGuard dg(ctx->device);
    *out_groups = 0;
    const int64_t cap = std::max<int64_t>((range + world - 1) / world, 1);
    QEH_TRY(alloc_column(ctx, key_dtype, cap, false, out_keys));
    DenseCols oc{};
    oc.n = n_vals;
    int made = 0, s = QEH_OK;
    for (; made < n_vals; ++made) {
        if ((s = alloc_column(ctx, out_dtypes[made], cap, false, &out_vals[made])) != QEH_OK) break;
        oc.vals[made] = out_vals[made].values;
        oc.dt[made] = out_dtypes[made];
    }
    DevBuf tot;
    if (s == QEH_OK) s = tot.alloc(ctx, 16);
    int64_t g = 0, gs[2] = {0, 0};
    if (s == QEH_OK) {
        hipLaunchKernelGGL(k_dense_take, dim3(1), dim3(1024), 0, ctx->stream, in, key_min, range, world, rank, key_dtype,
                           out_keys->values, oc, tot.as<int64_t>(), status ? 1 : 0);
        s = hipGetLastError() == hipSuccess ? read_small(ctx, gs, tot.p, status ? 16 : 8)
                                            : fail(QEH_E_HIP, "dense take launch failed");
        g = gs[0];
        if (status) *status = __builtin_bit_cast(double, gs[1]);
    }
    if (s != QEH_OK) {
        qeh_column_release(ctx, out_keys);
        for (int j = 0; j < made; ++j) qeh_column_release(ctx, &out_vals[j]);
        return s;
    }
    out_keys->length = g;
    for (int j = 0; j < n_vals; ++j) out_vals[j].length = g;
    *out_groups = g;
    return QEH_OK;
}

extern "C" int qeh_dense_states_take(qeh_ctx *ctx, const double *in, int n_vals, int64_t key_min, int64_t range, int world,
                                     int rank, int32_t key_dtype, const int32_t *out_dtypes, qeh_column *out_keys,
                                     qeh_column *out_vals, int64_t *out_groups) {
    return dense_states_take(ctx, in, n_vals, key_min, range, world, rank, key_dtype, out_dtypes, out_keys, out_vals,
                             out_groups, nullptr);
}

extern "C" int qeh_dense_states_take_status(qeh_ctx *ctx, const double *in, int n_vals, int64_t key_min, int64_t range,
                                            int world, int rank, int32_t key_dtype, const int32_t *out_dtypes,
                                            qeh_column *out_keys, qeh_column *out_vals, int64_t *out_groups,
                                            double *status) {
    if (!status) return fail(QEH_E_INVALID, "qeh_dense_states_take_status: bad argument");
    return dense_states_take(ctx, in, n_vals, key_min, range, world, rank, key_dtype, out_dtypes, out_keys, out_vals,
                             out_groups, status);
}

__global__ void k_seq_i64(int64_t *p, int64_t n, int64_t base, int as32) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (as32) ((int32_t *)p)[i] = (int32_t)(base + i);
        else p[i] = base + i;
    }
}

// The fused operator against a join table built elsewhere (the summed DIRECT u16 table of the
// table-form broadcast join, include/qeh.h): group g = entry - 1, key group_min + g.  The group
// keys are a synthesised column group_min + [0, G) with representative row g, so the aggregate and
// finalize are qeh_join_filter_aggregate's own.
static int join_filter_aggregate_table(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols, int probe_key_idx,
                                       const qeh_expr *predicate, const uint16_t *table, int64_t key_min,
                                       uint64_t key_range, int64_t group_min, int64_t n_groups, int32_t group_dtype,
                                       const qeh_agg *aggs, int n_aggs, qeh_column *out_keys, qeh_column *out_aggs,
                                       int64_t *out_groups, double *lanes, uint32_t *dev_status = nullptr) {
    if (!ctx || !out_groups || !table || key_range == 0 || key_range >= (1ull << 32) || n_groups < 1 ||
        n_groups >= 0xFFFE || (group_dtype != QEH_DT_INT64 && group_dtype != QEH_DT_INT32))
        return fail(QEH_E_INVALID, "qeh_join_filter_aggregate_table: bad argument");
    *out_groups = 0;
    if (n_aggs == 0) return QEH_OK;
    if (probe_key_idx < 0 || probe_key_idx >= n_probe_cols) return fail(QEH_E_INVALID, "probe key index out of range");
    const int64_t n = probe_cols[0].length;
    for (int i = 0; i < n_probe_cols; ++i)
        if (probe_cols[i].length != n) return fail(QEH_E_INVALID, "probe columns have different lengths");
    DeviceGuard dg(ctx->device);
    ColSet cols;
    QEH_TRY(make_colset(probe_cols, n_probe_cols, &cols));
    std::vector<int32_t> dts(n_probe_cols);
    std::vector<int> idx(n_probe_cols);
    for (int i = 0; i < n_probe_cols; ++i) {
        dts[i] = probe_cols[i].dtype;
        idx[i] = i;
    }
    PredPlan pp;
    QEH_TRY(plan_predicate(predicate, dts.data(), n_probe_cols, &pp));
    AggSpecs specs;
    QEH_TRY(plan_aggs(aggs, n_aggs, probe_cols, n_probe_cols, idx.data(), &specs));
    if (probe_cols[probe_key_idx].dtype != QEH_DT_INT64 && probe_cols[probe_key_idx].dtype != QEH_DT_INT32)
        return fail(QEH_E_UNSUPPORTED, "hash join keys must be Int32/Int64 on the device");
    SlicePre pre;
    std::shared_ptr<PendingSlice> pend = std::static_pointer_cast<PendingSlice>(ctx->pending_slice);
    ctx->pending_slice.reset();
    if (pend && pend->matches(probe_cols, n_probe_cols, probe_key_idx, predicate, aggs, n_aggs)) {
        if (pend->pre.dev_planned) QEH_TRY(resolve_dev_plan(ctx, &pend->pre, &pend->br));
        pend->take(&pre);
    }
    pend.reset();  // not adopted: waits for its phase A, frees its regions
    // (try_slice_join adopts `pre` only for this table's key range and tile count)
    DevBuf gkeys, rep;
    QEH_TRY(gkeys.alloc(ctx, (size_t)n_groups * 8));
    QEH_TRY(rep.alloc(ctx, (size_t)n_groups * 4));
    const int g = grid_for(ctx, n_groups, kBlock, 1);
    hipLaunchKernelGGL(k_seq_i64, dim3(g), dim3(kBlock), 0, ctx->stream, gkeys.as<int64_t>(), n_groups, group_min,
                       group_dtype == QEH_DT_INT32 ? 1 : 0);
    hipLaunchKernelGGL(k_iota, dim3(g), dim3(kBlock), 0, ctx->stream, rep.as<uint32_t>(), n_groups);
    QEH_HIP(hipGetLastError());
    qeh_column kc{};
    kc.dtype = group_dtype;
    kc.length = n_groups;
    kc.values = gkeys.p;
    KeyCols keys{};
    keys.n = 1;
    keys.c[0] = make_colref(kc);
    GidSource src{};
    src.jt.kind = TK_DIRECT;
    src.jt.payload16 = const_cast<uint16_t *>(table);
    src.jt.kmin = key_min;
    src.jt.kmax = (int64_t)((uint64_t)key_min + key_range - 1ull);
    src.jt.range = key_range;
    src.jt.unique = 1;
    src.key_col = probe_key_idx;
    const int32_t kd = group_dtype;
    if (lanes)
        for (int a = 0; a < specs.n; ++a)
            if (!((specs.a[a].kind == AK_SUM_F && specs.a[a].func == QEH_AGG_SUM && specs.a[a].cnt_slot == 0) ||
                  (specs.a[a].kind == AK_COUNT && specs.a[a].func == QEH_AGG_COUNT)))
                return fail(QEH_E_UNSUPPORTED, "dense lanes carry COUNT and non-null float SUM aggregates only");
    return aggregate_rows(ctx, GM_JOIN, cols, n, pp, src, specs, n_groups, keys, &kd, rep.as<uint32_t>(), true,
                          "join_filter_aggregate", out_keys, out_aggs, out_groups, &pre, lanes, dev_status);
}

extern "C" int qeh_join_filter_aggregate_table(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols,
                                               int probe_key_idx, const qeh_expr *predicate, const uint16_t *table,
                                               int64_t key_min, uint64_t key_range, int64_t group_min, int64_t n_groups,
                                               int32_t group_dtype, const qeh_agg *aggs, int n_aggs, qeh_column *out_keys,
                                               qeh_column *out_aggs, int64_t *out_groups) {
    return join_filter_aggregate_table(ctx, probe_cols, n_probe_cols, probe_key_idx, predicate, table, key_min, key_range,
                                       group_min, n_groups, group_dtype, aggs, n_aggs, out_keys, out_aggs, out_groups,
                                       nullptr);
}

extern "C" int qeh_join_filter_aggregate_table_lanes(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols,
                                                     int probe_key_idx, const qeh_expr *predicate, const uint16_t *table,
                                                     int64_t key_min, uint64_t key_range, int64_t n_groups,
                                                     const qeh_agg *aggs, int n_aggs, double *lanes) {
    if (!lanes) return fail(QEH_E_INVALID, "qeh_join_filter_aggregate_table_lanes: bad argument");
    if (n_aggs == 0) return fail(QEH_E_INVALID, "qeh_join_filter_aggregate_table_lanes: no aggregates");
    int64_t g = 0;
    return join_filter_aggregate_table(ctx, probe_cols, n_probe_cols, probe_key_idx, predicate, table, key_min, key_range,
                                       0, n_groups, QEH_DT_INT64, aggs, n_aggs, nullptr, nullptr, &g, lanes);
}

extern "C" int qeh_join_filter_aggregate_table_lanes_async(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols,
                                                           int probe_key_idx, const qeh_expr *predicate,
                                                           const uint16_t *table, int64_t key_min, uint64_t key_range,
                                                           int64_t n_groups, const qeh_agg *aggs, int n_aggs, double *lanes,
                                                           uint32_t *dev_status) {
    if (!lanes || !dev_status) return fail(QEH_E_INVALID, "qeh_join_filter_aggregate_table_lanes_async: bad argument");
    if (n_aggs == 0) return fail(QEH_E_INVALID, "qeh_join_filter_aggregate_table_lanes_async: no aggregates");
    int64_t g = 0;
    return join_filter_aggregate_table(ctx, probe_cols, n_probe_cols, probe_key_idx, predicate, table, key_min, key_range,
                                       0, n_groups, QEH_DT_INT64, aggs, n_aggs, nullptr, nullptr, &g, lanes, dev_status);
}

// ---- the fused pipeline (one bounded integer group key, unique Int64 build keys) ----------------
// Everything on the main queue, one host round trip per query (the status words after the finalize):
//   build key / group key min-max -> k_fused_plan (slice shape, group slots, status words zeroed)
//   -> states zeroed -> phase A (prologue: output group keys and the build rows grouped by slice into
//   per-(workgroup, slice) regions, 4 B each; then the probe rows with EARLY loads and the ragged tail
//   as a partial last tile) -> phase B (each slice's entries built in LDS from its build rows,
//   duplicate keys flagged) -> fold / compact / finalize.
// Returns kFusedNotEligible when the shape does not qualify (checked on the host) or the device plan,
// a region overflow or a duplicate build key rejected the run (outputs released): the caller runs
// the general path.
constexpr int kFusedNotEligible = -4;

static void launch_slice_partition_early(qeh_ctx *ctx, const FastIn &in, const PredPlan &pp, int nterms, int nacol,
                                         int64_t n_tiles, int64_t tail_rows, int grid, const SliceRegions &rg,
                                         const SlicePlan *dplan, const FusedPro &fp) {
    const bool nt = fast_nt_mode() == 1;
    KernelTimer kta(ctx, "slice_partition");
    const HashTable t{};
#define QEH_SE(NTV, NAV, NTB)                                                                                            \
    hipLaunchKernelGGL((k_slice_partition<NTV, NAV, NTB, 0, true>), dim3(grid), dim3(kSliceBlock), 0, ctx->stream, in,   \
                       pp.terms, 0, 0, n_tiles, rg, t, dplan, tail_rows, fp)
#define QEH_SE_NA(NTV, NTB)                      \
    if (nacol == 0) { QEH_SE(NTV, 0, NTB); }      \
    else if (nacol == 1) { QEH_SE(NTV, 1, NTB); } \
    else { QEH_SE(NTV, 2, NTB); }
#define QEH_SE_NT(NTB)                          \
    if (nterms == 0) { QEH_SE_NA(0, NTB) }      \
    else if (nterms == 1) { QEH_SE_NA(1, NTB) } \
    else { QEH_SE_NA(2, NTB) }
    if (nt) { QEH_SE_NT(true) } else { QEH_SE_NT(false) }
#undef QEH_SE_NT
#undef QEH_SE_NA
#undef QEH_SE
}

static int fused_join_filter_aggregate(qeh_ctx *ctx, const ColSet &cols, int64_t n, const PredPlan &pp,
                                       const AggSpecs &specs_in, int key_col, const qeh_column &bk, const qeh_column &gk,
                                       qeh_column *out_keys, qeh_column *out_aggs, int64_t *out_groups) {
    if (std::getenv("QEH_NO_FUSED") || std::getenv("QEH_NO_SLICES")) return kFusedNotEligible;
    const size_t timing_mark = ctx->timing_pending.size();
    const bool bk_nulls = bk.validity && bk.null_count != 0, gk_nulls = gk.validity && gk.null_count != 0;
    if (bk.dtype != QEH_DT_INT64 || bk_nulls || (gk.dtype != QEH_DT_INT64 && gk.dtype != QEH_DT_INT32) || gk_nulls)
        return kFusedNotEligible;
    const int64_t nd = bk.length;
    if (nd <= 0 || nd >= ((int64_t)1 << 32) || gk.length != nd) return kFusedNotEligible;
    FastIn in;
    int nterms, nacol;
    if (!fast_cols_eligible(cols, pp, key_col, specs_in, &in, &nterms, &nacol) || nacol > 2 ||
        (nacol == 2 && std::getenv("QEH_NO_FUSED_AGG2")))
        return kFusedNotEligible;
    // phase A: one 1024-thread workgroup per CU (two aggregate columns: 18-B items, half tiles)
    const int64_t tile_rows = nacol == 2 ? (int64_t)SliceShape<2, true>::TILE
                                         : (nacol ? SliceShape<1, true>::TILE : SliceShape<0, true>::TILE);
    const int chunk = nacol == 2 ? SliceShape<2, true>::CH : (nacol ? SliceShape<1, true>::CH : SliceShape<0, true>::CH);
    const int64_t n_tiles = n / tile_rows, tail = n - n_tiles * tile_rows;
    if (n_tiles == 0) return kFusedNotEligible;
    AggSpecs specs = specs_in;
    const int64_t g_cap = std::min<int64_t>(kSliceStateWords / std::max(specs.n_slots, 1), 0xFFFE);
    const int64_t Gs = g_cap;  // states and outputs for every possible slot; empty slots are dropped
    // one copy of the states: phase B folds each slice's LDS states into them once per workgroup, so
    // same-address contention is low and the shard fold launch is not worth its place in the chain
    // (A/B on one box, profiles/r04/ab_early_shape.txt); QEH_FUSED_SHARDS=1 restores the copies
    specs.shards = 1;
    if (std::getenv("QEH_FUSED_SHARDS"))
        while (specs.shards < 64 && (size_t)specs.n_slots * Gs * 8 * specs.shards * 2 <= (8u << 20)) specs.shards *= 2;
    const int64_t n_all = n_tiles + (tail ? 1 : 0);
    const int grid = (int)std::min<int64_t>({(int64_t)ctx->props.multiProcessorCount, n_all,
                                             (int64_t)kMaxSliceGrid});
    const uint64_t tiles_per_wg = (uint64_t)((n_all + grid - 1) / grid);

    DevBuf mm, plan, ditems, dcount, kbuf, vbuf, vbuf2, cbuf, states, errw, gkeys, rep;
    SlicePlanIn pi{};
    pi.min_bytes = 6ull << 20;
    if (const char *e = std::getenv("QEH_SLICE_MIN_BYTES")) pi.min_bytes = std::strtoull(e, nullptr, 10);
    pi.grid = grid;
    pi.n_slots = specs.n_slots;
    pi.sparse_ok = direct_sparse_allowed() ? 1 : 0;
    pi.chunk = chunk;
    pi.alloc_items = tiles_per_wg * grid * (uint64_t)tile_rows * 5 / 4 + (uint64_t)grid * kSliceMaxF * (256 + 2 * chunk);
    // build rows: uniform keys over the slices, +25 %, and per-region slack
    const uint64_t dim_items = (uint64_t)nd * 5 / 4 + (uint64_t)grid * kSliceMaxF * 64;
    if (dim_items >= (1ull << 32)) return kFusedNotEligible;  // phase B's region bases are 32-bit
    const uint64_t nreg_max = (uint64_t)grid * kSliceMaxF;
    QEH_TRY(mm.alloc(ctx, sizeof(MinMax) * 2 * (size_t)minmax_partials_max_blocks(ctx) + 16));  // the partials
    QEH_TRY(plan.alloc(ctx, sizeof(FusedPlan)));
    QEH_TRY(ditems.alloc(ctx, dim_items * 4 + 64));
    QEH_TRY(dcount.alloc(ctx, nreg_max * 4 + 64));
    QEH_TRY(kbuf.alloc(ctx, pi.alloc_items * 2 + 64));
    if (nacol) QEH_TRY(vbuf.alloc(ctx, pi.alloc_items * 8 + 64));
    if (nacol > 1) QEH_TRY(vbuf2.alloc(ctx, pi.alloc_items * 8 + 64));
    QEH_TRY(cbuf.alloc(ctx, nreg_max * 4 + 64));
    QEH_TRY(states.alloc(ctx, (size_t)specs.shards * specs.n_slots * Gs * 8));
    // status words (zeroed by k_fused_plan): [0] kernel error bits, [1] region overflow, [2..3] groups,
    // [4] duplicate build key, [5] the device plan's verdict
    QEH_TRY(errw.alloc(ctx, 32));
    QEH_TRY(gkeys.alloc(ctx, (size_t)Gs * 8));
    QEH_TRY(rep.alloc(ctx, (size_t)Gs * 4));
    uint32_t *st = errw.as<uint32_t>();
    SliceRegions rg{};
    rg.key = kbuf.as<uint16_t>();
    rg.val = nacol ? vbuf.as<int64_t>() : nullptr;
    rg.val2 = nacol > 1 ? vbuf2.as<int64_t>() : nullptr;
    rg.count = cbuf.as<uint32_t>();
    rg.overflow = st + 1;
    FusedPlan *dplan = plan.as<FusedPlan>();
    {
        KernelTimer kt(ctx, "fused_build");
        const qeh_column both[2] = {bk, gk};
        int nb = 0;
        QEH_TRY(columns_minmax_partials(ctx, both, 2, mm.as<MinMax>(), &nb));
        const int gp = (int)std::max<int64_t>(1, std::min<int64_t>(ctx->props.multiProcessorCount,
                                                                   (specs.shards * specs.n_slots * Gs + 4095) / 4096));
        hipLaunchKernelGGL(k_fused_plan, dim3(gp), dim3(1024), 0, ctx->stream, mm.as<MinMax>(), nb, pi, g_cap, nd, dim_items,
                           dplan, st, states.as<uint64_t>(), Gs, specs);
    }
    QEH_HIP(hipGetLastError());
    FusedPro fp{};
    fp.dk = (const int64_t *)bk.values + bk.offset;
    fp.dg = make_colref(gk);
    fp.nd = nd;
    fp.ditems = ditems.as<uint32_t>();
    fp.dcount = dcount.as<uint32_t>();
    fp.status = st;
    fp.gkeys = gkeys.p;
    fp.rep = rep.as<uint32_t>();
    fp.G = Gs;
    fp.as32 = gk.dtype == QEH_DT_INT32 ? 1 : 0;
    fp.plan = dplan;
    launch_slice_partition_early(ctx, in, pp, nterms, nacol, n_tiles, tail, grid, rg, &dplan->sp, fp);
    {
        KernelTimer ktb(ctx, "slice_probe");
        DimSlices dim{ditems.as<uint32_t>(), dcount.as<uint32_t>(), st + 4, dplan};
        const bool pf = slice_probe_prefetch();
        const int gridB = ctx->props.multiProcessorCount;
        const HashTable t{};
        // items loaded two per lane (PV, default; QEH_FUSED_PV=0: one per lane)
        static const bool pv = !(std::getenv("QEH_FUSED_PV") && std::atoi(std::getenv("QEH_FUSED_PV")) == 0);
#define QEH_SD(NAV, PFV, PVV)                                                                                              \
    hipLaunchKernelGGL((k_slice_probe<NAV, false, PFV, PVV, true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream, rg,   \
                       grid, 0, t, in, specs, Gs, states.as<uint64_t>(), dim)
        if (nacol == 0) {
            if (pf) QEH_SD(0, true, false);
            else QEH_SD(0, false, false);
        } else if (nacol == 2) {  // (item pairs carry one value column: two columns load per item)
            if (pf) QEH_SD(2, true, false);
            else QEH_SD(2, false, false);
        } else if (pv) {
            if (pf) QEH_SD(1, true, true);
            else QEH_SD(1, false, true);
        } else {
            if (pf) QEH_SD(1, true, false);
            else QEH_SD(1, false, false);
        }
#undef QEH_SD
    }
    QEH_HIP(hipGetLastError());
    // fold the shard copies (when there are several), then one workgroup compacts, writes the outputs
    // and the group count (st[2..3])
    if (specs.shards > 1) {
        const int64_t words = (int64_t)specs.n_slots * Gs;
        hipLaunchKernelGGL(k_states_fold, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, ctx->stream,
                           states.as<uint64_t>(), Gs, specs);
    }
    QEH_HIP(hipGetLastError());
    qeh_column kc{};
    kc.dtype = gk.dtype;
    kc.length = Gs;
    kc.values = gkeys.p;
    KeyCols keys{};
    keys.n = 1;
    keys.c[0] = make_colref(kc);
    OutCols oc{};
    int made = 0;
    auto cleanup = [&]() {
        for (int i = 0; i < made; ++i) qeh_column_release(ctx, i == 0 ? &out_keys[0] : &out_aggs[i - 1]);
        made = 0;
    };
    for (int i = 0; i < 1 + specs.n; ++i) {
        qeh_column *c = i == 0 ? &out_keys[0] : &out_aggs[i - 1];
        int dt;
        bool nullable;
        if (i == 0) {
            dt = gk.dtype;
            nullable = false;
        } else {
            const AggSpec &sp = specs.a[i - 1];
            dt = agg_output_type(sp.func, sp.in_type);
            nullable = sp.func != QEH_AGG_COUNT;
        }
        const int s = alloc_column(ctx, dt, Gs, nullable, c);
        if (s != QEH_OK) {
            cleanup();
            return s;
        }
        ++made;
        oc.c[i].values = c->values;
        oc.c[i].validity = (uint32_t *)c->validity;
        oc.c[i].dtype = dt;
    }
    {
        KernelTimer kt(ctx, "aggregate_finalize");
        hipLaunchKernelGGL(k_fused_finish, dim3(1), dim3(1024), 0, ctx->stream, states.as<uint64_t>(), Gs, keys,
                           rep.as<uint32_t>(), specs, oc, (uint64_t *)(st + 2));
    }
    uint32_t sw[8];
    int s = hipGetLastError() == hipSuccess ? QEH_OK : fail(QEH_E_HIP, "fused join-aggregate: launch failed");
    if (s == QEH_OK) s = read_small(ctx, sw, errw.p, 32);  // the one host round trip of the query
    if (s == QEH_OK && !sw[0] && (!sw[5] || sw[1] || sw[4])) s = kFusedNotEligible;  // plan, overflow, duplicates
    if (s == kFusedNotEligible && !sw[5]) {
        // the device plan declined: every kernel of this call returned at once, so its timing records
        // are not a query's phases (the general path that follows records its own)
        for (size_t i = timing_mark; i < ctx->timing_pending.size(); ++i) ctx->timing_pending[i].name += "_declined";
    }
    if (s == QEH_OK) s = kernel_error_status(sw[0], "aggregate");
    if (s != QEH_OK) {
        cleanup();
        return s;
    }
    const int64_t out_n = (int64_t)((uint64_t)sw[2] | ((uint64_t)sw[3] << 32));
    for (int i = 0; i < 1 + specs.n; ++i) {
        qeh_column *c = i == 0 ? &out_keys[0] : &out_aggs[i - 1];
        c->length = out_n;
        c->null_count = c->validity ? -1 : 0;
    }
    *out_groups = out_n;
    return QEH_OK;
}

// ---- the items form of the distributed broadcast join (BASELINE metric at N > 1) ---------------
// The fused pipeline with the build side sharded over the ranks: every rank groups ITS dimension rows by
// slice into 4-B items (key offset << 16 | group slot + 1) -- what phase A's prologue does with the
// whole dimension at N = 1 -- the caller all-gathers the item regions (4 B per dimension row over the
// wire, one region per rank and slice), and phase B builds each slice's LDS entries from the regions of
// every rank.  Phase A needs only the job-wide key range, which the plan takes from the gathered stats
// rows on the device (qeh_broadcast_stats), so it is launched before the host has read them:
//   qeh_fused_items_begin  plan + states + phase A (the EARLY kernel, no build rows in its prologue)
//   qeh_fused_items_build  this rank's build rows grouped by slice into caller buffers
//   (caller: all-gather of the items and counts)
//   qeh_fused_items_finish phase B over the gathered regions, then the dense final stage's lanes
// It replaces the table form's 2-B-per-key table insert, its all-reduce and the table's HBM reads in
// phase B; phase A is the fused pipeline's kernel (its loads issued a tile ahead) instead of the
// prelaunched kernel that keeps room for a build beside it.  A duplicate key (on any rank), a region
// overflow or a declined plan shows in the status lane of the lanes (every rank sees every rank's).

// The fused plan from the gathered stats rows ([rows, key min, max, group key min, max, has-bitmap,
// ...] per rank); states initialised, status words zeroed ([5] = the plan's verdict).
__global__ __launch_bounds__(1024) void k_fused_plan_stats(const int64_t *__restrict__ M, int world, int row_len,
                                                           SlicePlanIn pi, int64_t g_cap, FusedPlan *out,
                                                           uint32_t *__restrict__ st, uint64_t *__restrict__ states,
                                                           int64_t G, AggSpecs specs) {
    const int64_t words = (int64_t)specs.shards * specs.n_slots * G;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t slot = (i / G) % specs.n_slots;
        uint64_t v = 0;
        for (int a = 0; a < specs.n; ++a)
            if (specs.a[a].val_slot == slot) v = (uint64_t)agg_init_value(specs.a[a].kind);
        states[i] = v;
    }
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    int64_t tot = 0, kmn = INT64_MAX, kmx = INT64_MIN, gmn = INT64_MAX, gmx = INT64_MIN, bitmap = 0;
    for (int r = 0; r < world; ++r) {
        const int64_t *m = M + (int64_t)r * row_len;
        bitmap |= m[5];
        if (m[0] <= 0) continue;
        tot += m[0];
        kmn = m[1] < kmn ? m[1] : kmn, kmx = m[2] > kmx ? m[2] : kmx;
        gmn = m[3] < gmn ? m[3] : gmn, gmx = m[4] > gmx ? m[4] : gmx;
    }
    FusedPlan p{};
    p.sp = plan_slices(pi, kmn, kmx, tot, gmn, gmx, tot);
    const bool live = !bitmap && tot > 0 && kmn <= kmx && gmn <= gmx;
    p.gmin = gmn;
    p.ngroups = live ? (int64_t)((uint64_t)gmx - (uint64_t)gmn + 1ull) : 0;
    p.dcap = 0;  // the build regions' capacity comes with the gathered items
    p.sp.ok = p.sp.ok && live && p.ngroups >= 1 && p.ngroups <= g_cap && p.ngroups < 0xFFFF;
    *out = p;
    for (int i = 0; i < 8; ++i) st[i] = 0u;
    st[5] = p.sp.ok ? 1u : 0u;
}

// This rank's build rows grouped by slice, no global atomics (reserving ranges in one count word per
// slice from every workgroup serialised on those words) and no compaction: workgroup w takes rows
// [w * per, (w + 1) * per) (per = ceil(rows / gridDim.x)), counts them per slice in LDS, and writes them
// slice-major into its own span items[w * span ..], each slice's run starting at a multiple of 4 (phase
// B's 16-B loads) -- item = (key - kmin) mod 2^16 << 16 | (group key - gmin) + 1 -- with
// offs[w * 2 (S + 1) + b] = run start and offs[w * 2 (S + 1) + S + 1 + b] = run rows.  span >= per + 4 S.
// A key or group key outside the plan's ranges sets st[1] (the caller falls back).
__device__ __forceinline__ uint32_t dim_item(const FusedPlan &pl, int64_t k, int64_t g, uint32_t &it) {
    const uint64_t o = (uint64_t)k - (uint64_t)pl.sp.kmin;
    const uint64_t gs = (uint64_t)g - (uint64_t)pl.gmin;
    if (o >= pl.sp.range || gs >= (uint64_t)pl.ngroups) return 0xFFFFFFFFu;
    it = ((uint32_t)(o & (kSliceKeys - 1)) << 16) | ((uint32_t)gs + 1u);
    return (uint32_t)(o >> kSliceBits);
}
__global__ __launch_bounds__(1024) void k_dim_items(const int64_t *__restrict__ dk, ColRef dg, int64_t nd, uint64_t span,
                                                    const FusedPlan *__restrict__ plan, uint32_t *__restrict__ items,
                                                    uint32_t *__restrict__ offs, uint32_t *__restrict__ st) {
    constexpr int DR = 8, S = kSliceMaxF;
    __shared__ uint32_t lc[S], ls[S];
    const int tid = threadIdx.x;
    const FusedPlan pl = *plan;
    for (int i = tid; i < S; i += 1024) lc[i] = 0u;
    __syncthreads();
    const int64_t per = (nd + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per, hi = lo + per < nd ? lo + per : nd;
    bool bad = false;
    auto pass = [&](bool place) {
        for (int64_t c0 = lo; c0 < hi; c0 += 1024 * DR) {
            int64_t kk[DR], gg[DR];
#pragma unroll
            for (int q = 0; q < DR; ++q) {
                const int64_t i = c0 + (int64_t)q * 1024 + tid;
                kk[q] = i < hi ? dk[i] : 0;
                gg[q] = i < hi ? load_i64(dg, i) : 0;
            }
#pragma unroll
            for (int q = 0; q < DR; ++q) {
                if (c0 + (int64_t)q * 1024 + tid >= hi) continue;
                uint32_t it;
                const uint32_t b = dim_item(pl, kk[q], gg[q], it);
                if (b == 0xFFFFFFFFu) bad = true;
                else if (place) items[(uint64_t)blockIdx.x * span + atomicAdd(&ls[b], 1u)] = it;
                else atomicAdd(&lc[b], 1u);
            }
        }
    };
    if (pl.sp.ok) pass(false);  // slice counts
    __syncthreads();
    uint32_t *o = offs + (uint64_t)blockIdx.x * 2 * (S + 1);
    if (tid < 64) {  // run starts: exclusive scan of the counts padded to multiples of 4 (3 slices a lane)
        const int lane = tid;
        uint32_t c3[3], t = 0;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int b = lane * 3 + q;
            c3[q] = b < S ? (lc[b] + 3u) & ~3u : 0u;
            t += c3[q];
        }
        uint32_t incl = t;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t a = __shfl_up(incl, d, 64);
            if (lane >= d) incl += a;
        }
        uint32_t run = incl - t;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int b = lane * 3 + q;
            if (b < S) ls[b] = run;
            run += c3[q];
        }
        if (lane == 63) o[S] = incl;
    }
    __syncthreads();
    for (int b = tid; b < S; b += 1024) o[b] = ls[b], o[S + 1 + b] = lc[b];
    __syncthreads();
    if (pl.sp.ok) pass(true);  // the same rows again (L2), placed
    if (bad) st[1] = 1u;
}

struct FusedItems {
    DevBuf plan, kbuf, vbuf, cbuf, states, errw;
    SliceRegions rg{};
    FastIn in{};
    AggSpecs specs{};
    int nacol = 0, grid = 0;
    int64_t Gs = 0;
    // the shuffle join's items form (pw > 0): phase A in the partitioned layout, the packed send blocks
    int pw = 0, prank = 0, S = 0;
    uint64_t blockcap = 0, cap = 0;
    DevBuf pkey, pval, pcnt, prb, ptot, rrb, roff;
};

// begin's checks (check_only: nothing allocated or launched -- the caller's agreement flag)
static int fused_items_begin(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols, int probe_key_idx,
                             const qeh_expr *predicate, const qeh_agg *aggs, int n_aggs, const int64_t *stats_dev,
                             int world, int row_len, void **handle, bool check_only, int pw = 0, int prank = 0) {
    if (!ctx || (!check_only && (!handle || !stats_dev || world < 1 || row_len < 6)) || n_aggs < 1 || n_probe_cols < 1 ||
        probe_key_idx < 0 || probe_key_idx >= n_probe_cols)
        return fail(QEH_E_INVALID, "qeh_fused_items_begin: bad argument");
    if (handle) *handle = nullptr;
    DeviceGuard dg(ctx->device);
    const int64_t n = probe_cols[0].length;
    for (int i = 0; i < n_probe_cols; ++i)
        if (probe_cols[i].length != n) return fail(QEH_E_INVALID, "probe columns have different lengths");
    ColSet cols;
    QEH_TRY(make_colset(probe_cols, n_probe_cols, &cols));
    std::vector<int32_t> dts(n_probe_cols);
    std::vector<int> idx(n_probe_cols);
    for (int i = 0; i < n_probe_cols; ++i) dts[i] = probe_cols[i].dtype, idx[i] = i;
    PredPlan pp;
    QEH_TRY(plan_predicate(predicate, dts.data(), n_probe_cols, &pp));
    auto fi = std::make_unique<FusedItems>();
    QEH_TRY(plan_aggs(aggs, n_aggs, probe_cols, n_probe_cols, idx.data(), &fi->specs));
    for (int a = 0; a < fi->specs.n; ++a)
        if (!((fi->specs.a[a].kind == AK_SUM_F && fi->specs.a[a].func == QEH_AGG_SUM && fi->specs.a[a].cnt_slot == 0) ||
              (fi->specs.a[a].kind == AK_COUNT && fi->specs.a[a].func == QEH_AGG_COUNT)))
            return fail(QEH_E_UNSUPPORTED, "qeh_fused_items_begin: COUNT and non-null float SUM aggregates only");
    int nterms = 0;
    if (!fast_cols_eligible(cols, pp, probe_key_idx, fi->specs, &fi->in, &nterms, &fi->nacol) || fi->nacol > 1)
        return fail(QEH_E_UNSUPPORTED, "qeh_fused_items_begin: probe columns outside the fused pipeline's shapes");
    if (check_only) return QEH_OK;
    const int64_t tile_rows = fi->nacol ? SliceShape<1, true>::TILE : SliceShape<0, true>::TILE;
    const int chunk = fi->nacol ? SliceShape<1, true>::CH : SliceShape<0, true>::CH;
    const int64_t n_tiles = n / tile_rows, tail = n - n_tiles * tile_rows, n_all = n_tiles + (tail ? 1 : 0);
    AggSpecs &specs = fi->specs;
    specs.shards = 1;
    fi->Gs = std::min<int64_t>(kSliceStateWords / std::max(specs.n_slots, 1), 0xFFFE);
    // (the shuffle form: the same grid on every rank whatever its row count -- the receivers address the
    // regions of every sender as (source, slice, workgroup))
    fi->grid = pw > 1 ? (int)std::min<int64_t>(ctx->props.multiProcessorCount, kMaxSliceGrid)
                      : (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)ctx->props.multiProcessorCount, n_all,
                                                                     (int64_t)kMaxSliceGrid}));
    const uint64_t tiles_per_wg = (uint64_t)((n_all + fi->grid - 1) / fi->grid);
    SlicePlanIn pi{};
    pi.min_bytes = 6ull << 20;
    if (const char *e = std::getenv("QEH_SLICE_MIN_BYTES")) pi.min_bytes = std::strtoull(e, nullptr, 10);
    pi.grid = fi->grid;
    pi.n_slots = specs.n_slots;
    pi.sparse_ok = direct_sparse_allowed() ? 1 : 0;
    pi.chunk = chunk;
    pi.alloc_items = tiles_per_wg * fi->grid * (uint64_t)tile_rows * 5 / 4 + (uint64_t)fi->grid * kSliceMaxF * (256 + 2 * chunk);
    pi.world = pw;
    const uint64_t nreg_max = (uint64_t)fi->grid * (kSliceMaxF + (pw > 1 ? pw : 0));
    fi->pw = pw, fi->prank = prank;
    fi->rg.pw = pw, fi->rg.prank = prank;
    QEH_TRY(fi->plan.alloc(ctx, sizeof(FusedPlan)));
    QEH_TRY(fi->kbuf.alloc(ctx, pi.alloc_items * 2 + 64));
    if (fi->nacol) QEH_TRY(fi->vbuf.alloc(ctx, pi.alloc_items * 8 + 64));
    QEH_TRY(fi->cbuf.alloc(ctx, nreg_max * 4 + 64));
    QEH_TRY(fi->states.alloc(ctx, (size_t)specs.n_slots * fi->Gs * 8));
    QEH_TRY(fi->errw.alloc(ctx, 32));
    uint32_t *st = fi->errw.as<uint32_t>();
    fi->rg.key = fi->kbuf.as<uint16_t>();
    fi->rg.val = fi->nacol ? fi->vbuf.as<int64_t>() : nullptr;
    fi->rg.count = fi->cbuf.as<uint32_t>();
    fi->rg.overflow = st + 1;
    FusedPlan *dplan = fi->plan.as<FusedPlan>();
    {
        KernelTimer kt(ctx, "fused_build");
        const int gp = (int)std::max<int64_t>(1, std::min<int64_t>(ctx->props.multiProcessorCount,
                                                                   (specs.n_slots * fi->Gs + 4095) / 4096));
        hipLaunchKernelGGL(k_fused_plan_stats, dim3(gp), dim3(1024), 0, ctx->stream, stats_dev, world, row_len, pi, fi->Gs,
                           dplan, st, fi->states.as<uint64_t>(), fi->Gs, specs);
    }
    QEH_HIP(hipGetLastError());
    FusedPro fp{};  // no build rows in the prologue: they arrive gathered by slice
    fp.status = st;
    fp.plan = dplan;
    if (n_tiles > 0 || tail > 0)
        launch_slice_partition_early(ctx, fi->in, pp, nterms, fi->nacol, n_tiles, tail, fi->grid, fi->rg, &dplan->sp, fp);
    else  // (no fact rows on this rank: its regions are empty)
        QEH_HIP(hipMemsetAsync(fi->cbuf.p, 0, nreg_max * 4, ctx->stream));
    QEH_HIP(hipGetLastError());
    *handle = fi.release();
    return QEH_OK;
}

extern "C" int qeh_fused_items_begin(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols, int probe_key_idx,
                                     const qeh_expr *predicate, const qeh_agg *aggs, int n_aggs, const int64_t *stats_dev,
                                     int world, int row_len, void **handle) {
    return fused_items_begin(ctx, probe_cols, n_probe_cols, probe_key_idx, predicate, aggs, n_aggs, stats_dev, world, row_len,
                             handle, false);
}

extern "C" int qeh_fused_items_check(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols, int probe_key_idx,
                                     const qeh_expr *predicate, const qeh_agg *aggs, int n_aggs) {
    return fused_items_begin(ctx, probe_cols, n_probe_cols, probe_key_idx, predicate, aggs, n_aggs, nullptr, 0, 0, nullptr,
                             true);
}

extern "C" int qeh_fused_items_build(qeh_ctx *ctx, void *handle, const qeh_column *build_key, const qeh_column *group_key,
                                     int n_blocks, uint64_t span, uint32_t *items, uint32_t *offs) {
    if (!ctx || !handle || !build_key || !group_key || !offs || !items || n_blocks < 1 || n_blocks > kMaxSliceGrid ||
        (span & 3))
        return fail(QEH_E_INVALID, "qeh_fused_items_build: bad argument (1..512 blocks, span a multiple of 4)");
    FusedItems *fi = (FusedItems *)handle;
    DeviceGuard dg(ctx->device);
    if (build_key->dtype != QEH_DT_INT64 || (build_key->validity && build_key->null_count != 0) ||
        (group_key->dtype != QEH_DT_INT64 && group_key->dtype != QEH_DT_INT32) ||
        (group_key->validity && group_key->null_count != 0) || group_key->length != build_key->length)
        return fail(QEH_E_UNSUPPORTED, "qeh_fused_items_build: one non-null Int64 key and one non-null integer group key");
    const int64_t nd = build_key->length;
    if ((uint64_t)((nd + n_blocks - 1) / n_blocks) + 4ull * kSliceMaxF > span)
        return fail(QEH_E_INVALID, "qeh_fused_items_build: span below ceil(rows / n_blocks) + 640");
    KernelTimer kt(ctx, "fused_build");
    hipLaunchKernelGGL(k_dim_items, dim3(n_blocks), dim3(1024), 0, ctx->stream,
                       (const int64_t *)build_key->values + build_key->offset, make_colref(*group_key), nd, span,
                       fi->plan.as<FusedPlan>(), items, offs, fi->errw.as<uint32_t>());
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

extern "C" int qeh_fused_items_finish(qeh_ctx *ctx, void *handle, const uint32_t *items, uint64_t span,
                                      const uint32_t *offs, int n_regions, int64_t n_groups, double *lanes) {
    const int world = n_regions;
    if (!ctx || !handle || !offs || !lanes || world < 1 || world > kMaxSliceGrid || n_groups < 1 || (span & 3) ||
        (uint64_t)world * span >= (1ull << 32))
        return fail(QEH_E_INVALID, "qeh_fused_items_finish: bad argument");
    std::unique_ptr<FusedItems> fi((FusedItems *)handle);  // freed here: its buffers' users are queued ahead
    DeviceGuard dg(ctx->device);
    if (n_groups > fi->Gs) return fail(QEH_E_UNSUPPORTED, "qeh_fused_items_finish: more groups than the states hold");
    uint32_t *st = fi->errw.as<uint32_t>();
    {
        KernelTimer ktb(ctx, "slice_probe");
        DimSlices dim{items, nullptr, st + 4, fi->plan.as<FusedPlan>(), world, 0, span, offs};
        const int gridB = ctx->props.multiProcessorCount;
        const HashTable t{};
        const bool pf = slice_probe_prefetch();
        if (fi->nacol == 0) {
            if (pf) hipLaunchKernelGGL((k_slice_probe<0, false, true, false, true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream,
                                       fi->rg, fi->grid, 0, t, fi->in, fi->specs, fi->Gs, fi->states.as<uint64_t>(), dim);
            else hipLaunchKernelGGL((k_slice_probe<0, false, false, false, true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream,
                                    fi->rg, fi->grid, 0, t, fi->in, fi->specs, fi->Gs, fi->states.as<uint64_t>(), dim);
        } else {
            if (pf) hipLaunchKernelGGL((k_slice_probe<1, false, true, true, true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream,
                                       fi->rg, fi->grid, 0, t, fi->in, fi->specs, fi->Gs, fi->states.as<uint64_t>(), dim);
            else hipLaunchKernelGGL((k_slice_probe<1, false, false, true, true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream,
                                    fi->rg, fi->grid, 0, t, fi->in, fi->specs, fi->Gs, fi->states.as<uint64_t>(), dim);
        }
    }
    QEH_HIP(hipGetLastError());
    const int64_t ne = (int64_t)(1 + fi->specs.n) * n_groups;
    hipLaunchKernelGGL(k_states_lanes, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, ctx->stream,
                       (const uint64_t *)fi->states.as<uint64_t>(), fi->Gs, n_groups, fi->specs, lanes, (const uint32_t *)st, 1);
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

extern "C" int qeh_fused_items_abort(qeh_ctx *ctx, void *handle) {
    if (!ctx || !handle) return QEH_OK;
    DeviceGuard dg(ctx->device);
    std::unique_ptr<FusedItems> fi((FusedItems *)handle);
    QEH_HIP(hipStreamSynchronize(ctx->stream));  // its phase A may still be running
    return QEH_OK;
}

// ---- the items form of the shuffle join (BASELINE config 4: hash-partitioned join + aggregate) ----
// Each rank runs the fused pipeline's phase A over ITS fact shard in the partitioned layout -- the
// join key's slice b = (k - kmin) >> 16 decides the rank, b % world (the partition function: a modulo
// hash of the key's slice, so every key's fact and dimension rows meet on one rank) -- packs each
// destination's regions (10-B items: 16-bit key offset + value) into one block, and the all-to-all moves
// the blocks; the receiving rank runs phase B over what every rank sent it, with its slices' LDS
// entries built from the all-gathered dimension items (qeh_fused_items_build), and writes the dense
// final stage's lanes.  Per fact row: phase A's 24 B read + 10 B per selected row written, the pack's
// 10 + 10 B, phase B's 10 B read -- instead of the two-pass exchange (42 B) plus a local pipeline over
// the received (key, value) rows (16 B read, 10 + 10 B of its own items).

// Exclusive scan of each block's region counts (rounded up to 2: phase B's pair loads), written as
// absolute region starts base(q) + prefix; base(q) = bases[q], or q * blockcap without bases.  With
// F > 0 (the sender), counts of slices past the plan's last (j * pw + q >= F: never written by phase A)
// are taken as 0 and the cleaned counts go to cnt_out; totals[q] = the block's items.
__global__ __launch_bounds__(1024) void k_region_scan(const uint32_t *__restrict__ cnt, int64_t E, const int64_t *bases,
                                                      uint64_t blockcap, int F, int pw, int grid,
                                                      uint64_t *__restrict__ rbase, uint32_t *__restrict__ cnt_out,
                                                      int64_t *__restrict__ totals) {
    __shared__ uint64_t wsum[16];
    const int q = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint64_t base = bases ? (uint64_t)bases[q] : (uint64_t)q * blockcap;
    const int64_t per = (E + 1023) / 1024, e0 = (int64_t)t * per, e1 = e0 + per < E ? e0 + per : E;
    auto count = [&](int64_t e) -> uint32_t {
        if (F > 0 && (int64_t)(e / grid) * pw + q >= F) return 0u;
        return cnt[(uint64_t)q * E + e];
    };
    uint64_t tot = 0;
    for (int64_t e = e0; e < e1; ++e) tot += (count(e) + 1u) & ~1u;
    uint64_t incl = tot;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t a = __shfl_up(incl, d, 64);
        if (lane >= d) incl += a;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint64_t run = incl - tot;
    for (int w = 0; w < wave; ++w) run += wsum[w];
    for (int64_t e = e0; e < e1; ++e) {
        const uint32_t c = count(e);
        rbase[(uint64_t)q * E + e] = base + run;
        if (cnt_out) cnt_out[(uint64_t)q * E + e] = c;
        run += (c + 1u) & ~1u;
    }
    if (totals && t == 1023) totals[q] = (int64_t)run;  // (the last thread's run ends the block)
}

// Region r's items (count cnt[r], padded to 2) from the phase-A layout (r * cap) to rbase[r]: one
// workgroup per region, key pairs as 4-B words, value pairs as 16-B words.
__global__ __launch_bounds__(256) void k_region_pack(const uint16_t *__restrict__ kin, const int64_t *__restrict__ vin,
                                                     const uint32_t *__restrict__ cnt, const uint64_t *__restrict__ rbase,
                                                     uint64_t cap, uint16_t *__restrict__ kout, int64_t *__restrict__ vout,
                                                     int64_t E, int skip) {
    const uint64_t r = blockIdx.x;
    if ((int64_t)(r / E) == skip) return;  // (this rank's own block: phase B reads it in place)
    const uint32_t c2 = (cnt[r] + 1u) >> 1;  // item pairs
    const uint32_t *ks = (const uint32_t *)(kin + r * cap);
    uint32_t *kd = (uint32_t *)(kout + rbase[r]);
    const v2i64 *vs = (const v2i64 *)(vin + r * cap);
    v2i64 *vd = (v2i64 *)(vout + rbase[r]);
    constexpr int U = 4;  // pairs in flight per thread
    for (uint32_t i0 = 0; i0 < c2; i0 += 256 * U) {
        uint32_t kk[U];
        v2i64 vv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = i0 + u * 256 + threadIdx.x;
            if (i < c2) {
                kk[u] = __builtin_nontemporal_load(ks + i);
                if (vin) vv[u] = __builtin_nontemporal_load(vs + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = i0 + u * 256 + threadIdx.x;
            if (i < c2) {
                __builtin_nontemporal_store(kk[u], kd + i);
                if (vin) __builtin_nontemporal_store(vv[u], vd + i);
            }
        }
    }
}

extern "C" int qeh_shuffle_items_begin(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols, int probe_key_idx,
                                       const qeh_expr *predicate, const qeh_agg *aggs, int n_aggs, const int64_t *stats_dev,
                                       int world, int rank, int row_len, void **handle) {
    if (world < 2 || world > 64 || rank < 0 || rank >= world)
        return fail(QEH_E_INVALID, "qeh_shuffle_items_begin: bad argument (2..64 ranks)");
    return fused_items_begin(ctx, probe_cols, n_probe_cols, probe_key_idx, predicate, aggs, n_aggs, stats_dev, world, row_len,
                             handle, false, world, rank);
}

extern "C" int qeh_shuffle_items_pack(qeh_ctx *ctx, void *handle, uint16_t **keys, int64_t **vals, uint32_t **counts,
                                      uint64_t *blockcap, int64_t *block_regions, int64_t *totals, int *ok) {
    if (!ctx || !handle || !keys || !vals || !counts || !blockcap || !block_regions || !totals || !ok)
        return fail(QEH_E_INVALID, "qeh_shuffle_items_pack: bad argument");
    FusedItems *fi = (FusedItems *)handle;
    if (fi->pw < 2) return fail(QEH_E_INVALID, "qeh_shuffle_items_pack: not a shuffle handle");
    DeviceGuard dg(ctx->device);
    *ok = 0;
    FusedPlan pl;
    uint32_t sw[8];
    QEH_TRY(read_small(ctx, &pl, fi->plan.p, sizeof(FusedPlan)));  // (waits for phase A)
    QEH_TRY(read_small(ctx, sw, fi->errw.p, 32));
    for (int q = 0; q < fi->pw; ++q) totals[q] = 0;
    *keys = nullptr, *vals = nullptr, *counts = nullptr, *blockcap = 0, *block_regions = 0;
    if (!pl.sp.ok || sw[0] || sw[1]) return QEH_OK;  // declined plan, kernel error or a full region: *ok = 0
    const int pw = fi->pw, grid = fi->grid;
    fi->S = part_slices(pl.sp.F, pw);
    const int64_t E = (int64_t)fi->S * grid, P = E * pw;
    fi->blockcap = (uint64_t)E * pl.sp.cap;
    fi->cap = pl.sp.cap;
    QEH_TRY(fi->pkey.alloc(ctx, (fi->blockcap * pw + 4) * 2));
    if (fi->nacol) QEH_TRY(fi->pval.alloc(ctx, (fi->blockcap * pw + 4) * 8));
    QEH_TRY(fi->pcnt.alloc(ctx, (size_t)P * 4));
    QEH_TRY(fi->prb.alloc(ctx, (size_t)P * 8));
    QEH_TRY(fi->ptot.alloc(ctx, (size_t)pw * 8));
    {
        KernelTimer kt(ctx, "shuffle_pack");
        hipLaunchKernelGGL(k_region_scan, dim3(pw), dim3(1024), 0, ctx->stream, fi->cbuf.as<uint32_t>(), E,
                           (const int64_t *)nullptr, fi->blockcap, pl.sp.F, pw, grid, fi->prb.as<uint64_t>(),
                           fi->pcnt.as<uint32_t>(), fi->ptot.as<int64_t>());
        hipLaunchKernelGGL(k_region_pack, dim3((unsigned)P), dim3(256), 0, ctx->stream, fi->kbuf.as<uint16_t>(),
                           fi->nacol ? fi->vbuf.as<int64_t>() : nullptr, fi->pcnt.as<uint32_t>(), fi->prb.as<uint64_t>(),
                           pl.sp.cap, fi->pkey.as<uint16_t>(), fi->nacol ? fi->pval.as<int64_t>() : nullptr, E,
                           fi->prank);
    }
    QEH_HIP(hipGetLastError());
    QEH_TRY(read_small(ctx, totals, fi->ptot.p, (size_t)pw * 8));
    *keys = fi->pkey.as<uint16_t>();
    *vals = fi->nacol ? fi->pval.as<int64_t>() : nullptr;
    *counts = fi->pcnt.as<uint32_t>();
    *blockcap = fi->blockcap;
    *block_regions = E;
    *ok = 1;
    return QEH_OK;
}

extern "C" int qeh_shuffle_items_finish(qeh_ctx *ctx, void *handle, const uint16_t *keys, const int64_t *vals,
                                        const uint32_t *counts, const int64_t *src_offsets, const uint32_t *items,
                                        uint64_t span, const uint32_t *offs, int n_regions, int64_t n_groups,
                                        double *lanes) {
    if (!ctx || !handle || !keys || !counts || !src_offsets || !items || !offs || !lanes || n_regions < 1 ||
        n_regions > kMaxSliceGrid || n_groups < 1 || (span & 3) || (uint64_t)n_regions * span >= (1ull << 32))
        return fail(QEH_E_INVALID, "qeh_shuffle_items_finish: bad argument");
    std::unique_ptr<FusedItems> fi((FusedItems *)handle);  // freed here: its buffers' users are queued ahead
    DeviceGuard dg(ctx->device);
    if (fi->pw < 2 || fi->S < 1) return fail(QEH_E_INVALID, "qeh_shuffle_items_finish: pack did not run");
    if (n_groups > fi->Gs) return fail(QEH_E_UNSUPPORTED, "qeh_shuffle_items_finish: more groups than the states hold");
    if (fi->nacol && !vals) return fail(QEH_E_INVALID, "qeh_shuffle_items_finish: the values are missing");
    const int pw = fi->pw, grid = fi->grid;
    const int64_t E = (int64_t)fi->S * grid, P = E * pw;
    uint32_t *st = fi->errw.as<uint32_t>();
    QEH_TRY(fi->roff.alloc(ctx, (size_t)pw * 8));
    QEH_TRY(fi->rrb.alloc(ctx, (size_t)P * 8));
    QEH_HIP(hipMemcpyAsync(fi->roff.p, src_offsets, (size_t)pw * 8, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_region_scan, dim3(pw), dim3(1024), 0, ctx->stream, counts, E, fi->roff.as<int64_t>(), (uint64_t)0,
                       0, pw, grid, fi->rrb.as<uint64_t>(), (uint32_t *)nullptr, (int64_t *)nullptr);
    SliceRegions rg{};
    rg.key = (uint16_t *)keys;
    rg.val = (int64_t *)vals;
    rg.count = (uint32_t *)counts;
    rg.overflow = st + 1;
    rg.rbase = fi->rrb.as<uint64_t>();
    rg.pw = pw, rg.prank = fi->prank, rg.pgrid = grid;
    rg.okey = fi->kbuf.as<uint16_t>(), rg.oval = fi->nacol ? fi->vbuf.as<int64_t>() : nullptr, rg.ocap = fi->cap;
    {
        KernelTimer ktb(ctx, "slice_probe");
        DimSlices dim{items, nullptr, st + 4, fi->plan.as<FusedPlan>(), n_regions, 0, span, offs};
        const int gridB = ctx->props.multiProcessorCount;
        const HashTable t{};
        const bool pf = slice_probe_prefetch();
        const int nreg = pw * grid;
        if (fi->nacol == 0) {
            if (pf) hipLaunchKernelGGL((k_slice_probe<0, false, true, false, true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream,
                                       rg, nreg, 0, t, fi->in, fi->specs, fi->Gs, fi->states.as<uint64_t>(), dim);
            else hipLaunchKernelGGL((k_slice_probe<0, false, false, false, true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream,
                                    rg, nreg, 0, t, fi->in, fi->specs, fi->Gs, fi->states.as<uint64_t>(), dim);
        } else {
            if (pf) hipLaunchKernelGGL((k_slice_probe<1, false, true, true, true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream,
                                       rg, nreg, 0, t, fi->in, fi->specs, fi->Gs, fi->states.as<uint64_t>(), dim);
            else hipLaunchKernelGGL((k_slice_probe<1, false, false, true, true>), dim3(gridB), dim3(kSliceBlock), 0, ctx->stream,
                                    rg, nreg, 0, t, fi->in, fi->specs, fi->Gs, fi->states.as<uint64_t>(), dim);
        }
    }
    QEH_HIP(hipGetLastError());
    const int64_t ne = (int64_t)(1 + fi->specs.n) * n_groups;
    hipLaunchKernelGGL(k_states_lanes, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, ctx->stream,
                       (const uint64_t *)fi->states.as<uint64_t>(), fi->Gs, n_groups, fi->specs, lanes, (const uint32_t *)st, 1);
    QEH_HIP(hipGetLastError());
    // the handle's buffers (phase A's regions, the packed blocks) are freed when this returns: the
    // caller's collectives that read the packed blocks were issued before this call on its stream
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    return QEH_OK;
}

extern "C" int qeh_join_filter_aggregate(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols,
                                         int probe_key_idx, const qeh_expr *predicate, const qeh_column *build_key,
                                         const qeh_column *build_group_keys, int n_group_keys, const qeh_agg *aggs,
                                         int n_aggs, qeh_column *out_keys, qeh_column *out_aggs,
                                         int64_t *out_groups) {
    if (!ctx || !out_groups || !build_key) return fail(QEH_E_INVALID, "qeh_join_filter_aggregate: bad argument");
    *out_groups = 0;
    if (n_aggs == 0) return QEH_OK;
    if (probe_key_idx < 0 || probe_key_idx >= n_probe_cols) return fail(QEH_E_INVALID, "probe key index out of range");
    if (n_group_keys < 1) return fail(QEH_E_UNSUPPORTED, "fused join-aggregate needs at least one build-side group key");
    const int64_t n = probe_cols[0].length;
    for (int i = 0; i < n_probe_cols; ++i)
        if (probe_cols[i].length != n) return fail(QEH_E_INVALID, "probe columns have different lengths");
    for (int i = 0; i < n_group_keys; ++i)
        if (build_group_keys[i].length != build_key->length) return fail(QEH_E_INVALID, "build columns have different lengths");
    DeviceGuard dg(ctx->device);
    ColSet cols;
    QEH_TRY(make_colset(probe_cols, n_probe_cols, &cols));
    std::vector<int32_t> dts(n_probe_cols);
    std::vector<int> idx(n_probe_cols);
    for (int i = 0; i < n_probe_cols; ++i) {
        dts[i] = probe_cols[i].dtype;
        idx[i] = i;
    }
    PredPlan pp;
    QEH_TRY(plan_predicate(predicate, dts.data(), n_probe_cols, &pp));
    AggSpecs specs;
    QEH_TRY(plan_aggs(aggs, n_aggs, probe_cols, n_probe_cols, idx.data(), &specs));
    if (probe_cols[probe_key_idx].dtype != QEH_DT_INT64 && probe_cols[probe_key_idx].dtype != QEH_DT_INT32)
        return fail(QEH_E_UNSUPPORTED, "hash join keys must be Int32/Int64 on the device");
    MinMaxMemoScope memo(ctx);  // build key / group key ranges: read once for prelaunch, groups and join table

    // phase A of the slice path on the second queue, when its shape is known from the build key's
    // range (and the group count is bounded by one integer group key's range)
    SlicePre pre;
    std::shared_ptr<PendingSlice> pend = std::static_pointer_cast<PendingSlice>(ctx->pending_slice);
    ctx->pending_slice.reset();
    if (pend && n_group_keys == 1 && pend->matches(probe_cols, n_probe_cols, probe_key_idx, predicate, aggs, n_aggs)) {
        // adopt the phase A launched by qeh_join_filter_aggregate_prelaunch(_stats) if the build columns
        // that arrived have exactly the ranges it was planned from
        if (pend->pre.dev_planned) QEH_TRY(resolve_dev_plan(ctx, &pend->pre, &pend->br));
        const qeh_column both[2] = {*build_key, build_group_keys[0]};
        BuildRanges br;
        if (pend->pre.launched && build_key->dtype == QEH_DT_INT64 &&
            (build_group_keys[0].dtype == QEH_DT_INT64 || build_group_keys[0].dtype == QEH_DT_INT32)) {
            QEH_TRY(columns_minmax(ctx, both, 2, br.mn, br.mx, br.cnt));
            if (br == pend->br) pend->take(&pre);
        }
    }
    pend.reset();  // not adopted: waits for its phase A, frees its regions
    if (!pre.launched && n_group_keys == 1) {
        const int fs = fused_join_filter_aggregate(ctx, cols, n, pp, specs, probe_key_idx, *build_key, build_group_keys[0],
                                                   out_keys, out_aggs, out_groups);
        if (fs != kFusedNotEligible) return fs;
        QEH_TRY(slice_prelaunch(ctx, cols, n, pp, specs, probe_key_idx, *build_key, build_group_keys[0], &pre));
    }
    // build side: dense group ids of the build rows, then the join table with gid payloads
    GroupTable gt;
    DevBuf slot_of_row;
    QEH_TRY(group_slots_of_rows(ctx, build_group_keys, n_group_keys, build_key->length, &gt, &slot_of_row));
    BuiltTable bt;
    RowPayload rp;  // payload = dense group id of the build row, read through its slot
    rp.slot = slot_of_row.as<uint32_t>();
    rp.dense = gt.dense.as<uint64_t>();
    ctx->build_beside_rows = pre.launched ? n : 0;
    const int brc = build_join_table(ctx, *build_key, rp, (uint64_t)std::max<int64_t>(gt.groups - 1, 0), &bt);
    ctx->build_beside_rows = 0;
    QEH_TRY(brc);
    GidSource src{};
    src.jt = bt.t;
    src.key_col = probe_key_idx;
    std::vector<int32_t> kd(n_group_keys);
    for (int i = 0; i < n_group_keys; ++i) kd[i] = build_group_keys[i].dtype;
    return aggregate_rows(ctx, GM_JOIN, cols, n, pp, src, specs, gt.groups, gt.keys, kd.data(),
                          gt.rep_row.as<uint32_t>(), true, "join_filter_aggregate", out_keys, out_aggs, out_groups,
                          &pre);
}

#if QEH_PA_STAMPS
// diagnostic build only: the per-wave phase cycles of the last fused phase A (see QEH_PA_STAMPS)
extern "C" int qeh_debug_pa_stamps(uint64_t *out, uint64_t n_words) {
    using namespace qeh;
    const uint64_t w = std::min<uint64_t>(n_words, (uint64_t)kMaxSliceGrid * 16 * kPaStampWords);
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(qeh_pa_stamps), w * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
