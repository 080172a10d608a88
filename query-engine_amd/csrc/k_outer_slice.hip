// Order-preserving LDS-slice probe for LEFT / RIGHT / FULL joins over compact embedded records
// (the record tables of k_join.hip's k_embed_build32: one 2-B or 4-B record per key
// offset, 0 = no build row, FULL's matched flag in the top bit).
//
// An outer join over a unique DIRECT build writes one output row per probe row, in probe order.  The
// single-pass probe (k_outer_embed32) reads one record per probe row from a table that does not fit
// an XCD's L2 (20 MB for 1e7 keys): nearly every lookup is a line fill from the Infinity Cache, and
// that request rate bounds it (1.9 ms for 2e8 probe rows, 1e8 of them in range).  Here the lookups
// run in LDS, as in the metric's slice pipeline (k_aggregate.hip), and probe order comes back by
// replaying a deterministic partition instead of carrying row ids:
//   A  k_os_part: workgroup w walks its own contiguous range of 4096-row tiles.  A tile's rows are
//      ranked per table slice (2^16 keys of 2-B records or 2^15 of 4-B: 128 KB either way) with
//      returning LDS atomics on per-wave counters -- the lanes of one instruction are served in lane
//      order (lds_atomic_rank_ok) and the instructions in program order, so a row's rank is a function
//      of the keys alone -- and its 16-bit key offset joins the (w, slice) sequence.  Sequences live in
//      256-item chunks taken in a fixed order from w's own pool (no global atomics: chunk ids are a
//      function of the keys as well).  The tile's items are staged in LDS in (slice, rank) order and
//      stored run by run; each chunk is tagged with its slice and its item count.
//   B  chunk_lists groups the chunks by slice tag; k_os_probe, a workgroup per (slice, part of its
//      list), loads the slice's records into LDS and overwrites each item with its record's value
//      (FULL: sets the matched flag in the LDS copy and ORs the flags back into the table at the end).
//   C  k_os_emit: the same workgroups walk the same tiles, replay A's ranking and chunk choice, gather
//      each tile's results run by run into LDS, and write the build column (+ validity) in probe
//      order; FULL copies the probe columns beside the key read.
// HBM bytes per probe row: A 8 (key) + 2 per item, B 2 + 2 per item (4 + 4 for 4-B records), C 8 + 2
// per item read and 8 written (+ 8 read and 8 written per FULL probe column).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "ops.h"

namespace qeh {

namespace {

constexpr int kOsBlock = 512;                // phases A and C: two workgroups per CU overlap each other's waits
constexpr int kOsWaves = kOsBlock / 64;
#ifndef QEH_OS_R
#define QEH_OS_R 8
#endif
#ifndef QEH_OS_EXP  // timing ablations (experiment builds only, wrong results: 1 no item stores, 2 no ranking)
#define QEH_OS_EXP 0
#endif
constexpr int kOsR = QEH_OS_R;               // rows per thread per tile
constexpr int kOsTile = kOsBlock * kOsR;     // 4096 probe rows per tile
constexpr int kOsChunk = 256;                // items per pool chunk
constexpr int kOsMaxF = 256;                 // slices (key range <= 2^24 for 2-B records, 2^23 for 4-B)
constexpr int kOsSliceBytes = 128 * 1024;    // one slice of records in LDS
constexpr int kOsPBlock = 1024;              // phase B
constexpr int kOsPWaves = kOsPBlock / 64;
constexpr int kOsPU = 8;                     // chunks in flight per phase-B wave
constexpr int kOsLBlock = 256;               // the chunk-list passes
constexpr int kOsLGrid = 128;

struct OsShape {
    int64_t n;        // probe rows
    int64_t kmin;     // build key minimum (record 0)
    uint64_t range;   // records
    int32_t sbits;    // key bits per slice: 16 (2-B records) or 15 (4-B)
    int32_t F;        // slices
    int64_t tpw;      // tiles per workgroup (phases A and C)
    uint32_t pool;    // chunks per workgroup pool: tpw * (kOsTile / kOsChunk) + F bounds what one workgroup opens
};

typedef unsigned int os_u4 __attribute__((ext_vector_type(4)));

struct OsLds {
    uint32_t cnt[kOsWaves][kOsMaxF];  // per-wave counters, then the waves' bases
    // per slice, read by a row in one 16-B LDS load: x = items of (this workgroup, slice) before the
    // tile, y = the slice's first position in the staged tile, z = the chunk holding item x (when x is
    // not a chunk boundary), w = chunk id of sequence chunk kk for every chunk the tile opens, minus kk
    os_u4 ss[kOsMaxF];
    uint32_t wtot[4];
    uint32_t nxt;                     // next free chunk of the workgroup's pool
    alignas(16) uint32_t stage[kOsTile];  // A: item destinations; C: destinations, then results
};

// LDS barrier that keeps global loads in flight (the next tile's keys)
__device__ __forceinline__ void os_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int KES>
__device__ __forceinline__ void os_load_keys(const ColRef &key, int64_t n, int64_t t0, int tid, int64_t (&k)[kOsR],
                                             uint32_t &vm) {
    vm = 0;
#pragma unroll
    for (int q = 0; q < kOsR; ++q) {
        const int64_t row = t0 + (int64_t)q * kOsBlock + tid;
        const bool in = row < n;
        if (KES == 8)
            k[q] = in ? __builtin_nontemporal_load((const int64_t *)key.values + row) : 0;
        else
            k[q] = in ? (int64_t)__builtin_nontemporal_load((const int32_t *)key.values + row) : 0;
        vm |= (uint32_t)(in && col_valid(key, row)) << q;
    }
}

// The tile's ranking: slice s (-1: no item -- NULL key, outside the records, past n), key offset o
// inside the slice, rank r among the wave's rows of that slice.  Identical in phases A and C.
__device__ __forceinline__ void os_rank(OsLds &L, const OsShape &sh, int wave, const int64_t (&k)[kOsR], uint32_t vm,
                                        int (&s)[kOsR], uint32_t (&o)[kOsR], uint32_t (&r)[kOsR]) {
    const uint32_t omask = (1u << sh.sbits) - 1u;
#pragma unroll
    for (int q = 0; q < kOsR; ++q) {
        const uint64_t d = (uint64_t)k[q] - (uint64_t)sh.kmin;
        const bool in = ((vm >> q) & 1u) && d < sh.range;
        s[q] = in ? (int)(d >> sh.sbits) : -1;
        o[q] = (uint32_t)d & omask;
#if QEH_OS_EXP == 2
        r[q] = 0u;
#else
        r[q] = in ? atomicAdd(&L.cnt[wave][s[q]], 1u) : 0u;
#endif
    }
}

// After the ranking barrier: the waves' bases per slice (in place), the tile-local starts, and the
// chunks the tile opens -- one exclusive scan of (count | opened << 16) over the slices.  Threads
// 0..255 own slice tid.  Ends with a barrier; tc / need stay in the slice owner's registers.
__device__ __forceinline__ void os_plan(OsLds &L, int tid, int F, uint32_t my_pos, uint32_t &tc, uint32_t &need,
                                        uint32_t &abase) {
    uint32_t packed = 0, incl = 0;
    tc = 0, need = 0, abase = 0;
    if (tid < kOsMaxF) {
        if (tid < F) {
            uint32_t run = 0;
#pragma unroll
            for (int w = 0; w < kOsWaves; ++w) {
                const uint32_t c = L.cnt[w][tid];
                L.cnt[w][tid] = run;
                run += c;
            }
            tc = run;
        }
        const uint32_t k0 = (my_pos + kOsChunk - 1) / kOsChunk;
        need = (my_pos + tc + kOsChunk - 1) / kOsChunk - k0;
        packed = tc | (need << 16);
        incl = wave_incl_scan(packed);
        if ((tid & 63) == 63) L.wtot[tid >> 6] = incl;
    }
    os_barrier();
    if (tid < kOsMaxF) {
        uint32_t pre = 0;
        for (int w = 0; w < (tid >> 6); ++w) pre += L.wtot[w];
        const uint32_t ex = pre + incl - packed;
        abase = L.nxt + (ex >> 16);
        L.ss[tid].y = ex & 0xFFFFu;
        L.ss[tid].w = abase - (my_pos + kOsChunk - 1) / kOsChunk;  // (mod 2^32)
    }
    os_barrier();
}

// A row's tile-local staged position and its item's place in the pool.
__device__ __forceinline__ void os_place(const OsLds &L, int wave, int s, uint32_t r, uint32_t &p, uint32_t &dst) {
    const uint32_t wb = L.cnt[wave][s] + r;
    const os_u4 st = L.ss[s];
    const uint32_t j = st.x + wb;
    p = st.y + wb;
    const uint32_t kk = j / kOsChunk, k0 = (st.x + kOsChunk - 1) / kOsChunk;
    const uint32_t c = kk < k0 ? st.z : st.w + kk;
    dst = c * (uint32_t)kOsChunk + j % kOsChunk;
}

// After the placement barrier: the slice owners advance their sequence, counters are cleared for the
// next tile, the pool cursor moves past the chunks this tile opened.
__device__ __forceinline__ void os_advance(OsLds &L, int tid, int F, uint32_t &my_pos, uint32_t &my_cur, uint32_t tc,
                                           uint32_t abase) {
    if (tid < F) {
        const uint32_t np = my_pos + tc;
        if (np % kOsChunk) {
            const uint32_t kl = np / kOsChunk, k0 = (my_pos + kOsChunk - 1) / kOsChunk;
            if (kl >= k0) my_cur = abase + (kl - k0);
        }
        my_pos = np;
        L.ss[tid].x = my_pos;
        L.ss[tid].z = my_cur;
    }
    if (tid == 0) L.nxt += (L.wtot[0] + L.wtot[1] + L.wtot[2] + L.wtot[3]) >> 16;
    for (int i = tid; i < kOsWaves * kOsMaxF; i += kOsBlock) (&L.cnt[0][0])[i] = 0;
}

__device__ __forceinline__ uint32_t os_tile_total(const OsLds &L) {
    return (L.wtot[0] + L.wtot[1] + L.wtot[2] + L.wtot[3]) & 0xFFFFu;
}

__device__ __forceinline__ void os_init(OsLds &L, int tid, uint32_t pool_base) {
    for (int i = tid; i < kOsWaves * kOsMaxF; i += kOsBlock) (&L.cnt[0][0])[i] = 0;
    if (tid < kOsMaxF) L.ss[tid] = os_u4{0u, 0u, 0u, 0u};
    if (tid == 0) L.nxt = pool_base;
}

}  // namespace

// ---- phase A ----------------------------------------------------------------------------------------
template <int KES>
__global__ __launch_bounds__(kOsBlock) void k_os_part(ColRef key, OsShape sh, uint16_t *__restrict__ items,
                                                      uint16_t *__restrict__ tag, uint16_t *__restrict__ ccnt) {
    __shared__ OsLds L;
    __shared__ __attribute__((aligned(16))) uint16_t sval[kOsTile];
    const int tid = threadIdx.x, wave = tid >> 6;
    const int64_t ntiles = (sh.n + kOsTile - 1) / kOsTile;
    const int64_t t_lo = (int64_t)blockIdx.x * sh.tpw, t_hi = std::min<int64_t>(ntiles, t_lo + sh.tpw);
    os_init(L, tid, blockIdx.x * sh.pool);
    uint32_t my_pos = 0, my_cur = 0;
    int64_t k[kOsR];
    uint32_t vm;
    if (t_lo < t_hi) os_load_keys<KES>(key, sh.n, t_lo * kOsTile, tid, k, vm);
    __syncthreads();
    for (int64_t t = t_lo; t < t_hi; ++t) {
        int s[kOsR];
        uint32_t o[kOsR], r[kOsR];
        os_rank(L, sh, wave, k, vm, s, o, r);
        if (t + 1 < t_hi) os_load_keys<KES>(key, sh.n, (t + 1) * kOsTile, tid, k, vm);
        os_barrier();
        uint32_t tc, need, abase;
        os_plan(L, tid, sh.F, my_pos, tc, need, abase);
        // the chunks this tile opens: tagged with their slice, full until the last one is known
        if (tid < sh.F)
            for (uint32_t i = 0; i < need; ++i) {
                const uint32_t c = abase + i;
                tag[c] = (uint16_t)tid;
                ccnt[c] = (uint16_t)kOsChunk;
            }
#pragma unroll
        for (int q = 0; q < kOsR; ++q)
            if (s[q] >= 0) {
                uint32_t p, dst;
                os_place(L, wave, s[q], r[q], p, dst);
                L.stage[p] = dst;
                sval[p] = (uint16_t)o[q];
            }
        os_barrier();
        const uint32_t tot = os_tile_total(L);
#if QEH_OS_EXP != 1
        // staged items in pairs: two neighbours of one run at an even place leave as one 4-B store
        for (uint32_t p = 2 * tid; p < tot; p += 2 * kOsBlock) {
            const uint2 d = *(const uint2 *)&L.stage[p];
            const uint32_t v = *(const uint32_t *)&sval[p];
            if (p + 1 < tot && d.y == d.x + 1 && !(d.x & 1u)) {
                *(uint32_t *)(items + d.x) = v;
            } else {
                items[d.x] = (uint16_t)v;
                if (p + 1 < tot) items[d.y] = (uint16_t)(v >> 16);
            }
        }
#endif
        os_advance(L, tid, sh.F, my_pos, my_cur, tc, abase);
        os_barrier();
    }
    if (tid < sh.F && my_pos % kOsChunk) ccnt[my_cur] = (uint16_t)(my_pos % kOsChunk);
}

// ---- chunk lists: the pool's chunks grouped by slice (phase B reads its slice's list) ---------------
// (an entry is the chunk id (< 2^24: the pool holds < 2^32 items) | its item count - 1 << 24)
__global__ __launch_bounds__(kOsLBlock) void k_os_list_count(const uint16_t *__restrict__ tag, uint64_t nchunks, int F,
                                                           uint32_t *__restrict__ wg_hist, uint32_t *__restrict__ scount) {
    __shared__ uint32_t h[kOsMaxF];
    const int tid = threadIdx.x;
    for (int i = tid; i < F; i += kOsLBlock) h[i] = 0;
    __syncthreads();
    const uint64_t lo = nchunks * blockIdx.x / gridDim.x, hi = nchunks * (blockIdx.x + 1) / gridDim.x;
    for (uint64_t c = lo + tid; c < hi; c += kOsLBlock) {
        const uint32_t t = tag[c];
        if (t < (uint32_t)F) atomicAdd(&h[t], 1u);
    }
    __syncthreads();
    for (int i = tid; i < F; i += kOsLBlock) {
        wg_hist[(uint64_t)blockIdx.x * F + i] = h[i];
        if (h[i]) atomicAdd(&scount[i], h[i]);
    }
}

__global__ __launch_bounds__(kOsLBlock) void k_os_list_fill(const uint16_t *__restrict__ tag, uint64_t nchunks, int F,
                                                          const uint32_t *__restrict__ wg_hist,
                                                          const uint32_t *__restrict__ scount, uint32_t *__restrict__ sbase,
                                                          const uint16_t *__restrict__ ccnt, uint32_t *__restrict__ list) {
    __shared__ uint32_t cur[kOsMaxF];
    const int tid = threadIdx.x;
    for (int s = tid; s < F; s += kOsLBlock) {
        uint32_t base = 0, pre = 0;
        for (int i = 0; i < s; ++i) base += scount[i];
        for (uint32_t b = 0; b < blockIdx.x; ++b) pre += wg_hist[(uint64_t)b * F + s];
        cur[s] = base + pre;
        if (blockIdx.x == 0) {
            sbase[s] = base;
            if (s == F - 1) sbase[F] = base + scount[s];
        }
    }
    __syncthreads();
    const uint64_t lo = nchunks * blockIdx.x / gridDim.x, hi = nchunks * (blockIdx.x + 1) / gridDim.x;
    for (uint64_t c = lo + tid; c < hi; c += kOsLBlock) {
        const uint32_t t = tag[c];
        if (t < (uint32_t)F) list[atomicAdd(&cur[t], 1u)] = (uint32_t)c | ((uint32_t)(ccnt[c] - 1u) << 24);
    }
}

// ---- phase B ----------------------------------------------------------------------------------------
template <typename R, bool FULL>
__global__ __launch_bounds__(kOsPBlock) void k_os_probe(OsShape sh, int H, const uint32_t *__restrict__ sbase,
                                                        const uint32_t *__restrict__ list, uint16_t *__restrict__ items,
                                                        uint32_t *__restrict__ res32, R *__restrict__ rec) {
    constexpr int NK = kOsSliceBytes / (int)sizeof(R);
    constexpr uint32_t FLAG = 1u << (8 * sizeof(R) - 1), VAL = FLAG - 1u;
    __shared__ __attribute__((aligned(16))) R tab[NK];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int s = blockIdx.x / H, h = blockIdx.x % H;
    const uint32_t b0 = sbase[s], b1 = sbase[s + 1];
    const uint32_t lo = b0 + (uint32_t)((uint64_t)(b1 - b0) * h / H), hi = b0 + (uint32_t)((uint64_t)(b1 - b0) * (h + 1) / H);
    if (lo == hi) return;  // (uniform: nothing of this slice in this part)
    const uint64_t kb = (uint64_t)s << sh.sbits;
    const uint64_t have = std::min<uint64_t>((uint64_t)NK, sh.range - kb);  // records of this slice
    if (have == (uint64_t)NK) {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        const v4u *src = (const v4u *)(rec + kb);
        v4u *dst = (v4u *)tab;
        for (int i = tid; i < kOsSliceBytes / 16; i += kOsPBlock) dst[i] = src[i];
    } else {
        for (int i = tid; i < NK; i += kOsPBlock) tab[i] = (uint64_t)i < have ? rec[kb + i] : (R)0;
    }
    __syncthreads();
    // a wave per chunk, 4 items per lane, kOsPU chunks in flight per wave; the next batch's list entries
    // are read while this batch is looked up
    uint32_t ent[kOsPU];
#pragma unroll
    for (int u = 0; u < kOsPU; ++u) {
        const uint32_t e = lo + wave + u * kOsPWaves;
        ent[u] = e < hi ? list[e] : 0xFFFFFFFFu;
    }
    for (uint32_t e0 = lo + wave; e0 < hi; e0 += kOsPWaves * kOsPU) {
        uint32_t cid[kOsPU], cn[kOsPU];
        uint64_t it[kOsPU];
#pragma unroll
        for (int u = 0; u < kOsPU; ++u) {
            cid[u] = ent[u] & 0xFFFFFFu;
            cn[u] = ent[u] == 0xFFFFFFFFu ? 0u : (ent[u] >> 24) + 1u;
            it[u] = cn[u] ? *(const uint64_t *)(items + (uint64_t)cid[u] * kOsChunk + lane * 4) : 0ull;
        }
#pragma unroll
        for (int u = 0; u < kOsPU; ++u) {
            const uint32_t e = e0 + (uint32_t)(kOsPWaves * kOsPU) + u * kOsPWaves;
            ent[u] = e < hi ? list[e] : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int u = 0; u < kOsPU; ++u) {
            if (!cn[u]) continue;
            uint32_t v[4];
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                const uint32_t idx = lane * 4 + x;
                const uint32_t off = (uint32_t)(it[u] >> (16 * x)) & (uint32_t)(NK - 1);
                const uint32_t rr = idx < cn[u] ? (uint32_t)tab[off] : 0u;
                if (FULL && (rr & VAL) && !(rr & FLAG)) tab[off] = (R)(rr | FLAG);  // (idempotent)
                v[x] = rr & VAL;
            }
            if (sizeof(R) == 2) {
                *(uint64_t *)(items + (uint64_t)cid[u] * kOsChunk + lane * 4) =
                    (uint64_t)v[0] | ((uint64_t)v[1] << 16) | ((uint64_t)v[2] << 32) | ((uint64_t)v[3] << 48);
            } else {
                typedef unsigned int v4u __attribute__((ext_vector_type(4)));
                v4u o4 = {v[0], v[1], v[2], v[3]};
                *(v4u *)(res32 + (uint64_t)cid[u] * kOsChunk + lane * 4) = o4;
            }
        }
    }
    if (FULL) {
        // the matched flags this workgroup set, ORed into the table (the other parts of the slice set
        // theirs in their own LDS copies)
        __syncthreads();
        constexpr uint32_t FM = sizeof(R) == 2 ? 0x80008000u : 0x80000000u;
        const uint32_t *tw = (const uint32_t *)tab;
        uint32_t *gw = (uint32_t *)(rec + kb);
        const uint32_t nw = (uint32_t)((have * sizeof(R) + 3) / 4);
        for (uint32_t i = tid; i < nw; i += kOsPBlock) {
            const uint32_t f = tw[i] & FM;
            if (f) atomicOr(gw + i, f);
        }
    }
}

// ---- phase C ----------------------------------------------------------------------------------------
struct OsOut {
    const int64_t *pcol[3];
    int64_t *pout[3];
    uint64_t *pvalid[3];
    int64_t *bout;
    uint64_t *bvalid;
};

// alias: the probe column that is the key column itself (-1: none) -- copied from the key registers
template <typename R, int KES, int NP>
__global__ __launch_bounds__(kOsBlock) void k_os_emit(ColRef key, OsShape sh, const uint16_t *__restrict__ res16,
                                                      const uint32_t *__restrict__ res32, int64_t vmin, OsOut out,
                                                      int alias) {
    __shared__ OsLds L;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t ntiles = (sh.n + kOsTile - 1) / kOsTile;
    const int64_t t_lo = (int64_t)blockIdx.x * sh.tpw, t_hi = std::min<int64_t>(ntiles, t_lo + sh.tpw);
    os_init(L, tid, blockIdx.x * sh.pool);
    uint32_t my_pos = 0, my_cur = 0;
    int64_t k[kOsR];
    uint32_t vm;
    if (t_lo < t_hi) os_load_keys<KES>(key, sh.n, t_lo * kOsTile, tid, k, vm);
    __syncthreads();
    for (int64_t t = t_lo; t < t_hi; ++t) {
        const int64_t t0 = t * kOsTile;
        int s[kOsR];
        uint32_t o[kOsR], r[kOsR];
        os_rank(L, sh, wave, k, vm, s, o, r);
        int64_t kc[NP > 0 ? kOsR : 1];
#pragma unroll
        for (int q = 0; q < (NP > 0 ? kOsR : 0); ++q) kc[q] = k[q];
        if (t + 1 < t_hi) os_load_keys<KES>(key, sh.n, (t + 1) * kOsTile, tid, k, vm);
        os_barrier();
        uint32_t tc, need, abase;
        os_plan(L, tid, sh.F, my_pos, tc, need, abase);
        uint32_t p[kOsR] = {};
#pragma unroll
        for (int q = 0; q < kOsR; ++q)
            if (s[q] >= 0) {
                uint32_t dst;
                os_place(L, wave, s[q], r[q], p[q], dst);
                L.stage[p[q]] = dst;
            }
        // FULL's probe columns: loaded here, so their latency overlaps the result gather below
        int64_t pv[kOsR][NP > 0 ? NP : 1];
#pragma unroll
        for (int q = 0; q < kOsR; ++q)
#pragma unroll
            for (int c = 0; c < NP; ++c) {
                const int64_t row = t0 + (int64_t)q * kOsBlock + tid;
                pv[q][c] = c == alias ? kc[q] : row < sh.n ? __builtin_nontemporal_load(out.pcol[c] + row) : 0;
            }
        os_barrier();
        // the tile's results, run by run, into its staged positions
        const uint32_t tot = os_tile_total(L);
        for (uint32_t i = 2 * tid; i < tot; i += 2 * kOsBlock) {
            const uint2 d = *(const uint2 *)&L.stage[i];
            uint2 v;
            if (sizeof(R) == 2 && i + 1 < tot && d.y == d.x + 1 && !(d.x & 1u)) {
                const uint32_t w = *(const uint32_t *)(res16 + d.x);  // two neighbours of one run in one load
                v = make_uint2(w & 0xFFFFu, w >> 16);
            } else {
                v.x = sizeof(R) == 2 ? (uint32_t)res16[d.x] : res32[d.x];
                v.y = i + 1 < tot ? (sizeof(R) == 2 ? (uint32_t)res16[d.y] : res32[d.y]) : 0u;
            }
            *(uint2 *)&L.stage[i] = v;
        }
        os_advance(L, tid, sh.F, my_pos, my_cur, tc, abase);
        os_barrier();
#pragma unroll
        for (int q = 0; q < kOsR; ++q) {
            const int64_t row = t0 + (int64_t)q * kOsBlock + tid;
            const uint32_t v = s[q] >= 0 ? L.stage[p[q]] : 0u;
            const bool hit = v != 0;
            const uint64_t mask = __ballot(hit), rows = __ballot(row < sh.n);
            if (row < sh.n) {
                __builtin_nontemporal_store(hit ? vmin + (int64_t)v - 1 : (int64_t)0, out.bout + row);
#pragma unroll
                for (int c = 0; c < NP; ++c) __builtin_nontemporal_store(pv[q][c], out.pout[c] + row);
            }
            if (lane == 0 && row < sh.n) {
                out.bvalid[row >> 6] = mask;
#pragma unroll
                for (int c = 0; c < NP; ++c) out.pvalid[c][row >> 6] = rows;
            }
        }
        // (the next tile's ranking writes only the counters, cleared before the barrier above; the
        // staged results are read before the next tile's placement, two barriers later)
    }
}

// ---- host --------------------------------------------------------------------------------------------
// The chunks of a pool grouped by tag (k_os_list_count + k_os_list_fill): sbase[0..F] the tags' list
// ranges, list[] entries chunk id | (item count - 1) << 24.  Chunk ids < 2^24, F <= kOsMaxF.
size_t chunk_lists_work_words(int F) { return (size_t)kOsLGrid * F + F; }

int chunk_lists(qeh_ctx *ctx, const uint16_t *tag, const uint16_t *ccnt, uint64_t nchunks, int F, uint32_t *sbase,
                uint32_t *list, uint32_t *work) {
    if (F <= 0 || F > kOsMaxF || nchunks >= (1ull << 24)) return fail(QEH_E_INVALID, "chunk_lists: shape");
    uint32_t *wg_hist = work, *scount = wg_hist + (size_t)kOsLGrid * F;
    QEH_HIP(hipMemsetAsync(scount, 0, F * 4, ctx->stream));
    hipLaunchKernelGGL(k_os_list_count, dim3(kOsLGrid), dim3(kOsLBlock), 0, ctx->stream, tag, nchunks, F, wg_hist, scount);
    hipLaunchKernelGGL(k_os_list_fill, dim3(kOsLGrid), dim3(kOsLBlock), 0, ctx->stream, tag, nchunks, F, wg_hist, scount,
                       sbase, ccnt, list);
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}

int outer_slice_probe(qeh_ctx *ctx, const qeh_column &pk, void *rec, int rw, int64_t kmin, uint64_t range, int64_t vmin,
                      bool full, int np, const int64_t *const *pcol, int64_t *const *pout, uint64_t *const *pvalid,
                      int64_t *bout, uint64_t *bvalid) {
    const int64_t n = pk.length;
    if (std::getenv("QEH_NO_OUTER_SLICE")) return kOuterSliceNotEligible;
    const bool force = std::getenv("QEH_OUTER_SLICE") != nullptr;
    if ((rw != 2 && rw != 4) || np < 0 || np > 3 || (!full && np != 0)) return kOuterSliceNotEligible;
    if (pk.dtype != QEH_DT_INT64 && pk.dtype != QEH_DT_INT32) return kOuterSliceNotEligible;
    const int sbits = rw == 2 ? 16 : 15;
    const uint64_t F = (range + (1ull << sbits) - 1) >> sbits;
    if (n <= 0 || F == 0 || F > (uint64_t)kOsMaxF) return kOuterSliceNotEligible;
    // a table an XCD's L2 mostly holds is probed faster in one pass
    if (!force && (range * (uint64_t)rw < (8ull << 20) || n < (1 << 22))) return kOuterSliceNotEligible;
    if (!lds_atomic_rank_ok(ctx)) return kOuterSliceNotEligible;
    const int cus = ctx->props.multiProcessorCount;
    const int64_t ntiles = (n + kOsTile - 1) / kOsTile;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(2 * (int64_t)cus, ntiles));
    const int64_t tpw = (ntiles + grid - 1) / grid;
    const uint64_t pool = (uint64_t)tpw * (kOsTile / kOsChunk) + F;
    const uint64_t nchunks = pool * (uint64_t)grid;
    if (nchunks * kOsChunk >= (1ull << 32)) return kOuterSliceNotEligible;
    DevBuf items, res32, tag, ccnt, list, lwork;
    // (no room for the pool: the single-pass probe needs none)
    const size_t lw_words = chunk_lists_work_words((int)F) + F + 1;  // the list passes' scratch, slice bases
    if (items.alloc(ctx, nchunks * kOsChunk * 2) != QEH_OK || tag.alloc(ctx, nchunks * 2 + 16) != QEH_OK ||
        ccnt.alloc(ctx, nchunks * 2 + 16) != QEH_OK || list.alloc(ctx, nchunks * 4) != QEH_OK ||
        lwork.alloc(ctx, lw_words * 4) != QEH_OK ||
        (rw == 4 && res32.alloc(ctx, nchunks * kOsChunk * 4) != QEH_OK))
        return kOuterSliceNotEligible;
    uint32_t *sbase = lwork.as<uint32_t>() + chunk_lists_work_words((int)F);
    QEH_HIP(hipMemsetAsync(tag.p, 0xFF, nchunks * 2 + 16, ctx->stream));
    KernelTimer kt(ctx, "outer_slice");
    OsShape sh{n, kmin, range, sbits, (int32_t)F, tpw, (uint32_t)pool};
    const ColRef kr = make_colref(pk);
    const bool k8 = pk.dtype == QEH_DT_INT64;
    hipLaunchKernelGGL(k8 ? k_os_part<8> : k_os_part<4>, dim3(grid), dim3(kOsBlock), 0, ctx->stream, kr, sh,
                       items.as<uint16_t>(), tag.as<uint16_t>(), ccnt.as<uint16_t>());
    QEH_TRY(chunk_lists(ctx, tag.as<uint16_t>(), ccnt.as<uint16_t>(), nchunks, (int)F, sbase, list.as<uint32_t>(),
                        lwork.as<uint32_t>()));
    // phase B: about three rounds of workgroups (one per CU: the slice takes 128 KB of LDS) over the slices,
    // each slice's chunk list split evenly among its H workgroups
    const int H = (int)std::max<int64_t>(1, 3 * (int64_t)cus / (int64_t)F);
    auto probe = [&](auto rt) {
        typedef decltype(rt) R;
        auto kern = full ? k_os_probe<R, true> : k_os_probe<R, false>;
        hipLaunchKernelGGL(kern, dim3((unsigned)(F * H)), dim3(kOsPBlock), 0, ctx->stream, sh, H, sbase,
                           list.as<uint32_t>(), items.as<uint16_t>(), res32.as<uint32_t>(), (R *)rec);
    };
    if (rw == 2) probe(uint16_t{});
    else probe(uint32_t{});
    OsOut o{};
    for (int c = 0; c < np; ++c) o.pcol[c] = pcol[c], o.pout[c] = pout[c], o.pvalid[c] = pvalid[c];
    // a probe column that is the (non-null Int64) key itself is copied from the key read
    int alias = -1;
    for (int c = 0; c < np && alias < 0; ++c)
        if (k8 && !pk.validity && pcol[c] == (const int64_t *)pk.values + pk.offset) alias = c;
    o.bout = bout;
    o.bvalid = bvalid;
    auto emit = [&](auto rt, auto kes) {
        typedef decltype(rt) R;
        constexpr int KES = decltype(kes)::value;
        auto kern = np == 0 ? k_os_emit<R, KES, 0> : np == 1 ? k_os_emit<R, KES, 1> : np == 2 ? k_os_emit<R, KES, 2>
                                                                                          : k_os_emit<R, KES, 3>;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kOsBlock), 0, ctx->stream, kr, sh, items.as<uint16_t>(),
                           res32.as<uint32_t>(), vmin, o, alias);
    };
    if (rw == 2) {
        if (k8) emit(uint16_t{}, std::integral_constant<int, 8>{});
        else emit(uint16_t{}, std::integral_constant<int, 4>{});
    } else {
        if (k8) emit(uint32_t{}, std::integral_constant<int, 8>{});
        else emit(uint32_t{}, std::integral_constant<int, 4>{});
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(QEH_E_HIP, std::string("outer join (slices): ") + hipGetErrorString(e));
    // the buffers go back to the pool only after the kernels that use them have run
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    return QEH_OK;
}

}  // namespace qeh
