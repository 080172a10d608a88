// Window functions over one PARTITION BY key of at most 2^20 distinct consecutive values and one
// ORDER BY key, by three levels of 512-way partitioning with whole-chunk writes (BASELINE config 5:
// ROW_NUMBER() OVER (PARTITION BY k ORDER BY v), k in [0, 2^20), 1e9 rows).
//
// Semantics as qeh_row_number / qeh_window (k_sort.hip): rows numbered 1.. within each partition in
// ORDER BY order, ties by input position (docs/WINDOW_FUNCTIONS.md:44-65); RANK with gaps, NTILE's
// first size % n buckets one row larger (:67-140); output aligned to input order.
//
// The key k is folded to 20 bits (k mod 2^20: one-to-one over any range of <= 2^20 keys, checked from
// the min / max level 1 takes in the same read) and mixed by a bijection h of 20 bits, so the digits
// split the rows evenly whatever the key range: level 1 partitions by h >> 11 (512 ways), level 2 by
// the next 11 - sb bits, and a level-3 "sub-bucket" holds the rows of 2^sb PARTITION BY groups
// (sb = 2 at 1e9 rows: ~3.8 K rows, 4 groups):
//   L1 (k_w3_l1): per workgroup span of the input, a stable 512-way partition of (order key, h's low
//      11 bits) into regions (workgroup, digit) of fixed capacity; the digit also goes out in input
//      order (2 B) for the inverse pass.
//   L2 (k_w3_l2): a workgroup per level-1 digit reads that digit's regions in workgroup order (=
//      input order) and partitions them stably by the level-2 digit into sub-bucket regions: (order
//      key, sub-key byte).
//   L3 (k_w3_l3): a workgroup per sub-bucket ranks its rows by counting sort on (sub-key, top bits of
//      the order key), each row ranking itself exactly among its bucket's rows by (order key, position
//      in the sub-bucket = input order), and writes the function's value at the row's own position.
//   inverse L2 / inverse L1 (k_w3_il2 / k_w3_il1): both partitions are replayed (the ranking is
//      deterministic) and the results gathered back run by run: sub-bucket order -> level-1 order ->
//      input order (Int64 out).
// Both forward levels write every output stream in whole 64-B chunks: a digit's items are staged
// sorted, whole chunks go out, and the < chunk leftovers are carried in LDS to the next tile -- the
// 1024-way passes of k_window.hip wrote 8-row runs as partial sectors (2.5e8 partial-sector writes
// for 10 GB of runs).  Bytes per row: 16 read + 12 written (L1), 10 + 9 (L2), 9 + 2 (L3),
// 4 + 2 (inverse L2), 4 + 8 (inverse L1).
// Shapes outside it (a key range above 2^20, a region or sub-bucket over capacity -- heavy keys --,
// many equal order keys in one bucket, value functions, DENSE_RANK) return kWindowMsdNotEligible and
// the caller takes the k_window.hip pipeline.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "../../include/qeh_plan.h"
#include "device_common.h"
#include "ops.h"

namespace qeh {

constexpr int kW3Block = 1024;
constexpr int kW3Waves = kW3Block / 64;
constexpr int kW3Tile = 4096;                  // rows per partition tile
constexpr int kW3NJ = kW3Tile / kW3Block;      // rows per thread and tile
constexpr int kW3Dig = 512;                    // digits per level (9 bits)
constexpr int kW3CV = 8;                       // order-key chunk: 8 rows = 64 B
constexpr int kW3CK = 32;                      // level-1 key-bits chunk (u16): 64 B
constexpr int kW3CS = 64;                      // level-2 sub-key chunk (u8): 64 B
constexpr int kW3MaxCap2 = 8192;               // rows a sub-bucket may hold (L3's LDS)
constexpr int kW3E = kW3MaxCap2 / kW3Block;    // rows per L3 thread
constexpr int kW3Buckets = 8192;               // L3 counting-sort buckets (groups x 2^(13 - group bits))
constexpr uint32_t kW3BucketCap = 64;          // most rows one L3 bucket may hold (else: the other path)

// flags[0]: L1 region overflow, [1]: L2 sub-bucket overflow, [2]: an L3 bucket above kW3BucketCap
struct W3MinMax {
    int64_t mn, mx;
};

struct W3Shape {
    int64_t n;
    int64_t span;   // rows per level-1 workgroup (multiple of kW3Tile)
    int32_t g1;     // level-1 workgroups (= regions per level-1 digit)
    int32_t sb;     // sub-key bits handled by L3 (2..8); the level-2 digit is (h & 2047) >> sb
    uint32_t cap1;  // items per level-1 region (multiple of 64)
    uint32_t cap2;  // items per sub-bucket (multiple of 64, <= kW3MaxCap2)
};

__device__ __forceinline__ void w3_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// A bijection of 20 bits (odd multipliers and xorshifts modulo 2^20): equal keys share a digit path,
// distinct keys (of one 2^20 window) never do, and a narrow or clustered key range still fills all
// 512 digits of each level.
__host__ __device__ __forceinline__ uint32_t w3_hash(uint32_t x) {
    x &= 0xFFFFFu;
    x = (x * 0x9E3B5u) & 0xFFFFFu;
    x ^= x >> 11;
    x = (x * 0x5BD1Fu) & 0xFFFFFu;
    x ^= x >> 9;
    return x;
}

template <int ES>
__device__ __forceinline__ uint64_t w3_ld(const void *p, int64_t i) {
    if constexpr (ES == 4) return (uint64_t)__builtin_nontemporal_load((const uint32_t *)p + i);
    else return __builtin_nontemporal_load((const uint64_t *)p + i);
}
// order key as an unsigned integer whose order is the ORDER BY order (floats by totalOrder)
__device__ __forceinline__ uint64_t w3_order_bits(uint64_t raw, int dtype, int asc) {
    int64_t o;
    if (dtype == QEH_DT_INT32) o = (int64_t)(int32_t)(uint32_t)raw;
    else if (dtype == QEH_DT_FLOAT32) o = f64_order_key((double)__builtin_bit_cast(float, (uint32_t)raw));
    else if (dtype == QEH_DT_FLOAT64) o = f64_order_key(as_f64((int64_t)raw));
    else o = (int64_t)raw;
    const uint64_t u = (uint64_t)o ^ 0x8000000000000000ull;
    return asc ? u : ~u;
}

// ---- stable tile ranking by 512 digits ---------------------------------------------------------
// Tile rows are wave-contiguous (row = wave * 64 NJ + j * 64 + lane): input order is (wave, j, lane).
// One LDS atomic per row on the wave's packed u16 counters -- ds_add_rtn serves the lanes of one
// instruction that hit one word in lane order (lds_atomic_rank_ok checks exactly that) -- then a
// prefix over the waves: every row's slot in the digit-sorted tile, the same on every replay.
struct W3Rank {
    uint16_t wc[kW3Waves][kW3Dig];  // per-wave digit counts, then per-wave offsets
    uint32_t lofs[kW3Dig];          // digit start in the tile
    uint32_t cnt[kW3Dig];           // digit rows in the tile
    uint32_t wsum[kW3Waves];
};

template <int NJ>
__device__ __forceinline__ void w3_rank(const uint32_t (&d)[NJ], const bool (&live)[NJ], uint32_t (&slot)[NJ], W3Rank &R) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t *wz = (uint32_t *)R.wc[wave];
#pragma unroll
    for (int i = 0; i < kW3Dig / 2 / 64; ++i) wz[lane + 64 * i] = 0u;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint32_t r[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        r[j] = 0u;
        if (live[j]) {
            const uint32_t sh = (d[j] & 1u) * 16u;
            r[j] = (atomicAdd(&wz[d[j] >> 1], 1u << sh) >> sh) & 0xFFFFu;
        }
    }
    w3_barrier();
    uint32_t tot = 0;
    if (tid < kW3Dig) {
#pragma unroll
        for (int w = 0; w < kW3Waves; ++w) {
            const uint32_t c = R.wc[w][tid];
            R.wc[w][tid] = (uint16_t)tot;
            tot += c;
        }
    }
    const uint32_t inc = wave_incl_scan(tot);
    if (lane == 63) R.wsum[wave] = inc;
    w3_barrier();
    if (wave == 0) {
        const uint32_t w = lane < kW3Waves ? R.wsum[lane] : 0u;
        const uint32_t wi = wave_incl_scan(w);
        if (lane < kW3Waves) R.wsum[lane] = wi - w;
    }
    w3_barrier();
    if (tid < kW3Dig) {
        R.lofs[tid] = inc - tot + R.wsum[wave];
        R.cnt[tid] = tot;
    }
    w3_barrier();
#pragma unroll
    for (int j = 0; j < NJ; ++j) slot[j] = live[j] ? R.lofs[d[j]] + R.wc[wave][d[j]] + r[j] : 0u;
}

// A wave's lanes reserve n entries each of a list: one LDS atomic per wave (lanes asking for one word
// serialise), the lanes' offsets from a wave scan.  Wave-uniform call.
__device__ __forceinline__ uint32_t w3_list_base(uint32_t n, uint32_t *counter) {
    const uint32_t inc = wave_incl_scan(n);
    const uint32_t tot = __shfl(inc, 63, 64);
    uint32_t base = 0;
    if ((threadIdx.x & 63) == 63 && tot) base = atomicAdd(counter, tot);
    base = __shfl(base, 63, 64);
    return base + inc - n;
}

// ---- level 1 -------------------------------------------------------------------------------------
struct W3L1Lds {
    W3Rank R;
    uint64_t st_v[kW3Tile];        // staged order keys, digit-sorted
    uint32_t st_h[kW3Tile];        // staged h (digit = h >> 11, key bits = h & 2047)
    uint64_t cv[kW3Dig][kW3CV];    // carried order keys: the item at region position p sits at p % 8
    uint16_t ck[kW3Dig][kW3CK];    // carried key bits: p % 32
    uint32_t A[kW3Dig];            // items assigned to the digit's region so far
    uint32_t vl[kW3Tile / kW3CV + kW3Dig];  // chunks flushed this tile: chunk number << 9 | digit
    uint32_t kl[kW3Tile / kW3CK + kW3Dig];
    uint32_t nvl, nkl;
    int64_t mn[kW3Waves], mx[kW3Waves];
};

template <int KES, int OES>
__global__ __launch_bounds__(kW3Block) void k_w3_l1(ColRef key, ColRef ord, int asc, W3Shape sh,
                                                    uint64_t *__restrict__ v1, uint16_t *__restrict__ kl1,
                                                    uint16_t *__restrict__ d1s, uint32_t *__restrict__ count1,
                                                    uint32_t *__restrict__ flags, W3MinMax *__restrict__ mm) {
    __shared__ W3L1Lds L;
    constexpr int NJ = kW3NJ;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t r0 = (int64_t)blockIdx.x * sh.span, r1 = std::min<int64_t>(sh.n, r0 + sh.span);
    const uint64_t rb = (uint64_t)blockIdx.x * kW3Dig;  // this workgroup's first region
    const uint32_t cap = sh.cap1;
    if (tid < kW3Dig) L.A[tid] = 0u;
    if (tid == 0) L.nvl = L.nkl = 0u;
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    const int woff = wave * 64 * NJ + lane;
    uint64_t kr[NJ], vr[NJ];
    auto load = [&](int64_t t0) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int64_t i = t0 + woff + j * 64;
            const int64_t ii = i < r1 ? i : r0;
            kr[j] = w3_ld<KES>(key.values, ii);
            vr[j] = w3_ld<OES>(ord.values, ii);
        }
    };
    if (r0 < r1) load(r0);
    for (int64_t t0 = r0; t0 < r1; t0 += kW3Tile) {
        uint32_t d[NJ], h[NJ], slot[NJ];
        uint64_t ok[NJ];
        bool live[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int64_t i = t0 + woff + j * 64;
            live[j] = i < r1;
            const int64_t k = KES == 4 ? (int64_t)(int32_t)(uint32_t)kr[j] : (int64_t)kr[j];
            if (live[j]) {
                mn = k < mn ? k : mn;
                mx = k > mx ? k : mx;
            }
            h[j] = w3_hash((uint32_t)k);
            d[j] = h[j] >> 11;
            ok[j] = w3_order_bits(vr[j], ord.dtype, asc);
            if (live[j]) __builtin_nontemporal_store((uint16_t)d[j], d1s + i);
        }
        if (t0 + kW3Tile < r1) load(t0 + kW3Tile);  // in flight across the LDS phases
        w3_rank<NJ>(d, live, slot, L.R);
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            if (live[j]) {
                L.st_v[slot[j]] = ok[j];
                L.st_h[slot[j]] = h[j];
            }
        if (tid < kW3Dig) {  // the digit's whole chunks this tile (positions [a, e) join the region)
            const uint32_t a = L.A[tid], e = a + L.R.cnt[tid];
            if (e > cap) flags[0] = 1u;
            const uint32_t c0 = a / kW3CV, c1 = e / kW3CV;
            uint32_t p = w3_list_base(c1 - c0, &L.nvl);
            for (uint32_t c = c0; c < c1; ++c) L.vl[p++] = (c << 9) | (uint32_t)tid;
            const uint32_t q0 = a / kW3CK, q1 = e / kW3CK;
            p = w3_list_base(q1 - q0, &L.nkl);
            for (uint32_t c = q0; c < q1; ++c) L.kl[p++] = (c << 9) | (uint32_t)tid;
        }
        w3_barrier();
        // whole chunks out: an item below a (assigned before this tile) is a carried one
        {
            const uint32_t nv = L.nvl * kW3CV, nk = L.nkl * kW3CK;
#pragma unroll 4
            for (uint32_t tau = tid; tau < nv; tau += kW3Block) {
                const uint32_t ent = L.vl[tau / kW3CV], dd = ent & 511u;
                const uint32_t p = (ent >> 9) * kW3CV + (tau % kW3CV), a = L.A[dd];
                const uint64_t val = p < a ? L.cv[dd][p % kW3CV] : L.st_v[L.R.lofs[dd] + p - a];
                if (p < cap) __builtin_nontemporal_store(val, v1 + (rb + dd) * cap + p);
            }
#pragma unroll 4
            for (uint32_t tau = tid; tau < nk; tau += kW3Block) {
                const uint32_t ent = L.kl[tau / kW3CK], dd = ent & 511u;
                const uint32_t p = (ent >> 9) * kW3CK + (tau % kW3CK), a = L.A[dd];
                const uint16_t val = p < a ? L.ck[dd][p % kW3CK] : (uint16_t)(L.st_h[L.R.lofs[dd] + p - a] & 2047u);
                if (p < cap) __builtin_nontemporal_store(val, kl1 + (rb + dd) * cap + p);
            }
        }
        w3_barrier();
        // the tile's items past the last whole chunk: carried
        {
            const int m = (int)std::min<int64_t>(kW3Tile, r1 - t0);
#pragma unroll 4
            for (int s = tid; s < m; s += kW3Block) {
                const uint32_t hh = L.st_h[s], dd = hh >> 11;
                const uint32_t a = L.A[dd], e = a + L.R.cnt[dd], p = a + (uint32_t)s - L.R.lofs[dd];
                if (p >= (e & ~(uint32_t)(kW3CV - 1))) L.cv[dd][p % kW3CV] = L.st_v[s];
                if (p >= (e & ~(uint32_t)(kW3CK - 1))) L.ck[dd][p % kW3CK] = (uint16_t)(hh & 2047u);
            }
        }
        w3_barrier();
        if (tid < kW3Dig) L.A[tid] += L.R.cnt[tid];
        if (tid == 0) L.nvl = L.nkl = 0u;
    }
    w3_barrier();
    // the last partial chunks
    for (int tau = tid; tau < kW3Dig * kW3CV; tau += kW3Block) {
        const int dd = tau / kW3CV;
        const uint32_t a = L.A[dd], p = (a & ~(uint32_t)(kW3CV - 1)) + (uint32_t)(tau % kW3CV);
        if (p < a && p < cap) __builtin_nontemporal_store(L.cv[dd][p % kW3CV], v1 + (rb + dd) * cap + p);
    }
    for (int tau = tid; tau < kW3Dig * kW3CK; tau += kW3Block) {
        const int dd = tau / kW3CK;
        const uint32_t a = L.A[dd], p = (a & ~(uint32_t)(kW3CK - 1)) + (uint32_t)(tau % kW3CK);
        if (p < a && p < cap) __builtin_nontemporal_store(L.ck[dd][p % kW3CK], kl1 + (rb + dd) * cap + p);
    }
    if (tid < kW3Dig) count1[rb + tid] = std::min(L.A[tid], cap);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const int64_t a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    if (lane == 0) L.mn[wave] = mn, L.mx[wave] = mx;
    __syncthreads();
    if (tid == 0) {
        for (int w = 0; w < kW3Waves; ++w) mn = L.mn[w] < mn ? L.mn[w] : mn, mx = L.mx[w] > mx ? L.mx[w] : mx;
        mm[blockIdx.x] = W3MinMax{mn, mx};
    }
}

// ---- level 2 -------------------------------------------------------------------------------------
// The rows of level-1 digit d1 are its g1 regions in workgroup order; each region is taken in tiles of
// kW3Tile rows (its last one partial), so the replay in k_w3_il2 cuts the same tiles.
struct W3Cursor {  // the tile at row t0 of region w
    int w;
    uint32_t t0;
};
__device__ __forceinline__ W3Cursor w3_skip_empty(W3Cursor c, const uint32_t *rc, int g1) {
    while (c.w < g1 && c.t0 >= rc[c.w]) c.w++, c.t0 = 0;
    return c;
}

struct W3L2Lds {
    W3Rank R;
    uint64_t st_v[kW3Tile];
    uint16_t st_k[kW3Tile];        // staged key bits (digit = k >> sb, sub-key = k & (2^sb - 1))
    uint64_t cv[kW3Dig][kW3CV];
    uint8_t cs[kW3Dig][kW3CS];     // carried sub-keys: p % 64
    uint32_t A[kW3Dig];
    uint32_t vl[kW3Tile / kW3CV + kW3Dig];
    uint32_t sl[kW3Tile / kW3CS + kW3Dig];
    uint32_t rc[kW3Dig];           // the level-1 regions' row counts (g1 <= 512)
    uint32_t nvl, nsl;
};

__global__ __launch_bounds__(kW3Block) void k_w3_l2(W3Shape sh, const uint64_t *__restrict__ v1,
                                                    const uint16_t *__restrict__ kl1, const uint32_t *__restrict__ count1,
                                                    uint64_t *__restrict__ v2, uint8_t *__restrict__ s2,
                                                    uint32_t *__restrict__ count2, uint32_t *__restrict__ flags) {
    __shared__ W3L2Lds L;
    constexpr int NJ = kW3NJ;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int d1 = blockIdx.x, g1 = sh.g1, sbits = sh.sb;
    const int nd2 = 1 << (11 - sbits);
    const uint32_t smask = (1u << sbits) - 1u, cap = sh.cap2;
    const uint64_t ob = (uint64_t)d1 * nd2;  // this digit's first sub-bucket
    if (tid < kW3Dig) L.A[tid] = 0u;
    if (tid < g1) L.rc[tid] = count1[(uint64_t)tid * kW3Dig + d1];
    if (tid == 0) L.nvl = L.nsl = 0u;
    __syncthreads();
    const int woff = wave * 64 * NJ + lane;
    uint64_t vr[NJ];
    uint32_t kr[NJ];
    auto load = [&](W3Cursor c) {
        const uint64_t base = ((uint64_t)c.w * kW3Dig + d1) * sh.cap1 + c.t0;
        const uint32_t m = L.rc[c.w] - c.t0;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const uint32_t i = (uint32_t)(woff + j * 64);
            const uint64_t ii = base + (i < m ? i : 0u);
            vr[j] = __builtin_nontemporal_load(v1 + ii);
            kr[j] = __builtin_nontemporal_load(kl1 + ii);
        }
    };
    W3Cursor cur = w3_skip_empty(W3Cursor{0, 0u}, L.rc, g1);
    if (cur.w < g1) load(cur);
    while (cur.w < g1) {
        const uint32_t m = std::min<uint32_t>(kW3Tile, L.rc[cur.w] - cur.t0);
        uint32_t d[NJ], slot[NJ];
        uint64_t ok[NJ];
        uint32_t kk[NJ];
        bool live[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            live[j] = (uint32_t)(woff + j * 64) < m;
            ok[j] = vr[j];
            kk[j] = kr[j];
            d[j] = kk[j] >> sbits;
        }
        const W3Cursor nx = w3_skip_empty(W3Cursor{cur.w, cur.t0 + kW3Tile}, L.rc, g1);
        if (nx.w < g1) load(nx);
        w3_rank<NJ>(d, live, slot, L.R);
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            if (live[j]) {
                L.st_v[slot[j]] = ok[j];
                L.st_k[slot[j]] = (uint16_t)kk[j];
            }
        if (tid < kW3Dig) {  // (digits >= nd2 hold no rows)
            const uint32_t a = L.A[tid], e = a + L.R.cnt[tid];
            if (e > cap) flags[1] = 1u;
            const uint32_t c0 = a / kW3CV, c1 = e / kW3CV;
            uint32_t p = w3_list_base(c1 - c0, &L.nvl);
            for (uint32_t c = c0; c < c1; ++c) L.vl[p++] = (c << 9) | (uint32_t)tid;
            const uint32_t q0 = a / kW3CS, q1 = e / kW3CS;
            p = w3_list_base(q1 - q0, &L.nsl);
            for (uint32_t c = q0; c < q1; ++c) L.sl[p++] = (c << 9) | (uint32_t)tid;
        }
        w3_barrier();
        {
            const uint32_t nv = L.nvl * kW3CV, ns = L.nsl * kW3CS;
#pragma unroll 4
            for (uint32_t tau = tid; tau < nv; tau += kW3Block) {
                const uint32_t ent = L.vl[tau / kW3CV], dd = ent & 511u;
                const uint32_t p = (ent >> 9) * kW3CV + (tau % kW3CV), a = L.A[dd];
                const uint64_t val = p < a ? L.cv[dd][p % kW3CV] : L.st_v[L.R.lofs[dd] + p - a];
                if (p < cap) __builtin_nontemporal_store(val, v2 + (ob + dd) * cap + p);
            }
#pragma unroll 4
            for (uint32_t tau = tid; tau < ns; tau += kW3Block) {
                const uint32_t ent = L.sl[tau / kW3CS], dd = ent & 511u;
                const uint32_t p = (ent >> 9) * kW3CS + (tau % kW3CS), a = L.A[dd];
                const uint8_t val = p < a ? L.cs[dd][p % kW3CS] : (uint8_t)(L.st_k[L.R.lofs[dd] + p - a] & smask);
                if (p < cap) __builtin_nontemporal_store(val, s2 + (ob + dd) * cap + p);
            }
        }
        w3_barrier();
#pragma unroll 4
        for (int s = tid; s < (int)m; s += kW3Block) {
            const uint32_t kb = L.st_k[s], dd = kb >> sbits;
            const uint32_t a = L.A[dd], e = a + L.R.cnt[dd], p = a + (uint32_t)s - L.R.lofs[dd];
            if (p >= (e & ~(uint32_t)(kW3CV - 1))) L.cv[dd][p % kW3CV] = L.st_v[s];
            if (p >= (e & ~(uint32_t)(kW3CS - 1))) L.cs[dd][p % kW3CS] = (uint8_t)(kb & smask);
        }
        w3_barrier();
        if (tid < kW3Dig) L.A[tid] += L.R.cnt[tid];
        if (tid == 0) L.nvl = L.nsl = 0u;
        cur = nx;
    }
    w3_barrier();
    for (int tau = tid; tau < nd2 * kW3CV; tau += kW3Block) {
        const int dd = tau / kW3CV;
        const uint32_t a = L.A[dd], p = (a & ~(uint32_t)(kW3CV - 1)) + (uint32_t)(tau % kW3CV);
        if (p < a && p < cap) __builtin_nontemporal_store(L.cv[dd][p % kW3CV], v2 + (ob + dd) * cap + p);
    }
    for (int tau = tid; tau < nd2 * kW3CS; tau += kW3Block) {
        const int dd = tau / kW3CS;
        const uint32_t a = L.A[dd], p = (a & ~(uint32_t)(kW3CS - 1)) + (uint32_t)(tau % kW3CS);
        if (p < a && p < cap) __builtin_nontemporal_store(L.cs[dd][p % kW3CS], s2 + (ob + dd) * cap + p);
    }
    if (tid < nd2) count2[ob + tid] = std::min(L.A[tid], cap);
}

// ---- level 3: the sort ---------------------------------------------------------------------------
// Counting sort over (sub-key, top bits of (order key - the sub-bucket's minimum)): 2^13 buckets of
// 16-bit counters packed in LDS, rows placed by bucket start + arrival with their keys and positions
// at that slot, then each row ranks itself exactly among its bucket's rows by (order key, position).
// A bucket above kW3BucketCap rows (many equal order keys) sets flags[2]: the other path takes the job.
struct W3L3Lds {
    uint32_t cnt[kW3Buckets / 2];   // packed counters -> starts
    uint64_t sv[kW3MaxCap2];        // order keys by slot
    uint16_t sp[kW3MaxCap2];        // positions by slot
    uint32_t ws[kW3Waves];
    uint64_t wmn[kW3Waves], wmx[kW3Waves];
    uint32_t wmax[kW3Waves];
    uint16_t gmap[256];             // sub-key -> dense group number (sb >= 4)
};

template <int FN>
__global__ __launch_bounds__(kW3Block) void k_w3_l3(W3Shape sh, int nsub, const uint64_t *__restrict__ v2,
                                                    const uint8_t *__restrict__ s2, const uint32_t *__restrict__ count2,
                                                    uint16_t *__restrict__ res3, uint32_t *__restrict__ flags,
                                                    int64_t param) {
    __shared__ W3L3Lds L;
    // thread t holds the sub-bucket's row pairs 2048 q + 2t, + 1 (q < E / 2): every wave has rows
    constexpr int E = kW3E;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const bool remap = sh.sb >= 4;
    auto row = [&](int r) -> uint32_t { return (uint32_t)((r >> 1) * 2 * kW3Block + 2 * t + (r & 1)); };
    typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
    v2u64 vn[E / 2];
    uint64_t sn = 0;  // sub-keys, a byte per row
    uint32_t mnext = 0;
    auto issue = [&](int j) {
        mnext = count2[j];
        const uint64_t base = (uint64_t)j * sh.cap2;  // (pairs never straddle the even capacity)
        sn = 0;
#pragma unroll
        for (int q = 0; q < E / 2; ++q) {
            const uint32_t i = row(2 * q);
            if (i < mnext) {
                vn[q] = __builtin_nontemporal_load((const v2u64 *)(v2 + base + i));
                sn |= (uint64_t)__builtin_nontemporal_load((const uint16_t *)(s2 + base + i)) << (16 * q);
            }
        }
    };
    if ((int)blockIdx.x < nsub) issue(blockIdx.x);
    for (int j = blockIdx.x; j < nsub; j += gridDim.x) {
        const uint32_t m = mnext;
        uint64_t v[E];
#pragma unroll
        for (int q = 0; q < E / 2; ++q) v[2 * q] = vn[q][0], v[2 * q + 1] = vn[q][1];
        const uint64_t su8 = sn;
        const bool more = j + (int)gridDim.x < nsub;
        if (m == 0) {  // (uniform)
            if (more) issue(j + gridDim.x);
            continue;
        }
        const uint64_t base = (uint64_t)j * sh.cap2;
        uint64_t mn = ~0ull, mx = 0ull;
#pragma unroll
        for (int r = 0; r < E; ++r)
            if (row(r) < m) mn = v[r] < mn ? v[r] : mn, mx = v[r] > mx ? v[r] : mx;
#pragma unroll
        for (int q = 0; q < kW3Buckets / 2 / kW3Block; ++q) L.cnt[q * kW3Block + t] = 0u;
        if (remap && t < 256) L.gmap[t] = 0u;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const uint64_t a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
            mn = a < mn ? a : mn;
            mx = b > mx ? b : mx;
        }
        if (lane == 0) L.wmn[wave] = mn, L.wmx[wave] = mx;
        w3_barrier();
#pragma unroll
        for (int w = 0; w < kW3Waves; ++w) mn = L.wmn[w] < mn ? L.wmn[w] : mn, mx = L.wmx[w] > mx ? L.wmx[w] : mx;
        const uint64_t span = mx - mn;
        const int bits = span ? 64 - __clzll((long long)span) : 0;
        // With many sub-keys (small inputs: up to 256 groups per sub-bucket) most of them may be absent --
        // a narrow key range -- so the present ones are numbered densely and each group's share of the
        // 2^13 buckets follows the groups actually there (a group of 300 rows would otherwise get 32).
        int gbits = sh.sb;
        uint64_t gk8 = su8;  // group numbers, a byte per row
        if (remap) {
#pragma unroll
            for (int r = 0; r < E; ++r)
                if (row(r) < m) L.gmap[(su8 >> (8 * r)) & 0xFFu] = 1u;
            w3_barrier();
            const uint32_t g = t < (1 << sh.sb) ? L.gmap[t] : 0u;
            const uint32_t inc = wave_incl_scan(g);
            if (lane == 63) L.ws[wave] = inc;
            w3_barrier();
            uint32_t pre = 0, total = 0;
#pragma unroll
            for (int w2 = 0; w2 < 4; ++w2) pre += w2 < wave ? L.ws[w2] : 0u, total += L.ws[w2];
            if (t < (1 << sh.sb)) L.gmap[t] = (uint16_t)(inc - g + pre);
            w3_barrier();
            gbits = total > 1 ? 32 - __clz((int)(total - 1)) : 0;
            uint32_t lo = (uint32_t)su8, hi = (uint32_t)(su8 >> 32);
            asm volatile("" : "+v"(lo), "+v"(hi));  // (no address kept live from the marking loop)
            uint32_t nlo = 0, nhi = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                nlo |= (uint32_t)L.gmap[(lo >> (8 * r)) & 0xFFu] << (8 * r);
                nhi |= (uint32_t)L.gmap[(hi >> (8 * r)) & 0xFFu] << (8 * r);
            }
            gk8 = (uint64_t)nlo | ((uint64_t)nhi << 32);
        }
        const int B = 13 - gbits;  // bucket bits per group
        const int shift = bits > B ? bits - B : 0;
        uint32_t ba[E];  // bucket | arrival << 16
#pragma unroll
        for (int r = 0; r < E; ++r) {
            ba[r] = 0u;
            if (row(r) < m) {
                const uint32_t su = (uint32_t)(gk8 >> (8 * r)) & 0xFFu;
                const uint32_t bk = (su << B) | (uint32_t)((v[r] - mn) >> shift);
                const uint32_t s16 = (bk & 1u) * 16u;
                ba[r] = bk | (((atomicAdd(&L.cnt[bk >> 1], 1u << s16) >> s16) & 0xFFFFu) << 16);
            }
        }
        w3_barrier();
        {  // exclusive scan of the 8192 counters: thread t owns words 4t .. 4t + 3
            uint32_t w[4], tot = 0, big = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                w[q] = L.cnt[4 * t + q];
                const uint32_t lo = w[q] & 0xFFFFu, hi = w[q] >> 16;
                tot += lo + hi;
                big = std::max(big, std::max(lo, hi));
            }
            const uint32_t incl = wave_incl_scan(tot);
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) big = std::max(big, (uint32_t)__shfl_xor((int)big, o, 64));
            if (lane == 63) L.ws[wave] = incl;
            if (lane == 0) L.wmax[wave] = big;
            w3_barrier();
            uint32_t run = incl - tot;
#pragma unroll
            for (int w2 = 0; w2 < kW3Waves; ++w2) run += w2 < wave ? L.ws[w2] : 0u;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t lo = w[q] & 0xFFFFu, hi = w[q] >> 16;
                L.cnt[4 * t + q] = run | ((run + lo) << 16);
                run += lo + hi;
            }
        }
        w3_barrier();
        uint32_t maxc = 0;
#pragma unroll
        for (int w = 0; w < kW3Waves; ++w) maxc = std::max(maxc, L.wmax[w]);
        if (maxc > kW3BucketCap) {  // (uniform) many equal order keys: the other path
            if (t == 0) flags[2] = 1u;
            if (more) issue(j + gridDim.x);
            w3_barrier();
            continue;
        }
        auto start_of = [&](uint32_t b) -> uint32_t {
            return b < (uint32_t)kW3Buckets ? (L.cnt[b >> 1] >> ((b & 1u) * 16u)) & 0xFFFFu : m;
        };
#pragma unroll
        for (int r = 0; r < E; ++r) {
            if (row(r) < m) {
                const uint32_t slot = start_of(ba[r] & 0xFFFFu) + (ba[r] >> 16);
                L.sv[slot] = v[r];
                L.sp[slot] = (uint16_t)row(r);
            }
        }
        // the order keys now sit in LDS: the next sub-bucket's loads go out (in flight over the ranking)
        if (more) issue(j + gridDim.x);
        w3_barrier();
        // row by row: its rank among its bucket's rows (a handful on average), the function's value
        uint32_t res2[E / 2];
#pragma unroll
        for (int r = 0; r < E / 2; ++r) res2[r] = 0u;
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const uint32_t i = row(r);
            if (i >= m) continue;
            const uint32_t bk = ba[r] & 0xFFFFu, su = bk >> B;
            const uint32_t st = start_of(bk), en = start_of(bk + 1);
            const uint64_t vme = L.sv[st + (ba[r] >> 16)];
            uint32_t rank = 0;
            for (uint32_t q = st; q < en; ++q) {
                const uint64_t ov = L.sv[q];
                if constexpr (FN == QEH_WIN_RANK) rank += ov < vme ? 1u : 0u;
                else rank += (ov < vme || (ov == vme && (uint32_t)L.sp[q] < i)) ? 1u : 0u;
            }
        const uint32_t gs = start_of(su << B);  // the group's first sorted index
            const uint32_t idx = st + rank - gs;
            uint32_t res;
            if constexpr (FN == QEH_WIN_NTILE) {
                const int64_t mg = (int64_t)start_of((su + 1) << B) - gs;
                const int64_t qq = mg / param, rm = mg % param, r0 = idx;
                res = (uint32_t)(r0 < rm * (qq + 1) ? r0 / (qq + 1) + 1 : rm + (r0 - rm * (qq + 1)) / (qq > 0 ? qq : 1) + 1);
            } else {
                res = idx + 1u;
            }
            res2[r / 2] |= (res & 0xFFFFu) << (16 * (r % 2));
        }
#pragma unroll
        for (int q = 0; q < E / 2; ++q)  // a 4-B store per row pair
            if (row(2 * q) < m) __builtin_nontemporal_store(res2[q], (uint32_t *)(res3 + base + row(2 * q)));
        w3_barrier();  // every LDS read of this sub-bucket is done before the next one's writes
    }
}

// ---- inverse passes --------------------------------------------------------------------------------
struct W3InvLds {
    W3Rank R;
    uint16_t st_d[kW3Tile];
    uint16_t st_r[kW3Tile];
    uint32_t A[kW3Dig];
    uint32_t rc[kW3Dig];
};

// inverse of level 2: replay digit d1's tiles, gather the results run by run from the sub-buckets,
// write them at the rows' level-1 region positions
__global__ __launch_bounds__(kW3Block) __attribute__((amdgpu_waves_per_eu(8))) void k_w3_il2(
    W3Shape sh, const uint16_t *__restrict__ kl1, const uint32_t *__restrict__ count1, const uint16_t *__restrict__ res3,
    uint16_t *__restrict__ res2) {
    __shared__ W3InvLds L;
    constexpr int NJ = kW3NJ;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int d1 = blockIdx.x, g1 = sh.g1, sbits = sh.sb;
    const uint64_t ob = (uint64_t)d1 * (1u << (11 - sbits));
    const uint32_t cap2 = sh.cap2;
    if (tid < kW3Dig) L.A[tid] = 0u;
    if (tid < g1) L.rc[tid] = count1[(uint64_t)tid * kW3Dig + d1];
    __syncthreads();
    const int woff = wave * 64 * NJ + lane;
    uint32_t kr[NJ];
    auto load = [&](W3Cursor c) {
        const uint64_t base = ((uint64_t)c.w * kW3Dig + d1) * sh.cap1 + c.t0;
        const uint32_t m = L.rc[c.w] - c.t0;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const uint32_t i = (uint32_t)(woff + j * 64);
            kr[j] = __builtin_nontemporal_load(kl1 + base + (i < m ? i : 0u));
        }
    };
    W3Cursor cur = w3_skip_empty(W3Cursor{0, 0u}, L.rc, g1);
    if (cur.w < g1) load(cur);
    while (cur.w < g1) {
        const uint32_t m = std::min<uint32_t>(kW3Tile, L.rc[cur.w] - cur.t0);
        const uint64_t obase = ((uint64_t)cur.w * kW3Dig + d1) * sh.cap1 + cur.t0;
        uint32_t d[NJ], slot[NJ];
        bool live[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            live[j] = (uint32_t)(woff + j * 64) < m;
            d[j] = kr[j] >> sbits;
        }
        const W3Cursor nx = w3_skip_empty(W3Cursor{cur.w, cur.t0 + kW3Tile}, L.rc, g1);
        if (nx.w < g1) load(nx);
        w3_rank<NJ>(d, live, slot, L.R);
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            if (live[j]) L.st_d[slot[j]] = (uint16_t)d[j];
        w3_barrier();
        for (int s = tid; s < (int)m; s += kW3Block) {
            const uint32_t dd = L.st_d[s];
            L.st_r[s] = res3[(ob + dd) * cap2 + L.A[dd] + (uint32_t)s - L.R.lofs[dd]];
        }
        w3_barrier();
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            if (live[j]) __builtin_nontemporal_store(L.st_r[slot[j]], res2 + obase + woff + j * 64);
        if (tid < kW3Dig) L.A[tid] += L.R.cnt[tid];
        w3_barrier();
        cur = nx;
    }
}

// inverse of level 1: replay each span's tiles from the digit stream, gather the results run by run
// from the level-1 regions, write them in input order as Int64
__global__ __launch_bounds__(kW3Block) __attribute__((amdgpu_waves_per_eu(8))) void k_w3_il1(
    W3Shape sh, const uint16_t *__restrict__ d1s, const uint16_t *__restrict__ res2, int64_t *__restrict__ out) {
    __shared__ W3InvLds L;
    constexpr int NJ = kW3NJ;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t r0 = (int64_t)blockIdx.x * sh.span, r1 = std::min<int64_t>(sh.n, r0 + sh.span);
    const uint64_t rb = (uint64_t)blockIdx.x * kW3Dig;
    const uint32_t cap = sh.cap1;
    if (tid < kW3Dig) L.A[tid] = 0u;
    __syncthreads();
    const int woff = wave * 64 * NJ + lane;
    uint32_t dr[NJ];
    auto load = [&](int64_t t0) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int64_t i = t0 + woff + j * 64;
            dr[j] = __builtin_nontemporal_load(d1s + (i < r1 ? i : r0));
        }
    };
    if (r0 < r1) load(r0);
    for (int64_t t0 = r0; t0 < r1; t0 += kW3Tile) {
        uint32_t d[NJ], slot[NJ];
        bool live[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            live[j] = t0 + woff + j * 64 < r1;
            d[j] = dr[j];
        }
        if (t0 + kW3Tile < r1) load(t0 + kW3Tile);
        w3_rank<NJ>(d, live, slot, L.R);
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            if (live[j]) L.st_d[slot[j]] = (uint16_t)d[j];
        w3_barrier();
        const int m = (int)std::min<int64_t>(kW3Tile, r1 - t0);
        for (int s = tid; s < m; s += kW3Block) {
            const uint32_t dd = L.st_d[s];
            L.st_r[s] = res2[(rb + dd) * cap + L.A[dd] + (uint32_t)s - L.R.lofs[dd]];
        }
        w3_barrier();
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            if (live[j]) __builtin_nontemporal_store((int64_t)L.st_r[slot[j]], out + t0 + woff + j * 64);
        if (tid < kW3Dig) L.A[tid] += L.R.cnt[tid];
        w3_barrier();
    }
}

// ---- host ----------------------------------------------------------------------------------------
static uint32_t w3_round64(double x) { return (uint32_t)(((uint64_t)x + 63) & ~63ull); }

int window_w3(qeh_ctx *ctx, int func, const qeh_column &part, const qeh_column &order, bool asc, int64_t param,
              qeh_column *out) {
    // opt-in (QEH_WINDOW_W3=1): measured slower than k_window.hip's pipeline at config 5's size
    // (profiles/r06/cfg5_w3_kernel_stats.csv: 33.9 ms against 28.6), kept for that record and for its tests
    if (!std::getenv("QEH_WINDOW_W3")) return kWindowMsdNotEligible;
    if (func != QEH_WIN_ROW_NUMBER && func != QEH_WIN_RANK && func != QEH_WIN_NTILE) return kWindowMsdNotEligible;
    if (func == QEH_WIN_NTILE && param < 1) return kWindowMsdNotEligible;
    const int64_t n = part.length;
    if (n != order.length || n <= 0 || n >= ((int64_t)1 << 32) - 1) return kWindowMsdNotEligible;
    if (!std::getenv("QEH_WINDOW_MSD") && n < ((int64_t)1 << 20)) return kWindowMsdNotEligible;
    if (part.dtype != QEH_DT_INT64 && part.dtype != QEH_DT_INT32) return kWindowMsdNotEligible;
    if (order.dtype != QEH_DT_INT64 && order.dtype != QEH_DT_INT32 && order.dtype != QEH_DT_FLOAT64 &&
        order.dtype != QEH_DT_FLOAT32)
        return kWindowMsdNotEligible;
    if ((part.validity && part.null_count != 0) || (order.validity && order.null_count != 0)) return kWindowMsdNotEligible;
    if (!lds_atomic_rank_ok(ctx)) return kWindowMsdNotEligible;
    const int cus = ctx->props.multiProcessorCount;
    W3Shape sh{};
    sh.n = n;
    // level 1: two spans per CU at full size (the inverse pass runs two workgroups per CU), >= 64 K rows each
    sh.g1 = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * 2, (n + 65535) / 65536));
    sh.g1 = std::min(sh.g1, kW3Dig);
    sh.span = ((n + sh.g1 - 1) / sh.g1 + kW3Tile - 1) / kW3Tile * kW3Tile;
    sh.g1 = (int)((n + sh.span - 1) / sh.span);
    // region capacities: the rows of one key arrive as a lump, so few distinct keys spread unevenly
    // over the digits -- generous capacities (memory is not traffic: only what is written is touched),
    // and an overflow sends the query to the k_window.hip pipeline
    sh.cap1 = w3_round64((double)sh.span / kW3Dig * 1.5 + 1024);
    // level 2: digits so that a sub-bucket holds ~2-4 K rows
    // (at least 3 bits: sub-keys of <= 8 bits travel as bytes)
    int d2bits = 3;
    while (d2bits < 9 && ((double)n / kW3Dig / (double)(1 << d2bits)) > 4096.0) ++d2bits;
    sh.sb = 11 - d2bits;
    const double mean2 = (double)n / kW3Dig / (double)(1 << d2bits);
    const int64_t nsub = (int64_t)kW3Dig << d2bits;
    sh.cap2 = (double)nsub * kW3MaxCap2 * 11 <= std::max(2e9, (double)n * 24)
                  ? (uint32_t)kW3MaxCap2
                  : std::min<uint32_t>(kW3MaxCap2, w3_round64(mean2 * 1.5 + 512));
    const uint64_t nreg1 = (uint64_t)sh.g1 * kW3Dig, items1 = nreg1 * sh.cap1, items2 = (uint64_t)nsub * sh.cap2;
    DevBuf v1, kl1, d1s, c1, fl, mmb, v2, s2, c2, r3, r2;
    if (v1.alloc(ctx, items1 * 8) || kl1.alloc(ctx, items1 * 2) || d1s.alloc(ctx, (size_t)n * 2) ||
        c1.alloc(ctx, nreg1 * 4) || fl.alloc(ctx, 16) || mmb.alloc(ctx, sizeof(W3MinMax) * sh.g1))
        return fail(QEH_E_OOM, "window: out of device memory");
    QEH_HIP(hipMemsetAsync(fl.p, 0, 16, ctx->stream));
    const ColRef kc = make_colref(part), oc = make_colref(order);
    const int kes = part.dtype == QEH_DT_INT32 ? 4 : 8;
    const int oes = (order.dtype == QEH_DT_INT32 || order.dtype == QEH_DT_FLOAT32) ? 4 : 8;
    {
        KernelTimer kt(ctx, "w3_partition");
        hipLaunchKernelGGL(kes == 4 ? (oes == 4 ? k_w3_l1<4, 4> : k_w3_l1<4, 8>) : (oes == 4 ? k_w3_l1<8, 4> : k_w3_l1<8, 8>),
                           dim3(sh.g1), dim3(kW3Block), 0, ctx->stream, kc, oc, asc ? 1 : 0, sh, v1.as<uint64_t>(),
                           kl1.as<uint16_t>(), d1s.as<uint16_t>(), c1.as<uint32_t>(), fl.as<uint32_t>(), mmb.as<W3MinMax>());
    }
    QEH_HIP(hipGetLastError());
    // the fold to 20 bits is one-to-one only over a key range of <= 2^20: checked before going on
    std::vector<W3MinMax> mmh(sh.g1);
    uint32_t flh[4];
    QEH_TRY(read_small(ctx, mmh.data(), mmb.p, sizeof(W3MinMax) * sh.g1));
    QEH_TRY(read_small(ctx, flh, fl.p, 16));
    int64_t kmin = INT64_MAX, kmax = INT64_MIN;
    for (const W3MinMax &q : mmh) kmin = std::min(kmin, q.mn), kmax = std::max(kmax, q.mx);
    if ((uint64_t)kmax - (uint64_t)kmin >= (1ull << 20) || flh[0]) return kWindowMsdNotEligible;
    if (v2.alloc(ctx, items2 * 8) || s2.alloc(ctx, items2) || c2.alloc(ctx, (size_t)nsub * 4))
        return fail(QEH_E_OOM, "window: out of device memory");
    {
        KernelTimer kt(ctx, "w3_partition");
        hipLaunchKernelGGL(k_w3_l2, dim3(kW3Dig), dim3(kW3Block), 0, ctx->stream, sh, v1.as<uint64_t>(), kl1.as<uint16_t>(),
                           c1.as<uint32_t>(), v2.as<uint64_t>(), s2.as<uint8_t>(), c2.as<uint32_t>(), fl.as<uint32_t>());
    }
    QEH_HIP(hipGetLastError());
    v1.reset();
    if (r3.alloc(ctx, items2 * 2)) return fail(QEH_E_OOM, "window: out of device memory");
    {
        KernelTimer kt(ctx, "w3_sort");
        auto l3 = [&](auto fn) {
            constexpr int FN = decltype(fn)::value;
            hipLaunchKernelGGL(k_w3_l3<FN>, dim3(cus), dim3(kW3Block), 0, ctx->stream, sh, (int)nsub, v2.as<uint64_t>(),
                               s2.as<uint8_t>(), c2.as<uint32_t>(), r3.as<uint16_t>(), fl.as<uint32_t>(), param);
        };
        if (func == QEH_WIN_RANK) l3(std::integral_constant<int, QEH_WIN_RANK>{});
        else if (func == QEH_WIN_NTILE) l3(std::integral_constant<int, QEH_WIN_NTILE>{});
        else l3(std::integral_constant<int, QEH_WIN_ROW_NUMBER>{});
    }
    QEH_HIP(hipGetLastError());
    v2.reset();
    s2.reset();
    if (r2.alloc(ctx, items1 * 2)) return fail(QEH_E_OOM, "window: out of device memory");
    QEH_TRY(alloc_column(ctx, QEH_DT_INT64, n, false, out));
    {
        KernelTimer kt(ctx, "w3_place");
        hipLaunchKernelGGL(k_w3_il2, dim3(kW3Dig), dim3(kW3Block), 0, ctx->stream, sh, kl1.as<uint16_t>(), c1.as<uint32_t>(),
                           r3.as<uint16_t>(), r2.as<uint16_t>());
        hipLaunchKernelGGL(k_w3_il1, dim3(sh.g1), dim3(kW3Block), 0, ctx->stream, sh, d1s.as<uint16_t>(), r2.as<uint16_t>(),
                           (int64_t *)out->values);
    }
    if (hipGetLastError() != hipSuccess) {
        qeh_column_release(ctx, out);
        return fail(QEH_E_HIP, "window: kernel launch failed");
    }
    if (read_small(ctx, flh, fl.p, 16) != QEH_OK) {
        qeh_column_release(ctx, out);
        return fail(QEH_E_HIP, "window: kernel failed");
    }
    if (flh[1] || flh[2]) {  // a sub-bucket over capacity, or a bucket of many equal order keys
        qeh_column_release(ctx, out);
        return kWindowMsdNotEligible;
    }
    return QEH_OK;
}

}  // namespace qeh
