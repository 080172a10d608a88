// Window functions over one bounded integer PARTITION BY key and one ORDER BY key, by
// partitioning instead of a full sort (BASELINE config 5: ROW_NUMBER() OVER (PARTITION BY k
// ORDER BY v), k in [0, 2^20), 1e9 rows).
//
// Semantics as qeh_row_number / qeh_window (k_sort.hip): rows numbered 1.. within each partition
// in ORDER BY order, ties by input position (docs/WINDOW_FUNCTIONS.md:44-65); RANK with gaps,
// DENSE_RANK without, NTILE's first size % n buckets one row larger (:67-140); output aligned to
// input order.  The LSD path of k_sort.hip sorts 40-bit (k, v) pair keys in five 8-bit passes
// and scatters the numbers back with random 8-B stores; this path moves each row a bounded
// number of times with run-contiguous writes and no row ids:
//   1. k_wm_hist1 + k_wm2_pass1: a stable 1024-way partition of (order key, low key bits) by the
//      key's high bits (per-workgroup histograms, one scan, ballot-ranked LDS-staged runs);
//   2. k_wm2_chunk_hist + k_wm2_chunk_scan + k_wm2_pass2: inside each bucket a stable partition by
//      the key's low bits, chunk by chunk (two tiles each, the chunks of one bucket taken together by
//      one XCD's workgroups) -- every PARTITION BY group is now contiguous (in input order), its
//      start in pstart[];
//   3. k_wm2_csort_wg: a workgroup per group ranks its rows by counting sort (exact ties by
//      position in the group = input order) and writes the function's value at each row's own
//      position; groups whose keys cluster go to the bitonic network kernel (k_wm2_sort);
//   4. k_wm2_inv2 / k_wm2_inv1: the two partitions are replayed (the ranking is deterministic) and
//      the results gathered back run by run, into pass-1 order and then input order -- chunk by
//      chunk from the run positions both passes checkpoint every two tiles, one XCD's workgroups
//      on neighbouring chunks, so the short result runs are gathered through that XCD's L2.
// Value functions (LAG / LEAD / FIRST_VALUE / LAST_VALUE of the ORDER BY column) carry the value
// bits beside a valid flag.  Groups above 2048 rows (skew) and shapes outside the limits return
// kWindowMsdNotEligible and the caller takes the LSD path.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "../../include/qeh_plan.h"
#include "device_common.h"
#include "ops.h"

namespace qeh {

constexpr int kWmBlock = 1024;                // partition passes: one workgroup per CU
constexpr int kWmTile = 8192;                 // rows per partition-pass tile (8 per thread)
constexpr int kWmDig = 1024;                  // digits per partition pass
constexpr int kWmSortBlock = 256;             // group sort: 4 waves
constexpr int kWmCkTiles = 2;                 // pass 2 tiles per inverse-pass-2 chunk (a checkpoint each)

// Workgroup barrier ordering LDS only: the next tile's global loads stay in flight across it
// (__syncthreads would also drain vmcnt and serialise the prefetch).
__device__ __forceinline__ void wm_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// exclusive scan of one value per thread over a 1024-thread block
__device__ __forceinline__ uint32_t block_excl_scan1024(uint32_t v, uint32_t *wsum) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(v);
    if (lane == 63) wsum[wave] = inc;
    wm_barrier();
    if (wave == 0) {
        const uint32_t w = lane < kWmBlock / 64 ? wsum[lane] : 0u;
        const uint32_t wi = wave_incl_scan(w);
        if (lane < kWmBlock / 64) wsum[lane] = wi - w;
    }
    wm_barrier();
    return inc - v + wsum[wave];
}

// Typed element loads: the window kernels are instantiated per key / order-key element width, so the
// loads of a tile are plain vector loads with no dtype switch between them (a switch per element
// made the compiler wait for every load before issuing the next).  Values are converted after
// loading, in registers.
template <int ES>
__device__ __forceinline__ uint64_t wm_ld(const void *p, int64_t i) {
    if constexpr (ES == 4) return (uint64_t)((const uint32_t *)p)[i];
    else return ((const uint64_t *)p)[i];
}
// non-temporal: streamed columns should not evict the result runs an inverse pass re-reads from L2
template <int ES>
__device__ __forceinline__ uint64_t wm_ld_nt(const void *p, int64_t i) {
    if constexpr (ES == 4) return (uint64_t)__builtin_nontemporal_load((const uint32_t *)p + i);
    else return __builtin_nontemporal_load((const uint64_t *)p + i);
}
__device__ __forceinline__ int64_t wm_key_val(uint64_t raw, int dtype) {
    return dtype == QEH_DT_INT32 ? (int64_t)(int32_t)(uint32_t)raw : (int64_t)raw;
}
__device__ __forceinline__ uint64_t wm_order_bits(uint64_t raw, int dtype, int asc) {
    int64_t o;
    if (dtype == QEH_DT_INT32) o = (int64_t)(int32_t)(uint32_t)raw;
    else if (dtype == QEH_DT_FLOAT32) o = f64_order_key((double)__builtin_bit_cast(float, (uint32_t)raw));
    else if (dtype == QEH_DT_FLOAT64) o = f64_order_key(as_f64((int64_t)raw));
    else o = (int64_t)raw;
    const uint64_t u = (uint64_t)o ^ 0x8000000000000000ull;
    return asc ? u : ~u;
}

typedef unsigned int v4u32w __attribute__((ext_vector_type(4)));

struct WmShape {
    int64_t n;
    int64_t kmin;
    uint64_t kmask;    // key offset = (k - kmin) & kmask: all ones, or 2^20 - 1 with kmin = 0 (keys mod 2^20,
                       // one-to-one over any key range <= 2^20, so the histogram needs no minimum first)
    int32_t lb;        // low key bits (pass 2 digit); high digit = (k - kmin) >> lb
    int32_t sb;        // sub-key bits (key ranges above 2^20): pass 2's digit is the low bits >> sb, and a
                       // "group" is 2^sb consecutive keys, told apart by the group sort (ks below)
    int32_t nb;        // buckets (high digits in use)
    int64_t nparts;    // key range = number of PARTITION BY groups (some empty)
    int64_t span;      // rows per workgroup in pass 1 (multiple of kWmTile)
    int32_t exp;       // QEH_WM_EXP != 0 (-DQEH_EXPERIMENTS builds only: time pass 1 alone; the query then fails)
};

// Pass 1 and its inverse run by chunks of kWmCkTiles tiles of the input (kWmChunk rows; the histogram
// spans, sh.span, are whole chunks): per-chunk digit counts -> a scan over the chunks per digit gives
// every chunk its run positions ahead of pass 1 (and inverse pass 1 its checkpoints).
constexpr int64_t kWmChunk = (int64_t)kWmTile * kWmCkTiles;
constexpr int kWmScanB = 256;  // chunks per block of the chunk scan

// ---- pass 1: histogram of the high key digit per chunk ------------------------------------------
// One workgroup per span of whole chunks, the chunks in turn: counts[chunk][digit] (u16, a chunk holds
// <= kWmChunk = 16384 rows).  MM: also the key's min / max (per-workgroup partials) in the same read:
// the histogram is then taken on the key mod 2^20 (kmin = 0, kmask = 2^20 - 1, 1024 digits of 10
// bits), which is pass 1's digit for every key range of 2^19 .. 2^20 keys (config 5's shape) whatever
// its minimum; other ranges histogram again with their own shape (MM = false).
struct WmMinMax {
    int64_t mn, mx;
};
template <int KES, bool MM>
__global__ __launch_bounds__(kWmBlock) void k_wm_hist1(ColRef key, WmShape sh, uint16_t *__restrict__ counts,
                                                       WmMinMax *__restrict__ part) {
    __shared__ uint32_t h[kWmDig];
    __shared__ int64_t smn[kWmBlock / 64], smx[kWmBlock / 64];
    const int64_t r0 = (int64_t)blockIdx.x * sh.span, r1 = std::min<int64_t>(sh.n, r0 + sh.span);
    // 16-B loads (KES = 8: two keys, KES = 4: four) over the 16-B-aligned body, scalar edges
    constexpr int PER = 16 / KES, U = 4;  // keys per load, loads in flight per thread
    const char *kp = (const char *)key.values;
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    auto one = [&](uint64_t raw) {
        const int64_t x = wm_key_val(raw, key.dtype);
        if constexpr (MM) {
            mn = x < mn ? x : mn;
            mx = x > mx ? x : mx;
        }
        atomicAdd(&h[(((uint64_t)x - (uint64_t)sh.kmin) & sh.kmask) >> sh.lb], 1u);
    };
    for (int64_t c0 = r0; c0 < r1; c0 += kWmChunk) {
        const int64_t c1 = std::min<int64_t>(r1, c0 + kWmChunk);
        h[threadIdx.x] = 0;
        __syncthreads();
        int64_t a0 = c0;
        while (a0 < c1 && (((uintptr_t)(kp + a0 * KES)) & 15)) ++a0;
        const int64_t body = (c1 - a0) / (PER * U * kWmBlock) * (PER * U * kWmBlock);
        for (int64_t i = a0 + (int64_t)threadIdx.x * PER; i < a0 + body; i += (int64_t)kWmBlock * PER * U) {
            v4u32w w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) w[u] = __builtin_nontemporal_load((const v4u32w *)(kp + (i + (int64_t)u * kWmBlock * PER) * KES));
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr (KES == 8) {
                    one((uint64_t)w[u][0] | ((uint64_t)w[u][1] << 32));
                    one((uint64_t)w[u][2] | ((uint64_t)w[u][3] << 32));
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) one((uint64_t)w[u][q]);
                }
            }
        }
        for (int64_t i = c0 + threadIdx.x; i < a0; i += kWmBlock) one(wm_ld<KES>(key.values, i));
        for (int64_t i = a0 + body + threadIdx.x; i < c1; i += kWmBlock) one(wm_ld<KES>(key.values, i));
        __syncthreads();
        counts[(c0 / kWmChunk) * kWmDig + threadIdx.x] = (uint16_t)h[threadIdx.x];
        __syncthreads();
    }
    if constexpr (MM) {
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const int64_t a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64);
            mn = a < mn ? a : mn;
            mx = b > mx ? b : mx;
        }
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        if (lane == 0) smn[wave] = mn, smx[wave] = mx;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 0; w < kWmBlock / 64; ++w) mn = smn[w] < mn ? smn[w] : mn, mx = smx[w] > mx ? smx[w] : mx;
            part[blockIdx.x] = WmMinMax{mn, mx};
        }
    }
}

// The chunk scan, in three steps over blocks of kWmScanB chunks: (1) per block, rows per digit;
// (2) one workgroup: per digit the blocks' exclusive prefix and its total, then the digits' starts
// (bucket starts -> bst); (3) per block, every chunk's run positions -> cpos[chunk][digit].
__global__ __launch_bounds__(kWmBlock) void k_wm_cscan_blocks(const uint16_t *__restrict__ counts, int64_t nchunk,
                                                              uint32_t *__restrict__ bsum) {
    const int64_t c0 = (int64_t)blockIdx.x * kWmScanB, c1 = std::min<int64_t>(nchunk, c0 + kWmScanB);
    uint32_t t = 0;
    for (int64_t c = c0; c < c1; ++c) t += counts[c * kWmDig + threadIdx.x];
    bsum[(int64_t)blockIdx.x * kWmDig + threadIdx.x] = t;
}
__global__ __launch_bounds__(kWmBlock) void k_wm_cscan_top(uint32_t *__restrict__ bsum, int nblk, int nb,
                                                           uint32_t *__restrict__ dstart, uint64_t *__restrict__ bst) {
    __shared__ uint32_t wsum[kWmBlock / 64];
    uint32_t run = 0;
    for (int b = 0; b < nblk; ++b) {
        const uint32_t v = bsum[(int64_t)b * kWmDig + threadIdx.x];
        bsum[(int64_t)b * kWmDig + threadIdx.x] = run;  // -> the block's exclusive prefix
        run += v;
    }
    const uint32_t ex = block_excl_scan1024(run, wsum);
    dstart[threadIdx.x] = ex;
    if ((int)threadIdx.x < nb) bst[threadIdx.x] = ex;
}
__global__ __launch_bounds__(kWmBlock) void k_wm_cscan_pos(const uint16_t *__restrict__ counts, int64_t nchunk,
                                                           const uint32_t *__restrict__ bsum,
                                                           const uint32_t *__restrict__ dstart, uint32_t *__restrict__ cpos) {
    const int64_t c0 = (int64_t)blockIdx.x * kWmScanB, c1 = std::min<int64_t>(nchunk, c0 + kWmScanB);
    uint32_t pos = dstart[threadIdx.x] + bsum[(int64_t)blockIdx.x * kWmDig + threadIdx.x];
    for (int64_t c = c0; c < c1; ++c) {
        cpos[c * kWmDig + threadIdx.x] = pos;
        pos += counts[c * kWmDig + threadIdx.x];
    }
}

// ---- group sort: one wave per PARTITION BY group --------------------------------------------
// A group of m <= 64 R rows is sorted by a 32-bit composite key: the top 21 significant bits of
// (order key - the group's minimum) above the row's 11-bit position in the group.  The network
// (bitonic, lane-major: element e = lane * R + r, so distances below R are register swaps,
// unrolled by template recursion) therefore moves one dword per element.  Runs of equal 21-bit
// prefixes -- truncation collisions and true ties -- are then re-sorted exactly by (order key,
// row id) from the group's copy in LDS; a run above 64 rows (heavy ties) makes the operator
// fall back to the LSD path.
struct WmFunc {
    int32_t func;      // QEH_WIN_* (ROW_NUMBER .. LAST_VALUE)
    int64_t param;     // NTILE buckets / LAG, LEAD offset
    int32_t skip_sort; // QEH_WM_SKIP_SORT (-DQEH_EXPERIMENTS builds: load/emit cost without the network)
    int32_t no_count;  // QEH_WM_NO_COUNT (-DQEH_EXPERIMENTS builds: the bitonic network for every group)
    // value functions (LAG / LEAD / FIRST_VALUE / LAST_VALUE of the ORDER BY column itself): the
    // value is decoded from the group's order keys
    int32_t odt;       // order key dtype
    int32_t asc;
    int32_t has_dflt;
    int64_t dflt;      // default bits in the output width
    uint64_t *vout;    // id-free path, value functions: each row's value bits at its pass-2 position
};

// Value functions at sorted index i of a group of m rows: the source row's sorted index (false when
// the offset leaves the partition; LAST_VALUE spans the whole partition, as the reference's frame).
__device__ __forceinline__ bool wm_value_src(const WmFunc &f, int i, int m, int &js) {
    js = i;  // (param >= 0, checked by qeh_window; js is formed only inside the partition)
    if (f.func == QEH_WIN_LAG) {
        if (f.param > i) return false;
        js = (int)(i - f.param);
        return true;
    }
    if (f.func == QEH_WIN_LEAD) {
        if (f.param >= (int64_t)m - i) return false;
        js = (int)(i + f.param);
        return true;
    }
    js = f.func == QEH_WIN_FIRST_VALUE ? 0 : m - 1;
    return true;
}

// order key (wm_order_bits encoding) -> the column's value bits in its own width
__device__ __forceinline__ uint64_t wm_decode(uint64_t ok, int asc, int odt) {
    const uint64_t u = asc ? ok : ~ok;
    const int64_t o = (int64_t)(u ^ 0x8000000000000000ull);
    if (odt == QEH_DT_FLOAT64) return (uint64_t)f64_bits(f64_from_order_key(o));
    if (odt == QEH_DT_FLOAT32) return (uint64_t)__builtin_bit_cast(uint32_t, (float)f64_from_order_key(o));
    if (odt == QEH_DT_INT32) return (uint64_t)(uint32_t)(int32_t)o;
    return (uint64_t)o;
}

template <int R, int KK, int J>
__device__ __forceinline__ void bitonic_stage32(uint32_t (&k)[R], int lane) {
    if constexpr (J < R) {  // partner in this lane's registers
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int r2 = r ^ J;
            if (r2 > r) {
                const bool asc = ((lane * R + r) & KK) == 0;
                const uint32_t lo = min(k[r], k[r2]), hi = max(k[r], k[r2]);
                k[r] = asc ? lo : hi;
                k[r2] = asc ? hi : lo;
            }
        }
    } else {  // partner lane = lane ^ (J / R), same register
        constexpr int LJ = J / R;
        const bool lower = (lane & LJ) == 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool asc = ((lane * R + r) & KK) == 0;
            const uint32_t o = __shfl_xor(k[r], LJ, 64);
            k[r] = (lower == asc) ? min(k[r], o) : max(k[r], o);
        }
    }
}

template <int R, int KK, int J>
__device__ __forceinline__ void bitonic_merge32(uint32_t (&k)[R], int lane) {
    if constexpr (J > 0) {
        bitonic_stage32<R, KK, J>(k, lane);
        bitonic_merge32<R, KK, J / 2>(k, lane);
    }
}

template <int R, int KK>
__device__ __forceinline__ void bitonic_sort32(uint32_t (&k)[R], int lane) {
    if constexpr (KK <= 64 * R) {
        bitonic_merge32<R, KK, KK / 2>(k, lane);
        bitonic_sort32<R, KK * 2>(k, lane);
    }
}

__device__ __forceinline__ int wm_pad(int e) { return e + (e >> 5); }  // one pad dword per 32

// Lanes of one wave exchange data through LDS: the compiler must not move an LDS access across
// this point (it sees only per-lane dependences), and the wave's LDS operations complete.
__device__ __forceinline__ void wm_wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ bool wm_less(uint64_t a, uint32_t ia, uint64_t b, uint32_t ib) {
    return a < b || (a == b && ia < ib);
}

// per-wave LDS area for a group of up to P rows: order keys, row ids, composite keys (padded)
template <int P>
struct WmWaveLds {
    uint64_t ov[P];
    uint32_t id[P];
    uint32_t k[P + P / 32];
};

// ---- id-free pipeline (rank functions): stable passes replayed in reverse -------------------
// ROW_NUMBER / RANK / DENSE_RANK / NTILE carry no row ids.  Both partition passes rank a tile's
// rows STABLY (rows of one digit keep their input order), so every PARTITION BY group ends up in
// input order and ties sort by position in the group.  The sort writes each row's result (<= 2048,
// u16) back at the row's own position in the group; two inverse passes then replay the partition
// passes (same tiles, same deterministic ranks) and gather the results run by run, so the output
// is written in input order with coalesced stores.  Bytes per row: 8 (histogram) + 16 + 10 (pass
// 1) + 12 + 8 (pass 2) + 8 + 2 (sort) + 6 (inverse 2) + 10 + 8 (inverse 1) against 14 + 12 of ids
// and pairs moved through three more passes on the id path.

// Tile rows are wave-contiguous (row = wave * 64 * NJ + j * 64 + lane), so input order is
// (wave, j, lane).  A wave ranks its rows per digit by ballot matching (lanes of one digit ranked
// by lane, rounds in order) into per-wave LDS counters; a prefix over the waves gives every row its
// slot in the digit-sorted tile.  Deterministic: an inverse pass replays it exactly.
struct WmRankLds {
    uint16_t wc[kWmBlock / 64][kWmDig];  // per-wave digit counts, then per-wave offsets
    uint32_t lofs[kWmDig];               // digit start in the tile
    uint32_t wsum[16];
};

// Returns the tile's count of digit threadIdx.x.  DB >= 0: ballot matching with the digit width
// as a compile-time constant (the ballot loop unrolls); DB == -1: ballot matching over `dbits`
// bits at run time; DB == kWmAtomicRank: one LDS atomic per row on the wave's packed u16 counters
// -- ds_add_rtn serves the lanes of one instruction that hit the same word in lane order
// (tools/ubench/lds_order_ubench.hip checks exactly that), so the ranks are the same stable,
// replayable ones at a handful of instructions per row instead of ~5 per digit bit.
constexpr int kWmAtomicRank = -2;

template <int NJ, int DB = -1>
__device__ __forceinline__ uint32_t wm_stable_rank(const uint32_t (&d)[NJ], const bool (&live)[NJ], int dbits,
                                                   uint32_t (&slot)[NJ], WmRankLds &R) {
    if constexpr (DB >= 0) dbits = DB;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t *wz = (uint32_t *)R.wc[wave];
    for (int i = lane; i < kWmDig / 2; i += 64) wz[i] = 0u;
    wm_wave_sync();
    uint32_t r[NJ];
    if constexpr (DB == kWmAtomicRank) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            r[j] = 0u;
            if (live[j]) {
                const uint32_t sh = (d[j] & 1u) * 16u;
                r[j] = (atomicAdd(&wz[d[j] >> 1], 1u << sh) >> sh) & 0xFFFFu;
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            uint64_t m = __ballot(live[j]);
#pragma unroll
            for (int b = 0; b < (DB >= 0 ? DB : dbits); ++b) {
                // all ones where the lane's bit b is set (one signed bitfield extract)
                const uint32_t rep = (uint32_t)(__builtin_amdgcn_sbfe((int32_t)d[j], b, 1));
                const uint64_t bb = __ballot(rep != 0u);
                m &= ~(bb ^ (((uint64_t)rep << 32) | rep));  // lanes whose bit b equals this lane's
            }
            // every lane of a digit reads the digit's count (one LDS read, no broadcast from a leader);
            // the digit's lowest lane then adds the digit's row count (the read instruction precedes
            // the write in the wave's LDS order)
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const uint32_t old = live[j] ? (uint32_t)R.wc[wave][d[j]] : 0u;
            if (live[j] && below == 0) R.wc[wave][d[j]] = (uint16_t)(old + (uint32_t)__popcll(m));
            r[j] = old + below;
            wm_wave_sync();
        }
    }
    wm_barrier();
    uint32_t tot = 0;
#pragma unroll
    for (int w = 0; w < kWmBlock / 64; ++w) {
        const uint32_t c = R.wc[w][tid];
        R.wc[w][tid] = (uint16_t)tot;
        tot += c;
    }
    const uint32_t lo = block_excl_scan1024(tot, R.wsum);
    R.lofs[tid] = lo;
    wm_barrier();
#pragma unroll
    for (int j = 0; j < NJ; ++j) slot[j] = live[j] ? R.lofs[d[j]] + R.wc[wave][d[j]] + r[j] : 0u;
    return tot;
}

__host__ __device__ __forceinline__ int wm_digit_bits(int64_t ndig) {
    int b = 0;
    while (b < 11 && ((int64_t)1 << b) < ndig) ++b;
    return b;
}

// pass 1: stable 2^dbits-way partition of (order key, low key bits) by the high key digit, by chunks
// of the input, each from its precomputed run positions (cpos).  XCD x (blockIdx % 8) owns chunk ids
// [x nchunk / 8, (x + 1) nchunk / 8) and its workgroups claim them in order from one counter
// (claim[x]), so the chunks in flight on an XCD are always a window of consecutive ones: a digit's
// runs from neighbouring chunks are adjacent in the output and reach that XCD's L2 close in time.
// (Static striding let the workgroups drift thousands of chunks apart.)
template <int KES, int OES, int DB>
__global__ __launch_bounds__(kWmBlock) void k_wm2_pass1(ColRef key, ColRef ord, int asc, WmShape sh, int64_t nchunk,
                                                        const uint32_t *__restrict__ cpos, uint32_t *__restrict__ claim,
                                                        uint64_t *__restrict__ o_key, uint16_t *__restrict__ o_kl) {
    __shared__ WmRankLds R;
    __shared__ uint32_t lpos[kWmDig];  // run positions (< n < 2^32: window_msd's bound)
    __shared__ uint64_t st_key[kWmTile];
    __shared__ uint16_t st_kl[kWmTile], st_d[kWmTile];
    __shared__ uint32_t s_next;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int NJ = kWmTile / kWmBlock;
    const int dbits = wm_digit_bits(sh.nb);
    const uint32_t lmask = (1u << sh.lb) - 1u;
    const int woff = wave * 64 * NJ + lane;
    static_assert(kWmCkTiles == 2, "a whole chunk is two tiles below");
    const int xcd = blockIdx.x & 7;
    const int64_t j_lo = (int64_t)xcd * nchunk / 8, cnt = (int64_t)(xcd + 1) * nchunk / 8 - j_lo;
    if (tid == 0) s_next = atomicAdd(&claim[xcd], 1u);
    __syncthreads();
    int64_t jc = (int64_t)__builtin_amdgcn_readfirstlane(s_next);
    if (jc >= cnt) return;
    jc += j_lo;
    // the digits need only the key's low 32 bits ((k - kmin) < 2^24: see k_wm2_inv1)
    uint32_t kv[NJ];
    uint64_t ovv[NJ];
    // rows of [t0, t0 + kWmTile) inside [lo, hi) (the rest read row lo, not live)
    auto load = [&](int64_t t0, int64_t lo, int64_t hi) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int64_t i = t0 + woff + j * 64;
            const int64_t ii = i < hi ? i : lo;
            kv[j] = ((const uint32_t *)key.values)[ii * (KES / 4)];
            ovv[j] = wm_ld<OES>(ord.values, ii);
        }
    };
    int64_t c0 = jc * kWmChunk, c1 = std::min<int64_t>(sh.n, c0 + kWmChunk);
    uint32_t lp = cpos[jc * kWmDig + tid];
    load(c0, c0, c1);
    for (;;) {
        // claim the chunk after this one now: the chunk's last tile prefetches its first rows
        uint32_t nx = 0;
        if (tid == 0) nx = atomicAdd(&claim[xcd], 1u);
        lpos[tid] = lp;  // (own entry: every read of the previous chunk's run positions is behind a barrier)
        bool more = false;
        int64_t nj = 0, n0 = 0, n1 = 0;
        // One tile: FULL tiles store unconditionally (2 * NJ stores on every path), so waiting for the
        // next tile's prefetched loads never waits for this tile's run stores: the compiler counts
        // vmcnt exactly only when the store count between a load and its use is fixed -- a run-time
        // trip count there made it wait for every store ack (vmcnt(0)) before each tile.
        // LAST: the chunk's last tile (the claimed next chunk is known by then).
        auto tile = [&](int64_t t0, auto fullc, auto lastc) {
            constexpr bool FULL = decltype(fullc)::value, last = decltype(lastc)::value;
            uint32_t d[NJ], kl[NJ], slot[NJ];
            uint64_t ok[NJ];
            bool live[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                live[j] = FULL || woff + j * 64 < (int)(c1 - t0);
                const uint32_t kk = (kv[j] - (uint32_t)sh.kmin) & (uint32_t)sh.kmask;
                d[j] = kk >> sh.lb;
                kl[j] = kk & lmask;
                ok[j] = wm_order_bits(ovv[j], ord.dtype, asc);
            }
            // in flight across the LDS phases below: the chunk's next tile, or the next chunk's first
            if constexpr (!last) load(t0 + kWmTile, c0, c1);
            else if (more) load(n0, n0, n1);
            const uint32_t tcnt = wm_stable_rank<NJ, DB>(d, live, dbits, slot, R);
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                if (!live[j]) continue;
                st_key[slot[j]] = ok[j];
                st_kl[slot[j]] = (uint16_t)kl[j];
                st_d[slot[j]] = (uint16_t)d[j];
            }
            wm_barrier();
            if constexpr (FULL) {
#pragma unroll
                for (int q = 0; q < NJ; ++q) {
                    const int s = tid + q * kWmBlock;
                    const uint32_t dd = st_d[s];
                    const uint32_t p = lpos[dd] + (uint32_t)s - R.lofs[dd];
                    o_key[p] = st_key[s];
                    o_kl[p] = st_kl[s];
                }
            } else {
                const int m = (int)std::min<int64_t>(kWmTile, c1 - t0);
                for (int s = tid; s < m; s += kWmBlock) {
                    const uint32_t dd = st_d[s];
                    const uint32_t p = lpos[dd] + (uint32_t)s - R.lofs[dd];
                    o_key[p] = st_key[s];
                    o_kl[p] = st_kl[s];
                }
            }
            if constexpr (!last) {
                if (tid == 0) s_next = nx;
            }
            wm_barrier();
            lpos[tid] += tcnt;
        };
        auto next_known = [&]() {  // after a barrier behind the s_next store (uniform: kept scalar)
            const int64_t q = (int64_t)__builtin_amdgcn_readfirstlane(s_next);
            more = q < cnt;
            nj = j_lo + q;
            n0 = nj * kWmChunk;
            n1 = more ? std::min<int64_t>(sh.n, n0 + kWmChunk) : 0;
        };
        const int ntl = (int)((c1 - c0 + kWmTile - 1) / kWmTile);
        if (c1 - c0 == kWmChunk) {
            tile(c0, std::true_type{}, std::false_type{});
            next_known();
            if (more) lp = cpos[nj * kWmDig + tid];
            tile(c0 + kWmTile, std::true_type{}, std::true_type{});
        } else {
            // the input's last, partial chunk (the last id of the last XCD's range: nothing follows it),
            // its second tile loaded after the first
            tile(c0, std::false_type{}, std::true_type{});
            if (ntl > 1) {
                load(c0 + kWmTile, c0, c1);
                tile(c0 + kWmTile, std::false_type{}, std::true_type{});
            }
        }
        if (!more) break;
        jc = nj, c0 = n0, c1 = n1;
    }
}

// Pass 2 by chunks of kWmCkTiles tiles (default): the workgroups of one XCD partition consecutive
// chunks of one bucket together, so a group's runs from neighbouring chunks -- adjacent in the output
// -- are written into the same L2 at about the same time, and each chunk starts from run positions
// that k_wm2_chunk_hist + k_wm2_chunk_scan computed ahead (rows per group and chunk, then a scan over
// the bucket's chunks).  Those positions are also inverse pass 2's checkpoints.

// Chunk ids are dealt per XCD: XCD x (blockIdx % 8 -- the dispatcher deals workgroups to the XCDs in
// turn) takes buckets [x nb / 8, (x + 1) nb / 8), whose chunks are consecutive ids, and its
// workgroups take every per-th id, so neighbouring chunks run side by side in one L2 however many
// chunks a bucket has.  The bucket of chunk j: the last b with cbase[b] <= j (empty buckets share
// their successor's base and lose to it).
__device__ __forceinline__ int wm_chunk_bucket(const uint32_t *__restrict__ cbase, int lo, int hi, int64_t j) {
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((int64_t)cbase[mid] <= j) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// rows per low digit of each chunk (u16: a chunk holds <= kWmCkTiles * kWmTile = 16384 rows)
__global__ __launch_bounds__(kWmBlock) void k_wm2_chunk_hist(WmShape sh, const uint64_t *__restrict__ bstart,
                                                             const uint32_t *__restrict__ cbase,
                                                             const uint16_t *__restrict__ i_kl, uint16_t *__restrict__ ccnt) {
    __shared__ uint32_t h[kWmDig];
    const int tid = threadIdx.x, sbits = sh.sb;
    for (int b = blockIdx.x; b < sh.nb; b += gridDim.x) {
        const int64_t s0 = (int64_t)bstart[b], s1 = (int64_t)bstart[b + 1];
        const int64_t nch = (s1 - s0 + (int64_t)kWmTile * kWmCkTiles - 1) / ((int64_t)kWmTile * kWmCkTiles);
        for (int64_t c = 0; c < nch; ++c) {
            const int64_t c0 = s0 + c * kWmCkTiles * kWmTile, c1 = std::min<int64_t>(s1, c0 + (int64_t)kWmCkTiles * kWmTile);
            h[tid] = 0;
            __syncthreads();
            // 8 digits per 16-B load over the aligned body, single loads at the edges
            const int64_t a0 = std::min<int64_t>(c1, (c0 + 7) & ~(int64_t)7), a1 = std::max<int64_t>(a0, c1 & ~(int64_t)7);
            for (int64_t i = c0 + tid; i < a0; i += kWmBlock) atomicAdd(&h[i_kl[i] >> sbits], 1u);
            for (int64_t i = a1 + tid; i < c1; i += kWmBlock) atomicAdd(&h[i_kl[i] >> sbits], 1u);
            for (int64_t i = a0 + (int64_t)tid * 8; i < a1; i += (int64_t)kWmBlock * 8) {
                const v4u32w w = __builtin_nontemporal_load((const v4u32w *)(i_kl + i));
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    atomicAdd(&h[(w[q] & 0xFFFFu) >> sbits], 1u);
                    atomicAdd(&h[(w[q] >> 16) >> sbits], 1u);
                }
            }
            __syncthreads();
            ccnt[((int64_t)cbase[b] + c) * kWmDig + tid] = (uint16_t)h[tid];
            __syncthreads();
        }
    }
}

// per bucket (one workgroup each): group starts -> pstart, and every chunk's run positions -> ckpt
__global__ __launch_bounds__(kWmBlock) void k_wm2_chunk_scan(WmShape sh, const uint64_t *__restrict__ bstart,
                                                             const uint32_t *__restrict__ cbase,
                                                             const uint16_t *__restrict__ ccnt, uint32_t *__restrict__ ckpt,
                                                             uint64_t *__restrict__ pstart) {
    __shared__ uint32_t wsum[kWmBlock / 64];
    const int tid = threadIdx.x, b = blockIdx.x;
    const int64_t L = (int64_t)1 << (sh.lb - sh.sb);
    const int64_t s0 = (int64_t)bstart[b], s1 = (int64_t)bstart[b + 1];
    const int64_t nch = (s1 - s0 + (int64_t)kWmTile * kWmCkTiles - 1) / ((int64_t)kWmTile * kWmCkTiles);
    const int64_t base = cbase[b];
    uint32_t tot = 0;
    for (int64_t c = 0; c < nch; ++c) tot += ccnt[(base + c) * kWmDig + tid];
    const uint32_t ex = block_excl_scan1024(tot, wsum);
    const int64_t part = (int64_t)b * L + tid;
    if (tid < L && part < sh.nparts) pstart[part] = (uint64_t)(s0 + ex);
    uint32_t pos = (uint32_t)(s0 + ex);
    for (int64_t c = 0; c < nch; ++c) {
        ckpt[(base + c) * kWmDig + tid] = pos;
        pos += ccnt[(base + c) * kWmDig + tid];
    }
}

template <int DB, bool KS>
__global__ __launch_bounds__(kWmBlock) void k_wm2_pass2(WmShape sh, const uint64_t *__restrict__ bstart,
                                                         const uint32_t *__restrict__ cbase, const uint32_t *__restrict__ ckpt,
                                                         uint32_t *__restrict__ claim,
                                                         const uint64_t *__restrict__ i_key, const uint16_t *__restrict__ i_kl,
                                                         uint64_t *__restrict__ o_key, uint8_t *__restrict__ o_ks) {
    __shared__ WmRankLds R;
    __shared__ uint32_t lpos[kWmDig];  // run positions (< n < 2^32: window_msd's bound)
    __shared__ uint64_t st_key[kWmTile];
    __shared__ uint16_t st_d[kWmTile];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int NJ = kWmTile / kWmBlock;
    const int sbits = sh.sb;
    const int dbits = sh.lb - sbits;
    const int woff = wave * 64 * NJ + lane;
    // XCD x (blockIdx % 8) owns the consecutive chunk ids [x C / 8, (x + 1) C / 8) of all C chunks (an even
    // share whatever the buckets' sizes) and its workgroups claim them in order from one counter (as pass 1:
    // the chunks in flight stay consecutive, and adjacent chunk ids are adjacent rows of one bucket)
    const int xcd = blockIdx.x & 7;
    const int64_t nck = (int64_t)cbase[sh.nb], c_lo = (int64_t)xcd * nck / 8, c_hi = (int64_t)(xcd + 1) * nck / 8;
    __shared__ uint32_t s_next;
    if (c_lo < c_hi) {
        for (;;) {
            if (tid == 0) s_next = atomicAdd(&claim[xcd], 1u);
            __syncthreads();
            const int64_t jc = c_lo + (int64_t)__builtin_amdgcn_readfirstlane(s_next);
            if (jc >= c_hi) break;
            const int b = wm_chunk_bucket(cbase, 0, sh.nb - 1, jc);
            const int64_t s0 = (int64_t)bstart[b], s1 = (int64_t)bstart[b + 1], c = jc - (int64_t)cbase[b];
            const int64_t c0 = s0 + c * kWmCkTiles * kWmTile, c1 = std::min<int64_t>(s1, c0 + (int64_t)kWmCkTiles * kWmTile);
            lpos[tid] = ckpt[jc * kWmDig + tid];
            __syncthreads();
            uint64_t kx[NJ];
            uint32_t lx[NJ];
            // one base address, the rows at immediate offsets; a tile may read past the chunk (and past
            // n: i_key / i_kl carry kWmTile rows of padding) -- those rows are not live
            auto load = [&](int64_t t0) {
                const uint64_t *pk = i_key + t0 + woff;
                const uint16_t *pl = i_kl + t0 + woff;
#pragma unroll
                for (int j = 0; j < NJ; ++j) kx[j] = pk[j * 64], lx[j] = pl[j * 64];
            };
            // FULL tiles store unconditionally (see k_wm2_pass1: exact vmcnt accounting)
            auto tile = [&](int64_t t0, auto fullc) {
                constexpr bool FULL = decltype(fullc)::value;
                uint32_t d[NJ], slot[NJ];
                uint64_t keys[NJ];
                bool live[NJ];
                uint32_t ksub[NJ];
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    live[j] = FULL || woff + j * 64 < (int)(c1 - t0);
                    d[j] = KS ? lx[j] >> sbits : lx[j];
                    ksub[j] = KS ? lx[j] & ((1u << sbits) - 1u) : 0u;
                    keys[j] = kx[j];
                }
                if (t0 + kWmTile < c1) load(t0 + kWmTile);
                const uint32_t tcnt = wm_stable_rank<NJ, DB>(d, live, dbits, slot, R);
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    if (!live[j]) continue;
                    st_key[slot[j]] = keys[j];
                    st_d[slot[j]] = (uint16_t)(d[j] | (ksub[j] << 10));  // digit (10 bits) | sub-key (<= 4 bits)
                }
                wm_barrier();
                auto put = [&](int s) {
                    const uint32_t dd = st_d[s] & 1023u;
                    const uint32_t p = lpos[dd] + (uint32_t)s - R.lofs[dd];
                    o_key[p] = st_key[s];
                    if constexpr (KS) o_ks[p] = (uint8_t)(st_d[s] >> 10);
                };
                if constexpr (FULL) {
#pragma unroll
                    for (int q = 0; q < NJ; ++q) put(tid + q * kWmBlock);
                } else {
                    const int m = (int)std::min<int64_t>(kWmTile, c1 - t0);
                    for (int s = tid; s < m; s += kWmBlock) put(s);
                }
                wm_barrier();
                lpos[tid] += tcnt;
            };
            load(c0);
            if (c1 - c0 >= kWmTile) {
                tile(c0, std::true_type{});
                int64_t t0 = c0 + kWmTile;
                for (; t0 + kWmTile <= c1; t0 += kWmTile) tile(t0, std::true_type{});
                if (t0 < c1) tile(t0, std::false_type{});
            } else {
                tile(c0, std::false_type{});
            }
            __syncthreads();
        }
    }
}

template <int R, int P, bool VF>
__device__ __forceinline__ void wm2_group_tail(int64_t s, int m, const WmFunc &f, uint16_t *__restrict__ res_out,
                                               WmWaveLds<P> &L, int lane);

constexpr int kWmCsCap = 16;  // counting sort (k_wm2_csort_wg): most rows one bucket may hold

// group sort without row ids: ties by position in the group (= input order, the passes being
// stable); each row's result is written at its own position in the group
// `pre` holds the group's order keys register-major (element r * 64 + lane in pre[r]), loaded by
// the caller ahead of time.
template <int R, int P, int RP, bool VF>
__device__ void wm2_group(const uint64_t (&pre)[RP], int64_t s, int m, const WmFunc &f, uint16_t *__restrict__ res_out,
                          WmWaveLds<P> &L, uint32_t *__restrict__ too_big, int lane) {
    static_assert(R <= RP, "prefetch too short");
    wm_wave_sync();  // the previous group's LDS reads are done
    uint64_t mn = ~0ull, mx = 0ull;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        if (e < m) {
            const uint64_t o = pre[r];
            L.ov[e] = o;
            mn = o < mn ? o : mn;
            mx = o > mx ? o : mx;
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    const uint64_t span = mx - mn;
    const int sb = span ? 64 - __clzll((long long)span) : 0;
    wm_wave_sync();  // every lane's order keys are in LDS
    const int shift = sb > 21 ? sb - 21 : 0;
    uint32_t k[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = lane * R + r;  // lane-major: the network's layout
        k[r] = e < m ? ((uint32_t)((L.ov[e] - mn) >> shift) << 11) | (uint32_t)e : 0xFFFFFFFFu;
    }
    if (!f.skip_sort) bitonic_sort32<R, 2>(k, lane);
#pragma unroll
    for (int r = 0; r < R; ++r) L.k[wm_pad(lane * R + r)] = k[r];
    wm_wave_sync();
    // exact order inside runs of equal prefixes (insertion sort by (order key, position))
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        if (e >= m) continue;
        const uint32_t ke = L.k[wm_pad(e)] >> 11;
        const bool start = e == 0 || (L.k[wm_pad(e - 1)] >> 11) != ke;
        if (!start || e + 1 >= m || (L.k[wm_pad(e + 1)] >> 11) != ke) continue;
        int len = 2;
        while (e + len < m && (L.k[wm_pad(e + len)] >> 11) == ke) ++len;
        if (len > 64) {
            *too_big = 1u;
            continue;
        }
        for (int a = 1; a < len; ++a) {
            const uint32_t x = L.k[wm_pad(e + a)];
            const uint64_t xo = L.ov[x & 2047];
            int b = a - 1;
            while (b >= 0) {
                const uint32_t y = L.k[wm_pad(e + b)];
                if (!wm_less(xo, x & 2047, L.ov[y & 2047], y & 2047)) break;
                L.k[wm_pad(e + b + 1)] = y;
                --b;
            }
            L.k[wm_pad(e + b + 1)] = x;
        }
    }
    wm2_group_tail<R, P, VF>(s, m, f, res_out, L, lane);
}

// With the group's order (position in the low 11 bits of L.k[wm_pad(i)], i = sorted index): the
// function's value per row, written at the row's own position in the group.
// VF: value functions (valid flag in res_out, value bits in f.vout); else rank functions.
template <int R, int P, bool VF>
__device__ __forceinline__ void wm2_group_tail(int64_t s, int m, const WmFunc &f, uint16_t *__restrict__ res_out,
                                               WmWaveLds<P> &L, int lane) {
    wm_wave_sync();
    uint32_t carry_rank = 0, carry_dense = 0;
    uint64_t prev_ov = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        const bool live = e < m;
        const uint32_t x = live ? L.k[wm_pad(e)] : 0u;
        const uint32_t pos = x & 2047;
        const uint64_t ov = live ? L.ov[pos] : 0ull;
        uint32_t res;
        if (VF) {  // (valid flag, value bits of the source row at pos)
            int js;
            const bool ok = wm_value_src(f, e, m, js);
            uint64_t bits = f.has_dflt ? (uint64_t)f.dflt : 0ull;
            res = f.has_dflt ? 1u : 0u;
            if (live && ok) {
                bits = wm_decode(L.ov[L.k[wm_pad(js)] & 2047], f.asc, f.odt);
                res = 1u;
            }
            if (live) f.vout[s + pos] = bits;
        } else if (f.func == QEH_WIN_ROW_NUMBER) {
            res = (uint32_t)e + 1u;
        } else if (f.func == QEH_WIN_NTILE) {
            const int64_t q = m / f.param, rm = m % f.param, r0 = e;
            res = (uint32_t)(r0 < rm * (q + 1) ? r0 / (q + 1) + 1 : rm + (r0 - rm * (q + 1)) / (q > 0 ? q : 1) + 1);
        } else {
            uint64_t pv = __shfl_up(ov, 1, 64);
            if (lane == 0) pv = prev_ov;
            const uint32_t flag = (e == 0 || pv != ov) ? 1u : 0u;
            if (f.func == QEH_WIN_RANK) {
                uint32_t v = flag ? (uint32_t)e : 0u;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t t = __shfl_up(v, d, 64);
                    if (lane >= d) v = t > v ? t : v;
                }
                v = v > carry_rank ? v : carry_rank;
                res = v + 1u;
                carry_rank = __shfl(v, 63, 64);
            } else {  // DENSE_RANK
                const uint32_t v = wave_incl_scan(flag) + carry_dense;
                res = v;
                carry_dense = __shfl(v, 63, 64);
            }
            prev_ov = __shfl(ov, 63, 64);
        }
        if (live) L.id[pos] = res;
    }
    wm_wave_sync();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        if (e < m) res_out[s + e] = (uint16_t)L.id[e];
    }
}

// One wave per group, bitonic network.  BIG: the groups of 1025..2048 rows, a kernel of its own
// (larger LDS area).  LIST: the groups the counting sort (k_wm2_csort_wg) queued in fb (fb[0] =
// count, fb[1..] = group numbers); else every group of the size class.  (Loading the next group's
// keys while sorting this one needed 256 VGPRs and ran slower.)
template <bool BIG, bool LIST, bool VF>
__global__ __launch_bounds__(kWmSortBlock, 2) void k_wm2_sort(WmShape sh, WmFunc f, const uint64_t *__restrict__ pstart,
                                                              const uint64_t *__restrict__ gkey, uint16_t *__restrict__ res,
                                                              uint32_t *__restrict__ too_big, const uint32_t *__restrict__ fb) {
    constexpr int P = BIG ? 2048 : 1024;
    constexpr int W = kWmSortBlock / 64;
    __shared__ WmWaveLds<P> wl[W];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t i0, i1, di;
    if (LIST) {
        i0 = (int64_t)blockIdx.x * W + wave, i1 = (int64_t)fb[0], di = (int64_t)gridDim.x * W;
    } else {
        i0 = (int64_t)blockIdx.x * sh.nparts / gridDim.x + wave;
        i1 = (int64_t)(blockIdx.x + 1) * sh.nparts / gridDim.x;
        di = W;
    }
    for (int64_t i = i0; i < i1; i += di) {
        const int64_t g = LIST ? (int64_t)fb[1 + i] : i;
        const int64_t s = (int64_t)pstart[g];
        const int64_t m = (int64_t)pstart[g + 1] - s;
        if (m <= 0) continue;
        if (BIG) {
            if (m <= 1024) continue;
            if (m > 2048) {
                if (lane == 0) *too_big = 1u;
                continue;
            }
        } else if (m > 1024) {
            continue;
        }
        constexpr int RP = BIG ? 32 : 16;
        uint64_t pre[RP];
#pragma unroll
        for (int r = 0; r < RP; ++r) {
            const int e = r * 64 + lane;
            pre[r] = e < m ? gkey[s + e] : 0ull;
        }
        const int mi = (int)m;
        if (BIG) wm2_group<RP, P, RP, VF>(pre, s, mi, f, res, wl[wave], too_big, lane);
        else if (mi <= 64) wm2_group<1, P, RP, VF>(pre, s, mi, f, res, wl[wave], too_big, lane);
        else if (mi <= 128) wm2_group<2, P, RP, VF>(pre, s, mi, f, res, wl[wave], too_big, lane);
        else if (mi <= 256) wm2_group<4, P, RP, VF>(pre, s, mi, f, res, wl[wave], too_big, lane);
        else if (mi <= 512) wm2_group<8, P, RP, VF>(pre, s, mi, f, res, wl[wave], too_big, lane);
        else wm2_group<RP, P, RP, VF>(pre, s, mi, f, res, wl[wave], too_big, lane);
    }
}

// Counting sort of a group, a whole workgroup per group (E rows per thread: groups of (LO, 256 E]
// rows): buckets of the top log2(2P) bits of (order key - min), 16-bit counters packed in LDS,
// rows placed by bucket start + arrival with their keys at that slot, then each row ranks itself
// exactly among its bucket's rows by (order key, position) -- a few LDS operations per row instead
// of a bitonic network's log2(P)(log2(P)+1)/2 compare-exchange stages.  Buckets hold under one row
// on average for spread keys; a group with a bucket above kWmCsCap rows (clustered keys, many
// ties) is queued in fb for the network kernel.  The workgroup's group bounds sit in LDS and the
// next group's keys are loaded while this one is ranked (the barriers order LDS only, so the loads
// stay in flight).
constexpr int kWmCsMaxG = 512;  // groups per workgroup range (the grid is sized for it)

template <int E>
struct WmGroupLds {
    static constexpr int P = 256 * E;
    uint64_t ov[P];           // keys by bucket slot
    uint32_t k[P + P / 32];   // slot -> position; then sorted index -> position | slot << 12 (padded)
    uint32_t cnt[P];          // 2P packed 16-bit bucket counters, then starts; then results by position
    uint64_t bnd[kWmCsMaxG + 1];
    uint64_t mm[8];           // per-wave min / max
    uint32_t ws[4], wf[4], wc[4], wt[4];
    uint32_t subc[16], subst[16];  // SUB: rows per sub-key, then the sub-keys' starts in the sorted group
};

// FN: the window function as a compile-time constant (QEH_WIN_ROW_NUMBER .. NTILE; -1 = the value
// functions, selected by f.func at run time) -- the per-row dispatch left a third of the kernel's
// instructions scalar.
// SUB (key ranges above 2^20, sh.sb > 0): a group holds 2^sb consecutive keys, told apart by gks (the
// key's low sb bits): the buckets are (sub-key, order-key range), so a row's sorted index minus its
// sub-key's start is its index inside its own PARTITION BY group, and the sub-key's row count its
// size (the sorted entries carry the sub-key for DENSE_RANK's group starts and the value functions).
template <int E, int FN, bool SUB = false>
__global__ __launch_bounds__(256, E == 4 ? 5 : 2) void k_wm2_csort_wg(WmShape sh, WmFunc f, const uint64_t *__restrict__ pstart,
                                                      const uint64_t *__restrict__ gkey, uint16_t *__restrict__ res,
                                                      uint32_t *__restrict__ fb, uint32_t *__restrict__ too_big,
                                                      const uint8_t *__restrict__ gks) {
    constexpr int P = 256 * E, NB = E == 4 ? 11 : 12, LO = E == 4 ? 0 : 1024;  // groups of (LO, P] rows
    static_assert((1 << NB) == 2 * P, "two buckets per row of capacity");
    __shared__ WmGroupLds<E> L;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t g0 = (int64_t)blockIdx.x * sh.nparts / gridDim.x, g1 = (int64_t)(blockIdx.x + 1) * sh.nparts / gridDim.x;
    for (int64_t i = t; i <= g1 - g0; i += 256) L.bnd[i] = pstart[g0 + i];
    __syncthreads();
    uint64_t keyN[E];
    uint32_t ksN[SUB ? E : 1];
    auto issue = [&](int64_t gi) {
        const int64_t s = (int64_t)L.bnd[gi - g0];
        const int m = (int)((int64_t)L.bnd[gi - g0 + 1] - s);
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int e = r * 256 + t;
            keyN[r] = (m > LO && m <= P && e < m) ? __builtin_nontemporal_load(gkey + s + e) : 0ull;
            if constexpr (SUB) ksN[r] = (m > LO && m <= P && e < m) ? (uint32_t)gks[s + e] : 0u;
        }
    };
    if (g0 < g1) issue(g0);
    for (int64_t g = g0; g < g1; ++g) {
        const int64_t s = (int64_t)L.bnd[g - g0];
        const int m = (int)((int64_t)L.bnd[g - g0 + 1] - s);
        uint64_t key[E];
        uint32_t ks[SUB ? E : 1];
#pragma unroll
        for (int r = 0; r < E; ++r) key[r] = keyN[r];
        if constexpr (SUB) {
#pragma unroll
            for (int r = 0; r < E; ++r) ks[r] = ksN[r];
        }
        if (g + 1 < g1) issue(g + 1);
        if (m > P && E == 8 && t == 0) *too_big = 1u;  // above 2048 rows: the caller takes the LSD path
        if (m <= LO || m > P) continue;  // (uniform) empty, or the other kernel's size class
        uint64_t mn = ~0ull, mx = 0ull;
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int e = r * 256 + t;
            if (e < m) mn = min(mn, key[r]), mx = max(mx, key[r]);
            L.cnt[e] = 0u;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint64_t a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64);
            mn = a < mn ? a : mn;
            mx = b > mx ? b : mx;
        }
        if (lane == 0) L.mm[wave] = mn, L.mm[4 + wave] = mx;
        if (SUB && t < 16) L.subc[t] = 0u;
        wm_barrier();
        mn = min(min(L.mm[0], L.mm[1]), min(L.mm[2], L.mm[3]));
        mx = max(max(L.mm[4], L.mm[5]), max(L.mm[6], L.mm[7]));
        const uint64_t span = mx - mn;
        const int sb = span ? 64 - __clzll((long long)span) : 0;
        const int NBV = SUB ? NB - sh.sb : NB;  // bucket bits of the order key (the sub-key takes sh.sb)
        const int shift = sb > NBV ? sb - NBV : 0;
        uint32_t se[E], sl[E];  // bucket, then start | end << 16; arrival, then slot
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int e = r * 256 + t;
            se[r] = sl[r] = 0u;
            if (e < m) {
                uint32_t bk = (uint32_t)((key[r] - mn) >> shift);
                if constexpr (SUB) {
                    bk |= ks[r] << NBV;
                    atomicAdd(&L.subc[ks[r]], 1u);
                }
                const uint32_t sh16 = (bk & 1u) * 16u;
                const uint32_t old = atomicAdd(&L.cnt[bk >> 1], 1u << sh16);
                se[r] = bk;
                sl[r] = (old >> sh16) & 0xFFFFu;
            }
        }
        wm_barrier();
        {  // exclusive scan of the 2P counters: thread t owns words E t .. E t + E - 1
            uint32_t w[E], tot = 0, big = 0;
#pragma unroll
            for (int q = 0; q < E; ++q) {
                w[q] = L.cnt[E * t + q];
                const uint32_t lo = w[q] & 0xFFFFu, hi = w[q] >> 16;
                tot += lo + hi;
                big |= (lo > (uint32_t)kWmCsCap || hi > (uint32_t)kWmCsCap) ? 1u : 0u;
            }
            const uint32_t incl = wave_incl_scan(tot);
            const bool wbig = __ballot(big) != 0;
            if (lane == 63) L.ws[wave] = incl, L.wf[wave] = wbig ? 1u : 0u;
            wm_barrier();
            if (L.wf[0] | L.wf[1] | L.wf[2] | L.wf[3]) {  // (uniform) clustered keys: the network sorts it
                if (t == 0) {
                    if (SUB) *too_big = 1u;  // (the network knows no sub-keys: the LSD path takes the job)
                    else fb[1 + atomicAdd(&fb[0], 1u)] = (uint32_t)g;
                }
                wm_barrier();  // every thread has read the flags before the next group writes them
                continue;
            }
            if (SUB && t == 0) {  // sub-key starts in the group's sorted order (counts complete since the barrier)
                uint32_t run = 0;
                for (int q = 0; q < 16; ++q) {
                    L.subst[q] = run;
                    run += L.subc[q];
                }
            }
            uint32_t run = incl - tot;
#pragma unroll
            for (int v = 0; v < 3; ++v) run += v < wave ? L.ws[v] : 0u;
#pragma unroll
            for (int q = 0; q < E; ++q) {
                const uint32_t lo = w[q] & 0xFFFFu, hi = w[q] >> 16;
                L.cnt[E * t + q] = run | ((run + lo) << 16);
                run += lo + hi;
            }
        }
        wm_barrier();
        uint32_t maxc = 0;
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int e = r * 256 + t;
            if (e < m) {
                const uint32_t bk = se[r];
                const uint32_t st = (L.cnt[bk >> 1] >> ((bk & 1u) * 16u)) & 0xFFFFu;
                const uint32_t b1 = bk + 1;
                const uint32_t en = b1 < (1u << NB) ? (L.cnt[b1 >> 1] >> ((b1 & 1u) * 16u)) & 0xFFFFu : (uint32_t)m;
                const uint32_t slot = st + sl[r];
                L.k[wm_pad(slot)] = (uint32_t)e;
                L.ov[slot] = key[r];
                se[r] = st | (en << 16);
                sl[r] = slot;
                maxc = max(maxc, en - st);
            }
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) maxc = max(maxc, (uint32_t)__shfl_xor((int)maxc, d, 64));
        if (lane == 0) L.wc[wave] = maxc;
        wm_barrier();
        maxc = max(max(L.wc[0], L.wc[1]), max(L.wc[2], L.wc[3]));
        uint32_t rank[E];
#pragma unroll
        for (int r = 0; r < E; ++r) rank[r] = 0u;
        // ROW_NUMBER / NTILE: rank among the bucket's rows by (order key, position); RANK: by order
        // key alone (rows of earlier buckets all have smaller keys: buckets are key ranges)
        constexpr bool kDirect = FN == QEH_WIN_ROW_NUMBER || FN == QEH_WIN_RANK || FN == QEH_WIN_NTILE;
        for (uint32_t j = 0; maxc > 1 && j < maxc; ++j) {
#pragma unroll
            for (int r = 0; r < E; ++r) {
                const uint32_t st = se[r] & 0xFFFFu, en = se[r] >> 16;
                if (st + j < en) {
                    if constexpr (FN == QEH_WIN_RANK) {
                        rank[r] += L.ov[st + j] < key[r] ? 1u : 0u;
                    } else {
                        const uint32_t q = L.k[wm_pad(st + j)];
                        rank[r] += wm_less(L.ov[st + j], q, key[r], (uint32_t)(r * 256 + t)) ? 1u : 0u;
                    }
                }
            }
        }
        if constexpr (kDirect) {
            // the function's value follows from the row's sorted index (ROW_NUMBER, NTILE) or from
            // the count of smaller keys (RANK) alone: written straight to the row's position in the
            // group, without materialising the sorted order
#pragma unroll
            for (int r = 0; r < E; ++r) {
                const int e = r * 256 + t;
                if (e >= m) continue;
                uint32_t i = (se[r] & 0xFFFFu) + rank[r];
                int64_t mg = m;  // rows of the row's PARTITION BY group
                if constexpr (SUB) {
                    i -= L.subst[ks[r]];
                    mg = L.subc[ks[r]];
                }
                uint32_t v;
                if constexpr (FN == QEH_WIN_NTILE) {
                    const int64_t q = mg / f.param, rm = mg % f.param, r0 = i;
                    v = (uint32_t)(r0 < rm * (q + 1) ? r0 / (q + 1) + 1 : rm + (r0 - rm * (q + 1)) / (q > 0 ? q : 1) + 1);
                } else {
                    v = i + 1u;
                }
                res[s + e] = (uint16_t)v;
            }
            wm_barrier();  // the group's LDS reads are done before the next group's writes
            continue;
        }
        wm_barrier();  // every bucket read is done: L.k takes the sorted order
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int e = r * 256 + t;
            if (e < m) L.k[wm_pad((se[r] & 0xFFFFu) + rank[r])] = (uint32_t)e | (sl[r] << 12) | (SUB ? ks[r] << 24 : 0u);
        }
        wm_barrier();
        // the function: wave w takes sorted indices [64 E w, 64 E (w + 1)) in E steps of 64
        uint32_t rv[E], pos[E];
        uint32_t carry = 0;
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int i = wave * 64 * E + r * 64 + lane;
            const bool live = i < m;
            const uint32_t x = live ? L.k[wm_pad(i)] : 0u;
            pos[r] = x & 4095u;
            rv[r] = 0u;
            // SUB: the row's own PARTITION BY group is its sub-key's run [sst, sst + mg) of the sorted group
            const uint32_t sst = SUB ? L.subst[x >> 24] : 0u;
            const int mg = SUB ? (int)L.subc[x >> 24] : m;
            if constexpr (FN < 0) {  // (valid flag, value bits of the source row at pos)
                int js;
                const bool ok = wm_value_src(f, i - (int)sst, mg, js);
                uint64_t bits = f.has_dflt ? (uint64_t)f.dflt : 0ull;
                rv[r] = f.has_dflt ? 1u : 0u;
                if (live && ok) {
                    bits = wm_decode(L.ov[(L.k[wm_pad(js + (int)sst)] >> 12) & 4095u], f.asc, f.odt);
                    rv[r] = 1u;
                }
                if (live) f.vout[s + pos[r]] = bits;
            } else if constexpr (FN == QEH_WIN_ROW_NUMBER) {
                rv[r] = (uint32_t)i + 1u;
            } else if constexpr (FN == QEH_WIN_NTILE) {
                const int64_t q = m / f.param, rm = m % f.param, r0 = i;
                rv[r] = (uint32_t)(r0 < rm * (q + 1) ? r0 / (q + 1) + 1 : rm + (r0 - rm * (q + 1)) / (q > 0 ? q : 1) + 1);
            } else {
                const uint64_t ov = live ? L.ov[(x >> 12) & 4095u] : 0ull;
                const uint64_t pv = (live && i > 0) ? L.ov[(L.k[wm_pad(i - 1)] >> 12) & 4095u] : 0ull;
                const uint32_t flag = (live && (i == (int)sst || pv != ov)) ? 1u : 0u;
                if constexpr (FN == QEH_WIN_RANK) {  // index of the last peer-group start at or before i
                    uint32_t v = flag ? (uint32_t)i : 0u;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const uint32_t u = __shfl_up(v, d, 64);
                        if (lane >= d) v = u > v ? u : v;
                    }
                    v = v > carry ? v : carry;
                    rv[r] = v;
                    carry = __shfl(v, 63, 64);
                } else {  // DENSE_RANK: peer-group starts so far
                    const uint32_t v = wave_incl_scan(flag) + carry;
                    rv[r] = v;
                    carry = __shfl(v, 63, 64);
                }
            }
        }
        if constexpr (FN == QEH_WIN_RANK || FN == QEH_WIN_DENSE_RANK) {  // carries across waves
            if (lane == 0) L.wt[wave] = carry;
            wm_barrier();
            uint32_t c = 0;
#pragma unroll
            for (int v = 0; v < 3; ++v)
                if (v < wave) c = FN == QEH_WIN_RANK ? max(c, L.wt[v]) : c + L.wt[v];
#pragma unroll
            for (int r = 0; r < E; ++r) rv[r] = FN == QEH_WIN_RANK ? max(rv[r], c) + 1u : rv[r] + c;
            if constexpr (SUB && FN == QEH_WIN_DENSE_RANK) {
                // rv = peer-group starts up to i across the whole group; a row's DENSE_RANK counts them
                // from its sub-key's first row (every order-key read is done: L.ov takes the counts)
                uint32_t *pc = (uint32_t *)L.ov;
#pragma unroll
                for (int r = 0; r < E; ++r) {
                    const int i = wave * 64 * E + r * 64 + lane;
                    if (i < m) pc[i] = rv[r];
                }
                wm_barrier();
#pragma unroll
                for (int r = 0; r < E; ++r) {
                    const int i = wave * 64 * E + r * 64 + lane;
                    if (i < m) rv[r] = rv[r] - pc[L.subst[L.k[wm_pad(i)] >> 24]] + 1u;
                }
            }
        }
#pragma unroll
        for (int r = 0; r < E; ++r)
            if (wave * 64 * E + r * 64 + lane < m) L.cnt[pos[r]] = rv[r];
        wm_barrier();
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int e = r * 256 + t;
            if (e < m) res[s + e] = (uint16_t)L.cnt[e];
        }
        wm_barrier();  // the group's LDS reads are done before the next group's writes
    }
}

// chunks of kWmCkTiles pass-2 tiles per bucket: cbase[b] = first chunk of bucket b (exclusive scan of
// the chunk counts, one workgroup: nb <= kWmDig), cbase[nb] = all chunks
__global__ __launch_bounds__(kWmBlock) void k_wm_chunk_base(const uint64_t *__restrict__ bstart, int nb,
                                                            uint32_t *__restrict__ cbase) {
    __shared__ uint32_t wsum[kWmBlock / 64];
    const int b = threadIdx.x;
    const int64_t rows = b < nb ? (int64_t)(bstart[b + 1] - bstart[b]) : 0;
    const uint32_t c = (uint32_t)((rows + (int64_t)kWmTile * kWmCkTiles - 1) / ((int64_t)kWmTile * kWmCkTiles));
    const uint32_t ex = block_excl_scan1024(c, wsum);
    if (b < nb) cbase[b] = ex;
    if (b == nb - 1) cbase[nb] = ex + c;
}

// inverse of pass 2: replay each bucket's tiles, gather the results run by run (group order ->
// pass-1 order).  The workgroups of one XCD (blockIdx % 8 -- the dispatcher deals workgroups to the 8
// XCDs in turn) take the chunks of one bucket together, each resuming pass 2's replay at the chunk's
// checkpoint: a group's 8-row result runs of consecutive tiles share lines, and the bucket's 2 MB of
// results is then gathered through that XCD's L2 once instead of once per tile (a workgroup per
// bucket refetched each line for every tile it spans).
// VAL (value functions): the value bits move beside the flags (res2v -> res1v, staged in LDS).
template <int DB, bool VAL = false>
__global__ __launch_bounds__(kWmBlock) __attribute__((amdgpu_waves_per_eu(DB == kWmAtomicRank && !VAL ? 8 : 4))) void k_wm2_inv2(WmShape sh, const uint64_t *__restrict__ bstart,
                                                       const uint32_t *__restrict__ cbase, const uint32_t *__restrict__ ckpt,
                                                       const uint16_t *__restrict__ i_kl,
                                                       const uint16_t *__restrict__ res2, uint16_t *__restrict__ res1,
                                                       const uint64_t *__restrict__ res2v, uint64_t *__restrict__ res1v) {
    __shared__ WmRankLds R;
    __shared__ uint32_t lpos[kWmDig];  // run positions (< n < 2^32: window_msd's bound)
    __shared__ uint16_t st_d[kWmTile], st_r[kWmTile];
    __shared__ uint64_t st_v[VAL ? kWmTile : 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int NJ = kWmTile / kWmBlock;
    const int dbits = sh.lb - sh.sb;
    const int64_t woff = (int64_t)wave * 64 * NJ + lane;
    // chunk ids split evenly per XCD as in pass 2, every per-th id of the XCD's range per workgroup (the
    // launch grid is a multiple of 8: every XCD slot has a workgroup)
    const int xcd = blockIdx.x & 7, per = gridDim.x >> 3, slot = blockIdx.x >> 3;
    const int64_t nck = (int64_t)cbase[sh.nb], c_lo = (int64_t)xcd * nck / 8, c_hi = (int64_t)(xcd + 1) * nck / 8;
    {
        for (int64_t jc = c_lo + slot; jc < c_hi; jc += per) {
            const int b = wm_chunk_bucket(cbase, 0, sh.nb - 1, jc);
            const int64_t s0 = (int64_t)bstart[b], s1 = (int64_t)bstart[b + 1], c = jc - (int64_t)cbase[b];
            const int64_t c0 = s0 + c * kWmCkTiles * kWmTile, c1 = std::min<int64_t>(s1, c0 + (int64_t)kWmCkTiles * kWmTile);
            lpos[tid] = ckpt[jc * kWmDig + tid];
            __syncthreads();
            uint32_t lx[NJ];
            auto load = [&](int64_t t0) {
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int64_t i = t0 + woff + j * 64;
                    lx[j] = __builtin_nontemporal_load(i_kl + (i < c1 ? i : c0));
                }
            };
            load(c0);
            for (int64_t t0 = c0; t0 < c1; t0 += kWmTile) {
                uint32_t d[NJ], slt[NJ];
                bool live[NJ];
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    live[j] = t0 + woff + j * 64 < c1;
                    d[j] = lx[j] >> sh.sb;
                }
                if (t0 + kWmTile < c1) load(t0 + kWmTile);
                const uint32_t tcnt = wm_stable_rank<NJ, DB>(d, live, dbits, slt, R);
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    if (live[j]) st_d[slt[j]] = (uint16_t)d[j];
                wm_barrier();
                const int m = (int)std::min<int64_t>(kWmTile, c1 - t0);
#pragma unroll 8
                for (int s = tid; s < m; s += kWmBlock) {
                    const uint32_t dd = st_d[s];
                    const uint32_t src = lpos[dd] + (uint32_t)s - R.lofs[dd];
                    st_r[s] = res2[src];
                    if (VAL) st_v[s] = res2v[src];
                }
                wm_barrier();
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    if (live[j]) {
                        __builtin_nontemporal_store(st_r[slt[j]], res1 + t0 + woff + j * 64);
                        if (VAL) __builtin_nontemporal_store(st_v[slt[j]], res1v + t0 + woff + j * 64);
                    }
                lpos[tid] += tcnt;
                wm_barrier();
            }
            __syncthreads();
        }
    }
}

// inverse of pass 1: replay pass 1's tiles chunk by chunk from its run positions, gather the results
// run by run and write them in input order as Int64
// VAL = 0: rank functions, out = Int64 results.  VAL = 4 / 8 (value functions): res1 holds valid
// flags, res1v the value bits (gathered beside them through LDS), written in VAL bytes (zero when
// NULL) plus a validity byte.
template <int KES, int DB, int VAL = 0>
__global__ __launch_bounds__(kWmBlock) __attribute__((amdgpu_waves_per_eu(DB == kWmAtomicRank && !VAL ? 8 : 4))) void k_wm2_inv1(ColRef key, WmShape sh, int64_t nchunk, const uint32_t *__restrict__ ckpt,
                                                       const uint16_t *__restrict__ res1, void *__restrict__ out,
                                                       const uint64_t *__restrict__ res1v, uint8_t *__restrict__ valid8) {
    __shared__ WmRankLds R;
    __shared__ uint32_t lpos[kWmDig];  // run positions (< n < 2^32: window_msd's bound)
    __shared__ uint16_t st_d[kWmTile], st_r[kWmTile];
    __shared__ uint64_t st_v[VAL ? kWmTile : 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int NJ = kWmTile / kWmBlock;
    const int dbits = wm_digit_bits(sh.nb);
    const int64_t woff = (int64_t)wave * 64 * NJ + lane;
    // chunk ids dealt per XCD range, every per-th id (see k_wm2_inv2)
    const int xcd = blockIdx.x & 7, per = gridDim.x >> 3, wslot = blockIdx.x >> 3;
    const int64_t j_lo = (int64_t)xcd * nchunk / 8, j_hi = (int64_t)(xcd + 1) * nchunk / 8;
    {
        for (int64_t jc = j_lo + wslot; jc < j_hi; jc += per) {
            const int64_t c0 = jc * kWmChunk, c1 = std::min<int64_t>(sh.n, c0 + kWmChunk);
            lpos[tid] = ckpt[jc * kWmDig + tid];
            __syncthreads();
            // the digit needs only the key's low 32 bits: (k - kmin) < 2^24 here, so its low word is
            // (low word of k) - (low word of kmin) -- half the registers of the prefetched keys
            uint32_t kv[NJ];
            auto load = [&](int64_t t0) {
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int64_t i = t0 + woff + j * 64;
                    kv[j] = __builtin_nontemporal_load((const uint32_t *)key.values + (i < c1 ? i : c0) * (KES / 4));
                }
            };
            load(c0);
            for (int64_t t0 = c0; t0 < c1; t0 += kWmTile) {
                uint32_t d[NJ], slot[NJ];
                bool live[NJ];
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    live[j] = t0 + woff + j * 64 < c1;
                    d[j] = ((kv[j] - (uint32_t)sh.kmin) & (uint32_t)sh.kmask) >> sh.lb;
                }
                if (t0 + kWmTile < c1) load(t0 + kWmTile);
                const uint32_t tcnt = wm_stable_rank<NJ, DB>(d, live, dbits, slot, R);
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    if (live[j]) st_d[slot[j]] = (uint16_t)d[j];
                wm_barrier();
                const int m = (int)std::min<int64_t>(kWmTile, c1 - t0);
#pragma unroll 8
                for (int s = tid; s < m; s += kWmBlock) {
                    const uint32_t dd = st_d[s];
                    const uint32_t src = lpos[dd] + (uint32_t)s - R.lofs[dd];
                    st_r[s] = res1[src];
                    if (VAL) st_v[s] = res1v[src];
                }
                wm_barrier();
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    if (!live[j]) continue;
                    const int64_t i = t0 + woff + j * 64;
                    if constexpr (VAL == 0) {
                        __builtin_nontemporal_store((int64_t)st_r[slot[j]], (int64_t *)out + i);
                    } else {
                        const bool ok = st_r[slot[j]] != 0;
                        const uint64_t v = st_v[slot[j]];
                        if constexpr (VAL == 8) __builtin_nontemporal_store(ok ? v : 0ull, (uint64_t *)out + i);
                        else __builtin_nontemporal_store(ok ? (uint32_t)v : 0u, (uint32_t *)out + i);
                        valid8[i] = ok ? 1 : 0;
                    }
                }
                lpos[tid] += tcnt;
                wm_barrier();
            }
            __syncthreads();
        }
    }
}

__global__ void k_wm_set2(uint64_t *a, uint64_t *b, uint64_t v) {
    if (threadIdx.x == 0) *a = v, *b = v;
}

// The id-free pipeline for the rank functions (shapes checked by window_msd).
// Value functions (LAG / LEAD / FIRST_VALUE / LAST_VALUE of the ORDER BY column, dflt = the
// default's bits or null): the sort writes each row's value bits beside its valid flag and the
// inverse passes move both.
static int window_noid(qeh_ctx *ctx, int func, const qeh_column &part, const qeh_column &order, bool asc, int64_t param,
                       const int64_t *dflt, WmShape sh, qeh_column *out, DevBuf *pre_counts = nullptr) {
    const int64_t n = sh.n;
    const int cus = ctx->props.multiProcessorCount;
    // the chunked passes deal chunk ids to the 8 XCDs by blockIdx % 8: a grid of whole octets, >= 8
    const int gx = std::max(8, (cus + 7) / 8 * 8);
    const int g1 = (int)((n + sh.span - 1) / sh.span);
    const bool value_fn = func >= QEH_WIN_LAG;
    const int esz = (order.dtype == QEH_DT_INT32 || order.dtype == QEH_DT_FLOAT32) ? 4 : 8;
    DevBuf cnt1, bsum, dst, claim, key1, kl1, key2, pst, bst, res2, res1, flag, res2v, res1v, valid8, ks2, cbase, ckpt, ckpt1;
    // pass 1's chunks of the input, and the blocks of its chunk scan
    const int64_t nchunk = (n + kWmChunk - 1) / kWmChunk, nblk = (nchunk + kWmScanB - 1) / kWmScanB;
    // pass 2's chunks: at most n / kWmChunk whole ones plus one partial per bucket
    const int64_t nck = n / kWmChunk + sh.nb + 1;
    if ((!pre_counts && cnt1.alloc(ctx, nchunk * kWmDig * 2)) || bsum.alloc(ctx, nblk * kWmDig * 4) ||
        dst.alloc(ctx, kWmDig * 4) || claim.alloc(ctx, 16 * 4) || key1.alloc(ctx, (n + kWmTile) * 8) ||
        kl1.alloc(ctx, (n + kWmTile) * 2) || key2.alloc(ctx, n * 8) || pst.alloc(ctx, (sh.nparts + 1) * 8) ||
        bst.alloc(ctx, ((int64_t)sh.nb + 1) * 8) || flag.alloc(ctx, 8) || (sh.sb && ks2.alloc(ctx, n)) ||
        cbase.alloc(ctx, ((int64_t)sh.nb + 1) * 4) || ckpt.alloc(ctx, nck * kWmDig * 4) || ckpt1.alloc(ctx, nchunk * kWmDig * 4))
        return fail(QEH_E_OOM, "window: out of device memory");
    const ColRef kc = make_colref(part), oc = make_colref(order);
    const int kes = part.dtype == QEH_DT_INT32 ? 4 : 8;
    const int oes = (order.dtype == QEH_DT_INT32 || order.dtype == QEH_DT_FLOAT32) ? 4 : 8;
    // stable tile ranking by LDS atomics (default) or by ballot matching (QEH_WM_BALLOT=1, A/B)
    const bool at = std::getenv("QEH_WM_BALLOT") == nullptr && lds_atomic_rank_ok(ctx);
    {
        KernelTimer kt(ctx, "window_partition");
        const uint16_t *counts = pre_counts ? pre_counts->as<uint16_t>() : cnt1.as<uint16_t>();
        if (!pre_counts)
            hipLaunchKernelGGL((kes == 4 ? k_wm_hist1<4, false> : k_wm_hist1<8, false>), dim3(g1), dim3(kWmBlock), 0, ctx->stream,
                               kc, sh, cnt1.as<uint16_t>(), nullptr);
        // run positions of every chunk (-> ckpt1) and the bucket starts (-> bst)
        hipLaunchKernelGGL(k_wm_cscan_blocks, dim3((unsigned)nblk), dim3(kWmBlock), 0, ctx->stream, counts, nchunk,
                           bsum.as<uint32_t>());
        hipLaunchKernelGGL(k_wm_cscan_top, dim3(1), dim3(kWmBlock), 0, ctx->stream, bsum.as<uint32_t>(), (int)nblk, (int)sh.nb,
                           dst.as<uint32_t>(), bst.as<uint64_t>());
        hipLaunchKernelGGL(k_wm_cscan_pos, dim3((unsigned)nblk), dim3(kWmBlock), 0, ctx->stream, counts, nchunk,
                           bsum.as<uint32_t>(), dst.as<uint32_t>(), ckpt1.as<uint32_t>());
        QEH_HIP(hipMemsetAsync(claim.p, 0, 16 * 4, ctx->stream));  // pass 1: [0, 8), pass 2: [8, 16)
        const bool d1 = wm_digit_bits(sh.nb) == 10;
#define QEH_WM_P1(K, O) (at ? k_wm2_pass1<K, O, kWmAtomicRank> : d1 ? k_wm2_pass1<K, O, 10> : k_wm2_pass1<K, O, -1>)
        hipLaunchKernelGGL(kes == 4 ? (oes == 4 ? QEH_WM_P1(4, 4) : QEH_WM_P1(4, 8))
                                    : (oes == 4 ? QEH_WM_P1(8, 4) : QEH_WM_P1(8, 8)),
                           dim3(gx), dim3(kWmBlock), 0, ctx->stream, kc, oc, asc ? 1 : 0, sh, nchunk,
                           ckpt1.as<uint32_t>(), claim.as<uint32_t>(), key1.as<uint64_t>(), kl1.as<uint16_t>());
        hipLaunchKernelGGL(k_wm_set2, dim3(1), dim3(64), 0, ctx->stream, bst.as<uint64_t>() + sh.nb,
                           pst.as<uint64_t>() + sh.nparts, (uint64_t)n);
#undef QEH_WM_P1
        if (!sh.exp) {  // (experiment runs: pass 1 only)
            hipLaunchKernelGGL(k_wm_chunk_base, dim3(1), dim3(kWmBlock), 0, ctx->stream, bst.as<uint64_t>(), (int)sh.nb,
                               cbase.as<uint32_t>());
            {
                DevBuf ccnt;
                QEH_TRY(ccnt.alloc(ctx, nck * kWmDig * 2));
                hipLaunchKernelGGL(k_wm2_chunk_hist, dim3(sh.nb), dim3(kWmBlock), 0, ctx->stream, sh, bst.as<uint64_t>(),
                                   cbase.as<uint32_t>(), kl1.as<uint16_t>(), ccnt.as<uint16_t>());
                hipLaunchKernelGGL(k_wm2_chunk_scan, dim3(sh.nb), dim3(kWmBlock), 0, ctx->stream, sh, bst.as<uint64_t>(),
                                   cbase.as<uint32_t>(), ccnt.as<uint16_t>(), ckpt.as<uint32_t>(), pst.as<uint64_t>());
#define QEH_WM_P2(KS) (at ? k_wm2_pass2<kWmAtomicRank, KS> : sh.lb - sh.sb == 10 ? k_wm2_pass2<10, KS> : k_wm2_pass2<-1, KS>)
                hipLaunchKernelGGL(sh.sb ? QEH_WM_P2(true) : QEH_WM_P2(false), dim3(gx), dim3(kWmBlock), 0, ctx->stream,
                                   sh, bst.as<uint64_t>(), cbase.as<uint32_t>(), ckpt.as<uint32_t>(), claim.as<uint32_t>() + 8, key1.as<uint64_t>(),
                                   kl1.as<uint16_t>(), key2.as<uint64_t>(), ks2.as<uint8_t>());
#undef QEH_WM_P2
            }
        }
    }
    QEH_HIP(hipGetLastError());
    if (sh.exp) {  // experiment runs stop after the partition passes (their outputs are not valid)
        QEH_HIP(hipStreamSynchronize(ctx->stream));
        return fail(QEH_E_UNSUPPORTED, "QEH_WM_EXP: experiment run, partition passes only");
    }
    key1.reset();
    DevBuf fbl;  // groups the counting sort queues for the network: count, then group numbers
    if (res2.alloc(ctx, n * 2) || fbl.alloc(ctx, (sh.nparts + 1) * 4) || (value_fn && res2v.alloc(ctx, n * 8)))
        return fail(QEH_E_OOM, "window: out of device memory");
    QEH_HIP(hipMemsetAsync(flag.p, 0, 8, ctx->stream));
    QEH_HIP(hipMemsetAsync(fbl.p, 0, 4, ctx->stream));
    WmFunc wf{};
    wf.func = func;
    wf.param = param;
#ifdef QEH_EXPERIMENTS  // (A/B builds only: the first skips the network and returns wrong row numbers)
    wf.skip_sort = std::getenv("QEH_WM_SKIP_SORT") ? 1 : 0;
    wf.no_count = std::getenv("QEH_WM_NO_COUNT") ? 1 : 0;
#endif
    wf.odt = order.dtype;
    wf.asc = asc ? 1 : 0;
    wf.has_dflt = dflt != nullptr;
    if (dflt) wf.dflt = esz == 8 ? *dflt : (int64_t)(uint32_t)*dflt;
    wf.vout = res2v.as<uint64_t>();
    const int nsort = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * 4, sh.nparts));
    {
        KernelTimer kt(ctx, "window_sort");
        auto launch = [&](auto vf) {
            constexpr bool VF = decltype(vf)::value;
            if (wf.no_count || wf.skip_sort) {
                hipLaunchKernelGGL((k_wm2_sort<false, false, VF>), dim3(nsort), dim3(kWmSortBlock), 0, ctx->stream, sh, wf,
                                   pst.as<uint64_t>(), key2.as<uint64_t>(), res2.as<uint16_t>(), flag.as<uint32_t>(), nullptr);
                hipLaunchKernelGGL((k_wm2_sort<true, false, VF>), dim3(nsort), dim3(kWmSortBlock), 0, ctx->stream, sh, wf,
                                   pst.as<uint64_t>(), key2.as<uint64_t>(), res2.as<uint16_t>(), flag.as<uint32_t>(), nullptr);
                return;
            }
            // counting sort, a workgroup per group, ranges of <= kWmCsMaxG groups per workgroup; then
            // the network for the queued (clustered) groups of both size classes
            const int64_t ncs = std::max<int64_t>(std::min<int64_t>((int64_t)cus * 16, sh.nparts),
                                                  (sh.nparts + kWmCsMaxG - 1) / kWmCsMaxG);
            auto csort = [&](auto fn) {
                constexpr int FN = decltype(fn)::value;
                hipLaunchKernelGGL((k_wm2_csort_wg<4, FN>), dim3((unsigned)ncs), dim3(256), 0, ctx->stream, sh, wf,
                                   pst.as<uint64_t>(), key2.as<uint64_t>(), res2.as<uint16_t>(), fbl.as<uint32_t>(),
                                   flag.as<uint32_t>(), nullptr);
                hipLaunchKernelGGL((k_wm2_csort_wg<8, FN>), dim3((unsigned)ncs), dim3(256), 0, ctx->stream, sh, wf,
                                   pst.as<uint64_t>(), key2.as<uint64_t>(), res2.as<uint16_t>(), fbl.as<uint32_t>(),
                                   flag.as<uint32_t>(), nullptr);
            };
            // groups of 2^sb keys (sh.sb > 0): the sub-key-aware sort, direct functions only
            auto csort_sub = [&](auto fn) {
                constexpr int FN = decltype(fn)::value;
                hipLaunchKernelGGL((k_wm2_csort_wg<4, FN, true>), dim3((unsigned)ncs), dim3(256), 0, ctx->stream, sh, wf,
                                   pst.as<uint64_t>(), key2.as<uint64_t>(), res2.as<uint16_t>(), fbl.as<uint32_t>(),
                                   flag.as<uint32_t>(), ks2.as<uint8_t>());
                hipLaunchKernelGGL((k_wm2_csort_wg<8, FN, true>), dim3((unsigned)ncs), dim3(256), 0, ctx->stream, sh, wf,
                                   pst.as<uint64_t>(), key2.as<uint64_t>(), res2.as<uint16_t>(), fbl.as<uint32_t>(),
                                   flag.as<uint32_t>(), ks2.as<uint8_t>());
            };
            if (sh.sb) {
                if (VF) csort_sub(std::integral_constant<int, -1>{});
                else if (func == QEH_WIN_ROW_NUMBER) csort_sub(std::integral_constant<int, QEH_WIN_ROW_NUMBER>{});
                else if (func == QEH_WIN_RANK) csort_sub(std::integral_constant<int, QEH_WIN_RANK>{});
                else if (func == QEH_WIN_DENSE_RANK) csort_sub(std::integral_constant<int, QEH_WIN_DENSE_RANK>{});
                else csort_sub(std::integral_constant<int, QEH_WIN_NTILE>{});
                return;  // (nothing was queued for the network)
            }
            if (VF) csort(std::integral_constant<int, -1>{});
            else if (func == QEH_WIN_ROW_NUMBER) csort(std::integral_constant<int, QEH_WIN_ROW_NUMBER>{});
            else if (func == QEH_WIN_RANK) csort(std::integral_constant<int, QEH_WIN_RANK>{});
            else if (func == QEH_WIN_DENSE_RANK) csort(std::integral_constant<int, QEH_WIN_DENSE_RANK>{});
            else csort(std::integral_constant<int, QEH_WIN_NTILE>{});
            hipLaunchKernelGGL((k_wm2_sort<false, true, VF>), dim3(nsort), dim3(kWmSortBlock), 0, ctx->stream, sh, wf,
                               pst.as<uint64_t>(), key2.as<uint64_t>(), res2.as<uint16_t>(), flag.as<uint32_t>(),
                               fbl.as<uint32_t>());
            hipLaunchKernelGGL((k_wm2_sort<true, true, VF>), dim3(nsort), dim3(kWmSortBlock), 0, ctx->stream, sh, wf,
                               pst.as<uint64_t>(), key2.as<uint64_t>(), res2.as<uint16_t>(), flag.as<uint32_t>(),
                               fbl.as<uint32_t>());
        };
        if (value_fn) launch(std::true_type{});
        else launch(std::false_type{});
    }
    QEH_HIP(hipGetLastError());
    uint32_t too_big = 0;
    QEH_TRY(read_small(ctx, &too_big, flag.p, 4));
    if (too_big) return kWindowMsdNotEligible;  // a group above 2048 rows / a long tie run: the LSD path
    key2.reset();
    if (res1.alloc(ctx, n * 2) || (value_fn && (res1v.alloc(ctx, n * 8) || valid8.alloc(ctx, n))))
        return fail(QEH_E_OOM, "window: out of device memory");
    QEH_TRY(alloc_column(ctx, value_fn ? order.dtype : QEH_DT_INT64, n, value_fn, out));
    {
        KernelTimer kt(ctx, "window_place");
        const bool d10 = sh.lb - sh.sb == 10;
        // the inverse passes' workgroups, all resident: two per CU where the kernel fits 64 VGPRs
        // (atomic ranking, rank functions), else one
        const int ginv = at && !value_fn ? gx * 2 : gx;
        hipLaunchKernelGGL(value_fn ? (at ? k_wm2_inv2<kWmAtomicRank, true> : d10 ? k_wm2_inv2<10, true> : k_wm2_inv2<-1, true>)
                                    : (at ? k_wm2_inv2<kWmAtomicRank, false> : d10 ? k_wm2_inv2<10, false> : k_wm2_inv2<-1, false>),
                           dim3(ginv), dim3(kWmBlock), 0, ctx->stream, sh, bst.as<uint64_t>(), cbase.as<uint32_t>(),
                           ckpt.as<uint32_t>(), kl1.as<uint16_t>(), res2.as<uint16_t>(), res1.as<uint16_t>(),
                           res2v.as<uint64_t>(), res1v.as<uint64_t>());
        const bool d1i = wm_digit_bits(sh.nb) == 10;
#define QEH_WM_I1(V)                                                                                                     \
    (kes == 4 ? (at ? k_wm2_inv1<4, kWmAtomicRank, V> : d1i ? k_wm2_inv1<4, 10, V> : k_wm2_inv1<4, -1, V>)                 \
              : (at ? k_wm2_inv1<8, kWmAtomicRank, V> : d1i ? k_wm2_inv1<8, 10, V> : k_wm2_inv1<8, -1, V>))
        hipLaunchKernelGGL(!value_fn ? QEH_WM_I1(0) : esz == 8 ? QEH_WM_I1(8) : QEH_WM_I1(4), dim3(ginv), dim3(kWmBlock), 0,
                           ctx->stream, kc, sh, nchunk, ckpt1.as<uint32_t>(), res1.as<uint16_t>(), out->values,
                           res1v.as<uint64_t>(), valid8.as<uint8_t>());
#undef QEH_WM_I1
    }
    if (hipGetLastError() != hipSuccess) {
        qeh_column_release(ctx, out);
        return fail(QEH_E_HIP, "window: kernel launch failed");
    }
    if (value_fn) {
        const int st = qeh_bytes_to_validity(ctx, valid8.as<uint8_t>(), n, out->validity);
        if (st != QEH_OK) {
            qeh_column_release(ctx, out);
            return st;
        }
        out->null_count = -1;
    }
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) {
        qeh_column_release(ctx, out);
        return fail(QEH_E_HIP, "window: kernel failed");
    }
    return QEH_OK;
}

static bool msd_forced() { return std::getenv("QEH_WINDOW_MSD") != nullptr; }

// Returns kWindowMsdNotEligible (nothing allocated into *out) when the shapes do not fit.
int window_msd(qeh_ctx *ctx, int func, const qeh_column &part, const qeh_column &order, bool asc, int64_t param,
               const qeh_column *arg, const int64_t *dflt, qeh_column *out) {
    if (std::getenv("QEH_NO_WINDOW_MSD")) return kWindowMsdNotEligible;
    if (func < QEH_WIN_ROW_NUMBER || func > QEH_WIN_LAST_VALUE) return kWindowMsdNotEligible;
    const bool value_fn = func >= QEH_WIN_LAG;
    // value functions of the ORDER BY column itself (the value is decoded from its order key)
    if (value_fn && (!arg || arg->values != order.values || arg->offset != order.offset || arg->dtype != order.dtype ||
                     arg->length != order.length))
        return kWindowMsdNotEligible;
    const int64_t n = part.length;
    if (n != order.length || n <= 0 || n >= ((int64_t)1 << 32) - 1) return kWindowMsdNotEligible;
    if (!msd_forced() && n < ((int64_t)1 << 20)) return kWindowMsdNotEligible;
    if (part.dtype != QEH_DT_INT64 && part.dtype != QEH_DT_INT32) return kWindowMsdNotEligible;
    if (order.dtype != QEH_DT_INT64 && order.dtype != QEH_DT_INT32 && order.dtype != QEH_DT_FLOAT64 &&
        order.dtype != QEH_DT_FLOAT32)
        return kWindowMsdNotEligible;
    if ((part.validity && part.null_count != 0) || (order.validity && order.null_count != 0)) return kWindowMsdNotEligible;
    if (!value_fn) {  // the three-level pipeline first (k_window3.hip); it declines shapes it cannot take
        const int s = window_w3(ctx, func, part, order, asc, param, out);
        if (s != kWindowMsdNotEligible) return s;
    }
    const int cus = ctx->props.multiProcessorCount;
    // pass-1 workgroups (row spans): two per CU by default, so the replaying inverse pass (80 KB of
    // LDS) runs two per CU and one's barrier phases overlap the other's memory phases
    int g1x = 2;
    if (const char *e = std::getenv("QEH_WM_G1X")) g1x = std::max(1, std::atoi(e));
    const int g1w = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * g1x, (n + kWmTile - 1) / kWmTile));
    const int64_t span = ((n + g1w - 1) / g1w + kWmChunk - 1) / kWmChunk * kWmChunk;  // whole chunks
    const int g1 = (int)((n + span - 1) / span);  // window_noid's pass-1 grid (histogram layout)
    // the key's min / max and the 20-bit shape's pass-1 histogram in one read (k_wm_hist1<KES, true>)
    WmShape sh{};
    sh.n = n;
    sh.span = span;
    sh.kmin = 0;
    sh.kmask = (1ull << 20) - 1;
    sh.lb = 10;
    DevBuf pre, mmp;
    QEH_TRY(pre.alloc(ctx, (size_t)kWmDig * ((n + kWmChunk - 1) / kWmChunk) * 2));
    QEH_TRY(mmp.alloc(ctx, sizeof(WmMinMax) * (size_t)g1));
    {
        KernelTimer kt(ctx, "window_partition");
        hipLaunchKernelGGL((part.dtype == QEH_DT_INT32 ? k_wm_hist1<4, true> : k_wm_hist1<8, true>), dim3(g1), dim3(kWmBlock), 0,
                           ctx->stream, make_colref(part), sh, pre.as<uint16_t>(), mmp.as<WmMinMax>());
        QEH_HIP(hipGetLastError());
    }
    std::vector<WmMinMax> mmh(g1);
    QEH_TRY(read_small(ctx, mmh.data(), mmp.p, sizeof(WmMinMax) * (size_t)g1));
    int64_t kmin = INT64_MAX, kmax = INT64_MIN;
    for (const WmMinMax &q : mmh) kmin = q.mn < kmin ? q.mn : kmin, kmax = q.mx > kmax ? q.mx : kmax;
    const uint64_t range = (uint64_t)kmax - (uint64_t)kmin + 1ull;
    // up to 2^20 keys: a group per key; up to 2^24: a group per 2^sb consecutive keys, told apart inside
    // the group sort
    const bool sub_ok = !std::getenv("QEH_WM_NO_SUB");
    if (range == 0 || range > (1ull << (sub_ok ? 24 : 20))) return kWindowMsdNotEligible;
    int bits = 0;
    while (bits < 64 && ((range - 1) >> bits)) ++bits;
    const bool folded = bits == 20 && !std::getenv("QEH_WM_LB") && !std::getenv("QEH_WM_NO_FOLD");
    sh.kmin = kmin;
    sh.kmask = ~0ull;
    sh.lb = bits > 10 ? bits - 10 : 0;
    sh.sb = bits > 20 ? bits - 20 : 0;
    if (const char *e = std::getenv("QEH_WM_LB")) {  // experiments: digit split between the passes
        const int lb = std::atoi(e);
        if (!sh.sb && lb >= sh.lb && lb <= 10 && lb <= bits) sh.lb = lb;
    }
    sh.nb = (int32_t)(((range - 1) >> sh.lb) + 1);
    sh.nparts = (int64_t)(((range - 1) >> sh.sb) + 1);  // groups (of 2^sb keys)
    if (folded) {  // groups = keys mod 2^20 (some empty): the histogram already taken is pass 1's
        sh.kmin = 0;
        sh.kmask = (1ull << 20) - 1;
        sh.lb = 10;
        sh.nb = kWmDig;
        sh.nparts = (int64_t)1 << 20;
    }
#ifdef QEH_EXPERIMENTS
    if (const char *e = std::getenv("QEH_WM_EXP")) sh.exp = std::atoi(e);
#endif
    return window_noid(ctx, func, part, order, asc, param, dflt, sh, out, folded ? &pre : nullptr);
}


// composite[i] = sum_j (k_j[i] - mn_j) * mul_j (mixed radix, the first key most significant)
struct WmKeys {
    ColRef c[4];
    int64_t mn[4], mul[4];
    int32_t n;
};
__global__ void k_wm_composite(WmKeys ks, int64_t n, int64_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t v = 0;
        for (int j = 0; j < ks.n; ++j) v += ((uint64_t)load_i64(ks.c[j], i) - (uint64_t)ks.mn[j]) * (uint64_t)ks.mul[j];
        out[i] = (int64_t)v;
    }
}

int window_msd_keys(qeh_ctx *ctx, int func, const qeh_column *parts, int n_part, const qeh_column &order, bool asc,
                    int64_t param, const qeh_column *arg, const int64_t *dflt, qeh_column *out) {
    if (n_part == 1) return window_msd(ctx, func, parts[0], order, asc, param, arg, dflt, out);
    if (n_part < 2 || n_part > 4 || std::getenv("QEH_NO_WINDOW_MSD")) return kWindowMsdNotEligible;
    const int64_t n = parts[0].length;
    if (!msd_forced() && n < ((int64_t)1 << 20)) return kWindowMsdNotEligible;
    const uint64_t bound = 1ull << (std::getenv("QEH_WM_NO_SUB") ? 20 : 24);
    WmKeys ks{};
    ks.n = n_part;
    uint64_t prod = 1, rng[4] = {};
    for (int j = 0; j < n_part; ++j) {
        const qeh_column &c = parts[j];
        if (c.length != n || (c.dtype != QEH_DT_INT64 && c.dtype != QEH_DT_INT32) || (c.validity && c.null_count != 0))
            return kWindowMsdNotEligible;
        int64_t mn, mx, cnt;
        QEH_TRY(column_minmax(ctx, c, &mn, &mx, &cnt));
        if (cnt != n) return kWindowMsdNotEligible;
        rng[j] = (uint64_t)mx - (uint64_t)mn + 1ull;
        if (rng[j] == 0 || rng[j] > bound || prod * rng[j] > bound) return kWindowMsdNotEligible;
        ks.c[j] = make_colref(c);
        ks.mn[j] = mn;
        prod *= rng[j];
    }
    // multipliers: the product of the ranges of the keys after j (the last key least significant)
    uint64_t m = 1;
    for (int j = n_part - 1; j >= 0; --j) {
        ks.mul[j] = (int64_t)m;
        m *= rng[j];
    }
    qeh_column comp{};
    QEH_TRY(alloc_column(ctx, QEH_DT_INT64, n, false, &comp));
    {
        KernelTimer kt(ctx, "window_partition");
        hipLaunchKernelGGL(k_wm_composite, dim3(grid_for(ctx, n, 256 * 8, 8)), dim3(256), 0, ctx->stream, ks, n,
                           (int64_t *)comp.values);
    }
    if (hipGetLastError() != hipSuccess) {
        qeh_column_release(ctx, &comp);
        return fail(QEH_E_HIP, "window: composite key launch failed");
    }
    const int s = window_msd(ctx, func, comp, order, asc, param, arg, dflt, out);
    qeh_column_release(ctx, &comp);
    return s;
}

}  // namespace qeh
