// Window functions over one bounded integer PARTITION BY key and one ORDER BY key, by
// partitioning instead of a full sort (BASELINE config 5: ROW_NUMBER() OVER (PARTITION BY k
// ORDER BY v), k in [0, 2^20), 1e9 rows).
//
// Semantics as qeh_row_number / qeh_window (k_sort.hip): rows numbered 1.. within each partition
// in ORDER BY order, ties by input position (docs/WINDOW_FUNCTIONS.md:44-65); RANK with gaps,
// DENSE_RANK without, NTILE's first size % n buckets one row larger (:67-140); output aligned to
// input order.  The LSD path of k_sort.hip sorts 40-bit (k, v) pair keys in five 8-bit passes
// and scatters the numbers back with random 8-B stores; this path moves each row a bounded
// number of times with coalesced writes:
//   1. k_wm_hist1 + k_wm_pass1: a 1024-way partition of (order key, row id, low key bits) by the
//      key's high bits (per-workgroup histograms, one scan, LDS-staged runs);
//   2. k_wm_pass2: inside each bucket (one workgroup per bucket) a 1024-way partition by the
//      key's low bits -- every PARTITION BY group is now contiguous, its start in pstart[];
//   3. k_wm_sort: one wave per group sorts (order key, row id) in registers (bitonic network,
//      lane-major layout: distances below the per-lane width are register swaps), computes the
//      function, emits (row id, result) pairs in group order, and counts them per output window;
//   4. k_wm_pass5a / k_wm_pass5b: the pairs are partitioned by row id into windows of 2^15 rows
//      (window starts are exact: every row id occurs once);
//   5. k_wm_place: a workgroup stages one window's results in LDS and writes its rows in order.
// Partitions are ranked with LDS atomics (unordered within a tile): the sort compares
// (order key, row id), so nothing depends on stability.  Groups above 2048 rows (skew) and
// shapes outside the limits return kWindowMsdNotEligible and the caller takes the LSD path.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "../../include/qeh_plan.h"
#include "device_common.h"
#include "ops.h"

namespace qeh {

constexpr int kWmBlock = 1024;                // partition passes: one workgroup per CU
constexpr int kWmTile = 8192;                 // rows per partition-pass tile (8 per thread)
constexpr int kWmDig = 1024;                  // digits per partition pass
constexpr int kWmSortBlock = 256;             // group sort: 4 waves
constexpr int kWmMaxR = 32;                   // rows per lane in the group sort -> groups <= 2048
constexpr int kWmWinBits = 15;                // output window = 2^15 rows (128 KB of u32 in LDS)

// exclusive scan of one value per thread over a 1024-thread block; *total gets the sum
__device__ __forceinline__ uint32_t block_excl_scan1024(uint32_t v, uint32_t *wsum, uint32_t *total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(v);
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    if (wave == 0) {
        const uint32_t w = lane < kWmBlock / 64 ? wsum[lane] : 0u;
        const uint32_t wi = wave_incl_scan(w);
        if (lane < kWmBlock / 64) wsum[lane] = wi - w;
        if (lane == kWmBlock / 64 - 1 && total) *total = wi;
    }
    __syncthreads();
    return inc - v + wsum[wave];
}

// order key -> unsigned sortable 64-bit (ascending; descending flips every bit)
__device__ __forceinline__ uint64_t wm_order_key(const ColRef &c, int64_t row, int asc) {
    const int64_t x = load_i64(c, row);
    const int64_t o = (c.dtype == QEH_DT_FLOAT32 || c.dtype == QEH_DT_FLOAT64) ? f64_order_key(as_f64(x)) : x;
    const uint64_t u = (uint64_t)o ^ 0x8000000000000000ull;
    return asc ? u : ~u;
}

struct WmShape {
    int64_t n;
    int64_t kmin;
    int32_t lb;        // low key bits (pass 2 digit); high digit = (k - kmin) >> lb
    int32_t nb;        // buckets (high digits in use)
    int64_t nparts;    // key range = number of PARTITION BY groups (some empty)
    int64_t span;      // rows per workgroup in pass 1 (multiple of kWmTile)
};

// ---- pass 1: histogram of the high key digit per workgroup row range -------------------------
__global__ __launch_bounds__(kWmBlock) void k_wm_hist1(ColRef key, WmShape sh, uint32_t *__restrict__ counts) {
    __shared__ uint32_t h[kWmDig];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t r0 = (int64_t)blockIdx.x * sh.span, r1 = std::min<int64_t>(sh.n, r0 + sh.span);
    for (int64_t i = r0 + threadIdx.x; i < r1; i += kWmBlock) {
        const uint64_t kk = (uint64_t)load_i64(key, i) - (uint64_t)sh.kmin;
        atomicAdd(&h[kk >> sh.lb], 1u);
    }
    __syncthreads();
    counts[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] = h[threadIdx.x];  // digit-major
}

// ---- pass 1: partition (order key, row id, low key bits) by the high digit -------------------
__global__ __launch_bounds__(kWmBlock) void k_wm_pass1(ColRef key, ColRef ord, int asc, WmShape sh,
                                                       const uint64_t *__restrict__ base, uint64_t *__restrict__ o_key,
                                                       uint32_t *__restrict__ o_id, uint16_t *__restrict__ o_kl) {
    __shared__ uint32_t cnt[kWmDig], lofs[kWmDig], wsum[16];
    __shared__ uint64_t lpos[kWmDig];
    __shared__ uint64_t st_key[kWmTile];
    __shared__ uint32_t st_id[kWmTile];
    __shared__ uint16_t st_kl[kWmTile], st_d[kWmTile];
    const int tid = threadIdx.x;
    cnt[tid] = 0;
    lpos[tid] = base[(int64_t)tid * gridDim.x + blockIdx.x];
    __syncthreads();
    const uint32_t lmask = (1u << sh.lb) - 1u;
    const int64_t r0 = (int64_t)blockIdx.x * sh.span, r1 = std::min<int64_t>(sh.n, r0 + sh.span);
    for (int64_t t0 = r0; t0 < r1; t0 += kWmTile) {
        uint32_t d[8], rk[8], kl[8];
        uint64_t ok[8];
        bool live[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int64_t i = t0 + j * kWmBlock + tid;
            live[j] = i < r1;
            const int64_t ii = live[j] ? i : r0;
            const uint64_t kk = (uint64_t)load_i64(key, ii) - (uint64_t)sh.kmin;
            d[j] = (uint32_t)(kk >> sh.lb);
            kl[j] = (uint32_t)kk & lmask;
            ok[j] = wm_order_key(ord, ii, asc);
            rk[j] = live[j] ? atomicAdd(&cnt[d[j]], 1u) : 0u;
        }
        __syncthreads();
        const uint32_t c = cnt[tid];
        lofs[tid] = block_excl_scan1024(c, wsum, nullptr);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (!live[j]) continue;
            const uint32_t s = lofs[d[j]] + rk[j];
            st_key[s] = ok[j];
            st_id[s] = (uint32_t)(t0 + j * kWmBlock + tid);
            st_kl[s] = (uint16_t)kl[j];
            st_d[s] = (uint16_t)d[j];
        }
        __syncthreads();
        const int m = (int)std::min<int64_t>(kWmTile, r1 - t0);
        for (int s = tid; s < m; s += kWmBlock) {
            const uint32_t dd = st_d[s];
            const uint64_t p = lpos[dd] + (uint64_t)(s - (int)lofs[dd]);
            o_key[p] = st_key[s];
            o_id[p] = st_id[s];
            o_kl[p] = st_kl[s];
        }
        __syncthreads();
        lpos[tid] += c;
        cnt[tid] = 0;
        __syncthreads();
    }
}

// ---- pass 2: inside each bucket, partition by the low digit; group starts -> pstart ----------
__global__ __launch_bounds__(kWmBlock) void k_wm_pass2(WmShape sh, const uint64_t *__restrict__ bstart,
                                                       const uint64_t *__restrict__ i_key, const uint32_t *__restrict__ i_id,
                                                       const uint16_t *__restrict__ i_kl, uint64_t *__restrict__ o_key,
                                                       uint32_t *__restrict__ o_id, uint64_t *__restrict__ pstart) {
    __shared__ uint32_t cnt[kWmDig], lofs[kWmDig], wsum[16];
    __shared__ uint64_t lpos[kWmDig];
    __shared__ uint64_t st_key[kWmTile];
    __shared__ uint32_t st_id[kWmTile];
    __shared__ uint16_t st_d[kWmTile];
    const int tid = threadIdx.x;
    const int64_t L = (int64_t)1 << sh.lb;
    for (int b = blockIdx.x; b < sh.nb; b += gridDim.x) {
        const uint64_t s0 = bstart[b], s1 = bstart[b + 1];
        cnt[tid] = 0;
        __syncthreads();
        for (uint64_t i = s0 + tid; i < s1; i += kWmBlock) atomicAdd(&cnt[i_kl[i]], 1u);
        __syncthreads();
        const uint32_t c = cnt[tid];
        const uint32_t ex = block_excl_scan1024(c, wsum, nullptr);
        const int64_t part = (int64_t)b * L + tid;
        if (tid < L && part < sh.nparts) pstart[part] = s0 + ex;
        lpos[tid] = s0 + ex;
        cnt[tid] = 0;
        __syncthreads();
        for (uint64_t t0 = s0; t0 < s1; t0 += kWmTile) {
            uint32_t d[8], rk[8];
            bool live[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint64_t i = t0 + (uint64_t)(j * kWmBlock + tid);
                live[j] = i < s1;
                d[j] = live[j] ? i_kl[i] : 0u;
                rk[j] = live[j] ? atomicAdd(&cnt[d[j]], 1u) : 0u;
            }
            __syncthreads();
            const uint32_t cc = cnt[tid];
            lofs[tid] = block_excl_scan1024(cc, wsum, nullptr);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (!live[j]) continue;
                const uint64_t i = t0 + (uint64_t)(j * kWmBlock + tid);
                const uint32_t s = lofs[d[j]] + rk[j];
                st_key[s] = i_key[i];
                st_id[s] = i_id[i];
                st_d[s] = (uint16_t)d[j];
            }
            __syncthreads();
            const int m = (int)std::min<uint64_t>(kWmTile, s1 - t0);
            for (int s = tid; s < m; s += kWmBlock) {
                const uint32_t dd = st_d[s];
                const uint64_t p = lpos[dd] + (uint64_t)(s - (int)lofs[dd]);
                o_key[p] = st_key[s];
                o_id[p] = st_id[s];
            }
            __syncthreads();
            lpos[tid] += cc;
            cnt[tid] = 0;
            __syncthreads();
        }
    }
}

// ---- group sort: one wave per PARTITION BY group --------------------------------------------
__device__ __forceinline__ bool kv_less(uint64_t ak, uint32_t ai, uint64_t bk, uint32_t bi) {
    return ak < bk || (ak == bk && ai < bi);
}

struct WmFunc {
    int32_t func;      // QEH_WIN_ROW_NUMBER / RANK / DENSE_RANK / NTILE
    int64_t param;     // NTILE buckets
    int32_t win_shift; // pass-5a digit = row id >> win_shift
};

// Elements in lane-major order: element e = lane * R + r.  Sorted ascending by (key, id).
// The network is unrolled by template recursion (stage KK, distance J), so every register
// index is a compile-time constant: no dynamic indexing, no scratch.
template <int R, int KK, int J>
__device__ __forceinline__ void bitonic_stage(uint64_t (&k)[R], uint32_t (&id)[R], int lane) {
    if constexpr (J < R) {  // partner in this lane's registers
#pragma unroll
        for (int r = 0; r < R; ++r) {
            constexpr int dummy = 0;
            (void)dummy;
            const int r2 = r ^ J;
            if (r2 > r) {
                const int e = lane * R + r;
                const bool asc = (e & KK) == 0;
                const bool sw = asc ? kv_less(k[r2], id[r2], k[r], id[r]) : kv_less(k[r], id[r], k[r2], id[r2]);
                const uint64_t a = k[r], b = k[r2];
                const uint32_t ia = id[r], ib = id[r2];
                k[r] = sw ? b : a, k[r2] = sw ? a : b;
                id[r] = sw ? ib : ia, id[r2] = sw ? ia : ib;
            }
        }
    } else {  // partner lane = lane ^ (J / R), same register
        constexpr int LJ = J / R;
        const bool lower = (lane & LJ) == 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int e = lane * R + r;
            const bool asc = (e & KK) == 0;
            const uint64_t ok = __shfl_xor(k[r], LJ, 64);
            const uint32_t oi = __shfl_xor(id[r], LJ, 64);
            // the lower element keeps the min when ascending, the upper the max
            const bool take = (lower == asc) ? kv_less(ok, oi, k[r], id[r]) : kv_less(k[r], id[r], ok, oi);
            k[r] = take ? ok : k[r];
            id[r] = take ? oi : id[r];
        }
    }
}

template <int R, int KK, int J>
__device__ __forceinline__ void bitonic_merge(uint64_t (&k)[R], uint32_t (&id)[R], int lane) {
    if constexpr (J > 0) {
        bitonic_stage<R, KK, J>(k, id, lane);
        bitonic_merge<R, KK, J / 2>(k, id, lane);
    }
}

template <int R, int KK>
__device__ __forceinline__ void bitonic_sort(uint64_t (&k)[R], uint32_t (&id)[R], int lane) {
    if constexpr (KK <= 64 * R) {
        bitonic_merge<R, KK, KK / 2>(k, id, lane);
        bitonic_sort<R, KK * 2>(k, id, lane);
    }
}

template <int R>
__device__ __forceinline__ void wave_bitonic(uint64_t (&k)[R], uint32_t (&id)[R], int lane) {
    bitonic_sort<R, 2>(k, id, lane);
}

template <int R>
__device__ void wm_group(const uint64_t *__restrict__ gkey, const uint32_t *__restrict__ gid, int64_t s, int m,
                         const WmFunc &f, uint64_t *__restrict__ pairs, uint32_t *__restrict__ whist, int lane) {
    uint64_t k[R];
    uint32_t id[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = lane * R + r;
        k[r] = e < m ? gkey[s + e] : ~0ull;
        id[r] = e < m ? gid[s + e] : 0xFFFFFFFFu;
    }
    wave_bitonic<R>(k, id, lane);
    uint32_t res[R];
    if (f.func == QEH_WIN_ROW_NUMBER) {
#pragma unroll
        for (int r = 0; r < R; ++r) res[r] = (uint32_t)(lane * R + r + 1);
    } else if (f.func == QEH_WIN_NTILE) {
        const int64_t q = m / f.param, rm = m % f.param;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t r0 = lane * R + r;
            res[r] = (uint32_t)(r0 < rm * (q + 1) ? r0 / (q + 1) + 1 : rm + (r0 - rm * (q + 1)) / (q > 0 ? q : 1) + 1);
        }
    } else {
        // peer flags (a new ORDER BY value starts a peer group); the previous element of
        // register 0 is the previous lane's last register
        const uint64_t prev_last = __shfl_up(k[R - 1], 1, 64);
        uint32_t flag[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint64_t pk = r > 0 ? k[r - 1] : prev_last;
            flag[r] = (lane == 0 && r == 0) || pk != k[r] ? 1u : 0u;
        }
        if (f.func == QEH_WIN_RANK) {
            // rank = 1 + position of the last peer-group start at or before e (max-scan)
            uint32_t run = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (flag[r]) run = (uint32_t)(lane * R + r);
                res[r] = run;
            }
            uint32_t carry = run;  // lane's last start (0 if none: lane 0 always has one)
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t t = __shfl_up(carry, d, 64);
                if (lane >= d) carry = t > carry ? t : carry;
            }
            uint32_t before = __shfl_up(carry, 1, 64);
            if (lane == 0) before = 0;
            bool seen = false;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                seen = seen || flag[r];
                res[r] = (seen ? res[r] : before) + 1u;
            }
        } else {  // DENSE_RANK: inclusive count of peer-group starts
            uint32_t tot = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) tot += flag[r];
            const uint32_t incl = wave_incl_scan(tot);
            uint32_t acc = incl - tot;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                acc += flag[r];
                res[r] = acc;
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = lane * R + r;
        if (e < m) {
            pairs[s + e] = ((uint64_t)id[r] << 32) | res[r];
            atomicAdd(&whist[id[r] >> f.win_shift], 1u);
        }
    }
}

// Workgroup w owns groups [g0, g1) (contiguous rows [pstart[g0], pstart[g1])); its waves take
// the groups in turn.  Window histograms are added to counts[digit * grid + w] for pass 5a.
// BIG = false: groups of <= 1024 rows (register width <= 16); BIG = true: 1025..2048 rows, in a
// kernel of its own so the wide network's registers do not limit the common case.
template <bool BIG>
__global__ __launch_bounds__(kWmSortBlock) void k_wm_sort(WmShape sh, WmFunc f, const uint64_t *__restrict__ pstart,
                                                          const uint64_t *__restrict__ gkey, const uint32_t *__restrict__ gid,
                                                          uint64_t *__restrict__ pairs, uint32_t *__restrict__ counts,
                                                          uint32_t *__restrict__ too_big) {
    __shared__ uint32_t whist[kWmDig];
    for (int i = threadIdx.x; i < kWmDig; i += kWmSortBlock) whist[i] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t g0 = (int64_t)blockIdx.x * sh.nparts / gridDim.x, g1 = (int64_t)(blockIdx.x + 1) * sh.nparts / gridDim.x;
    for (int64_t g = g0 + wave; g < g1; g += kWmSortBlock / 64) {
        const int64_t s = (int64_t)pstart[g];
        const int64_t m = (int64_t)pstart[g + 1] - s;
        if (m <= 0) continue;
        if (BIG) {
            if (m <= 1024) continue;
            if (m > 64 * kWmMaxR) {
                if (lane == 0) *too_big = 1u;
                continue;
            }
            wm_group<32>(gkey, gid, s, (int)m, f, pairs, whist, lane);
        } else {
            const int mi = (int)m;
            if (mi > 1024) continue;
            if (mi <= 64) wm_group<1>(gkey, gid, s, mi, f, pairs, whist, lane);
            else if (mi <= 128) wm_group<2>(gkey, gid, s, mi, f, pairs, whist, lane);
            else if (mi <= 256) wm_group<4>(gkey, gid, s, mi, f, pairs, whist, lane);
            else if (mi <= 512) wm_group<8>(gkey, gid, s, mi, f, pairs, whist, lane);
            else wm_group<16>(gkey, gid, s, mi, f, pairs, whist, lane);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kWmDig; i += kWmSortBlock)
        if (whist[i]) atomicAdd(&counts[(int64_t)i * gridDim.x + blockIdx.x], whist[i]);
}

// ---- pass 5a: pairs partitioned by row id into windows (global, ranges = k_wm_sort's) --------
__global__ __launch_bounds__(kWmBlock) void k_wm_pass5a(WmShape sh, int nsort, int win_shift,
                                                        const uint64_t *__restrict__ pstart,
                                                        const uint64_t *__restrict__ base, const uint64_t *__restrict__ in,
                                                        uint64_t *__restrict__ out) {
    __shared__ uint32_t cnt[kWmDig], lofs[kWmDig], wsum[16];
    __shared__ uint64_t lpos[kWmDig];
    __shared__ uint64_t st[kWmTile];
    __shared__ uint16_t st_d[kWmTile];
    const int tid = threadIdx.x;
    for (int w = blockIdx.x; w < nsort; w += gridDim.x) {
        const int64_t g0 = (int64_t)w * sh.nparts / nsort, g1 = (int64_t)(w + 1) * sh.nparts / nsort;
        const uint64_t r0 = pstart[g0], r1 = pstart[g1];
        cnt[tid] = 0;
        lpos[tid] = base[(int64_t)tid * nsort + w];
        __syncthreads();
        for (uint64_t t0 = r0; t0 < r1; t0 += kWmTile) {
            uint32_t d[8], rk[8];
            uint64_t v[8];
            bool live[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint64_t i = t0 + (uint64_t)(j * kWmBlock + tid);
                live[j] = i < r1;
                v[j] = live[j] ? in[i] : 0ull;
                d[j] = (uint32_t)((v[j] >> 32) >> win_shift);
                rk[j] = live[j] ? atomicAdd(&cnt[d[j]], 1u) : 0u;
            }
            __syncthreads();
            const uint32_t c = cnt[tid];
            lofs[tid] = block_excl_scan1024(c, wsum, nullptr);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (!live[j]) continue;
                const uint32_t s = lofs[d[j]] + rk[j];
                st[s] = v[j];
                st_d[s] = (uint16_t)d[j];
            }
            __syncthreads();
            const int m = (int)std::min<uint64_t>(kWmTile, r1 - t0);
            for (int s = tid; s < m; s += kWmBlock) {
                const uint32_t dd = st_d[s];
                out[lpos[dd] + (uint64_t)(s - (int)lofs[dd])] = st[s];
            }
            __syncthreads();
            lpos[tid] += c;
            cnt[tid] = 0;
            __syncthreads();
        }
        __syncthreads();
    }
}

// ---- pass 5b: inside each window, pairs partitioned by output sub-window ----------------------
// Window w holds exactly the row ids [w << win_shift, (w + 1) << win_shift): its region and
// every sub-window's place are known without a histogram.
__global__ __launch_bounds__(kWmBlock) void k_wm_pass5b(int64_t n, int win_shift, int64_t nwin,
                                                        const uint64_t *__restrict__ in, uint64_t *__restrict__ out) {
    __shared__ uint32_t cnt[kWmDig], lofs[kWmDig], wsum[16];
    __shared__ uint64_t lpos[kWmDig];
    __shared__ uint64_t st[kWmTile];
    __shared__ uint16_t st_d[kWmTile];
    const int tid = threadIdx.x;
    const uint32_t dmask = (1u << (win_shift - kWmWinBits)) - 1u;
    for (int64_t w = blockIdx.x; w < nwin; w += gridDim.x) {
        const uint64_t r0 = (uint64_t)w << win_shift, r1 = std::min<uint64_t>((uint64_t)n, (uint64_t)(w + 1) << win_shift);
        cnt[tid] = 0;
        lpos[tid] = r0 + ((uint64_t)tid << kWmWinBits);
        __syncthreads();
        for (uint64_t t0 = r0; t0 < r1; t0 += kWmTile) {
            uint32_t d[8], rk[8];
            uint64_t v[8];
            bool live[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint64_t i = t0 + (uint64_t)(j * kWmBlock + tid);
                live[j] = i < r1;
                v[j] = live[j] ? in[i] : 0ull;
                d[j] = (uint32_t)((v[j] >> 32) >> kWmWinBits) & dmask;
                rk[j] = live[j] ? atomicAdd(&cnt[d[j]], 1u) : 0u;
            }
            __syncthreads();
            const uint32_t c = cnt[tid];
            lofs[tid] = block_excl_scan1024(c, wsum, nullptr);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (!live[j]) continue;
                const uint32_t s = lofs[d[j]] + rk[j];
                st[s] = v[j];
                st_d[s] = (uint16_t)d[j];
            }
            __syncthreads();
            const int m = (int)std::min<uint64_t>(kWmTile, r1 - t0);
            for (int s = tid; s < m; s += kWmBlock) {
                const uint32_t dd = st_d[s];
                out[lpos[dd] + (uint64_t)(s - (int)lofs[dd])] = st[s];
            }
            __syncthreads();
            lpos[tid] += c;
            cnt[tid] = 0;
            __syncthreads();
        }
        __syncthreads();
    }
}

// ---- placement: one output window at a time through LDS, rows written in order ---------------
__global__ __launch_bounds__(kWmBlock) void k_wm_place(int64_t n, const uint64_t *__restrict__ pairs,
                                                       int64_t *__restrict__ out) {
    __shared__ uint32_t buf[1 << kWmWinBits];
    const int64_t nw = (n + (1 << kWmWinBits) - 1) >> kWmWinBits;
    for (int64_t w = blockIdx.x; w < nw; w += gridDim.x) {
        const int64_t r0 = w << kWmWinBits, r1 = std::min<int64_t>(n, r0 + (1 << kWmWinBits));
        for (int64_t i = r0 + threadIdx.x; i < r1; i += kWmBlock) {
            const uint64_t p = pairs[i];
            buf[(uint32_t)(p >> 32) - (uint32_t)r0] = (uint32_t)p;
        }
        __syncthreads();
        for (int64_t i = r0 + threadIdx.x; i < r1; i += kWmBlock) out[i] = (int64_t)buf[i - r0];
        __syncthreads();
    }
}

__global__ void k_wm_set2(uint64_t *a, uint64_t *b, uint64_t v) {
    if (threadIdx.x == 0) *a = v, *b = v;
}

static bool msd_forced() { return std::getenv("QEH_WINDOW_MSD") != nullptr; }

// Returns kWindowMsdNotEligible (nothing allocated into *out) when the shapes do not fit.
int window_msd(qeh_ctx *ctx, int func, const qeh_column &part, const qeh_column &order, bool asc, int64_t param,
               qeh_column *out) {
    if (std::getenv("QEH_NO_WINDOW_MSD")) return kWindowMsdNotEligible;
    if (func != QEH_WIN_ROW_NUMBER && func != QEH_WIN_RANK && func != QEH_WIN_DENSE_RANK && func != QEH_WIN_NTILE)
        return kWindowMsdNotEligible;
    const int64_t n = part.length;
    if (n != order.length || n <= 0 || n >= ((int64_t)1 << 32) - 1) return kWindowMsdNotEligible;
    if (!msd_forced() && n < ((int64_t)1 << 20)) return kWindowMsdNotEligible;
    if (part.dtype != QEH_DT_INT64 && part.dtype != QEH_DT_INT32) return kWindowMsdNotEligible;
    if (order.dtype != QEH_DT_INT64 && order.dtype != QEH_DT_INT32 && order.dtype != QEH_DT_FLOAT64 &&
        order.dtype != QEH_DT_FLOAT32)
        return kWindowMsdNotEligible;
    if ((part.validity && part.null_count != 0) || (order.validity && order.null_count != 0)) return kWindowMsdNotEligible;
    int64_t kmin, kmax, kval;
    QEH_TRY(column_minmax(ctx, part, &kmin, &kmax, &kval));
    if (kval != n) return kWindowMsdNotEligible;
    const uint64_t range = (uint64_t)kmax - (uint64_t)kmin + 1ull;
    if (range == 0 || range > (1ull << 20)) return kWindowMsdNotEligible;
    int bits = 0;
    while (bits < 64 && ((range - 1) >> bits)) ++bits;
    WmShape sh{};
    sh.n = n;
    sh.kmin = kmin;
    sh.lb = bits > 10 ? bits - 10 : 0;
    sh.nb = (int32_t)(((range - 1) >> sh.lb) + 1);
    sh.nparts = (int64_t)range;
    const int cus = ctx->props.multiProcessorCount;
    const int g1 = (int)std::max<int64_t>(1, std::min<int64_t>(cus, (n + kWmTile - 1) / kWmTile));
    sh.span = ((n + g1 - 1) / g1 + kWmTile - 1) / kWmTile * kWmTile;
    // output windows: nwb bits of row id above the 2^15-row placement window
    int nbits = 0;
    while (nbits < 63 && ((uint64_t)(n - 1) >> nbits)) ++nbits;
    const int above = std::max(0, nbits - kWmWinBits);
    const int d2 = std::max(0, above - 10);                 // pass-5b digit bits
    const int win_shift = kWmWinBits + d2;                  // pass-5a digit = id >> win_shift
    const int64_t nwin = ((n - 1) >> win_shift) + 1;

    DevBuf cnt1, base1, key1, id1, kl1, key2, id2, pst, cnt5, base5, pa, pb, flag;
    const int64_t nc1 = (int64_t)kWmDig * g1;
    const int nsort = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * 4, sh.nparts));
    const int64_t nc5 = (int64_t)kWmDig * nsort;
    if (cnt1.alloc(ctx, nc1 * 4) || base1.alloc(ctx, (nc1 + 1) * 8) || key1.alloc(ctx, n * 8) || id1.alloc(ctx, n * 4) ||
        kl1.alloc(ctx, n * 2) || key2.alloc(ctx, n * 8) || id2.alloc(ctx, n * 4) || pst.alloc(ctx, (sh.nparts + 1) * 8) ||
        cnt5.alloc(ctx, nc5 * 4) || base5.alloc(ctx, (nc5 + 1) * 8) || flag.alloc(ctx, 8))
        return fail(QEH_E_OOM, "window: out of device memory");
    const ColRef kc = make_colref(part), oc = make_colref(order);
    {
        KernelTimer kt(ctx, "window_partition");
        hipLaunchKernelGGL(k_wm_hist1, dim3(g1), dim3(kWmBlock), 0, ctx->stream, kc, sh, cnt1.as<uint32_t>());
        QEH_TRY(exclusive_scan_u32(ctx, cnt1.as<uint32_t>(), base1.as<uint64_t>(), nc1, nullptr));
        hipLaunchKernelGGL(k_wm_pass1, dim3(g1), dim3(kWmBlock), 0, ctx->stream, kc, oc, asc ? 1 : 0, sh, base1.as<uint64_t>(),
                           key1.as<uint64_t>(), id1.as<uint32_t>(), kl1.as<uint16_t>());
    }
    QEH_HIP(hipGetLastError());
    // bucket starts = the scanned bases of workgroup 0 per digit, then n
    DevBuf bst;
    if (bst.alloc(ctx, ((int64_t)sh.nb + 1) * 8)) return fail(QEH_E_OOM, "window: out of device memory");
    QEH_HIP(hipMemcpy2DAsync(bst.p, 8, base1.p, (size_t)g1 * 8, 8, sh.nb, hipMemcpyDeviceToDevice, ctx->stream));
    hipLaunchKernelGGL(k_wm_set2, dim3(1), dim3(64), 0, ctx->stream, bst.as<uint64_t>() + sh.nb, pst.as<uint64_t>() + sh.nparts,
                       (uint64_t)n);
    {
        KernelTimer kt(ctx, "window_partition");
        hipLaunchKernelGGL(k_wm_pass2, dim3(std::min(cus, sh.nb)), dim3(kWmBlock), 0, ctx->stream, sh, bst.as<uint64_t>(),
                           key1.as<uint64_t>(), id1.as<uint32_t>(), kl1.as<uint16_t>(), key2.as<uint64_t>(),
                           id2.as<uint32_t>(), pst.as<uint64_t>());
    }
    QEH_HIP(hipGetLastError());
    key1.reset();
    id1.reset();
    kl1.reset();
    if (pa.alloc(ctx, n * 8) || pb.alloc(ctx, n * 8)) return fail(QEH_E_OOM, "window: out of device memory");
    QEH_HIP(hipMemsetAsync(flag.p, 0, 8, ctx->stream));
    QEH_HIP(hipMemsetAsync(cnt5.p, 0, (size_t)nc5 * 4, ctx->stream));
    WmFunc wf{};
    wf.func = func;
    wf.param = param;
    wf.win_shift = win_shift;
    {
        KernelTimer kt(ctx, "window_sort");
        hipLaunchKernelGGL(k_wm_sort<false>, dim3(nsort), dim3(kWmSortBlock), 0, ctx->stream, sh, wf, pst.as<uint64_t>(),
                           key2.as<uint64_t>(), id2.as<uint32_t>(), pa.as<uint64_t>(), cnt5.as<uint32_t>(),
                           flag.as<uint32_t>());
        hipLaunchKernelGGL(k_wm_sort<true>, dim3(nsort), dim3(kWmSortBlock), 0, ctx->stream, sh, wf, pst.as<uint64_t>(),
                           key2.as<uint64_t>(), id2.as<uint32_t>(), pa.as<uint64_t>(), cnt5.as<uint32_t>(),
                           flag.as<uint32_t>());
    }
    QEH_HIP(hipGetLastError());
    uint32_t too_big = 0;
    QEH_TRY(read_small(ctx, &too_big, flag.p, 4));
    if (too_big) return kWindowMsdNotEligible;  // a group above 2048 rows: the LSD path handles skew
    key2.reset();
    id2.reset();
    QEH_TRY(alloc_column(ctx, QEH_DT_INT64, n, false, out));
    {
        KernelTimer kt(ctx, "window_place");
        const uint64_t *placed = pa.as<uint64_t>();
        if (nwin > 1) {
            QEH_TRY(exclusive_scan_u32(ctx, cnt5.as<uint32_t>(), base5.as<uint64_t>(), nc5, nullptr));
            hipLaunchKernelGGL(k_wm_pass5a, dim3(std::min(cus, nsort)), dim3(kWmBlock), 0, ctx->stream, sh, nsort, win_shift,
                               pst.as<uint64_t>(), base5.as<uint64_t>(), pa.as<uint64_t>(), pb.as<uint64_t>());
            placed = pb.as<uint64_t>();
            if (d2 > 0) {
                hipLaunchKernelGGL(k_wm_pass5b, dim3((unsigned)std::min<int64_t>(cus, nwin)), dim3(kWmBlock), 0, ctx->stream, n,
                                   win_shift, nwin, pb.as<uint64_t>(), pa.as<uint64_t>());
                placed = pa.as<uint64_t>();
            }
        }
        const int64_t nw = (n + (1 << kWmWinBits) - 1) >> kWmWinBits;
        hipLaunchKernelGGL(k_wm_place, dim3((unsigned)std::min<int64_t>((int64_t)cus * 2, nw)), dim3(kWmBlock), 0, ctx->stream,
                           n, placed, (int64_t *)out->values);
    }
    if (hipGetLastError() != hipSuccess) {
        qeh_column_release(ctx, out);
        return fail(QEH_E_HIP, "window: kernel launch failed");
    }
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) {
        qeh_column_release(ctx, out);
        return fail(QEH_E_HIP, "window: stream synchronize failed");
    }
    return QEH_OK;
}

}  // namespace qeh
