// SortExec, ROW_NUMBER() window and hash partitioning: LSD radix sort with
// LDS histograms producing a stable permutation.
//
// Reference: execute_sort is the identity (crates/query-executor/src/executor.rs:290-297)
// and the Window arm passes its input through (executor.rs:76-80), so the
// semantics are the intended ones of SURVEY.md §8.0: stable lexicographic sort
// by `exprs` with a per-key ascending flag, NULLs first (arrow SortOptions
// default; the only explicit null ordering in the tree is
// distributed/operators.rs:97-104), floats by totalOrder; ROW_NUMBER numbers
// rows 1.. within each PARTITION BY group in ORDER BY order, ties by input
// position (docs/WINDOW_FUNCTIONS.md:44-65), output aligned to input order.
// Hash partitioning follows Partitioner::partition_by_hash
// (crates/query-distributed/src/partition.rs:151-212) with a device hash.
//
// Key encoding: each key column becomes an unsigned integer in [0, 2^bits):
// NULL -> 0, value -> (ordered(x) - min + 1) ascending or (max - ordered(x) + 1)
// descending, where ordered() is sign-flip for ints and totalOrder for floats
// and min/max come from one reduction.  Only `bits` = bit length of the range
// are sorted (e.g. 21 bits for k in [0, 2^20)), 8 bits per pass; keys are
// processed last column first, each column's passes reading its encoding
// through the current permutation, so the result is lexicographic and stable.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/qeh_plan.h"
#include "device_common.h"
#include "expr_device.h"
#include "fast_tile.h"
#include "ops.h"

namespace qeh {

constexpr int kRadixBits = 8;
constexpr int kRadix = 1 << kRadixBits;

struct KeyStats {
    int64_t mn, mx;
};

__device__ __forceinline__ int64_t ordered_key(const ColRef &c, int64_t row) {
    const int64_t x = load_i64(c, row);
    if (c.dtype == QEH_DT_FLOAT32 || c.dtype == QEH_DT_FLOAT64) return f64_order_key(as_f64(x));
    return x;
}

constexpr int kRsMaxSegs = 16;  // Merge::sorted partitions read in place (RsEncode, KeySegs)

// (block bid of nb over the rows: k_key_stats runs it for one column, k_key_stats_segs for one segment each)
__device__ __forceinline__ void key_stats_body(const ColRef &c, const uint32_t *__restrict__ perm, int64_t n, KeyStats *out,
                                               int64_t bid, int64_t nb) {
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    if (!perm && !c.validity && c.dtype == QEH_DT_INT64 && ((uintptr_t)c.values & 15) == 0) {
        // plain int64 column: 16-B loads, four in flight per thread
        typedef long long v2 __attribute__((ext_vector_type(2)));
        const v2 *kv = (const v2 *)c.values;
        const int64_t pairs = n / 2, stride = nb * blockDim.x;
        for (int64_t i = bid * blockDim.x + threadIdx.x; i < pairs; i += 4 * stride) {
            v2 q[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) q[u] = kv[i + u * stride < pairs ? i + u * stride : i];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                mn = q[u].x < mn ? q[u].x : mn;
                mx = q[u].x > mx ? q[u].x : mx;
                mn = q[u].y < mn ? q[u].y : mn;
                mx = q[u].y > mx ? q[u].y : mx;
            }
        }
        if ((n & 1) && bid == 0 && threadIdx.x == 0) {
            const int64_t k = ((const int64_t *)c.values)[n - 1];
            mn = k < mn ? k : mn;
            mx = k > mx ? k : mx;
        }
    } else if (!perm && c.dtype == QEH_DT_INT64 && (c.vbit0 & 7) == 0 && ((uintptr_t)c.values & 15) == 0) {
        // nullable int64 column whose validity bytes line up with the rows: eight rows per thread
        // (one validity byte, four 16-B loads), rows of NULLs skipped by mask
        typedef long long v2 __attribute__((ext_vector_type(2)));
        const uint8_t *vb = c.validity + (c.vbit0 >> 3);
        // (four groups per iteration: 16 loads in flight per thread, the grid is one workgroup per CU)
        const int64_t groups = n / 8, stride = nb * blockDim.x;
        for (int64_t g0 = bid * blockDim.x + threadIdx.x; g0 < groups; g0 += 4 * stride) {
            uint32_t m[4];
            v2 q[4][4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const int64_t g = g0 + w * stride < groups ? g0 + w * stride : g0;
                m[w] = g0 + w * stride < groups ? vb[g] : 0u;  // (a clamped repeat counts nothing)
                const v2 *kv = (const v2 *)c.values + g * 4;
#pragma unroll
                for (int u = 0; u < 4; ++u) q[w][u] = kv[u];
            }
#pragma unroll
            for (int w = 0; w < 4; ++w)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if ((m[w] >> (2 * u)) & 1u) mn = q[w][u].x < mn ? q[w][u].x : mn, mx = q[w][u].x > mx ? q[w][u].x : mx;
                    if ((m[w] >> (2 * u + 1)) & 1u) mn = q[w][u].y < mn ? q[w][u].y : mn, mx = q[w][u].y > mx ? q[w][u].y : mx;
                }
        }
        for (int64_t i = groups * 8 + bid * blockDim.x + threadIdx.x; i < n; i += stride) {
            if (!col_valid(c, i)) continue;
            const int64_t k = ((const int64_t *)c.values)[i];
            mn = k < mn ? k : mn;
            mx = k > mx ? k : mx;
        }
    } else {
        for (int64_t i = bid * blockDim.x + threadIdx.x; i < n; i += nb * blockDim.x) {
            const int64_t r = perm ? perm[i] : i;
            if (!col_valid(c, r)) continue;
            const int64_t k = ordered_key(c, r);
            mn = k < mn ? k : mn;
            mx = k > mx ? k : mx;
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const int64_t a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin((long long *)&out->mn, (long long)mn);
        atomicMax((long long *)&out->mx, (long long)mx);
    }
}

__global__ void k_key_stats(ColRef c, const uint32_t *__restrict__ perm, int64_t n, KeyStats *out) {
    key_stats_body(c, perm, n, out, blockIdx.x, gridDim.x);
}

// one launch over up to kRsMaxSegs columns (Merge::sorted's partitions): gps blocks per segment
struct KeySegs {
    int32_t ns, gps;
    ColRef c[kRsMaxSegs];
    int64_t n[kRsMaxSegs];
};
__global__ void k_key_stats_segs(KeySegs ks, KeyStats *out) {
    const int seg = blockIdx.x / ks.gps;
    key_stats_body(ks.c[seg], nullptr, ks.n[seg], out, blockIdx.x % ks.gps, ks.gps);
}

__global__ void k_stats_init(KeyStats *s) {
    s->mn = INT64_MAX;
    s->mx = INT64_MIN;
}

// encoded key of row perm[i] (or i) -> keys[i]; perm_out[i] = perm[i] (or i)
// mode 0: value encoding (NULL -> 0, values biased by `bias`); mode 1: null flag only
// `null_code`: the key of a NULL row (0 = NULLs first; above every value code = NULLs last)
template <typename KeyT>
__global__ void k_encode(ColRef c, const uint32_t *__restrict__ perm, int64_t n, int64_t mn, int64_t mx, int asc,
                         uint64_t bias, int mode, uint64_t null_code, KeyT *__restrict__ keys,
                         uint32_t *__restrict__ perm_out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = perm ? perm[i] : i;
        uint64_t k = null_code;
        if (col_valid(c, r)) {
            if (mode == 1) {
                k = null_code ? 0 : 1;
            } else {
                const int64_t x = ordered_key(c, r);
                k = asc ? (uint64_t)x - (uint64_t)mn + bias : (uint64_t)mx - (uint64_t)x + bias;
            }
        }
        keys[i] = (KeyT)k;
        perm_out[i] = (uint32_t)r;
    }
}

// ---- one LSD pass ----------------------------------------------------------------------
// Block b owns elements [b*seg, (b+1)*seg) and walks them in tiles of kRsTile;
// inside a tile wave w owns the contiguous run [w*64*kRsIpt, (w+1)*64*kRsIpt)
// and its item j is element w*64*kRsIpt + j*64 + lane, so (wave, j, lane) is
// input order and every load is a full 512-byte wave line.  hist is digit-major
// [kRadix][nblocks].
constexpr int kRsIpt = 8;
constexpr int kRsThreads = 1024;
constexpr int kRsSTile = kRsThreads * kRsIpt;  // 8192

// lanes of this wave whose digit equals mine (wave64 has no match_any: 8 ballots)
__device__ __forceinline__ uint64_t digit_peers(uint32_t dg, bool live) {
    uint64_t peers = __ballot(live);
#pragma unroll
    for (int b = 0; b < kRadixBits; ++b) {
        const uint64_t m = __ballot((dg >> b) & 1);
        peers &= ((dg >> b) & 1) ? m : ~m;
    }
    return peers;
}

// Stable rank of this lane's row among the rows of digit dg ranked so far by this wave (wc = the
// wave's counters): one returning LDS atomic when the device serves a wave's lanes in lane order
// (AT, the default after the lds_atomic_rank_ok self-check), else ballot peers; dead lanes get 0.
template <bool AT>
__device__ __forceinline__ uint32_t tile_rank(uint32_t *wc, uint32_t dg, bool live) {
    if constexpr (AT) {
        return live ? atomicAdd(&wc[dg], 1u) : 0u;
    } else {
        const uint32_t d = live ? dg : 0u;
        const uint64_t peers = digit_peers(d, live);
        const uint32_t before = wc[d];
        if (live && mbcnt(peers) == 0) wc[d] = before + (uint32_t)popc64(peers);
        return live ? before + mbcnt(peers) : 0u;
    }
}

// The payload sort's first pass reads the raw key column and encodes on load (KES = 4 / 8: Int32 /
// Int64 values) instead of a separate encode pass; KES = 0 reads the codes.
// ns > 0: the first pass reads the key and payload in place from ns row segments (qeh_merge_sorted's
// partitions: rows [start[s], start[s + 1]) are segment s's rows 0..) instead of one column -- no
// concatenation copy ahead of the sort (kRsMaxSegs: at the top of the file)
struct RsEncode {
    ColRef c;
    int64_t mn, mx;
    uint64_t bias, null_code;
    int32_t asc;
    int32_t ns;
    int64_t start[kRsMaxSegs + 1];
    ColRef sk[kRsMaxSegs];
    const uint64_t *sv[kRsMaxSegs];
    // KES = 1 (the MSD payload sort's second pass): the keys are the low 32 code bits, and the byte
    // stream nd holds code bits [nd_shift, nd_shift + 8) -- all the pass reads of a code
    const uint8_t *nd;
    int32_t nd_shift;
};

// the segment of row i (branch-free count of the segment starts at or below i)
__device__ __forceinline__ int rs_seg(const RsEncode &e, int64_t i) {
    int s = 0;
#pragma unroll
    for (int q = 1; q < kRsMaxSegs; ++q) s += (q < e.ns && i >= e.start[q]) ? 1 : 0;
    return s;
}

// the segment of a tile's rows [a, b] when they share one (wave-uniform: a scalar index into the kernel
// arguments), else -1 (rows straddle a partition boundary: looked up per row)
__device__ __forceinline__ int rs_tile_seg(const RsEncode &e, int64_t a, int64_t b) {
    if (!e.ns) return 0;
    const int sa = rs_seg(e, a), sb = rs_seg(e, b);
    return __builtin_amdgcn_readfirstlane(sa == sb ? sa : -1);
}

template <int KES>
__device__ __forceinline__ uint64_t rs_code(const RsEncode &e, const ColRef &c, int64_t i) {
    const int64_t x = KES == 4 ? (int64_t)__builtin_nontemporal_load((const int32_t *)c.values + i)
                               : __builtin_nontemporal_load((const int64_t *)c.values + i);
    const uint64_t code = e.asc ? (uint64_t)x - (uint64_t)e.mn + e.bias : (uint64_t)e.mx - (uint64_t)x + e.bias;
    return col_valid(c, i) ? code : e.null_code;
}

// (segments are only ever indexed by a wave-uniform value: a per-lane index into the kernel arguments
// would copy the whole RsEncode to scratch)
template <int KES, typename KeyT>
__device__ __forceinline__ KeyT rs_load_key(const KeyT *__restrict__ keys, const RsEncode &e, int64_t i, int ts = 0) {
    if constexpr (KES == 0) {
        return __builtin_nontemporal_load(&keys[i]);
    } else if constexpr (KES == 1) {
        const uint32_t lo = __builtin_nontemporal_load((const uint32_t *)keys + i);
        return ((KeyT)e.nd[i] << e.nd_shift) | (KeyT)(lo & ((1u << e.nd_shift) - 1u));
    } else {
        if (!e.ns) return (KeyT)rs_code<KES>(e, e.c, i);
        if (ts >= 0) return (KeyT)rs_code<KES>(e, e.sk[ts], i - e.start[ts]);
        uint64_t code = 0;
        for (int s = 0; s < e.ns; ++s)  // (a tile across a partition boundary)
            if (i >= e.start[s] && i < e.start[s + 1]) code = rs_code<KES>(e, e.sk[s], i - e.start[s]);
        return (KeyT)code;
    }
}

// the first pass's payload of row i (in place from the segments when ns > 0)
template <int KES, typename ValT>
__device__ __forceinline__ ValT rs_load_val(const ValT *__restrict__ vals, const RsEncode &e, int64_t i, int ts = 0) {
    if constexpr (KES >= 4 && sizeof(ValT) == 8) {
        if (e.ns) {
            if (ts >= 0) return (ValT)__builtin_nontemporal_load(e.sv[ts] + (i - e.start[ts]));
            ValT v = 0;
            for (int s = 0; s < e.ns; ++s)
                if (i >= e.start[s] && i < e.start[s + 1]) v = (ValT)__builtin_nontemporal_load(e.sv[s] + (i - e.start[s]));
            return v;
        }
    }
    return __builtin_nontemporal_load(&vals[i]);
}

template <typename KeyT, int KES = 0>
__global__ __launch_bounds__(kRsThreads) void k_rs_hist(const KeyT *__restrict__ keys, int64_t n, int64_t seg,
                                                        int shift, uint32_t *__restrict__ hist, int nblocks, RsEncode enc) {
    constexpr int W = kRsThreads / 64;
    __shared__ uint32_t h[W][kRadix];  // per-wave counters: one LDS atomic per row
    for (int i = threadIdx.x; i < W * kRadix; i += kRsThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const int64_t lo = (int64_t)blockIdx.x * seg, hi = lo + seg < n ? lo + seg : n;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int64_t c0 = lo; c0 < hi; c0 += kRsSTile) {
        const int64_t base = c0 + (int64_t)wave * 64 * kRsIpt + lane;
        const int ts = KES != 0 ? rs_tile_seg(enc, c0, (c0 + kRsSTile < hi ? c0 + kRsSTile : hi) - 1) : 0;
        KeyT k[kRsIpt];
#pragma unroll
        for (int j = 0; j < kRsIpt; ++j) {
            const int64_t i = base + j * 64;
            k[j] = rs_load_key<KES>(keys, enc, i < hi ? i : hi - 1, ts);
        }
#pragma unroll
        for (int j = 0; j < kRsIpt; ++j) {
            const bool live = base + j * 64 < hi;
            const uint32_t dg = (uint32_t)((k[j] >> shift) & (kRadix - 1));
            if (live) atomicAdd(&h[wave][dg], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < kRadix) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) c += h[w][threadIdx.x];
        hist[(int64_t)threadIdx.x * nblocks + blockIdx.x] = c;
    }
}

// The payload sort's first histogram (KES = 8 / 4: Int64 / Int32 keys, encoded as rs_code does): a
// lane reads 8 consecutive rows of a partition with 16-B loads and their validity byte at once (row
// order does not matter to a histogram), four such groups in flight; a segment's head and tail rows,
// and columns whose values or validity do not line up, one row at a time.  Same block row ranges
// [b * seg, (b + 1) * seg) and hist layout as k_rs_hist<KeyT, KES>.
template <int KES>
__global__ __launch_bounds__(kRsThreads) void k_rs_hist_enc(int64_t n, int64_t seg, int shift, uint32_t *__restrict__ hist,
                                                            int nblocks, RsEncode enc) {
    constexpr int W = kRsThreads / 64;
    constexpr int NL = KES / 2;  // 16-B loads per 8-row group
    typedef long long v2 __attribute__((ext_vector_type(2)));
    __shared__ uint32_t h[W][kRadix];
    for (int i = threadIdx.x; i < W * kRadix; i += kRsThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    const int64_t lo = (int64_t)blockIdx.x * seg, hi = lo + seg < n ? lo + seg : n;
    const bool asc = enc.asc != 0;
    const uint64_t emn = (uint64_t)enc.mn, emx = (uint64_t)enc.mx, bias = enc.bias, null_code = enc.null_code;
    uint32_t *hw = &h[wave][0];
    auto count = [=](int64_t x, bool ok) {
        const uint64_t code = ok ? (asc ? (uint64_t)x - emn + bias : emx - (uint64_t)x + bias) : null_code;
        atomicAdd(&hw[(uint32_t)(code >> shift) & (kRadix - 1)], 1u);
    };
    const int ns = enc.ns ? enc.ns : 1;
    for (int sg0 = 0; sg0 < ns; ++sg0) {
        // a scalar index into the kernel arguments (else the compiler copies RsEncode to scratch)
        const int sg = __builtin_amdgcn_readfirstlane(sg0);
        const ColRef c = enc.ns ? enc.sk[sg] : enc.c;
        const int64_t st = enc.ns ? enc.start[sg] : 0, en = enc.ns ? enc.start[sg + 1] : n;
        const int64_t a = (lo > st ? lo : st) - st, e = (hi < en ? hi : en) - st;  // local rows [a, e)
        if (a >= e) continue;
        auto row = [=](int64_t i) {
            const int64_t x = KES == 4 ? (int64_t)__builtin_nontemporal_load((const int32_t *)c.values + i)
                                       : __builtin_nontemporal_load((const int64_t *)c.values + i);
            count(x, col_valid(c, i));
        };
        const bool vec = ((uintptr_t)c.values & 15) == 0 && (!c.validity || (c.vbit0 & 7) == 0);
        int64_t ga = (a + 7) / 8, gb = e / 8;  // whole 8-row groups [ga, gb)
        if (!vec || ga >= gb) ga = gb = 0;
        const int64_t h0 = ga < gb ? ga * 8 : e, t0 = ga < gb ? gb * 8 : e;
        for (int64_t i = a + threadIdx.x; i < h0; i += kRsThreads) row(i);
        for (int64_t i = (t0 > a ? t0 : a) + threadIdx.x; i < e; i += kRsThreads) row(i);
        const uint8_t *vb = c.validity ? c.validity + (c.vbit0 >> 3) : nullptr;
        for (int64_t g0 = ga + threadIdx.x; g0 < gb; g0 += 4 * kRsThreads) {
            uint32_t m[4];
            v2 q[4][NL];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const bool live = g0 + w * kRsThreads < gb;
                const int64_t g = live ? g0 + w * kRsThreads : g0;
                m[w] = live ? (vb ? (uint32_t)vb[g] : 0xFFu) : 0u;
                const v2 *kv = (const v2 *)((const char *)c.values + g * 8 * KES);
#pragma unroll
                for (int u = 0; u < NL; ++u) q[w][u] = __builtin_nontemporal_load(kv + u);
            }
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                if (g0 + w * kRsThreads >= gb) continue;
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    int64_t x;
                    if constexpr (KES == 8) {
                        x = (r & 1) ? q[w][r >> 1].y : q[w][r >> 1].x;
                    } else {
                        const long long wd = (r & 2) ? q[w][r >> 2].y : q[w][r >> 2].x;
                        x = (int64_t)(int32_t)(uint32_t)((r & 1) ? ((unsigned long long)wd >> 32) : (unsigned long long)wd);
                    }
                    count(x, (m[w] >> r) & 1u);
                }
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < kRadix) {
        uint32_t cnt = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) cnt += h[w][threadIdx.x];
        hist[(int64_t)threadIdx.x * nblocks + blockIdx.x] = cnt;
    }
}

// Histogram of a pass whose digits the previous scatter wrote as a byte stream
// (nd_out): 1 B per element instead of the 8-B key, 16 digits per 16-B load,
// per-wave LDS counters (no cross-wave atomics on hot digits).
__global__ __launch_bounds__(kRsThreads) void k_rs_hist_u8(const uint8_t *__restrict__ dg, int64_t n, int64_t seg,
                                                           uint32_t *__restrict__ hist, int nblocks) {
    constexpr int W = kRsThreads / 64;
    __shared__ uint32_t h[W][kRadix];
    for (int i = threadIdx.x; i < W * kRadix; i += kRsThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    const int64_t lo = (int64_t)blockIdx.x * seg, hi = lo + seg < n ? lo + seg : n;
    // segments start at multiples of seg; the 16-B body is [a, b), head/tail bytewise
    const int64_t a = (lo + 15) & ~(int64_t)15, b = hi & ~(int64_t)15;
    if (a < b) {
        for (int64_t i = a + 16 * (int64_t)threadIdx.x; i < b; i += 16 * (int64_t)kRsThreads) {
            typedef unsigned int v4u32s __attribute__((ext_vector_type(4)));
            const v4u32s w = __builtin_nontemporal_load((const v4u32s *)(dg + i));
            const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) atomicAdd(&h[wave][(ws[q] >> (8 * r)) & 0xff], 1u);
        }
        for (int64_t i = lo + threadIdx.x; i < a; i += kRsThreads) atomicAdd(&h[wave][dg[i]], 1u);
        for (int64_t i = b + threadIdx.x; i < hi; i += kRsThreads) atomicAdd(&h[wave][dg[i]], 1u);
    } else {
        for (int64_t i = lo + threadIdx.x; i < hi; i += kRsThreads) atomicAdd(&h[wave][dg[i]], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kRadix) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) c += h[w][threadIdx.x];
        hist[(int64_t)threadIdx.x * nblocks + blockIdx.x] = c;
    }
}

// Stable scatter, one 1024-thread workgroup per CU: rank each 8192-element
// tile by digit (ballot peers + per-wave counters), reorder it in LDS, then
// write every digit's run (≈ 32 elements = whole 128-byte lines) contiguously.
// Few, long-lived workgroups keep the open output lines of an XCD within its
// L2 (32 workgroups × 256 digits × 2 arrays), and the next tile's loads are
// issued before the current tile is ranked (LDS-only barriers below do not
// wait for them).

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The payload sort's last pass writes the decoded key column itself (DEC): code -> Int64 / Int32 value
// as rs_load_key's inverse, and one valid byte per row for the bitmap packed afterwards.
struct RsDecode {
    int64_t mn, mx;
    uint64_t bias, null_code;
    int32_t asc, dt;
    void *out;
    uint8_t *validb;  // nullable key: 1 = value, 0 = NULL (else nullptr)
};

// AT: tile ranks by LDS atomics (ds_add_rtn serves one instruction's lanes in lane order, so the
// rank is stable: tools/ubench/lds_order_ubench.hip), else by ballot peers (QEH_RS_BALLOT=1, A/B).
// ValT: the carried value -- a u32 row id, or (qeh_merge_sorted's payload sort) an 8-B payload.
// SEG (the MSD payload sort's second pass): block b's rows [lo, hi) and its offsets come from a
// segment table (lo, hi, hb, nbb per block): offsets[hb + digit * nbb], so every block stays inside
// one first-pass bucket and the scan orders (bucket, digit, block).
template <typename KeyT, bool AT = true, typename ValT = uint32_t, bool DEC = false, int KES = 0, bool SEG = false,
          typename KOutT = KeyT>
__global__ __launch_bounds__(kRsThreads) void k_rs_scatter(const KeyT *__restrict__ keys, const ValT *__restrict__ vals,
                                                           int64_t n, int64_t seg, int shift, const uint64_t *__restrict__ offs,
                                                           int nblocks, KOutT *__restrict__ keys_out,
                                                           ValT *__restrict__ vals_out, uint8_t *__restrict__ nd_out,
                                                           int nshift, RsDecode dec, RsEncode enc,
                                                           const int64_t *__restrict__ segtab = nullptr) {
    constexpr int W = kRsThreads / 64;
    constexpr int DW = kRadix / 64;       // waves that own one digit per lane in the bookkeeping
    __shared__ KeyT s_keys[kRsSTile];
    __shared__ ValT s_vals[kRsSTile];
    __shared__ uint32_t wcnt[W][kRadix];  // per-wave digit counts, then per-wave start inside the digit
    __shared__ uint32_t loc[kRadix];      // tile-local start of each digit
    __shared__ uint32_t tot_s[kRadix];
    __shared__ uint32_t wsum[DW];
    __shared__ uint64_t run[kRadix];      // global position of the block's next element of each digit
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    int64_t lo, hi;
    if constexpr (SEG) {
        const int64_t *e = segtab + 4 * (int64_t)blockIdx.x;
        lo = e[0], hi = e[1];
        if (t < kRadix) run[t] = offs[e[2] + (int64_t)t * e[3]];
    } else {
        if (t < kRadix) run[t] = offs[(int64_t)t * nblocks + blockIdx.x];
        lo = (int64_t)blockIdx.x * seg, hi = lo + seg < n ? lo + seg : n;
    }
    KeyT k[kRsIpt];
    ValT v[kRsIpt];
    // loads are unconditional (indices clamped into [lo, hi)): no branches around
    // them, so the compiler's wait counts stay exact and the prefetch really
    // stays in flight across the ranking of the current tile
    auto load_tile = [&](int64_t c0, KeyT *kk, ValT *vv) {
        const int64_t base = c0 + (int64_t)wave * 64 * kRsIpt + lane;
        const int ts = KES != 0 ? rs_tile_seg(enc, c0, (c0 + kRsSTile < hi ? c0 + kRsSTile : hi) - 1) : 0;
#pragma unroll
        for (int j = 0; j < kRsIpt; ++j) {
            const int64_t i = base + j * 64;
            const int64_t ii = i < hi ? i : hi - 1;
            kk[j] = rs_load_key<KES>(keys, enc, ii, ts);
            vv[j] = rs_load_val<KES>(vals, enc, ii, ts);
        }
    };
    if (lo < hi) load_tile(lo, k, v);
    for (int64_t c0 = lo; c0 < hi; c0 += kRsSTile) {
        for (int i = t; i < W * kRadix; i += kRsThreads) (&wcnt[0][0])[i] = 0;
        KeyT kn[kRsIpt];
        ValT vn[kRsIpt];
        const int64_t c1 = c0 + kRsSTile;
        load_tile(c1 < hi ? c1 : c0, kn, vn);  // in flight while this tile is ranked and written
        lds_barrier();
        const int64_t base = c0 + (int64_t)wave * 64 * kRsIpt + lane;
        uint32_t rk[kRsIpt];
#pragma unroll
        for (int j = 0; j < kRsIpt; ++j) {
            const bool live = base + j * 64 < hi;
            const uint32_t dg = (uint32_t)((k[j] >> shift) & (kRadix - 1));
            if constexpr (AT) {
                // LDS atomics serve the lanes of one instruction in lane order: the same stable rank
                rk[j] = live ? atomicAdd(&wcnt[wave][dg], 1u) : 0u;
            } else {
                const uint64_t peers = digit_peers(dg, live);
                const uint32_t before = wcnt[wave][dg];
                rk[j] = before + mbcnt(peers);
                if (live && mbcnt(peers) == 0) wcnt[wave][dg] = before + (uint32_t)popc64(peers);
            }
        }
        lds_barrier();
        // thread t < 256 = digit t: wave starts inside the digit, tile total, scan -> loc
        uint32_t tot = 0, incl = 0;
        if (t < kRadix) {
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint32_t c = wcnt[w][t];
                wcnt[w][t] = tot;
                tot += c;
            }
            tot_s[t] = tot;
            incl = wave_incl_scan(tot);
            if (lane == 63) wsum[wave] = incl;
        }
        lds_barrier();
        if (t < kRadix) {
            uint32_t wbase = 0;
#pragma unroll
            for (int w = 0; w < DW; ++w) wbase += w < wave ? wsum[w] : 0;
            loc[t] = wbase + incl - tot;
        }
        lds_barrier();
#pragma unroll
        for (int j = 0; j < kRsIpt; ++j) {
            if (base + j * 64 < hi) {
                const uint32_t dg = (uint32_t)((k[j] >> shift) & (kRadix - 1));
                const uint32_t p = loc[dg] + wcnt[wave][dg] + rk[j];
                s_keys[p] = k[j];
                s_vals[p] = v[j];
            }
        }
        lds_barrier();
        const int cnt = (int)(hi - c0 < kRsSTile ? hi - c0 : kRsSTile);
        for (int p = t; p < cnt; p += kRsThreads) {
            const KeyT key = s_keys[p];
            const uint32_t dg = (uint32_t)((key >> shift) & (kRadix - 1));
            const uint64_t pos = run[dg] + (uint64_t)(p - (int)loc[dg]);
            if constexpr (DEC) {
                const uint64_t c = (uint64_t)key;
                const bool ok = !dec.validb || c != dec.null_code;  // no NULLs: every code is a value
                const int64_t x = ok ? (dec.asc ? (int64_t)(c - dec.bias + (uint64_t)dec.mn)
                                               : (int64_t)((uint64_t)dec.mx - (c - dec.bias)))
                                     : 0;
                if (dec.dt == QEH_DT_INT32) ((int32_t *)dec.out)[pos] = (int32_t)x;
                else ((int64_t *)dec.out)[pos] = x;
                if (dec.validb) dec.validb[pos] = ok ? 1 : 0;
            } else {
                keys_out[pos] = (KOutT)key;  // (KOutT narrower: the low code bits the next stage needs)
            }
            vals_out[pos] = s_vals[p];
            if (nd_out) nd_out[pos] = (uint8_t)(key >> nshift);  // the next pass's digit (its histogram input)
        }
        lds_barrier();
        if (t < kRadix) run[t] += tot_s[t];
#pragma unroll
        for (int j = 0; j < kRsIpt; ++j) {
            k[j] = kn[j];
            v[j] = vn[j];
        }
    }
}

// Partition move (the device side of Exchange): one stable pass over u8 partition ids that
// carries up to 4 non-null 8-byte payload columns to their partition-major positions, with the
// same tile ranking and run-contiguous writes as k_rs_scatter — instead of a permutation
// followed by one gather per column (a gather re-reads every source line once per partition).
constexpr int kPmMaxCols = 4;
constexpr int kPmIpt = 4;
constexpr int kPmTile = kRsThreads * kPmIpt;  // 4096 rows: ids + 4 columns fit in LDS

struct PmCols {
    const uint64_t *src[kPmMaxCols];
    uint64_t *dst[kPmMaxCols];
    int32_t n;
};

// Rows whose id is >= `drop` (the filtered-out rows of a fused filter + exchange) are ranked last
// and not written.
template <int NC, bool AT = true>
__global__ __launch_bounds__(kRsThreads) void k_part_scatter(const uint8_t *__restrict__ ids, int64_t n, int64_t seg,
                                                             const uint64_t *__restrict__ offs, int nblocks, PmCols cols,
                                                             uint32_t drop) {
    constexpr int W = kRsThreads / 64;
    constexpr int DW = kRadix / 64;
    __shared__ uint64_t s_val[NC > 0 ? NC : 1][kPmTile];
    __shared__ uint8_t s_id[kPmTile];
    __shared__ uint32_t wcnt[W][kRadix];
    __shared__ uint32_t loc[kRadix];
    __shared__ uint32_t tot_s[kRadix];
    __shared__ uint32_t wsum[DW];
    __shared__ uint64_t run[kRadix];
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    if (t < kRadix) run[t] = offs[(int64_t)t * nblocks + blockIdx.x];
    const int64_t lo = (int64_t)blockIdx.x * seg, hi = lo + seg < n ? lo + seg : n;
    // the next tile's ids and columns are loaded into registers while this tile is ranked, staged
    // and written (the barriers below order LDS only, so those loads stay in flight)
    uint32_t dgn[kPmIpt];
    uint64_t vn[kPmIpt][NC > 0 ? NC : 1];
    auto load = [&](int64_t c0) {
        const int64_t base = c0 + (int64_t)wave * 64 * kPmIpt + lane;
#pragma unroll
        for (int j = 0; j < kPmIpt; ++j) {
            const int64_t i = base + j * 64;
            const int64_t ii = i < hi ? i : hi - 1;
            dgn[j] = ids[ii];
#pragma unroll
            for (int c = 0; c < NC; ++c) vn[j][c] = __builtin_nontemporal_load(&cols.src[c][ii]);
        }
    };
    if (lo < hi) load(lo);
    __syncthreads();  // run[]
    for (int64_t c0 = lo; c0 < hi; c0 += kPmTile) {
        for (int i = t; i < W * kRadix; i += kRsThreads) (&wcnt[0][0])[i] = 0;
        const int64_t base = c0 + (int64_t)wave * 64 * kPmIpt + lane;
        uint32_t dg[kPmIpt];
        uint64_t v[kPmIpt][NC > 0 ? NC : 1];
#pragma unroll
        for (int j = 0; j < kPmIpt; ++j) {
            dg[j] = dgn[j];
#pragma unroll
            for (int c = 0; c < NC; ++c) v[j][c] = vn[j][c];
        }
        if (c0 + kPmTile < hi) load(c0 + kPmTile);
        lds_barrier();
        uint32_t rk[kPmIpt];
#pragma unroll
        for (int j = 0; j < kPmIpt; ++j) {
            const bool live = base + j * 64 < hi;
            rk[j] = tile_rank<AT>(wcnt[wave], dg[j], live);  // stable
        }
        lds_barrier();
        uint32_t tot = 0, incl = 0;
        if (t < kRadix) {
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint32_t c = wcnt[w][t];
                wcnt[w][t] = tot;
                tot += c;
            }
            tot_s[t] = tot;
            incl = wave_incl_scan(tot);
            if (lane == 63) wsum[wave] = incl;
        }
        lds_barrier();
        if (t < kRadix) {
            uint32_t wbase = 0;
#pragma unroll
            for (int w = 0; w < DW; ++w) wbase += w < wave ? wsum[w] : 0;
            loc[t] = wbase + incl - tot;
        }
        lds_barrier();
#pragma unroll
        for (int j = 0; j < kPmIpt; ++j) {
            if (base + j * 64 < hi) {
                const uint32_t p = loc[dg[j]] + wcnt[wave][dg[j]] + rk[j];
                s_id[p] = (uint8_t)dg[j];
#pragma unroll
                for (int c = 0; c < NC; ++c) s_val[c][p] = v[j][c];
            }
        }
        lds_barrier();
        const int cnt = (int)(hi - c0 < kPmTile ? hi - c0 : kPmTile);
        for (int p = t; p < cnt; p += kRsThreads) {
            const uint32_t d = s_id[p];
            if (d >= drop) continue;
            const uint64_t pos = run[d] + (uint64_t)(p - (int)loc[d]);
#pragma unroll
            for (int c = 0; c < NC; ++c) cols.dst[c][pos] = s_val[c][p];
        }
        lds_barrier();
        if (t < kRadix) run[t] += tot_s[t];
    }
}

// k_part_scatter for at most kPsDig partitions (an Exchange to the GPUs of one node, config 4's 8):
// the same stable, run-contiguous placement with the bookkeeping sized to the partitions instead of
// 256 digits (16 per-wave counters, a 16-lane scan), 8192-row tiles for up to two columns, and rows
// with an id >= drop (the filtered-out rows) neither ranked nor staged, so the write loop covers only
// the rows that move.
constexpr int kPsDig = 16;
template <int NC, bool AT = true>
__global__ __launch_bounds__(kRsThreads) void k_part_scatter_small(const uint8_t *__restrict__ ids, int64_t n, int64_t seg,
                                                                   const uint64_t *__restrict__ offs, int nblocks, PmCols cols,
                                                                   uint32_t drop) {
    constexpr int W = kRsThreads / 64;
    constexpr int IPT = NC <= 2 ? 8 : 4;
    constexpr int TILE = kRsThreads * IPT;
    __shared__ uint64_t s_val[NC > 0 ? NC : 1][TILE];
    __shared__ uint8_t s_id[TILE];
    __shared__ uint32_t wcnt[W][kPsDig];  // per-wave counts, then per-wave starts inside the partition
    __shared__ uint32_t loc[kPsDig], tot_s[kPsDig + 1];
    __shared__ uint64_t run[kPsDig];
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    if (drop > (uint32_t)kPsDig) drop = kPsDig;
    if (t < kPsDig) run[t] = offs[(int64_t)t * nblocks + blockIdx.x];
    const int64_t lo = (int64_t)blockIdx.x * seg, hi = lo + seg < n ? lo + seg : n;
    uint32_t dgn[IPT];
    uint64_t vn[IPT][NC > 0 ? NC : 1];
    auto load = [&](int64_t c0) {
        const int64_t base = c0 + (int64_t)wave * 64 * IPT + lane;
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int64_t i = base + j * 64;
            const int64_t ii = i < hi ? i : hi - 1;
            dgn[j] = ids[ii];
#pragma unroll
            for (int c = 0; c < NC; ++c) vn[j][c] = __builtin_nontemporal_load(&cols.src[c][ii]);
        }
    };
    if (lo < hi) load(lo);
    __syncthreads();  // run[]
    for (int64_t c0 = lo; c0 < hi; c0 += TILE) {
        if (t < W * kPsDig) (&wcnt[0][0])[t] = 0u;
        const int64_t base = c0 + (int64_t)wave * 64 * IPT + lane;
        uint32_t dg[IPT];
        uint64_t v[IPT][NC > 0 ? NC : 1];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            dg[j] = dgn[j];
#pragma unroll
            for (int c = 0; c < NC; ++c) v[j][c] = vn[j][c];
        }
        if (c0 + TILE < hi) load(c0 + TILE);
        lds_barrier();
        uint32_t rk[IPT];
        bool mv[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            mv[j] = base + j * 64 < hi && dg[j] < drop;
            rk[j] = tile_rank<AT>(wcnt[wave], dg[j], mv[j]);  // stable
        }
        lds_barrier();
        if (t < 64) {  // lane d < kPsDig: per-wave starts inside partition d, its tile total, the scan
            uint32_t tot = 0;
            if (lane < kPsDig) {
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    const uint32_t c = wcnt[w][lane];
                    wcnt[w][lane] = tot;
                    tot += c;
                }
            }
            const uint32_t incl = wave_incl_scan(tot);
            if (lane < kPsDig) loc[lane] = incl - tot, tot_s[lane] = tot;
            if (lane == kPsDig - 1) tot_s[kPsDig] = incl;  // rows that move in this tile
        }
        lds_barrier();
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            if (mv[j]) {
                const uint32_t p = loc[dg[j]] + wcnt[wave][dg[j]] + rk[j];
                s_id[p] = (uint8_t)dg[j];
#pragma unroll
                for (int c = 0; c < NC; ++c) s_val[c][p] = v[j][c];
            }
        }
        lds_barrier();
        const int cnt = (int)tot_s[kPsDig];
        for (int p = t; p < cnt; p += kRsThreads) {
            const uint32_t d = s_id[p];
            const uint64_t pos = run[d] + (uint64_t)(p - (int)loc[d]);
#pragma unroll
            for (int c = 0; c < NC; ++c) cols.dst[c][pos] = s_val[c][p];
        }
        lds_barrier();
        if (t < kPsDig) run[t] += tot_s[t];
    }
}

// The inverse of k_part_scatter_small (qeh_partition_hash_unmove): the same stable ranking of each
// tile's rows by partition, but every row reads its value from the partition-major column at the
// position the forward move gave it (run start + its rank in the partition) and writes it at its own
// input position.  A stable partition places row i at (rows of lower partitions) + (rows of its
// partition before i) whatever the tiling, so this reproduces any stable forward move.
template <int NC, bool AT = true>
__global__ __launch_bounds__(kRsThreads) void k_part_gather_small(const uint8_t *__restrict__ ids, int64_t n, int64_t seg,
                                                                  const uint64_t *__restrict__ offs, int nblocks, PmCols cols) {
    constexpr int W = kRsThreads / 64;
    constexpr int IPT = 8;
    constexpr int TILE = kRsThreads * IPT;
    __shared__ uint32_t wcnt[W][kPsDig];
    __shared__ uint32_t tot_s[kPsDig];
    __shared__ uint64_t run[kPsDig];
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    if (t < kPsDig) run[t] = offs[(int64_t)t * nblocks + blockIdx.x];
    const int64_t lo = (int64_t)blockIdx.x * seg, hi = lo + seg < n ? lo + seg : n;
    __syncthreads();  // run[]
    for (int64_t c0 = lo; c0 < hi; c0 += TILE) {
        if (t < W * kPsDig) (&wcnt[0][0])[t] = 0u;
        const int64_t base = c0 + (int64_t)wave * 64 * IPT + lane;
        uint32_t dg[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int64_t i = base + j * 64;
            dg[j] = ids[i < hi ? i : hi - 1];
        }
        lds_barrier();
        uint32_t rk[IPT];
        bool live[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            live[j] = base + j * 64 < hi;
            rk[j] = tile_rank<AT>(wcnt[wave], dg[j], live[j]);  // stable, as the forward move
        }
        lds_barrier();
        if (t < kPsDig) {  // thread d: per-wave starts inside partition d, its tile total
            uint32_t tot = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint32_t c = wcnt[w][t];
                wcnt[w][t] = tot;
                tot += c;
            }
            tot_s[t] = tot;
        }
        lds_barrier();
        uint64_t v[IPT][NC];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const uint64_t pos = live[j] ? run[dg[j]] + wcnt[wave][dg[j]] + rk[j] : 0;
#pragma unroll
            for (int c = 0; c < NC; ++c) v[j][c] = live[j] ? cols.src[c][pos] : 0;
        }
#pragma unroll
        for (int j = 0; j < IPT; ++j)
            if (live[j])
#pragma unroll
                for (int c = 0; c < NC; ++c) __builtin_nontemporal_store(v[j][c], &cols.dst[c][base + j * 64]);
        lds_barrier();
        if (t < kPsDig) run[t] += tot_s[t];
    }
}

// Filter + partition ids + per-segment histogram in one pass (config 4's probe side, fewer than
// kPsDig partitions): block b streams its segment [b * seg, (b + 1) * seg) -- seg a multiple of the
// 8192-row tile -- with FastTile's 16-B loads of the key and up to two term columns (every load of a
// tile issued before the predicate), writes the ids as u16 pairs and counts them per partition in
// byte-packed register counters, so no histogram pass re-reads the id stream.  The generic id pass
// (k_hash_ids8_pred) evaluated the predicate and loaded the key in two dependent rounds of 4-row
// loads (3.1 TB/s).  Rows past the last whole tile (the tail of the last segment) go row by row.
__device__ __forceinline__ uint32_t part_of_key(int64_t k, uint32_t parts) {
    uint64_t h = 0x9E3779B97F4A7C15ull;  // k_hash_ids8's hash of one non-null key column
    h = hash64(h ^ (hash64((uint64_t)k) + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2)));
    return (uint32_t)(h % parts);
}

template <int NTERMS>
__global__ __launch_bounds__(kRsThreads) void k_ids_hist_pred(FastIn in, PredTerms terms, int64_t n, int64_t seg,
                                                              uint32_t parts, uint8_t *__restrict__ ids,
                                                              uint32_t *__restrict__ hist, int nblocks) {
    constexpr int W = kRsThreads / 64, TILE = kRsThreads * kFastR;
    __shared__ uint32_t wc[W][kPsDig];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t lo = (int64_t)blockIdx.x * seg, hi = lo + seg < n ? lo + seg : n;
    const int64_t full = hi > lo ? lo + (hi - lo) / TILE * TILE : lo;
    uint32_t cnt[kPsDig];
#pragma unroll
    for (int d = 0; d < kPsDig; ++d) cnt[d] = 0u;
    uint64_t acc[2] = {0ull, 0ull};  // byte counters of partitions 0-7 / 8-15 (flushed before 256)
    auto flush = [&]() {
#pragma unroll
        for (int d = 0; d < kPsDig; ++d) cnt[d] += (uint32_t)(acc[d >> 3] >> (8 * (d & 7))) & 0xFFu;
        acc[0] = acc[1] = 0ull;
    };
    FastTile<NTERMS, 0, true> ft;
    int tiles = 0;
    if (lo < full) ft.issue(in, lo + (int64_t)wave * 512 + 2 * lane);
    for (int64_t t0 = lo; t0 < full; t0 += TILE) {
        ft.eval(in, terms);
        uint32_t id[kFastR];
#pragma unroll
        for (int r = 0; r < kFastR; ++r) id[r] = ((ft.sel >> r) & 1u) ? part_of_key(ft.k(r), parts) : parts;
        if (t0 + TILE < full) ft.issue(in, t0 + TILE + (int64_t)wave * 512 + 2 * lane);
        const int64_t base = t0 + (int64_t)wave * 512 + 2 * lane;
#pragma unroll
        for (int j = 0; j < kFastPairs; ++j) {
            *(uint16_t *)(ids + base + j * 128) = (uint16_t)(id[2 * j] | (id[2 * j + 1] << 8));
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const uint32_t d = id[2 * j + q];
                const uint64_t one = 1ull << (8 * (d & 7));
                acc[0] += d < 8 ? one : 0ull;
                acc[1] += d < 8 ? 0ull : one;
            }
        }
        if (++tiles == 31) {  // 31 tiles x 8 rows < 256 per byte counter
            flush();
            tiles = 0;
        }
    }
    flush();
    for (int64_t i = full + t; i < hi; i += kRsThreads) {  // ragged tail, one row per thread
        bool ok = NTERMS == 0 || !terms.is_or;
#pragma unroll
        for (int q = 0; q < NTERMS; ++q) {
            const PredTerm pt = terms.t[q];
            int64_t v = in.term[q][i];
            if (pt.ctype == QEH_DT_FLOAT64) v = f64_order_key(in.term_dt[q] == QEH_DT_FLOAT64 ? as_f64(v) : (double)v);
            const bool tr = cmp_i64(pt.op, v, pt.lit);
            ok = terms.is_or ? (q == 0 ? tr : (ok || tr)) : (ok && tr);
        }
        const uint32_t d = ok ? part_of_key(in.key[i], parts) : parts;
        ids[i] = (uint8_t)d;
#pragma unroll
        for (int e = 0; e < kPsDig; ++e) cnt[e] += d == (uint32_t)e ? 1u : 0u;
    }
#pragma unroll
    for (int d = 0; d < kPsDig; ++d) {
        uint32_t c = cnt[d];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
        if (lane == 0) wc[wave][d] = c;
    }
    __syncthreads();
    if (t < kPsDig) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) c += wc[w][t];
        hist[(int64_t)t * nblocks + blockIdx.x] = c;  // digit-major, as k_rs_hist_u8
    }
}

// Sort state: encoded keys + permutation, double-buffered.
struct RadixState {
    DevBuf k[2], v[2];
    int cur = 0;
    int64_t n = 0;
    bool enc_injective = false;  // k[cur] encodes the last-sorted column one-to-one (no null-flag pass)
    int part_shift = -1;         // >= 0: k[cur] holds (first key << part_shift) | ..., the pair encoding
    bool key32 = false;          // k[] currently holds 32-bit keys (column range fits 32 bits)
};

// ballot ranking when asked for (QEH_RS_BALLOT=1, A/B) or when the device's LDS atomics failed the
// lane-order self-check (lds_atomic_rank_ok)
static bool rs_ballot(qeh_ctx *ctx) {
    return std::getenv("QEH_RS_BALLOT") != nullptr || !lds_atomic_rank_ok(ctx);
}

// Stable LSD passes over the low `bits` of the encoded keys in rs.
template <typename KeyT>
static int radix_passes_t(qeh_ctx *ctx, RadixState &rs, int bits) {
    const int64_t n = rs.n;
    if (n <= 1 || bits <= 0) return QEH_OK;
    // one long-lived scatter workgroup per CU (see k_rs_scatter); hist uses the same segments
    const int nblocks = (int)std::min<int64_t>(std::max<int64_t>((n + kRsSTile - 1) / kRsSTile, 1), (int64_t)ctx->props.multiProcessorCount);
    const int64_t seg = (n + nblocks - 1) / nblocks;
    DevBuf hist, offs, nd;
    QEH_TRY(hist.alloc(ctx, (size_t)kRadix * nblocks * 4));
    QEH_TRY(offs.alloc(ctx, (size_t)kRadix * nblocks * 8));
    // every scatter but the last also writes the next pass's digit as one byte per element, so
    // that pass's histogram reads 1 B instead of the key (sizeof(KeyT) B)
    const bool multi = bits > kRadixBits && n >= (int64_t)kRsSTile;
    if (multi) QEH_TRY(nd.alloc(ctx, (size_t)n));
    for (int shift = 0; shift < bits; shift += kRadixBits) {
        KernelTimer kt(ctx, "radix_pass");
        const int c = rs.cur;
        if (multi && shift > 0)
            hipLaunchKernelGGL(k_rs_hist_u8, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, nd.as<uint8_t>(), n, seg,
                               hist.as<uint32_t>(), nblocks);
        else
            hipLaunchKernelGGL(k_rs_hist<KeyT>, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, rs.k[c].as<KeyT>(), n, seg,
                               shift, hist.as<uint32_t>(), nblocks, RsEncode{});
        QEH_HIP(hipGetLastError());
        QEH_TRY(exclusive_scan_u32(ctx, hist.as<uint32_t>(), offs.as<uint64_t>(), (int64_t)kRadix * nblocks, nullptr));
        const bool next = multi && shift + kRadixBits < bits;
        auto scat = rs_ballot(ctx) ? k_rs_scatter<KeyT, false> : k_rs_scatter<KeyT, true>;
        hipLaunchKernelGGL(scat, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, rs.k[c].as<KeyT>(), rs.v[c].as<uint32_t>(), n, seg, shift, offs.as<uint64_t>(),
                           nblocks, rs.k[1 - c].as<KeyT>(), rs.v[1 - c].as<uint32_t>(), next ? nd.as<uint8_t>() : nullptr,
                           shift + kRadixBits, RsDecode{}, RsEncode{}, nullptr);
        QEH_HIP(hipGetLastError());
        rs.cur = 1 - c;
    }
    return QEH_OK;
}

// One stable pass on the 8-bit digit at `shift` (u32 / u64 keys as KeyT).
template <typename KeyT>
static int radix_pass_at(qeh_ctx *ctx, RadixState &rs, int shift) {
    const int64_t n = rs.n;
    if (n <= 1) return QEH_OK;
    const int nblocks = (int)std::min<int64_t>(std::max<int64_t>((n + kRsSTile - 1) / kRsSTile, 1), (int64_t)ctx->props.multiProcessorCount);
    const int64_t seg = (n + nblocks - 1) / nblocks;
    DevBuf hist, offs;
    QEH_TRY(hist.alloc(ctx, (size_t)kRadix * nblocks * 4));
    QEH_TRY(offs.alloc(ctx, (size_t)kRadix * nblocks * 8));
    KernelTimer kt(ctx, "radix_pass");
    const int c = rs.cur;
    hipLaunchKernelGGL(k_rs_hist<KeyT>, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, rs.k[c].as<KeyT>(), n, seg, shift,
                       hist.as<uint32_t>(), nblocks, RsEncode{});
    QEH_HIP(hipGetLastError());
    QEH_TRY(exclusive_scan_u32(ctx, hist.as<uint32_t>(), offs.as<uint64_t>(), (int64_t)kRadix * nblocks, nullptr));
    auto scat = rs_ballot(ctx) ? k_rs_scatter<KeyT, false> : k_rs_scatter<KeyT, true>;
    hipLaunchKernelGGL(scat, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, rs.k[c].as<KeyT>(), rs.v[c].as<uint32_t>(), n, seg, shift, offs.as<uint64_t>(), nblocks,
                       rs.k[1 - c].as<KeyT>(), rs.v[1 - c].as<uint32_t>(), nullptr, 0, RsDecode{}, RsEncode{}, nullptr);
    QEH_HIP(hipGetLastError());
    rs.cur = 1 - c;
    return QEH_OK;
}

static int gc_of(qeh_ctx *ctx, int64_t nchunks) {
    return (int)std::min<int64_t>(nchunks, (int64_t)ctx->props.multiProcessorCount * 8);
}

// Stable LSD passes over the low `bits` of the encoded keys in rs.
static int radix_passes(qeh_ctx *ctx, RadixState &rs, int bits) {
    return rs.key32 ? radix_passes_t<uint32_t>(ctx, rs, bits) : radix_passes_t<uint64_t>(ctx, rs, bits);
}

static int bit_length(uint64_t x) {
    int b = 0;
    while (b < 64 && (x >> b) != 0) ++b;
    return b;
}

// Encode key column `c` through the current permutation (or identity) and
// sort by it.  Returns the key range bits used.
static int sort_by_column(qeh_ctx *ctx, RadixState &rs, const qeh_column &col, bool asc, bool first,
                          bool nulls_last = false) {
    const ColRef c = make_colref(col);
    const int64_t n = rs.n;
    DevBuf st;
    QEH_TRY(st.alloc(ctx, sizeof(KeyStats)));
    KeyStats ks{};
    {
        KernelTimer kt(ctx, "sort_encode");
        hipLaunchKernelGGL(k_stats_init, dim3(1), dim3(1), 0, ctx->stream, st.as<KeyStats>());
        // min/max do not depend on row order: read the column directly, not through the permutation
        hipLaunchKernelGGL(k_key_stats, dim3(grid_for(ctx, n, kBlock * 8, 1)), dim3(kBlock), 0, ctx->stream, c, nullptr, n,
                           st.as<KeyStats>());
    }
    QEH_HIP(hipGetLastError());
    QEH_TRY(read_small(ctx, &ks, st.p, sizeof ks));
    const bool nullable = col.validity != nullptr && col.null_count != 0;
    int bits = 1;  // all NULL (or empty)
    // NULLs first: NULL -> 0, values -> 1 .. span+1; NULLs last: values -> 0 .. span, NULL -> span+1
    uint64_t bias = (nullable && !nulls_last) ? 1 : 0;
    uint64_t null_code = 0;
    bool null_pass = false;
    if (ks.mn <= ks.mx) {
        const uint64_t span = (uint64_t)ks.mx - (uint64_t)ks.mn;
        if (nullable && span == UINT64_MAX) {  // 2^64 values + NULL: 65 bits -> separate null-flag pass
            bias = 0;
            null_pass = true;
        }
        const uint64_t top = span + ((nullable && !null_pass) ? 1 : 0);
        if (nullable && nulls_last && !null_pass) null_code = top;
        bits = bit_length(top);
        if (bits == 0) bits = 1;
    }
    for (int pass = 0; pass < (null_pass ? 2 : 1); ++pass) {
        const uint32_t *pm = (first && pass == 0) ? nullptr : rs.v[rs.cur].as<uint32_t>();
        const int o = 1 - rs.cur;  // encode into the spare buffers, then swap
        const int pbits = pass == 0 ? bits : 1;
        rs.key32 = pbits <= 32;  // narrow keys halve the key traffic of every pass
        {
            KernelTimer kt(ctx, "sort_encode");
            const int g = grid_for(ctx, n, kBlock * 8, 8);
            // the null-flag pass (pass 1) orders NULL vs value: code 1 for NULL when NULLs go last
            const uint64_t nc = pass == 0 ? null_code : (nulls_last ? 1 : 0);
            if (rs.key32)
                hipLaunchKernelGGL(k_encode<uint32_t>, dim3(g), dim3(kBlock), 0, ctx->stream, c, pm, n, ks.mn, ks.mx,
                                   asc ? 1 : 0, bias, pass, nc, rs.k[o].as<uint32_t>(), rs.v[o].as<uint32_t>());
            else
                hipLaunchKernelGGL(k_encode<uint64_t>, dim3(g), dim3(kBlock), 0, ctx->stream, c, pm, n, ks.mn, ks.mx,
                                   asc ? 1 : 0, bias, pass, nc, rs.k[o].as<uint64_t>(), rs.v[o].as<uint32_t>());
        }
        QEH_HIP(hipGetLastError());
        rs.cur = o;
        QEH_TRY(radix_passes(ctx, rs, pbits));
    }
    rs.enc_injective = !null_pass;
    return QEH_OK;
}

// ---- two-key sorts (ROW_NUMBER's PARTITION BY k ORDER BY v, ORDER BY a, b) ----------------
// One LSD sort over the pair encoding K = (enc(k) << bv) | (enc(v) >> shift)
// instead of one sort per column.  When the two ranges need more than 64 bits,
// v keeps only its top bv bits (total 48 or 64) and a fix-up pass sorts the
// runs of equal K (rare: rows that share k and the top bits of v) by the
// dropped low bits, ties by row index, so the order stays exact.
constexpr int64_t kPairMaxRun = 64;

__device__ __forceinline__ uint64_t enc_key(const ColRef &c, int64_t row, int64_t mn, int64_t mx, int asc) {
    const int64_t x = ordered_key(c, row);
    return asc ? (uint64_t)x - (uint64_t)mn : (uint64_t)mx - (uint64_t)x;
}

template <typename KeyT>
__global__ void k_encode_pair(ColRef a, ColRef b, int64_t n, int64_t amn, int64_t amx, int aasc, int64_t bmn, int64_t bmx,
                              int basc, int bv, int shift, KeyT *__restrict__ keys, uint32_t *__restrict__ perm) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t ka = enc_key(a, i, amn, amx, aasc), kb = enc_key(b, i, bmn, bmx, basc);
        keys[i] = (KeyT)((bv >= 64 ? 0ull : ka << bv) | (kb >> shift));
        perm[i] = (uint32_t)i;
    }
}

__global__ void k_fix_pair_runs(const uint64_t *__restrict__ K, uint32_t *__restrict__ perm, int64_t n, ColRef b, int64_t bmn,
                                int64_t bmx, int basc, int shift, uint32_t *overflow) {
    const uint64_t mask = (1ull << shift) - 1ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = K[i];
        if (K[i + 1] != k || (i > 0 && K[i - 1] == k)) continue;  // not the start of a run of equal K
        int64_t j = i + 1;
        while (j + 1 < n && K[j + 1] == k && j - i < kPairMaxRun) ++j;
        if (j + 1 < n && K[j + 1] == k) {
            *overflow = 1u;  // a long run: the caller falls back to the per-column sort
            continue;
        }
        // stable LSD from the identity left the run in row order: insertion-sort it by the low bits
        for (int64_t a = i + 1; a <= j; ++a) {
            const uint32_t r = perm[a];
            const uint64_t lo = enc_key(b, r, bmn, bmx, basc) & mask;
            int64_t c = a - 1;
            while (c >= i) {
                const uint32_t rc = perm[c];
                const uint64_t lc = enc_key(b, rc, bmn, bmx, basc) & mask;
                if (lc < lo || (lc == lo && rc < r)) break;
                perm[c + 1] = rc;
                --c;
            }
            perm[c + 1] = r;
        }
    }
}

constexpr int kPairNotEligible = -1;

static int sort_perm_pair(qeh_ctx *ctx, const qeh_column &ca, const qeh_column &cb, bool aasc, bool basc, int64_t n,
                          RadixState &rs) {
    if (std::getenv("QEH_NO_PAIR_SORT")) return kPairNotEligible;
    if ((ca.validity && ca.null_count != 0) || (cb.validity && cb.null_count != 0)) return kPairNotEligible;
    const ColRef a = make_colref(ca), b = make_colref(cb);
    DevBuf st;
    QEH_TRY(st.alloc(ctx, 2 * sizeof(KeyStats) + 16));
    KeyStats ks[2];
    {
        KernelTimer kt(ctx, "sort_encode");
        KeyStats *d = st.as<KeyStats>();
        hipLaunchKernelGGL(k_stats_init, dim3(1), dim3(1), 0, ctx->stream, d);
        hipLaunchKernelGGL(k_stats_init, dim3(1), dim3(1), 0, ctx->stream, d + 1);
        const int g = grid_for(ctx, n, kBlock * 8, 1);
        hipLaunchKernelGGL(k_key_stats, dim3(g), dim3(kBlock), 0, ctx->stream, a, nullptr, n, d);
        hipLaunchKernelGGL(k_key_stats, dim3(g), dim3(kBlock), 0, ctx->stream, b, nullptr, n, d + 1);
    }
    QEH_HIP(hipGetLastError());
    QEH_TRY(read_small(ctx, ks, st.p, sizeof ks));
    const int ba = bit_length((uint64_t)ks[0].mx - (uint64_t)ks[0].mn);
    const int bb = bit_length((uint64_t)ks[1].mx - (uint64_t)ks[1].mn);
    int bv, shift, total;
    if (ba + bb <= 64) {
        bv = bb;
        shift = 0;
        total = ba + bb;
    } else if (ba <= 40) {
        // K keeps a's bits and the top bits of b; equal-K runs (fixed up exactly below) stay rare
        // when K has ~10 bits more than the row count needs: total = roundup8(log2 n + 10), at
        // least 16 bits of b, at most 64 (1e9 rows: 40 bits = 5 passes instead of 6)
        total = std::min(64, (bit_length((uint64_t)n) + 10 + 7) / 8 * 8);
        if (total < ba + 16) total = std::min(64, (ba + 16 + 7) / 8 * 8);
        if (total < 40) total = 40;  // 64-bit keys (k_fix_pair_runs reads them as such)
        bv = total - ba;
        shift = bb - bv;
    } else {
        return kPairNotEligible;
    }
    if (total == 0) total = 1;
    rs.key32 = total <= 32;
    {
        KernelTimer kt(ctx, "sort_encode");
        const int g = grid_for(ctx, n, kBlock * 8, 8);
        const int o = 1 - rs.cur;
        if (rs.key32)
            hipLaunchKernelGGL(k_encode_pair<uint32_t>, dim3(g), dim3(kBlock), 0, ctx->stream, a, b, n, ks[0].mn, ks[0].mx,
                               aasc ? 1 : 0, ks[1].mn, ks[1].mx, basc ? 1 : 0, bv, shift, rs.k[o].as<uint32_t>(),
                               rs.v[o].as<uint32_t>());
        else
            hipLaunchKernelGGL(k_encode_pair<uint64_t>, dim3(g), dim3(kBlock), 0, ctx->stream, a, b, n, ks[0].mn, ks[0].mx,
                               aasc ? 1 : 0, ks[1].mn, ks[1].mx, basc ? 1 : 0, bv, shift, rs.k[o].as<uint64_t>(),
                               rs.v[o].as<uint32_t>());
        rs.cur = o;
    }
    QEH_HIP(hipGetLastError());
    QEH_TRY(radix_passes(ctx, rs, total));
    if (shift > 0) {
        DevBuf flag;
        QEH_TRY(flag.alloc(ctx, 8));
        QEH_HIP(hipMemsetAsync(flag.p, 0, 8, ctx->stream));
        {
            KernelTimer kt(ctx, "sort_encode");
            hipLaunchKernelGGL(k_fix_pair_runs, dim3(grid_for(ctx, n, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream,
                               rs.k[rs.cur].as<uint64_t>(), rs.v[rs.cur].as<uint32_t>(), n, b, ks[1].mn, ks[1].mx,
                               basc ? 1 : 0, shift, flag.as<uint32_t>());
        }
        QEH_HIP(hipGetLastError());
        uint32_t of = 0;
        QEH_TRY(read_small(ctx, &of, flag.p, 4));
        if (of) return kPairNotEligible;
    }
    rs.enc_injective = false;
    rs.part_shift = bv;
    return QEH_OK;
}

// Stable lexicographic permutation by keys (last key sorted first).
static int sort_perm(qeh_ctx *ctx, const qeh_column *keys, int n_keys, const int8_t *ascending, int64_t n,
                     RadixState &rs, const int8_t *nulls_first = nullptr) {
    rs.n = n;
    for (int b = 0; b < 2; ++b) {
        QEH_TRY(rs.k[b].alloc(ctx, (size_t)std::max<int64_t>(n, 1) * 8));
        QEH_TRY(rs.v[b].alloc(ctx, (size_t)std::max<int64_t>(n, 1) * 4));
    }
    rs.cur = 0;
    rs.part_shift = -1;
    if (n == 0) return QEH_OK;
    if (n_keys == 2) {
        const int r = sort_perm_pair(ctx, keys[0], keys[1], ascending ? ascending[0] != 0 : true,
                                     ascending ? ascending[1] != 0 : true, n, rs);
        if (r != kPairNotEligible) return r;
        rs.cur = 0;  // fall back: the per-column sort starts from the identity
        rs.part_shift = -1;
    }
    for (int j = n_keys - 1; j >= 0; --j)
        QEH_TRY(sort_by_column(ctx, rs, keys[j], ascending ? ascending[j] != 0 : true, j == n_keys - 1,
                               nulls_first ? nulls_first[j] == 0 : false));
    return QEH_OK;
}

static int check_sort_keys(const qeh_column *keys, int n_keys, int64_t *n) {
    if (n_keys < 1) return fail(QEH_E_INVALID, "sort needs at least one key");
    *n = keys[0].length;
    for (int j = 0; j < n_keys; ++j) {
        QEH_TRY(check_column(keys[j], "sort key"));
        if (keys[j].dtype == QEH_DT_UTF8) return fail(QEH_E_UNSUPPORTED, "Utf8 sort keys are not supported on the device");
        if (keys[j].length != *n) return fail(QEH_E_INVALID, "sort keys have different lengths");
    }
    return QEH_OK;
}

// ---- ROW_NUMBER ----------------------------------------------------------------------------
// flags[i] = 1 when sorted row i starts a new partition (partition columns differ from row i-1)
// One gather per row: each lane loads its row's keys through the permutation and takes the
// previous row's from the lane below (lane 0 loads its predecessor itself), halving the random
// reads of comparing perm[i-1] with perm[i] directly.  Whole workgroups step together, so every
// lane of a wave reaches the shuffles.
__global__ void k_part_flags(KeyCols part, const uint32_t *__restrict__ perm, int64_t n, uint32_t *__restrict__ flags) {
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
        const int64_t i = base + threadIdx.x;
        const bool act = i < n;
        const int64_t b = act ? (int64_t)perm[i] : 0;
        const bool own_prev = act && lane == 0 && i > 0;
        const int64_t a = own_prev ? (int64_t)perm[i - 1] : 0;
        uint32_t f = 0;
        for (int c = 0; c < part.n; ++c) {
            const int vb = act && col_valid(part.c[c], b) ? 1 : 0;
            const int64_t xb = vb ? load_i64(part.c[c], b) : 0;
            int va = __shfl_up(vb, 1, 64);
            int64_t xa = __shfl_up(xb, 1, 64);
            if (own_prev) {
                va = col_valid(part.c[c], a) ? 1 : 0;
                xa = va ? load_i64(part.c[c], a) : 0;
            }
            if (va != vb || (va && xa != xb)) f = 1;
        }
        if (act) flags[i] = i == 0 ? 1u : f;
    }
}

// single partition key: compare the sorted encodings (coalesced) instead of
// gathering the key column through the permutation.  shift >= the key width means the
// partition key occupies no bits (one distinct value): only row 0 starts a partition (a shift
// by the full width would be undefined and the hardware masks it to 0).
template <typename KeyT>
__global__ void k_part_flags_enc(const KeyT *__restrict__ enc, int64_t n, uint32_t *__restrict__ flags, int shift = 0) {
    const bool one_part = shift >= (int)(8 * sizeof(KeyT));
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        flags[i] = i == 0 || (!one_part && (enc[i] >> shift) != (enc[i - 1] >> shift));
}

// Row numbers without materialising partition ids: rn(i) = i - start(i) + 1,
// start(i) = the last partition start <= i.  Chunks of kRnChunk sorted
// positions: (1) each chunk's last start, (2) an exclusive prefix max over
// chunks, (3) per chunk a block max-scan seeded with (2), then the scatter
// rn[perm[i]] into input order.  No partition count is read back.
constexpr int kRnPer = 16;
constexpr int64_t kRnChunk = (int64_t)kBlock * kRnPer;

__global__ __launch_bounds__(kBlock) void k_rn_chunk_last(const uint32_t *__restrict__ flags, int64_t n, int64_t nchunks,
                                                          int64_t *__restrict__ last) {
    __shared__ int64_t red[kBlock / 64];
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        int64_t m = -1;
        const int64_t base = c * kRnChunk;
        for (int j = 0; j < kRnPer; ++j) {
            const int64_t i = base + (int64_t)j * kBlock + threadIdx.x;
            if (i < n && flags[i]) m = i > m ? i : m;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const int64_t o = __shfl_xor(m, d, 64);
            m = o > m ? o : m;
        }
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 1; w < kBlock / 64; ++w) m = red[w] > m ? red[w] : m;
            last[c] = m;
        }
        __syncthreads();
    }
}

// in place: last[c] <- max(last[0..c-1]) (exclusive), one workgroup
__global__ __launch_bounds__(1024) void k_rn_prefix_max(int64_t *__restrict__ last, int64_t nchunks) {
    __shared__ int64_t part[1024];
    const int t = threadIdx.x;
    const int64_t per = (nchunks + 1023) / 1024, lo = (int64_t)t * per, hi = lo + per < nchunks ? lo + per : nchunks;
    int64_t m = -1;
    for (int64_t c = lo; c < hi; ++c) m = last[c] > m ? last[c] : m;
    part[t] = m;
    __syncthreads();
    if (t == 0) {
        int64_t run = -1;
        for (int i = 0; i < 1024; ++i) {
            const int64_t x = part[i];
            part[i] = run;
            run = x > run ? x : run;
        }
    }
    __syncthreads();
    int64_t run = part[t];
    for (int64_t c = lo; c < hi; ++c) {
        const int64_t x = last[c];
        last[c] = run;
        run = x > run ? x : run;
    }
}

// PAIRS: instead of scattering rn[perm[i]] (1e9 random 8-byte writes), write the pairs
// (perm[i], rn) in sorted order; one stable radix pass on the destination's top bits then
// groups them by output window and k_rn_scatter_windows writes one window at a time
template <bool PAIRS>
__global__ __launch_bounds__(kBlock) void k_rn_write(const uint32_t *__restrict__ flags, const int64_t *__restrict__ carry,
                                                     const uint32_t *__restrict__ perm, int64_t n, int64_t nchunks,
                                                     int64_t *__restrict__ rn, uint32_t *__restrict__ pair_dst,
                                                     uint32_t *__restrict__ pair_rn) {
    __shared__ int64_t wmax[kBlock / 64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        // thread t owns kRnPer consecutive positions
        const int64_t base = c * kRnChunk + (int64_t)t * kRnPer;
        uint32_t f[kRnPer];
        int64_t m = -1;
#pragma unroll
        for (int j = 0; j < kRnPer; ++j) {
            const int64_t i = base + j;
            f[j] = i < n ? flags[i] : 0u;
            if (f[j]) m = i;
        }
        // exclusive max-scan of the threads' last starts, seeded with the chunks before
        int64_t incl = m;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t o = __shfl_up(incl, d, 64);
            if (lane >= d) incl = o > incl ? o : incl;
        }
        if (lane == 63) wmax[w] = incl;
        __syncthreads();
        int64_t start = carry[c];
        for (int q = 0; q < w; ++q) start = wmax[q] > start ? wmax[q] : start;
        const int64_t prev = __shfl_up(incl, 1, 64);
        if (lane > 0) start = prev > start ? prev : start;
#pragma unroll
        for (int j = 0; j < kRnPer; ++j) {
            const int64_t i = base + j;
            if (f[j]) start = i;
            if (i < n) {
                if (PAIRS) {
                    pair_dst[i] = perm[i];
                    pair_rn[i] = (uint32_t)(i - start + 1);
                } else {
                    rn[perm[i]] = i - start + 1;
                }
            }
        }
        __syncthreads();
    }
}

// pairs grouped by output window (destination >> shift): consecutive workgroups write inside
// one window at a time, so the partial-line writes meet in L2 / the Infinity Cache instead of HBM
__global__ void k_rn_scatter_windows(const uint32_t *__restrict__ dst, const uint32_t *__restrict__ val, int64_t n,
                                     int64_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[dst[i]] = (int64_t)val[i];
}

// start of every window in the window-grouped pairs (empty windows start where the next begins)
__global__ void k_rn_window_starts(const uint32_t *__restrict__ dst, int64_t n, int shift, int64_t nwin,
                                   int64_t *__restrict__ start) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t w = i < n ? (int64_t)(dst[i] >> shift) : nwin;
        const int64_t wp = i > 0 ? (int64_t)(dst[i - 1] >> shift) : -1;
        for (int64_t q = wp + 1; q <= w; ++q) start[q] = i;  // windows (wp, w] begin at i
    }
}

// XCD-local windows: workgroup b runs on XCD b % 8 (round-robin dispatch), and the workgroups of
// one XCD walk that XCD's windows (w = xcd, xcd + 8, ...) together, so a window's output lines
// (2 MB) are completed inside one L2 before they are written back
__global__ void k_rn_scatter_xcd(const uint32_t *__restrict__ dst, const uint32_t *__restrict__ val,
                                 const int64_t *__restrict__ start, int64_t nwin, int64_t *__restrict__ out) {
    constexpr int kXcd = 8;
    const int xcd = blockIdx.x % kXcd;
    const int64_t per = gridDim.x / kXcd, me = blockIdx.x / kXcd;
    for (int64_t w = xcd; w < nwin; w += kXcd) {
        const int64_t a = start[w], b = start[w + 1];
        for (int64_t i = a + me * blockDim.x + threadIdx.x; i < b; i += per * blockDim.x) out[dst[i]] = (int64_t)val[i];
    }
}

// ---- hash partition ---------------------------------------------------------------------------
__global__ void k_partition_ids(ColRef key, int64_t n, uint32_t parts, uint64_t *__restrict__ keys,
                                uint32_t *__restrict__ idx) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t p = 0;  // NULL keys hash like an empty key (partition.rs:292-316 skips them)
        if (col_valid(key, i)) p = (uint32_t)(hash64((uint64_t)load_i64(key, i)) % parts);
        keys[i] = p;
        idx[i] = (uint32_t)i;
    }
}

// range partition: NULL -> 0 (NULLs sort first); value -> number of splitters
// strictly below (ascending) / above (descending) its order key, so equal keys
// share a partition and partition p precedes p+1 in sort order
__global__ void k_range_ids(ColRef key, int64_t n, const int64_t *__restrict__ split, int n_split, int asc,
                            uint64_t *__restrict__ keys, uint32_t *__restrict__ idx) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t p = 0;
        if (col_valid(key, i)) {
            const int64_t k = ordered_key(key, i);
            for (int j = 0; j < n_split; ++j) p += asc ? split[j] < k : split[j] > k;
        }
        keys[i] = p;
        idx[i] = (uint32_t)i;
    }
}

// PartitionStrategy::Hash over several key columns (partition.rs:151-212, compute_row_hash
// :292-316): NULL cells contribute nothing to the row hash, as the reference skips them; Int32 /
// Int64 values and Utf8 bytes are mixed into one 64-bit hash (the hash function is not
// observable in results).
struct HashKeys {
    ColRef c[kMaxCols];
    const int32_t *offs[kMaxCols];
    const uint8_t *data[kMaxCols];
    int32_t n;
};

__global__ void k_hash_ids_multi(HashKeys keys, int64_t n, uint32_t parts, uint64_t *__restrict__ ids,
                                 uint32_t *__restrict__ idx) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t h = 0x9E3779B97F4A7C15ull;
        for (int j = 0; j < keys.n; ++j) {
            const ColRef &c = keys.c[j];
            if (!col_valid(c, i)) continue;
            uint64_t v;
            if (c.dtype == QEH_DT_UTF8) {
                v = 0xcbf29ce484222325ull;  // FNV-1a over the bytes
                for (int32_t b = keys.offs[j][i]; b < keys.offs[j][i + 1]; ++b) v = (v ^ keys.data[j][b]) * 0x100000001b3ull;
            } else {
                v = (uint64_t)load_i64(c, i);
            }
            h = hash64(h ^ (hash64(v) + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2)));
        }
        ids[i] = h % parts;
        idx[i] = (uint32_t)i;
    }
}

__global__ void k_hash_ids8(HashKeys keys, int64_t n, uint32_t parts, uint8_t *__restrict__ ids) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t h = 0x9E3779B97F4A7C15ull;
        for (int j = 0; j < keys.n; ++j) {
            const ColRef &c = keys.c[j];
            if (!col_valid(c, i)) continue;
            uint64_t v;
            if (c.dtype == QEH_DT_UTF8) {
                v = 0xcbf29ce484222325ull;
                for (int32_t b = keys.offs[j][i]; b < keys.offs[j][i + 1]; ++b) v = (v ^ keys.data[j][b]) * 0x100000001b3ull;
            } else {
                v = (uint64_t)load_i64(c, i);
            }
            h = hash64(h ^ (hash64(v) + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2)));
        }
        ids[i] = (uint8_t)(h % parts);
    }
}

// k_hash_ids8 for one non-null Int64 key column: eight rows per thread (four 16-B loads, one 8-B
// store of ids), the same hash.
__global__ __launch_bounds__(kBlock) void k_hash_ids8_i64(const int64_t *__restrict__ key, int64_t n, uint32_t parts,
                                                          uint8_t *__restrict__ ids) {
    typedef long long v2i64h __attribute__((ext_vector_type(2)));
    for (int64_t i0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 8; i0 < n; i0 += (int64_t)gridDim.x * kBlock * 8) {
        uint64_t v[8];
        if (i0 + 8 <= n && (((uintptr_t)(key + i0)) & 15) == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const v2i64h w = __builtin_nontemporal_load((const v2i64h *)(key + i0) + q);
                v[2 * q] = (uint64_t)w[0], v[2 * q + 1] = (uint64_t)w[1];
            }
        } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = i0 + q < n ? (uint64_t)key[i0 + q] : 0ull;
        }
        uint64_t out = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            uint64_t h = 0x9E3779B97F4A7C15ull;
            h = hash64(h ^ (hash64(v[q]) + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2)));
            out |= (uint64_t)(uint8_t)(h % parts) << (8 * q);
        }
        if (i0 + 8 <= n) {
            *(uint64_t *)(ids + i0) = out;
        } else {
            for (int q = 0; q < 8 && i0 + q < n; ++q) ids[i0 + q] = (uint8_t)(out >> (8 * q));
        }
    }
}

// The filter of a shuffle fused into the Exchange's id pass (config 4's probe side): rows whose
// predicate (an AND / OR list of column-literal comparisons) is TRUE get hash(key) % parts,
// the others `parts` (dropped by k_part_scatter).  One key column, Int32 / Int64.
__global__ __launch_bounds__(kBlock) void k_hash_ids8_pred(ColRef key, ColSet cols, PredTerms terms, int64_t n,
                                                           uint32_t parts, uint8_t *__restrict__ ids) {
    constexpr int R = 4;
    for (int64_t t0 = (int64_t)blockIdx.x * kBlock * R; t0 < n; t0 += (int64_t)gridDim.x * kBlock * R) {
        const int64_t row0 = t0 + threadIdx.x;
        const uint32_t m = eval_terms<R>(terms, cols, row0, kBlock, n);
        int64_t kv[R];
        uint32_t kvalid;
        load_rows<R>(key, row0, kBlock, n, kv, kvalid);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t i = row0 + (int64_t)r * kBlock;
            if (i >= n) continue;
            uint64_t h = 0x9E3779B97F4A7C15ull;  // k_hash_ids8's hash of one key column (NULL skipped)
            if ((kvalid >> r) & 1u) h = hash64(h ^ (hash64((uint64_t)kv[r]) + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2)));
            ids[i] = ((m >> r) & 1u) ? (uint8_t)(h % parts) : (uint8_t)parts;
        }
    }
}

// PartitionStrategy::Range (find_range_partition, partition.rs:320-341): the first boundary the
// value is below, or len(boundaries); NULL -> 0; only Int64 keys are ranged (every other column
// type lands in partition 0, as in the reference)
__global__ void k_range_ids_first_below(ColRef key, int64_t n, const int64_t *__restrict__ b, int nb, int is_i64,
                                        uint64_t *__restrict__ ids, uint32_t *__restrict__ idx) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t p = 0;
        if (is_i64 && col_valid(key, i)) {
            const int64_t v = ((const int64_t *)key.values)[i];
            p = (uint32_t)nb;
            for (int j = 0; j < nb; ++j)
                if (v < b[j]) {
                    p = (uint32_t)j;
                    break;
                }
        }
        ids[i] = p;
        idx[i] = (uint32_t)i;
    }
}

template <typename T>
__global__ void k_scatter(const T *__restrict__ src, const uint32_t *__restrict__ idx, int64_t m, T *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        out[idx[i]] = src[i];
}

__global__ void k_count_parts(const uint64_t *__restrict__ ids, int64_t n, int parts, unsigned long long *__restrict__ counts) {
    __shared__ uint32_t h[kRadix];
    for (int i = threadIdx.x; i < kRadix; i += blockDim.x) h[i] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&h[ids[i]], 1u);
    __syncthreads();
    for (int p = threadIdx.x; p < parts; p += blockDim.x)
        if (h[p]) atomicAdd(&counts[p], (unsigned long long)h[p]);
}

__global__ void k_u64_to_u32_idx(const int64_t *__restrict__ in, int64_t n, int64_t limit, uint32_t *__restrict__ out,
                                 uint32_t *__restrict__ bad) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v = in[i];
        if (v < 0 || v >= limit) *bad = 1u;
        out[i] = (uint32_t)(v < 0 || v >= limit ? 0 : v);
    }
}

}  // namespace qeh

using namespace qeh;

extern "C" int qeh_sort_indices(qeh_ctx *ctx, const qeh_column *keys, int n_keys, const int8_t *ascending,
                                qeh_column *out_perm) {
    if (!ctx || !keys || !out_perm) return fail(QEH_E_INVALID, "qeh_sort_indices: bad argument");
    DeviceGuard dg(ctx->device);
    int64_t n;
    QEH_TRY(check_sort_keys(keys, n_keys, &n));
    RadixState rs;
    QEH_TRY(sort_perm(ctx, keys, n_keys, ascending, n, rs));
    QEH_TRY(alloc_column(ctx, QEH_DT_UINT32, n, false, out_perm));
    if (n > 0) QEH_HIP(hipMemcpyAsync(out_perm->values, rs.v[rs.cur].p, (size_t)n * 4, hipMemcpyDeviceToDevice, ctx->stream));
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    return QEH_OK;
}

// ---- payload-carrying sort (qeh_merge_sorted of one Int64 / Int32 key and one 8-byte column) ----
// The key is encoded as in sort_by_column (asc: x - mn, desc: mx - x; NULL = 0 below every value
// code when NULLs go first, or above them when last) and sorted with the payload itself as the carried
// value, so no permutation is gathered afterwards: the sorted key column is decoded from the sorted
// codes, and the last pass writes the payload straight into the output column.

// valid bytes (the last pass's, one per row, each 0 or 1) -> the key's validity bitmap: one 64-row word
// per thread from four 16-B loads (bit i of a dword's 4 flags = bit 8 i of the dword)
__global__ void k_pack_valid(const uint8_t *__restrict__ vb, int64_t n, uint64_t *__restrict__ valid) {
    typedef unsigned int v4u32p __attribute__((ext_vector_type(4)));
    const int64_t nw = (n + 63) >> 6;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r0 = w << 6;
        uint64_t m = 0;
        if (r0 + 64 <= n) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const v4u32p x = __builtin_nontemporal_load((const v4u32p *)(vb + r0) + q);
                const uint32_t d[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint32_t y = d[t];
                    const uint32_t b4 = (y & 1u) | ((y >> 7) & 2u) | ((y >> 14) & 4u) | ((y >> 21) & 8u);
                    m |= (uint64_t)b4 << (q * 16 + t * 4);
                }
            }
        } else {
            for (int64_t i = r0; i < n; ++i) m |= (uint64_t)(vb[i] != 0) << (i - r0);
        }
        valid[w] = m;
    }
}

// ---- MSD payload sort ----------------------------------------------------------------------
// Codes of 24..45 bits over >= 2^20 rows: two stable 256-way passes on the top 16 bits (k_rs_scatter
// over the whole array, then the same scatter inside every first-pass bucket: SEG blocks never straddle
// a bucket and the scan orders (bucket, digit, block)), then one workgroup per sub-bucket sorts its
// rows by the remaining low bits in LDS -- stable 8-bit LDS passes over (low code, row) pairs, ranks
// by lane-ordered LDS atomics as the global passes -- and writes the decoded key, the payload
// (gathered inside the sub-bucket) and the valid byte.  Three passes over the rows instead of
// ceil(bits / 8) hist + scatter pairs.  A sub-bucket above kMsdCap rows is copied through when its
// codes are all equal (the NULLs, a repeated key), else the caller redoes the sort on the LSD path.
constexpr int kMsdCap = 4096;
constexpr int kMsdThreads = 512;
constexpr int kMsdBits = 16;  // code bits the two global passes consume
constexpr uint32_t kMsdMaxBig = 255;  // sub-buckets above kMsdCap rows handled by k_msd_big
constexpr int kMsdLdsBits = 9;        // digit of the in-LDS passes: 25 low bits in three passes
constexpr int kMsdMaxLow = 29;        // low code bits the LDS sort packs beside a 12-bit row index

__global__ __launch_bounds__(kRsThreads) void k_rs_hist_u8_seg(const uint8_t *__restrict__ dg, const int64_t *__restrict__ segtab,
                                                               uint32_t *__restrict__ hist) {
    constexpr int W = kRsThreads / 64;
    __shared__ uint32_t h[W][kRadix];
    for (int i = threadIdx.x; i < W * kRadix; i += kRsThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const int64_t *e = segtab + 4 * (int64_t)blockIdx.x;
    const int64_t lo = e[0], hi = e[1];
    const int wave = threadIdx.x >> 6;
    const int64_t a = std::min<int64_t>(hi, (lo + 15) & ~(int64_t)15), b = std::max<int64_t>(a, hi & ~(int64_t)15);
    for (int64_t i = lo + threadIdx.x; i < a; i += kRsThreads) atomicAdd(&h[wave][dg[i]], 1u);
    for (int64_t i = b + threadIdx.x; i < hi; i += kRsThreads) atomicAdd(&h[wave][dg[i]], 1u);
    for (int64_t i = a + 16 * (int64_t)threadIdx.x; i < b; i += 16 * (int64_t)kRsThreads) {
        typedef unsigned int v4u32s __attribute__((ext_vector_type(4)));
        const v4u32s w = __builtin_nontemporal_load((const v4u32s *)(dg + i));
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r) atomicAdd(&h[wave][(ws[q] >> (8 * r)) & 0xff], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kRadix) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) c += h[w][threadIdx.x];
        hist[e[2] + (int64_t)threadIdx.x * e[3]] = c;
    }
}

// sub-bucket (bucket b, digit d) starts: the scanned second-pass offset of the bucket's first block
// (btab per bucket: hist base, blocks, start); sb[65536] = n
__global__ void k_msd_sbstart(const uint64_t *__restrict__ offs2, const int64_t *__restrict__ btab, int64_t n,
                              uint64_t *__restrict__ sb) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id > kRadix * kRadix) return;
    if (id == kRadix * kRadix) {
        sb[id] = (uint64_t)n;
        return;
    }
    const int b = id >> kRadixBits, d = id & (kRadix - 1);
    const int64_t base = btab[3 * b], nb = btab[3 * b + 1];
    sb[id] = nb ? offs2[base * kRadix + (int64_t)d * nb] : (uint64_t)btab[3 * b + 2];
}

__device__ __forceinline__ void msd_emit(const RsDecode &dec, uint64_t *__restrict__ vout, int64_t pos, uint64_t c,
                                         uint64_t val) {
    const bool ok = !dec.validb || c != dec.null_code;
    const int64_t x = ok ? (dec.asc ? (int64_t)(c - dec.bias + (uint64_t)dec.mn) : (int64_t)((uint64_t)dec.mx - (c - dec.bias)))
                         : 0;
    if (dec.dt == QEH_DT_INT32) ((int32_t *)dec.out)[pos] = (int32_t)x;
    else ((int64_t *)dec.out)[pos] = x;
    if (dec.validb) dec.validb[pos] = ok ? 1 : 0;
    vout[pos] = val;
}

// one workgroup per sub-bucket (blockIdx.x = bucket << 8 | digit): the codes here share their top 16
// bits; pass 2 left their low 32 bits.  Rows e = wave * 64 J + j * 64 + lane keep input order in
// (wave, j, lane).  The first LDS pass ranks (low code, row e) and leaves packed words
// (remaining code bits << 12 | e), so the later passes move one dword per row (lbits <= 29).
// list (optional): only the sub-buckets list[1 .. list[0]] (the ones k_msd_csort queued), one per
// workgroup; else sub-bucket blockIdx.x
__global__ __launch_bounds__(kMsdThreads) void k_msd_lds_sort(const uint32_t *__restrict__ codes, const uint64_t *__restrict__ vin,
                                                              const uint64_t *__restrict__ sb, int lbits, RsDecode dec,
                                                              uint64_t *__restrict__ vout, uint32_t *__restrict__ flag,
                                                              uint32_t *__restrict__ big, const uint32_t *__restrict__ list) {
    constexpr int W = kMsdThreads / 64, J = kMsdCap / kMsdThreads;
    constexpr int DB = kMsdLdsBits, ND = 1 << DB, DPT = ND / kMsdThreads;  // digits per thread in the scan
    static_assert(DPT >= 1, "one digit per thread at least");
    constexpr int IB = 12;                                                 // row bits (kMsdCap = 2^12)
    static_assert(kMsdCap == 1 << IB, "row index bits");
    __shared__ uint32_t buf[2][kMsdCap];
    __shared__ uint32_t wc[W][ND];
    __shared__ uint32_t loc[ND], wsum[W];
    const uint32_t nlist = list ? list[0] : 0u;
    // list mode: the grid strides over the queued sub-buckets; else sub-bucket blockIdx.x
    for (uint32_t it = blockIdx.x; list ? it < nlist : it == blockIdx.x; it += gridDim.x) {
    const uint32_t id = list ? list[1 + it] : it;
    const int64_t s0 = (int64_t)sb[id], s1 = (int64_t)sb[id + 1];
    const int64_t m = s1 - s0;
    if (m <= 0) continue;
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    if (m > kMsdCap) {  // k_msd_big takes it, with the whole grid
        if (t == 0) {
            const uint32_t q = atomicAdd(big, 1u);
            if (q < kMsdMaxBig) big[1 + q] = id;
            else atomicOr(flag, 1u);
        }
        continue;
    }
    const int mm = (int)m;
    const uint64_t hi_code = (uint64_t)id << lbits;
    const uint32_t lmask = lbits >= 32 ? 0xFFFFFFFFu : ((1u << lbits) - 1u);
    for (int e = t; e < mm; e += kMsdThreads) buf[0][e] = codes[s0 + e] & lmask;
    int cur = 0;
    for (int sh = 0; sh < lbits; sh += DB) {
        const bool first = sh == 0;
        for (int i = t; i < W * ND; i += kMsdThreads) (&wc[0][0])[i] = 0;
        __syncthreads();
        uint32_t kk[J], rk[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int e = wave * 64 * J + j * 64 + lane;
            const bool live = e < mm;
            kk[j] = live ? buf[cur][e] : 0u;
            // the first pass reads raw low codes; later passes packed words (digit above the row bits)
            const uint32_t dg = first ? (kk[j] & (ND - 1)) : ((kk[j] >> IB) & (ND - 1));
            rk[j] = live ? atomicAdd(&wc[wave][dg], 1u) : 0u;
        }
        __syncthreads();
        // thread t owns digits t * DPT .. + DPT - 1: wave starts inside each digit, then one scan
        uint32_t dt[DPT], tot = 0;
#pragma unroll
        for (int q = 0; q < DPT; ++q) {
            const int d = t * DPT + q;
            uint32_t c0 = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint32_t c = wc[w][d];
                wc[w][d] = c0;
                c0 += c;
            }
            dt[q] = c0;
            tot += c0;
        }
        const uint32_t inc = wave_incl_scan(tot);
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        uint32_t wb = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) wb += w < wave ? wsum[w] : 0u;
        uint32_t run = wb + inc - tot;
#pragma unroll
        for (int q = 0; q < DPT; ++q) {
            loc[t * DPT + q] = run;
            run += dt[q];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int e = wave * 64 * J + j * 64 + lane;
            if (e >= mm) continue;
            const uint32_t dg = first ? (kk[j] & (ND - 1)) : ((kk[j] >> IB) & (ND - 1));
            const uint32_t p = loc[dg] + wc[wave][dg] + rk[j];
            // packed: the code bits above this pass's digit, then the row
            buf[cur ^ 1][p] = first ? (((kk[j] >> DB) << IB) | (uint32_t)e)
                                    : ((((kk[j] >> IB) >> DB) << IB) | (kk[j] & (kMsdCap - 1)));
        }
        __syncthreads();
        cur ^= 1;
    }
    // every pass ran (lbits > 0): buf holds rows in code order; the code is re-read from the row
    for (int e = t; e < mm; e += kMsdThreads) {
        const uint32_t r = buf[cur][e] & (kMsdCap - 1);
        msd_emit(dec, vout, s0 + e, hi_code | (codes[s0 + r] & lmask), vin[s0 + r]);
    }
    __syncthreads();  // (list mode: buf is read before the next sub-bucket overwrites it)
    }
}

// Counting sort of a sub-bucket in one LDS pass (replaces the three radix passes of k_msd_lds_sort for
// spread codes): 2^12 buckets of the top bits of the remaining code, each row placed by its bucket's
// start + arrival beside its (code, row) word, then ranked exactly among its bucket's rows by
// (code, row) -- the row order within equal codes is the input order, as the radix passes keep it.
// The ranked words then move to their sorted slots in LDS, and the output is written in sorted order
// (coalesced stores, the payload gathered by row): scattered stores measured 5.20 ms for the
// Merge::sorted shape against 4.09 ms for the radix passes, sorted-order stores 3.93 ms.
// A sub-bucket with a bucket above kCsCap rows (clustered or repeated codes) is queued in fb for
// k_msd_lds_sort (list mode); one above kMsdCap rows goes to k_msd_big as before.
// 12 bits measured best: 10 / 11 / 13 / 14 bits 3.96 / 3.85 / 4.05 / 5.06 ms vs 3.76, and 13 bits again
// with 32-bit rank words 3.71 vs 3.62 (ab_merge_csort.txt)
constexpr int kCsBits = 12, kCsCap = 24;
static_assert(kMsdCap <= 4096 && (kMsdCap & (kMsdCap - 1)) == 0, "row index packs into the low 12 bits");
template <int CB>
__global__ __launch_bounds__(kMsdThreads) void k_msd_csort(const uint32_t *__restrict__ codes, const uint64_t *__restrict__ vin,
                                                           const uint64_t *__restrict__ sb, int lbits, RsDecode dec,
                                                           uint64_t *__restrict__ vout, uint32_t *__restrict__ flag,
                                                           uint32_t *__restrict__ big, uint32_t *__restrict__ fb) {
    constexpr int W = kMsdThreads / 64, J = kMsdCap / kMsdThreads, NB = 1 << CB, BPT = NB / kMsdThreads;
    static_assert(NB >= kMsdCap, "cnt holds the sorted codes at the end");
    __shared__ uint32_t cnt[NB];      // counts, then starts; at the end the codes in sorted order
    __shared__ uint32_t ce[kMsdCap];  // by slot: the code bits below the bucket's << 12 | row; then rows in sorted order
    __shared__ uint32_t wsum[W], wmax[W];
    const int64_t s0 = (int64_t)sb[blockIdx.x], s1 = (int64_t)sb[blockIdx.x + 1];
    const int64_t m = s1 - s0;
    if (m <= 0) return;
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    if (m > kMsdCap) {
        if (t == 0) {
            const uint32_t q = atomicAdd(big, 1u);
            if (q < kMsdMaxBig) big[1 + q] = blockIdx.x;
            else atomicOr(flag, 1u);
        }
        return;
    }
    const int mm = (int)m;
    const uint64_t hi_code = (uint64_t)blockIdx.x << lbits;
    const uint32_t lmask = lbits >= 32 ? 0xFFFFFFFFu : ((1u << lbits) - 1u);
    const int bshift = lbits > CB ? lbits - CB : 0;
    const uint32_t lowm = (1u << bshift) - 1u;  // bshift <= kMsdMaxLow - CB: the rank words fit 32 bits
    static_assert(kMsdMaxLow - CB + 12 <= 32, "rank words: low code bits + 12-bit row");
    for (int i = t; i < NB; i += kMsdThreads) cnt[i] = 0;
    uint32_t c[J], arr[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int e = j * kMsdThreads + t;
        c[j] = e < mm ? codes[s0 + e] & lmask : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int e = j * kMsdThreads + t;
        arr[j] = e < mm ? atomicAdd(&cnt[c[j] >> bshift], 1u) : 0u;
    }
    __syncthreads();
    {  // exclusive scan of the NB counts: thread t owns t * BPT .. + BPT - 1; the largest count on the side
        uint32_t w[BPT], tot = 0, mx = 0;
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            w[q] = cnt[t * BPT + q];
            tot += w[q];
            mx = max(mx, w[q]);
        }
        const uint32_t inc = wave_incl_scan(tot);
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
        if (lane == 63) wsum[wave] = inc;
        if (lane == 0) wmax[wave] = mx;
        __syncthreads();
        uint32_t run = inc - tot;
        for (int v = 0; v < wave; ++v) run += wsum[v];
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            cnt[t * BPT + q] = run;
            run += w[q];
        }
    }
    uint32_t mxall = 0;
#pragma unroll
    for (int v = 0; v < W; ++v) mxall = max(mxall, wmax[v]);
    if (mxall > (uint32_t)kCsCap) {  // (uniform) clustered codes: the radix passes sort this one
        if (t == 0) fb[1 + atomicAdd(&fb[0], 1u)] = blockIdx.x;
        return;
    }
    __syncthreads();
    uint32_t slot[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int e = j * kMsdThreads + t;
        slot[j] = 0;
        if (e < mm) {
            slot[j] = cnt[c[j] >> bshift] + arr[j];
            ce[slot[j]] = ((c[j] & lowm) << 12) | (uint32_t)e;
        }
    }
    __syncthreads();
    uint32_t rank[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int e = j * kMsdThreads + t;
        rank[j] = 0;
        if (e >= mm) continue;
        const uint32_t b = c[j] >> bshift;
        const uint32_t st = cnt[b], en = b + 1 < (uint32_t)NB ? cnt[b + 1] : (uint32_t)mm;
        const uint32_t me = ((c[j] & lowm) << 12) | (uint32_t)e;  // (a bucket shares the bits above)
        uint32_t rk = st;
        for (uint32_t x = st; x < en; ++x) rk += ce[x] < me ? 1u : 0u;
        rank[j] = rk;
    }
    __syncthreads();  // every rank read its bucket: the entries move to their sorted places
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int e = j * kMsdThreads + t;
        if (e < mm) {
            ce[rank[j]] = (uint32_t)e;
            cnt[rank[j]] = c[j];
        }
    }
    __syncthreads();
    // written in sorted order (coalesced), the payload gathered from its row
    for (int p = t; p < mm; p += kMsdThreads) msd_emit(dec, vout, s0 + p, hi_code | cnt[p], vin[s0 + ce[p]]);
}

// The sub-buckets above kMsdCap rows (big[0] of them, ids in big[1..]), every workgroup of the grid on
// each in turn: rows whose codes all equal the first one (the NULLs, one repeated key) are already in
// order and are copied through; any other code sets the redo flag (the LSD passes then rewrite all).
__global__ __launch_bounds__(256) void k_msd_big(const uint32_t *__restrict__ codes, const uint64_t *__restrict__ vin,
                                                 const uint64_t *__restrict__ sb, int lbits, RsDecode dec, uint64_t *__restrict__ vout,
                                                 uint32_t *__restrict__ flag, const uint32_t *__restrict__ big) {
    const uint32_t nbig = big[0] < kMsdMaxBig ? big[0] : kMsdMaxBig;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (uint32_t q = 0; q < nbig; ++q) {
        const uint32_t id = big[1 + q];
        const int64_t s0 = (int64_t)sb[id], s1 = (int64_t)sb[id + 1];
        const uint32_t c0 = codes[s0];
        const uint64_t full = ((uint64_t)id << lbits) | c0;
        bool bad = false;
        for (int64_t i = s0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < s1; i += stride) {
            if (codes[i] != c0) bad = true;
            else msd_emit(dec, vout, i, full, vin[i]);
        }
        if (bad) atomicOr(flag, 1u);
    }
}

// Returns QEH_OK (outputs written, validity bytes in validb) or kMsdRedo (a sub-bucket too large to
// sort in LDS: the caller runs the LSD passes over the same buffers).
constexpr int kMsdRedo = -5;
static int msd_payload_passes(qeh_ctx *ctx, const qeh_column &key, const uint64_t *vsrc, int64_t n, int bits, const RsEncode &enc,
                              const RsDecode &dec, uint64_t *kb0, uint64_t *kb1, uint64_t *vtmp, uint64_t *vout) {
    const bool k32 = key.dtype == QEH_DT_INT32;
    const int cus = ctx->props.multiProcessorCount;
    const int nblocks = (int)std::min<int64_t>(std::max<int64_t>((n + kRsSTile - 1) / kRsSTile, 1), (int64_t)cus);
    const int64_t seg = (n + nblocks - 1) / nblocks;
    const int shift1 = bits - kRadixBits, shift2 = bits - kMsdBits;
    DevBuf hist, offs, nd, vtmp2, tabd, btabd, sbd, flag, fbl;
    QEH_TRY(hist.alloc(ctx, (size_t)kRadix * nblocks * 4));
    QEH_TRY(offs.alloc(ctx, (size_t)kRadix * nblocks * 8));
    QEH_TRY(nd.alloc(ctx, (size_t)n + 16));
    QEH_TRY(vtmp2.alloc(ctx, (size_t)n * 8));
    QEH_TRY(sbd.alloc(ctx, ((size_t)kRadix * kRadix + 1) * 8));
    QEH_TRY(flag.alloc(ctx, 8 + 4 * (kMsdMaxBig + 1)));
    QEH_TRY(fbl.alloc(ctx, 4 * ((size_t)kRadix * kRadix + 1)));
    {
        KernelTimer kt(ctx, "radix_pass");
        if (std::getenv("QEH_RS_HIST_LANE")) {  // (A/B: the lane-strided histogram of the scatter's layout)
            auto hk = k32 ? k_rs_hist<uint64_t, 4> : k_rs_hist<uint64_t, 8>;
            hipLaunchKernelGGL(hk, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, kb0, n, seg, shift1, hist.as<uint32_t>(), nblocks,
                               enc);
        } else {
            auto hk = k32 ? k_rs_hist_enc<4> : k_rs_hist_enc<8>;
            hipLaunchKernelGGL(hk, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, n, seg, shift1, hist.as<uint32_t>(), nblocks, enc);
        }
        QEH_TRY(exclusive_scan_u32(ctx, hist.as<uint32_t>(), offs.as<uint64_t>(), (int64_t)kRadix * nblocks, nullptr));
        // the codes leave as their low 32 bits (the second pass takes its digit from the byte stream nd)
        auto sk = k32 ? k_rs_scatter<uint64_t, true, uint64_t, false, 4, false, uint32_t>
                      : k_rs_scatter<uint64_t, true, uint64_t, false, 8, false, uint32_t>;
        hipLaunchKernelGGL(sk, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, kb0, vsrc, n, seg, shift1, offs.as<uint64_t>(),
                           nblocks, (uint32_t *)kb1, vtmp, nd.as<uint8_t>(), shift2, dec, enc, nullptr);
        QEH_HIP(hipGetLastError());
    }
    // the buckets' starts (the scanned offsets of block 0), then blocks of <= S rows inside each bucket
    std::vector<uint64_t> bst(kRadix + 1);
    QEH_HIP(hipMemcpy2DAsync(bst.data(), 8, offs.p, (size_t)nblocks * 8, 8, kRadix, hipMemcpyDeviceToHost, ctx->stream));
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    bst[kRadix] = (uint64_t)n;
    // ~4 blocks per CU: the buckets differ in size, so many shorter blocks balance the last round
    const int64_t S = std::max<int64_t>(kRsSTile, ((n + 4 * cus - 1) / (4 * cus) + kRsSTile - 1) / kRsSTile * kRsSTile);
    std::vector<int64_t> tab, btab;
    int64_t base = 0;
    for (int b = 0; b < kRadix; ++b) {
        const int64_t lo = (int64_t)bst[b], hi = (int64_t)bst[b + 1], size = hi - lo;
        const int64_t nb = size > 0 ? (size + S - 1) / S : 0;
        for (int64_t j = 0; j < nb; ++j) {
            tab.push_back(lo + j * S);
            tab.push_back(std::min<int64_t>(lo + (j + 1) * S, hi));
            tab.push_back(base * kRadix + j);
            tab.push_back(nb);
        }
        btab.push_back(base);
        btab.push_back(nb);
        btab.push_back(lo);
        base += nb;
    }
    const int64_t B = base;
    QEH_TRY(tabd.alloc(ctx, tab.size() * 8));
    QEH_TRY(btabd.alloc(ctx, btab.size() * 8));
    QEH_HIP(hipMemcpyAsync(tabd.p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    QEH_HIP(hipMemcpyAsync(btabd.p, btab.data(), btab.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    DevBuf hist2, offs2;
    QEH_TRY(hist2.alloc(ctx, (size_t)kRadix * B * 4));
    QEH_TRY(offs2.alloc(ctx, (size_t)kRadix * B * 8));
    {
        KernelTimer kt(ctx, "radix_pass");
        hipLaunchKernelGGL(k_rs_hist_u8_seg, dim3((unsigned)B), dim3(kRsThreads), 0, ctx->stream, nd.as<uint8_t>(), tabd.as<int64_t>(),
                           hist2.as<uint32_t>());
        QEH_TRY(exclusive_scan_u32(ctx, hist2.as<uint32_t>(), offs2.as<uint64_t>(), (int64_t)kRadix * B, nullptr));
        uint32_t *codes2 = (uint32_t *)kb0;  // the low 32 code bits: all the LDS sort needs (lbits <= 29)
        RsEncode enc2{};  // codes = (nd << shift2) | low shift2 bits of the first pass's 32-bit codes
        enc2.nd = nd.as<uint8_t>();
        enc2.nd_shift = shift2;
        hipLaunchKernelGGL((k_rs_scatter<uint64_t, true, uint64_t, false, 1, true, uint32_t>), dim3((unsigned)B), dim3(kRsThreads), 0,
                           ctx->stream, kb1, vtmp, n, 0, shift2, offs2.as<uint64_t>(), (int)B, codes2, vtmp2.as<uint64_t>(), nullptr, 0,
                           dec, enc2, tabd.as<int64_t>());
        hipLaunchKernelGGL(k_msd_sbstart, dim3((kRadix * kRadix + 256) / 256), dim3(256), 0, ctx->stream, offs2.as<uint64_t>(),
                           btabd.as<int64_t>(), n, sbd.as<uint64_t>());
        QEH_HIP(hipMemsetAsync(flag.p, 0, 16, ctx->stream));
        uint32_t *bigl = flag.as<uint32_t>() + 2;
        if (std::getenv("QEH_MSD_RADIX_LDS")) {  // (A/B: the three-pass radix sort for every sub-bucket)
            hipLaunchKernelGGL(k_msd_lds_sort, dim3(kRadix * kRadix), dim3(kMsdThreads), 0, ctx->stream, codes2,
                               vtmp2.as<uint64_t>(), sbd.as<uint64_t>(), shift2, dec, vout, flag.as<uint32_t>(), bigl,
                               (const uint32_t *)nullptr);
        } else {
            // one counting pass per sub-bucket; the ones with a crowded bucket queued for the radix passes
            QEH_HIP(hipMemsetAsync(fbl.p, 0, 4, ctx->stream));
            hipLaunchKernelGGL(k_msd_csort<kCsBits>, dim3(kRadix * kRadix), dim3(kMsdThreads), 0, ctx->stream, codes2, vtmp2.as<uint64_t>(),
                               sbd.as<uint64_t>(), shift2, dec, vout, flag.as<uint32_t>(), bigl, fbl.as<uint32_t>());
            hipLaunchKernelGGL(k_msd_lds_sort, dim3(cus * 4), dim3(kMsdThreads), 0, ctx->stream, codes2,
                               vtmp2.as<uint64_t>(), sbd.as<uint64_t>(), shift2, dec, vout, flag.as<uint32_t>(), bigl,
                               (const uint32_t *)fbl.as<uint32_t>());
        }
        hipLaunchKernelGGL(k_msd_big, dim3(cus * 4), dim3(256), 0, ctx->stream, codes2, vtmp2.as<uint64_t>(), sbd.as<uint64_t>(),
                           shift2, dec, vout, flag.as<uint32_t>(), bigl);
        QEH_HIP(hipGetLastError());
    }
    uint32_t redo = 0;
    QEH_TRY(read_small(ctx, &redo, flag.p, 4));
    return redo ? kMsdRedo : QEH_OK;
}

int qeh::sort_pairs_payload(qeh_ctx *ctx, const qeh_column &key, const qeh_column &val, bool asc, bool nulls_first,
                            qeh_column *out_key, qeh_column *out_val) {
    return sort_pairs_payload_parts(ctx, &key, &val, 1, asc, nulls_first, out_key, out_val);
}

// The key / payload as nparts row segments (Merge::sorted's partitions, concatenated in order): the first
// pass reads them in place (RsEncode.ns); every later pass works on the sort's own buffers.
int qeh::sort_pairs_payload_parts(qeh_ctx *ctx, const qeh_column *keys, const qeh_column *vals, int nparts, bool asc,
                                  bool nulls_first, qeh_column *out_key, qeh_column *out_val) {
    if (nparts < 1 || nparts > kRsMaxSegs) return kPayloadSortNotEligible;
    const qeh_column &key = keys[0], &val = vals[0];
    int64_t n = 0;
    bool nullable = false;
    for (int p = 0; p < nparts; ++p) {
        if (keys[p].dtype != key.dtype || vals[p].dtype != val.dtype || vals[p].length != keys[p].length)
            return kPayloadSortNotEligible;
        if (vals[p].validity && vals[p].null_count != 0) return kPayloadSortNotEligible;
        nullable = nullable || (keys[p].validity && keys[p].null_count != 0);
        n += keys[p].length;
    }
    if (std::getenv("QEH_NO_PAYLOAD_SORT") || n <= 1 || n >= ((int64_t)1 << 32)) return kPayloadSortNotEligible;
    if (key.dtype != QEH_DT_INT64 && key.dtype != QEH_DT_INT32) return kPayloadSortNotEligible;
    if (rs_ballot(ctx)) return kPayloadSortNotEligible;  // its passes rank by LDS atomics only
    if (val.dtype != QEH_DT_INT64 && val.dtype != QEH_DT_FLOAT64) return kPayloadSortNotEligible;
    const ColRef kc = make_colref(key);
    DevBuf st;
    QEH_TRY(st.alloc(ctx, sizeof(KeyStats)));
    KeyStats ks{};
    {
        KernelTimer kt(ctx, "sort_encode");
        hipLaunchKernelGGL(k_stats_init, dim3(1), dim3(1), 0, ctx->stream, st.as<KeyStats>());
        if (nparts == 1) {
            hipLaunchKernelGGL(k_key_stats, dim3(grid_for(ctx, n, kBlock * 8, 1)), dim3(kBlock), 0, ctx->stream, kc, nullptr,
                               n, st.as<KeyStats>());
        } else {  // every partition in one launch
            KeySegs kss{};
            kss.ns = nparts;
            kss.gps = std::max(1, grid_for(ctx, n, kBlock * 8, 1) / nparts);
            for (int p = 0; p < nparts; ++p) kss.c[p] = make_colref(keys[p]), kss.n[p] = keys[p].length;
            hipLaunchKernelGGL(k_key_stats_segs, dim3(nparts * kss.gps), dim3(kBlock), 0, ctx->stream, kss, st.as<KeyStats>());
        }
    }
    QEH_TRY(read_small(ctx, &ks, st.p, sizeof ks));
    const bool any_valid = ks.mn <= ks.mx;
    const int64_t mn = any_valid ? ks.mn : 0, mx = any_valid ? ks.mx : 0;
    const uint64_t range = (uint64_t)mx - (uint64_t)mn;  // value codes 0 .. range (+ bias)
    const uint64_t bias = nullable && nulls_first ? 1 : 0;
    const uint64_t null_code = nullable && nulls_first ? 0 : range + 1;  // (no NULLs: never produced)
    // the largest code: range (+ 1 for the NULL code when nullable); a nullable key spanning the
    // whole Int64 range has no free code left, so it takes the permutation sort
    if (nullable && range == UINT64_MAX) return kPayloadSortNotEligible;
    const uint64_t max_code = range + (nullable ? 1 : 0);
    int bits = 1;
    while (bits < 64 && (max_code >> bits) != 0) ++bits;
    const int npass = (bits + kRadixBits - 1) / kRadixBits;
    // ping-pong buffers; pass 0 reads the payload column itself, the last pass writes the output
    // columns: the payload, and the key decoded from its codes (+ one valid byte per row when nullable)
    QEH_TRY(alloc_column(ctx, val.dtype, n, false, out_val));
    int s = alloc_column(ctx, key.dtype, n, nullable, out_key);
    if (s != QEH_OK) {
        qeh_column_release(ctx, out_val);
        return s;
    }
    DevBuf kb[2], vtmp, hist, offs, validb;
    const int nblocks = (int)std::min<int64_t>(std::max<int64_t>((n + kRsSTile - 1) / kRsSTile, 1), (int64_t)ctx->props.multiProcessorCount);
    const int64_t seg = (n + nblocks - 1) / nblocks;
    if (kb[0].alloc(ctx, n * 8) || kb[1].alloc(ctx, n * 8) || vtmp.alloc(ctx, n * 8) ||
        hist.alloc(ctx, (size_t)kRadix * nblocks * 4) || offs.alloc(ctx, (size_t)kRadix * nblocks * 8) ||
        (nullable && validb.alloc(ctx, n)))
        s = fail(QEH_E_OOM, "payload sort: out of device memory");
    // pass p reads buffer p % 2 (pass 0: the input column) and writes (p + 1) % 2
    const uint64_t *vsrc = (const uint64_t *)((const char *)val.values + (size_t)val.offset * 8);
    uint64_t *vb[2];
    vb[npass % 2] = (uint64_t *)out_val->values;
    vb[(npass + 1) % 2] = vtmp.as<uint64_t>();
    // pass 0 encodes the key column on load (histogram and scatter), the last pass decodes on store
    RsEncode enc{kc, mn, mx, bias, null_code, asc ? 1 : 0};
    auto segs = [&](RsEncode &e) {
        if (nparts == 1) return;
        e.ns = nparts;
        int64_t at = 0;
        for (int p = 0; p < nparts; ++p) {
            e.start[p] = at;
            e.sk[p] = make_colref(keys[p]);
            e.sv[p] = (const uint64_t *)((const char *)vals[p].values + (size_t)vals[p].offset * 8);
            at += keys[p].length;
        }
        e.start[nparts] = at;
    };
    segs(enc);
    const RsDecode dec{mn, mx, bias, null_code, asc ? 1 : 0, key.dtype, out_key->values, nullable ? validb.as<uint8_t>() : nullptr};
    const bool k32 = key.dtype == QEH_DT_INT32;
    // codes of 24..45 bits over many rows: the MSD passes (three passes over the rows); a sub-bucket
    // too large for its LDS sort sends the job on to the LSD passes below.  The NULL code gets a
    // sub-bucket (top 16 bits) of its own: the first one (NULLS FIRST: values biased past it) or the
    // one after the largest value's, so the NULLs are copied through instead of sharing an LDS sort.
    int mbits = 0;
    uint64_t mbias = 0, mnull = 0;
    if (s == QEH_OK && bits >= 24 && n >= ((int64_t)1 << 20) && !std::getenv("QEH_NO_MSD_SORT") &&
        range < (1ull << (kMsdBits + kMsdMaxLow))) {
        for (int bm = std::max(24, bits); bm <= kMsdBits + kMsdMaxLow && !mbits; ++bm) {
            const int s2 = bm - kMsdBits;
            const uint64_t top = range >> s2;  // the largest value's sub-bucket (unbiased)
            if (!nullable) mbits = bm;
            else if (top + 1 < (1ull << kMsdBits)) {
                mbits = bm;
                if (nulls_first) mbias = 1ull << s2, mnull = 0;
                else mnull = (top + 1) << s2;
            }
        }
    }
    bool done = false;
    if (mbits) {
        RsEncode encm{kc, mn, mx, mbias, mnull, asc ? 1 : 0};
        segs(encm);
        const RsDecode decm{mn, mx, mbias, mnull, asc ? 1 : 0, key.dtype, out_key->values, nullable ? validb.as<uint8_t>() : nullptr};
        const int r = msd_payload_passes(ctx, key, vsrc, n, mbits, encm, decm, kb[0].as<uint64_t>(), kb[1].as<uint64_t>(),
                                         vtmp.as<uint64_t>(), (uint64_t *)out_val->values);
        if (r == QEH_OK) done = true;
        else if (r != kMsdRedo) s = r;
    }
    for (int p = 0; p < npass && s == QEH_OK && !done; ++p) {
        KernelTimer kt(ctx, "radix_pass");
        const int c = p & 1, shift = p * kRadixBits;
        const bool first = p == 0, last = p + 1 == npass;
        if (first) {  // the key columns themselves, encoded on load
            auto hk = k32 ? k_rs_hist_enc<4> : k_rs_hist_enc<8>;
            hipLaunchKernelGGL(hk, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, n, seg, shift, hist.as<uint32_t>(), nblocks, enc);
        } else {
            hipLaunchKernelGGL((k_rs_hist<uint64_t, 0>), dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, kb[c].as<uint64_t>(), n, seg,
                               shift, hist.as<uint32_t>(), nblocks, enc);
        }
        s = exclusive_scan_u32(ctx, hist.as<uint32_t>(), offs.as<uint64_t>(), (int64_t)kRadix * nblocks, nullptr);
        if (s != QEH_OK) break;
        const uint64_t *vin = first ? vsrc : vb[c];
        auto sk = first ? (last ? (k32 ? k_rs_scatter<uint64_t, true, uint64_t, true, 4> : k_rs_scatter<uint64_t, true, uint64_t, true, 8>)
                                : (k32 ? k_rs_scatter<uint64_t, true, uint64_t, false, 4> : k_rs_scatter<uint64_t, true, uint64_t, false, 8>))
                        : (last ? k_rs_scatter<uint64_t, true, uint64_t, true, 0> : k_rs_scatter<uint64_t, true, uint64_t, false, 0>);
        hipLaunchKernelGGL(sk, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, kb[c].as<uint64_t>(), vin, n, seg, shift,
                           offs.as<uint64_t>(), nblocks, kb[1 - c].as<uint64_t>(), vb[1 - c], nullptr, 0, dec, enc, nullptr);
        if (hipGetLastError() != hipSuccess) s = fail(QEH_E_HIP, "payload sort: pass launch failed");
    }
    if (s == QEH_OK && nullable) {
        KernelTimer kt(ctx, "sort_encode");
        hipLaunchKernelGGL(k_pack_valid, dim3(grid_for(ctx, (n + 63) / 64, kBlock, 8)), dim3(kBlock), 0, ctx->stream, validb.as<uint8_t>(),
                           n, (uint64_t *)out_key->validity);
        if (hipGetLastError() != hipSuccess) s = fail(QEH_E_HIP, "payload sort: validity launch failed");
    }
    if (s == QEH_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) s = fail(QEH_E_HIP, "payload sort failed");
    if (s != QEH_OK) {
        qeh_column_release(ctx, out_key);
        qeh_column_release(ctx, out_val);
        return s;
    }
    out_key->null_count = nullable ? -1 : 0;
    out_val->null_count = 0;
    return QEH_OK;
}

extern "C" int qeh_sort_indices_nulls(qeh_ctx *ctx, const qeh_column *keys, int n_keys, const int8_t *ascending,
                                      const int8_t *nulls_first, qeh_column *out_perm) {
    if (!ctx || !keys || !out_perm) return fail(QEH_E_INVALID, "qeh_sort_indices_nulls: bad argument");
    DeviceGuard dg(ctx->device);
    int64_t n;
    QEH_TRY(check_sort_keys(keys, n_keys, &n));
    RadixState rs;
    QEH_TRY(sort_perm(ctx, keys, n_keys, ascending, n, rs, nulls_first));
    QEH_TRY(alloc_column(ctx, QEH_DT_UINT32, n, false, out_perm));
    if (n > 0) QEH_HIP(hipMemcpyAsync(out_perm->values, rs.v[rs.cur].p, (size_t)n * 4, hipMemcpyDeviceToDevice, ctx->stream));
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    return QEH_OK;
}

extern "C" int qeh_take(qeh_ctx *ctx, const qeh_column *col, const qeh_column *indices, qeh_column *out) {
    if (!ctx || !col || !indices || !out) return fail(QEH_E_INVALID, "qeh_take: bad argument");
    DeviceGuard dg(ctx->device);
    if (indices->validity) return fail(QEH_E_UNSUPPORTED, "take: nullable indices");
    const int64_t m = indices->length;
    if (indices->dtype == QEH_DT_UINT32) {
        const uint32_t *idx = (const uint32_t *)indices->values + indices->offset;
        QEH_TRY(gather_column(ctx, *col, idx, m, out));
        QEH_HIP(hipStreamSynchronize(ctx->stream));
        return QEH_OK;
    }
    if (indices->dtype != QEH_DT_INT64) return fail(QEH_E_INVALID, "take: indices must be UInt32 or Int64");
    DevBuf idx, bad;
    QEH_TRY(idx.alloc(ctx, (size_t)std::max<int64_t>(m, 1) * 4));
    QEH_TRY(bad.alloc(ctx, 8));
    QEH_HIP(hipMemsetAsync(bad.p, 0, 8, ctx->stream));
    if (m > 0)
        hipLaunchKernelGGL(k_u64_to_u32_idx, dim3(grid_for(ctx, m, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream,
                           (const int64_t *)indices->values + indices->offset, m, col->length, idx.as<uint32_t>(),
                           bad.as<uint32_t>());
    uint32_t b = 0;
    QEH_TRY(read_small(ctx, &b, bad.p, 4));
    if (b) return fail(QEH_E_INVALID, "take: index out of bounds");
    QEH_TRY(gather_column(ctx, *col, idx.as<uint32_t>(), m, out));
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    return QEH_OK;
}

extern "C" int qeh_row_number(qeh_ctx *ctx, const qeh_column *part_keys, int n_part, const qeh_column *order_keys,
                              int n_order, const int8_t *ascending, qeh_column *out_rn) {
    if (!ctx || !out_rn || (n_part + n_order) < 1) return fail(QEH_E_INVALID, "qeh_row_number: bad argument");
    if (n_part > kMaxGroupKeys) return fail(QEH_E_UNSUPPORTED, "at most 4 PARTITION BY keys on the device");
    DeviceGuard dg(ctx->device);
    std::vector<qeh_column> all;
    std::vector<int8_t> asc;
    for (int j = 0; j < n_part; ++j) {
        all.push_back(part_keys[j]);
        asc.push_back(1);
    }
    for (int j = 0; j < n_order; ++j) {
        all.push_back(order_keys[j]);
        asc.push_back(ascending ? ascending[j] : 1);
    }
    int64_t n;
    QEH_TRY(check_sort_keys(all.data(), (int)all.size(), &n));
    if (n_part >= 1 && n_order == 1) {  // bounded integer partition keys: partition instead of sorting
        const int s = window_msd_keys(ctx, QEH_WIN_ROW_NUMBER, part_keys, n_part, order_keys[0], asc[n_part] != 0, 0, nullptr,
                                      nullptr, out_rn);
        if (s != kWindowMsdNotEligible) return s;
    }
    RadixState rs;
    QEH_TRY(sort_perm(ctx, all.data(), (int)all.size(), asc.data(), n, rs));
    QEH_TRY(alloc_column(ctx, QEH_DT_INT64, n, false, out_rn));
    if (n == 0) return QEH_OK;
    const uint32_t *perm = rs.v[rs.cur].as<uint32_t>();
    DevBuf flags, seg;
    int s = flags.alloc(ctx, (size_t)n * 4);
    if (s != QEH_OK) {
        qeh_column_release(ctx, out_rn);
        return s;
    }
    KeyCols pk{};
    pk.n = n_part;
    for (int j = 0; j < n_part; ++j) pk.c[j] = make_colref(part_keys[j]);
    const int grid = grid_for(ctx, n, kBlock * 8, 8);
    {
        KernelTimer kt(ctx, "row_number");
        const int sh = rs.part_shift >= 0 ? rs.part_shift : 0;
        const bool enc_ok = n_part == 1 && (rs.enc_injective || (rs.part_shift >= 0 && n_order == 1));
        if (enc_ok && rs.key32)
            hipLaunchKernelGGL(k_part_flags_enc<uint32_t>, dim3(grid), dim3(kBlock), 0, ctx->stream,
                               rs.k[rs.cur].as<uint32_t>(), n, flags.as<uint32_t>(), sh);
        else if (enc_ok)
            hipLaunchKernelGGL(k_part_flags_enc<uint64_t>, dim3(grid), dim3(kBlock), 0, ctx->stream,
                               rs.k[rs.cur].as<uint64_t>(), n, flags.as<uint32_t>(), sh);
        else
            hipLaunchKernelGGL(k_part_flags, dim3(grid), dim3(kBlock), 0, ctx->stream, pk, perm, n, flags.as<uint32_t>());
    }
    const int64_t nchunks = (n + kRnChunk - 1) / kRnChunk;
    s = seg.alloc(ctx, (size_t)nchunks * 8);
    if (s != QEH_OK) {
        qeh_column_release(ctx, out_rn);
        return s;
    }
    {
        KernelTimer kt(ctx, "row_number");
        hipLaunchKernelGGL(k_rn_chunk_last, dim3(gc_of(ctx, nchunks)), dim3(kBlock), 0, ctx->stream, flags.as<uint32_t>(), n, nchunks,
                           seg.as<int64_t>());
        hipLaunchKernelGGL(k_rn_prefix_max, dim3(1), dim3(1024), 0, ctx->stream, seg.as<int64_t>(), nchunks);
    }
    const int dbits = bit_length((uint64_t)(n - 1));
    // Direct scatter by default.  QEH_RN_WINDOWED (experiment, slower): group the (destination,
    // rn) pairs into 2 MB output windows with two radix passes and scatter window by window with
    // the workgroups of one XCD per window — 138 vs 104 ms for cfg 5 (the passes cost 23 ms and
    // the windowed scatter did not beat the direct one; with one pass and 32 MB windows: 61 vs
    // 40 ms for the row-number stage).
    if (dbits <= 22 || !std::getenv("QEH_RN_WINDOWED")) {
        KernelTimer kt(ctx, "row_number");
        hipLaunchKernelGGL(k_rn_write<false>, dim3(gc_of(ctx, nchunks)), dim3(kBlock), 0, ctx->stream, flags.as<uint32_t>(),
                           seg.as<int64_t>(), perm, n, nchunks, (int64_t *)out_rn->values, nullptr, nullptr);
    } else {
        // (destination, rn) pairs in sorted order into the spare radix buffers, one stable 8-bit
        // pass on the destination's top bits (windows of 2^(dbits-8) rows), windowed scatter
        const int o = 1 - rs.cur;
        {
            KernelTimer kt(ctx, "row_number");
            hipLaunchKernelGGL(k_rn_write<true>, dim3(gc_of(ctx, nchunks)), dim3(kBlock), 0, ctx->stream,
                               flags.as<uint32_t>(), seg.as<int64_t>(), perm, n, nchunks, nullptr, rs.k[o].as<uint32_t>(),
                               rs.v[o].as<uint32_t>());
        }
        rs.cur = o;
        rs.key32 = true;
        // 2 MB output windows (2^18 rows): two stable passes on destination bits [dbits-12, dbits)
        const int wshift = dbits - 12;
        s = radix_pass_at<uint32_t>(ctx, rs, wshift);
        if (s == QEH_OK) s = radix_pass_at<uint32_t>(ctx, rs, wshift + 8);
        DevBuf starts;
        const int64_t nwin = (int64_t)(((uint64_t)(n - 1) >> wshift) + 1);
        if (s == QEH_OK) s = starts.alloc(ctx, (size_t)(nwin + 1) * 8);
        if (s != QEH_OK) {
            qeh_column_release(ctx, out_rn);
            return s;
        }
        KernelTimer kt(ctx, "row_number");
        hipLaunchKernelGGL(k_rn_window_starts, dim3(grid_for(ctx, n + 1, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream,
                           rs.k[rs.cur].as<uint32_t>(), n, wshift, nwin, starts.as<int64_t>());
        const int gx = (int)std::max<int64_t>(8, ctx->props.multiProcessorCount * 4 / 8 * 8);
        hipLaunchKernelGGL(k_rn_scatter_xcd, dim3(gx), dim3(kBlock), 0, ctx->stream, rs.k[rs.cur].as<uint32_t>(),
                           rs.v[rs.cur].as<uint32_t>(), starts.as<int64_t>(), nwin, (int64_t *)out_rn->values);
    }
    QEH_HIP(hipGetLastError());
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    return QEH_OK;
}

// ---- RANK / DENSE_RANK / NTILE / LAG / LEAD / FIRST_VALUE / LAST_VALUE -------------------
// Same sorted order as ROW_NUMBER.  In sorted positions: ps[i] = start of i's partition and
// qs[i] = start of its peer group (last flagged position <= i: the chunked max-scan of the row
// numbers), peer-group counts by an exclusive scan (DENSE_RANK), partition ends stored at their
// start (NTILE / LEAD / LAST_VALUE); one kernel then writes every row's result into input order.

// L[i] = last j <= i with flags[j] (k_rn_write's scan, writing the start instead of i - start + 1)
__global__ __launch_bounds__(kBlock) void k_seg_start(const uint32_t *__restrict__ flags, const int64_t *__restrict__ carry,
                                                      int64_t n, int64_t nchunks, int64_t *__restrict__ L) {
    __shared__ int64_t wmax[kBlock / 64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const int64_t base = c * kRnChunk + (int64_t)t * kRnPer;
        uint32_t f[kRnPer];
        int64_t m = -1;
#pragma unroll
        for (int j = 0; j < kRnPer; ++j) {
            const int64_t i = base + j;
            f[j] = i < n ? flags[i] : 0u;
            if (f[j]) m = i;
        }
        int64_t incl = m;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t o = __shfl_up(incl, d, 64);
            if (lane >= d) incl = o > incl ? o : incl;
        }
        if (lane == 63) wmax[w] = incl;
        __syncthreads();
        int64_t start = carry[c];
        for (int q = 0; q < w; ++q) start = wmax[q] > start ? wmax[q] : start;
        const int64_t prev = __shfl_up(incl, 1, 64);
        if (lane > 0) start = prev > start ? prev : start;
#pragma unroll
        for (int j = 0; j < kRnPer; ++j) {
            const int64_t i = base + j;
            if (f[j]) start = i;
            if (i < n) L[i] = start;
        }
        __syncthreads();
    }
}

__global__ void k_or_flags(uint32_t *__restrict__ a, const uint32_t *__restrict__ b, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        a[i] |= b[i];
}

// pend[ps[i]] = end of i's partition, written by its last row
__global__ void k_part_end(const uint32_t *__restrict__ fp, const int64_t *__restrict__ ps, int64_t n,
                           int64_t *__restrict__ pend) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (i == n - 1 || fp[i + 1]) pend[ps[i]] = i + 1;
}

__global__ void k_win_iota(uint32_t *__restrict__ p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)i;
}

struct WinArgs {
    const uint32_t *perm;
    const int64_t *ps, *qs, *pend;
    const uint64_t *excl;  // exclusive scan of the peer flags
    const uint32_t *fq;    // peer flags
    ColRef arg;
    int64_t param;
    int64_t dflt;
    int has_dflt;
    int esz;               // argument element bytes (value functions)
};

template <int FUNC>
__global__ void k_window_out(WinArgs a, int64_t n, void *__restrict__ out, uint8_t *__restrict__ valid8) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = a.ps[i], row = a.perm[i];
        int64_t v = 0, src = -1;
        uint8_t ok = 1;
        if (FUNC == QEH_WIN_ROW_NUMBER) {
            v = i - s + 1;
        } else if (FUNC == QEH_WIN_RANK) {
            v = a.qs[i] - s + 1;
        } else if (FUNC == QEH_WIN_DENSE_RANK) {
            v = (int64_t)(a.excl[i] + a.fq[i] - a.excl[s]);
        } else if (FUNC == QEH_WIN_NTILE) {
            const int64_t size = a.pend[s] - s, r0 = i - s, q = size / a.param, r = size % a.param;
            v = r0 < r * (q + 1) ? r0 / (q + 1) + 1 : r + (r0 - r * (q + 1)) / q + 1;
        } else if (FUNC == QEH_WIN_LAG) {
            src = a.param <= i - s ? (int64_t)a.perm[i - a.param] : -2;
        } else if (FUNC == QEH_WIN_LEAD) {
            src = a.param < a.pend[s] - i ? (int64_t)a.perm[i + a.param] : -2;  // no i + param overflow
        } else if (FUNC == QEH_WIN_FIRST_VALUE) {
            src = a.perm[s];
        } else {  // LAST_VALUE: the partition's last row (whole-partition frame)
            src = a.perm[a.pend[s] - 1];
        }
        if (FUNC >= QEH_WIN_LAG) {
            if (src == -2) {
                ok = (uint8_t)a.has_dflt;
                v = a.dflt;
            } else {
                ok = col_valid(a.arg, src) ? 1 : 0;
                v = a.esz == 8 ? ((const int64_t *)a.arg.values)[src] : (int64_t)((const uint32_t *)a.arg.values)[src];
            }
            valid8[row] = ok;
            if (a.esz == 8) ((int64_t *)out)[row] = ok ? v : 0;
            else ((uint32_t *)out)[row] = ok ? (uint32_t)v : 0u;
        } else {
            ((int64_t *)out)[row] = v;
        }
    }
}

extern "C" int qeh_window(qeh_ctx *ctx, int32_t func, const qeh_column *part_keys, int n_part, const qeh_column *order_keys,
                          int n_order, const int8_t *ascending, const qeh_column *arg, int64_t param, const int64_t *dflt,
                          qeh_column *out) {
    if (!ctx || !out || n_part < 0 || n_order < 0) return fail(QEH_E_INVALID, "qeh_window: bad argument");
    if (func < QEH_WIN_ROW_NUMBER || func > QEH_WIN_LAST_VALUE) return fail(QEH_E_INVALID, "qeh_window: unknown function");
    if (n_part > kMaxGroupKeys || n_order > kMaxGroupKeys)
        return fail(QEH_E_UNSUPPORTED, "at most 4 PARTITION BY and 4 ORDER BY keys on the device");
    const bool value_fn = func >= QEH_WIN_LAG;
    if (func == QEH_WIN_NTILE && param < 1) return fail(QEH_E_INVALID, "NTILE needs a bucket count >= 1");
    if ((func == QEH_WIN_LAG || func == QEH_WIN_LEAD) && param < 0) return fail(QEH_E_INVALID, "LAG/LEAD offset must be >= 0");
    int esz = 8;
    if (value_fn) {
        if (!arg) return fail(QEH_E_INVALID, "window value function needs an argument column");
        QEH_TRY(check_column(*arg, "window argument"));
        if (arg->dtype == QEH_DT_INT32 || arg->dtype == QEH_DT_FLOAT32) esz = 4;
        else if (arg->dtype != QEH_DT_INT64 && arg->dtype != QEH_DT_FLOAT64)
            return fail(QEH_E_UNSUPPORTED, "window value functions take Int32/Int64/Float32/Float64 on the device");
    }
    DeviceGuard dg(ctx->device);
    std::vector<qeh_column> all;
    std::vector<int8_t> asc;
    for (int j = 0; j < n_part; ++j) all.push_back(part_keys[j]), asc.push_back(1);
    for (int j = 0; j < n_order; ++j) all.push_back(order_keys[j]), asc.push_back(ascending ? ascending[j] : 1);
    int64_t n = arg ? arg->length : 0;  // OVER (): the argument column gives the row count
    if (!all.empty()) {
        QEH_TRY(check_sort_keys(all.data(), (int)all.size(), &n));
        if (value_fn && arg->length != n) return fail(QEH_E_INVALID, "window argument length mismatch");
    } else if (!arg) {
        return fail(QEH_E_INVALID, "qeh_window: OVER () needs a column for the row count");
    }
    if (func == QEH_WIN_ROW_NUMBER && !all.empty())  // the dedicated path (pair-key sort, no peer state)
        return qeh_row_number(ctx, part_keys, n_part, order_keys, n_order, ascending, out);
    if (n_part >= 1 && n_order == 1) {  // bounded integer partition keys: partition instead of sorting
        const int s = window_msd_keys(ctx, func, part_keys, n_part, order_keys[0], asc[n_part] != 0, param, arg, dflt, out);
        if (s != kWindowMsdNotEligible) return s;
    }
    const int odt = value_fn ? arg->dtype : QEH_DT_INT64;
    QEH_TRY(alloc_column(ctx, odt, n, value_fn, out));
    if (n == 0) return QEH_OK;
    auto bail = [&](int s) {
        qeh_column_release(ctx, out);
        return s;
    };
    RadixState rs;
    DevBuf iota;
    const uint32_t *perm;
    if (!all.empty()) {
        int s = sort_perm(ctx, all.data(), (int)all.size(), asc.data(), n, rs);
        if (s != QEH_OK) return bail(s);
        perm = rs.v[rs.cur].as<uint32_t>();
    } else {
        if (iota.alloc(ctx, (size_t)n * 4) != QEH_OK) return bail(QEH_E_OOM);
        hipLaunchKernelGGL(k_win_iota, dim3(grid_for(ctx, n, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream, iota.as<uint32_t>(), n);
        perm = iota.as<uint32_t>();
    }
    const int grid = grid_for(ctx, n, kBlock * 8, 8);
    const int64_t nchunks = (n + kRnChunk - 1) / kRnChunk;
    DevBuf fp, fq, ps, qs, pend, excl, carry, valid8;
    if (fp.alloc(ctx, (size_t)n * 4) != QEH_OK || ps.alloc(ctx, (size_t)n * 8) != QEH_OK ||
        carry.alloc(ctx, (size_t)nchunks * 8) != QEH_OK)
        return bail(QEH_E_OOM);
    KernelTimer kt(ctx, "window");
    KeyCols pk{};
    pk.n = n_part;
    for (int j = 0; j < n_part; ++j) pk.c[j] = make_colref(part_keys[j]);
    // partition flags from the sorted encodings when they determine the partition key (as in
    // qeh_row_number), else by comparing the key columns through the permutation
    const int sh = rs.part_shift >= 0 ? rs.part_shift : 0;
    const bool enc_ok = !all.empty() && n_part == 1 && (rs.enc_injective || (rs.part_shift >= 0 && n_order == 1));
    if (enc_ok && rs.key32)
        hipLaunchKernelGGL(k_part_flags_enc<uint32_t>, dim3(grid), dim3(kBlock), 0, ctx->stream, rs.k[rs.cur].as<uint32_t>(), n,
                           fp.as<uint32_t>(), sh);
    else if (enc_ok)
        hipLaunchKernelGGL(k_part_flags_enc<uint64_t>, dim3(grid), dim3(kBlock), 0, ctx->stream, rs.k[rs.cur].as<uint64_t>(), n,
                           fp.as<uint32_t>(), sh);
    else
        hipLaunchKernelGGL(k_part_flags, dim3(grid), dim3(kBlock), 0, ctx->stream, pk, perm, n, fp.as<uint32_t>());
    auto seg_start = [&](const uint32_t *flags, int64_t *L) {
        hipLaunchKernelGGL(k_rn_chunk_last, dim3(gc_of(ctx, nchunks)), dim3(kBlock), 0, ctx->stream, flags, n, nchunks,
                           carry.as<int64_t>());
        hipLaunchKernelGGL(k_rn_prefix_max, dim3(1), dim3(1024), 0, ctx->stream, carry.as<int64_t>(), nchunks);
        hipLaunchKernelGGL(k_seg_start, dim3(gc_of(ctx, nchunks)), dim3(kBlock), 0, ctx->stream, flags, carry.as<int64_t>(), n,
                           nchunks, L);
    };
    seg_start(fp.as<uint32_t>(), ps.as<int64_t>());
    WinArgs a{};
    a.perm = perm;
    a.ps = ps.as<int64_t>();
    a.param = param;
    a.esz = esz;
    if (func == QEH_WIN_RANK || func == QEH_WIN_DENSE_RANK) {
        // peer flags: partition start or any ORDER BY key changes
        if (fq.alloc(ctx, (size_t)n * 4) != QEH_OK) return bail(QEH_E_OOM);
        KeyCols ok{};
        ok.n = n_order;
        for (int j = 0; j < n_order; ++j) ok.c[j] = make_colref(order_keys[j]);
        if (n_order > 0) {
            hipLaunchKernelGGL(k_part_flags, dim3(grid), dim3(kBlock), 0, ctx->stream, ok, perm, n, fq.as<uint32_t>());
            hipLaunchKernelGGL(k_or_flags, dim3(grid), dim3(kBlock), 0, ctx->stream, fq.as<uint32_t>(), fp.as<uint32_t>(), n);
        } else if (hipMemcpyAsync(fq.p, fp.p, (size_t)n * 4, hipMemcpyDeviceToDevice, ctx->stream) != hipSuccess) {
            return bail(fail(QEH_E_HIP, "qeh_window: device copy failed"));
        }
        a.fq = fq.as<uint32_t>();
        if (func == QEH_WIN_RANK) {
            if (qs.alloc(ctx, (size_t)n * 8) != QEH_OK) return bail(QEH_E_OOM);
            seg_start(fq.as<uint32_t>(), qs.as<int64_t>());
            a.qs = qs.as<int64_t>();
        } else {
            if (excl.alloc(ctx, (size_t)n * 8) != QEH_OK) return bail(QEH_E_OOM);
            int s = exclusive_scan_u32(ctx, fq.as<uint32_t>(), excl.as<uint64_t>(), n, nullptr);
            if (s != QEH_OK) return bail(s);
            a.excl = excl.as<uint64_t>();
        }
    }
    if (func == QEH_WIN_NTILE || func == QEH_WIN_LEAD || func == QEH_WIN_LAST_VALUE) {
        if (pend.alloc(ctx, (size_t)n * 8) != QEH_OK) return bail(QEH_E_OOM);
        hipLaunchKernelGGL(k_part_end, dim3(grid), dim3(kBlock), 0, ctx->stream, fp.as<uint32_t>(), ps.as<int64_t>(), n,
                           pend.as<int64_t>());
        a.pend = pend.as<int64_t>();
    }
    if (value_fn) {
        if (valid8.alloc(ctx, (size_t)n) != QEH_OK) return bail(QEH_E_OOM);
        a.arg = make_colref(*arg);
        a.has_dflt = dflt != nullptr;
        if (dflt) a.dflt = esz == 8 ? *dflt : (int64_t)(uint32_t)*dflt;
    }
#define QEH_WIN(F)                                                                                                        \
    hipLaunchKernelGGL(k_window_out<F>, dim3(grid), dim3(kBlock), 0, ctx->stream, a, n, out->values, valid8.as<uint8_t>())
    switch (func) {
        case QEH_WIN_ROW_NUMBER: QEH_WIN(QEH_WIN_ROW_NUMBER); break;  // OVER (): input order
        case QEH_WIN_RANK: QEH_WIN(QEH_WIN_RANK); break;
        case QEH_WIN_DENSE_RANK: QEH_WIN(QEH_WIN_DENSE_RANK); break;
        case QEH_WIN_NTILE: QEH_WIN(QEH_WIN_NTILE); break;
        case QEH_WIN_LAG: QEH_WIN(QEH_WIN_LAG); break;
        case QEH_WIN_LEAD: QEH_WIN(QEH_WIN_LEAD); break;
        case QEH_WIN_FIRST_VALUE: QEH_WIN(QEH_WIN_FIRST_VALUE); break;
        default: QEH_WIN(QEH_WIN_LAST_VALUE); break;
    }
#undef QEH_WIN
    if (hipGetLastError() != hipSuccess) return bail(fail(QEH_E_HIP, "qeh_window: kernel launch failed"));
    if (value_fn) {
        int s = qeh_bytes_to_validity(ctx, valid8.as<uint8_t>(), n, out->validity);
        if (s != QEH_OK) return bail(s);
        out->null_count = -1;
    }
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return bail(fail(QEH_E_HIP, "qeh_window: stream synchronize failed"));
    return QEH_OK;
}

// Stable partition-major permutation from per-row partition ids written by `ids`.
template <typename IdLaunch>
static int partition_perm(qeh_ctx *ctx, int64_t n, int n_parts, IdLaunch ids, const char *timer, int64_t *counts,
                          qeh_column *out_perm) {
    RadixState rs;
    rs.n = n;
    for (int b = 0; b < 2; ++b) {
        QEH_TRY(rs.k[b].alloc(ctx, (size_t)std::max<int64_t>(n, 1) * 8));
        QEH_TRY(rs.v[b].alloc(ctx, (size_t)std::max<int64_t>(n, 1) * 4));
    }
    std::fill(counts, counts + n_parts, 0);
    if (n > 0) {
        {
            KernelTimer kt(ctx, timer);
            ids(rs.k[0].as<uint64_t>(), rs.v[0].as<uint32_t>());
        }
        QEH_HIP(hipGetLastError());
        QEH_TRY(radix_passes(ctx, rs, n_parts > 1 ? bit_length((uint64_t)n_parts - 1) : 0));
    }
    QEH_TRY(alloc_column(ctx, QEH_DT_UINT32, n, false, out_perm));
    if (n > 0) {
        QEH_HIP(hipMemcpyAsync(out_perm->values, rs.v[rs.cur].p, (size_t)n * 4, hipMemcpyDeviceToDevice, ctx->stream));
        DevBuf cnt;
        int s = cnt.alloc(ctx, (size_t)n_parts * 8);
        if (s == QEH_OK) {
            QEH_HIP(hipMemsetAsync(cnt.p, 0, (size_t)n_parts * 8, ctx->stream));
            hipLaunchKernelGGL(k_count_parts, dim3(grid_for(ctx, n, kBlock * 16, 4)), dim3(kBlock), 0, ctx->stream,
                               rs.k[rs.cur].as<uint64_t>(), n, n_parts, cnt.as<unsigned long long>());
            s = read_small(ctx, counts, cnt.p, (size_t)n_parts * 8);
        }
        if (s != QEH_OK) {
            qeh_column_release(ctx, out_perm);
            return s;
        }
    }
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    return QEH_OK;
}

extern "C" int qeh_hash_partition(qeh_ctx *ctx, const qeh_column *key, int n_parts, int64_t *counts,
                                  qeh_column *out_perm) {
    if (!ctx || !key || !counts || !out_perm || n_parts < 1 || n_parts > kRadix)
        return fail(QEH_E_INVALID, "qeh_hash_partition: bad argument (1..256 partitions)");
    DeviceGuard dg(ctx->device);
    QEH_TRY(check_column(*key, "partition key"));
    if (key->dtype != QEH_DT_INT64 && key->dtype != QEH_DT_INT32)
        return fail(QEH_E_UNSUPPORTED, "partition keys must be Int32/Int64 on the device");
    const int64_t n = key->length;
    const ColRef kc = make_colref(*key);
    return partition_perm(
        ctx, n, n_parts,
        [&](uint64_t *ids, uint32_t *idx) {
            hipLaunchKernelGGL(k_partition_ids, dim3(grid_for(ctx, n, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream, kc,
                               n, (uint32_t)n_parts, ids, idx);
        },
        "hash_partition", counts, out_perm);
}

extern "C" int qeh_range_partition(qeh_ctx *ctx, const qeh_column *key, int ascending, const int64_t *splitters,
                                   int n_splitters, int64_t *counts, qeh_column *out_perm) {
    if (!ctx || !key || !counts || !out_perm || n_splitters < 0 || n_splitters >= kRadix ||
        (n_splitters > 0 && !splitters))
        return fail(QEH_E_INVALID, "qeh_range_partition: bad argument (0..255 splitters)");
    DeviceGuard dg(ctx->device);
    QEH_TRY(check_column(*key, "partition key"));
    if (key->dtype == QEH_DT_UTF8) return fail(QEH_E_UNSUPPORTED, "Utf8 range partition keys are not supported on the device");
    for (int j = 1; j < n_splitters; ++j)
        if (splitters[j] < splitters[j - 1]) return fail(QEH_E_INVALID, "qeh_range_partition: splitters must be ascending");
    const int64_t n = key->length;
    DevBuf sp;
    QEH_TRY(sp.alloc(ctx, (size_t)std::max(n_splitters, 1) * 8));
    if (n_splitters > 0)
        QEH_HIP(hipMemcpyAsync(sp.p, splitters, (size_t)n_splitters * 8, hipMemcpyHostToDevice, ctx->stream));
    QEH_HIP(hipStreamSynchronize(ctx->stream));  // host splitter array may go away
    const ColRef kc = make_colref(*key);
    return partition_perm(
        ctx, n, n_splitters + 1,
        [&](uint64_t *ids, uint32_t *idx) {
            hipLaunchKernelGGL(k_range_ids, dim3(grid_for(ctx, n, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream, kc, n,
                               sp.as<int64_t>(), n_splitters, ascending ? 1 : 0, ids, idx);
        },
        "range_partition", counts, out_perm);
}

extern "C" int qeh_partition_hash(qeh_ctx *ctx, const qeh_column *keys, int n_keys, int n_parts, int64_t *counts,
                                  qeh_column *out_perm) {
    if (!ctx || !keys || n_keys < 1 || n_keys > kMaxCols || !counts || !out_perm || n_parts < 1 || n_parts > kRadix)
        return fail(QEH_E_INVALID, "qeh_partition_hash: bad argument (1..12 keys, 1..256 partitions)");
    DeviceGuard dg(ctx->device);
    HashKeys hk{};
    hk.n = n_keys;
    const int64_t n = keys[0].length;
    for (int j = 0; j < n_keys; ++j) {
        QEH_TRY(check_column(keys[j], "partition key"));
        if (keys[j].length != n) return fail(QEH_E_INVALID, "partition keys have different lengths");
        if (keys[j].dtype != QEH_DT_INT64 && keys[j].dtype != QEH_DT_INT32 && keys[j].dtype != QEH_DT_UTF8)
            return fail(QEH_E_UNSUPPORTED, "hash partition keys must be Int32 / Int64 / Utf8 (compute_row_hash)");
        hk.c[j] = make_colref(keys[j]);
        if (keys[j].dtype == QEH_DT_UTF8) {
            hk.offs[j] = keys[j].offsets + keys[j].offset;
            hk.data[j] = (const uint8_t *)keys[j].values;
        }
    }
    return partition_perm(
        ctx, n, n_parts,
        [&](uint64_t *ids, uint32_t *idx) {
            hipLaunchKernelGGL(k_hash_ids_multi, dim3(grid_for(ctx, n, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream, hk, n,
                               (uint32_t)n_parts, ids, idx);
        },
        "hash_partition", counts, out_perm);
}

static int make_hash_keys(const qeh_column *keys, int n_keys, HashKeys *hk, int64_t *n) {
    hk->n = n_keys;
    *n = keys[0].length;
    for (int j = 0; j < n_keys; ++j) {
        QEH_TRY(check_column(keys[j], "partition key"));
        if (keys[j].length != *n) return fail(QEH_E_INVALID, "partition keys have different lengths");
        if (keys[j].dtype != QEH_DT_INT64 && keys[j].dtype != QEH_DT_INT32 && keys[j].dtype != QEH_DT_UTF8)
            return fail(QEH_E_UNSUPPORTED, "hash partition keys must be Int32 / Int64 / Utf8 (compute_row_hash)");
        hk->c[j] = make_colref(keys[j]);
        if (keys[j].dtype == QEH_DT_UTF8) {
            hk->offs[j] = keys[j].offsets + keys[j].offset;
            hk->data[j] = (const uint8_t *)keys[j].values;
        }
    }
    return QEH_OK;
}

// Exchange's device side in one pass: partition ids, per-segment histograms, then the payload
// columns moved to partition-major order (k_part_scatter).  Columns that are not non-null
// 8-byte go through the permutation + gather path.
// qeh_partition_hash_unmove: out_cols[c][i] = moved[c][position of row i in the stable partition-major
// order of qeh_partition_hash_move over the same key] -- the reverse of an Exchange's move, for results
// computed on the partition-major rows (distributed window functions return them into input order).
extern "C" int qeh_partition_hash_unmove(qeh_ctx *ctx, const qeh_column *key, int n_parts, const qeh_column *moved,
                                         int n_cols, qeh_column *out_cols) {
    if (!ctx || !key || !moved || !out_cols || n_cols < 1 || n_cols > 2 || n_parts < 1 || n_parts > kPsDig)
        return fail(QEH_E_INVALID, "qeh_partition_hash_unmove: bad argument (1..2 columns, 1..16 partitions)");
    DeviceGuard dg(ctx->device);
    const int64_t n = key->length;
    QEH_TRY(check_column(*key, "partition key"));
    if (key->dtype != QEH_DT_INT64 || (key->validity && key->null_count != 0) ||
        (((uintptr_t)key->values + (uintptr_t)key->offset * 8) & 15) != 0)
        return fail(QEH_E_UNSUPPORTED, "qeh_partition_hash_unmove: one non-null, 16-B aligned Int64 key");
    for (int c = 0; c < n_cols; ++c) {
        QEH_TRY(check_column(moved[c], "moved column"));
        if (moved[c].length != n || (moved[c].dtype != QEH_DT_INT64 && moved[c].dtype != QEH_DT_FLOAT64) ||
            (moved[c].validity && moved[c].null_count != 0))
            return fail(QEH_E_UNSUPPORTED, "qeh_partition_hash_unmove: non-null Int64 / Float64 columns of the key's length");
    }
    constexpr int64_t kFusedTile = (int64_t)kRsThreads * kFastR;
    int nblocks = (int)std::min<int64_t>(std::max<int64_t>((n + kFusedTile - 1) / kFusedTile, 1), (int64_t)ctx->props.multiProcessorCount);
    int64_t seg = (n + nblocks - 1) / nblocks;
    seg = std::max<int64_t>((seg + kFusedTile - 1) / kFusedTile * kFusedTile, kFusedTile);
    nblocks = (int)std::max<int64_t>((n + seg - 1) / seg, 1);
    int made = 0, s = QEH_OK;
    for (; made < n_cols; ++made)
        if ((s = alloc_column(ctx, moved[made].dtype, n, false, &out_cols[made])) != QEH_OK) break;
    if (s == QEH_OK && n > 0) {
        DevBuf ids, hist, offs;
        if (ids.alloc(ctx, (size_t)n) || hist.alloc(ctx, (size_t)kPsDig * nblocks * 4) ||
            offs.alloc(ctx, (size_t)kPsDig * nblocks * 8))
            s = fail(QEH_E_OOM, "partition unmove: out of device memory");
        KernelTimer kt(ctx, "partition_move");
        if (s == QEH_OK) {
            FastIn fin{};
            fin.key = (const int64_t *)key->values + key->offset;
            hipLaunchKernelGGL(k_ids_hist_pred<0>, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, fin, PredTerms{}, n, seg,
                               (uint32_t)n_parts, ids.as<uint8_t>(), hist.as<uint32_t>(), nblocks);
            s = exclusive_scan_u32(ctx, hist.as<uint32_t>(), offs.as<uint64_t>(), (int64_t)kPsDig * nblocks, nullptr);
        }
        if (s == QEH_OK) {
            PmCols pc{};
            pc.n = n_cols;
            for (int c = 0; c < n_cols; ++c) {
                pc.src[c] = (const uint64_t *)moved[c].values + moved[c].offset;
                pc.dst[c] = (uint64_t *)out_cols[c].values;
            }
            const bool ballot = rs_ballot(ctx);
            auto kf = n_cols == 1 ? (ballot ? k_part_gather_small<1, false> : k_part_gather_small<1, true>)
                                  : (ballot ? k_part_gather_small<2, false> : k_part_gather_small<2, true>);
            hipLaunchKernelGGL(kf, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, ids.as<uint8_t>(), n, seg,
                               offs.as<uint64_t>(), nblocks, pc);
            if (hipGetLastError() != hipSuccess) s = fail(QEH_E_HIP, "partition unmove launch failed");
        }
        if (s == QEH_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) s = fail(QEH_E_HIP, "partition unmove failed");
    }
    if (s != QEH_OK)
        for (int c = 0; c < made; ++c) qeh_column_release(ctx, &out_cols[c]);
    return s;
}

extern "C" int qeh_partition_hash_move(qeh_ctx *ctx, const qeh_column *keys, int n_keys, int n_parts,
                                       const qeh_column *cols, int n_cols, int64_t *counts, qeh_column *out_cols) {
    if (!ctx || !keys || n_keys < 1 || n_keys > kMaxCols || !counts || n_parts < 1 || n_parts > kRadix || n_cols < 0 ||
        (n_cols > 0 && (!cols || !out_cols)))
        return fail(QEH_E_INVALID, "qeh_partition_hash_move: bad argument (1..12 keys, 1..256 partitions)");
    DeviceGuard dg(ctx->device);
    HashKeys hk{};
    int64_t n;
    QEH_TRY(make_hash_keys(keys, n_keys, &hk, &n));
    for (int c = 0; c < n_cols; ++c) {
        QEH_TRY(check_column(cols[c], "partition column"));
        if (cols[c].length != n) return fail(QEH_E_INVALID, "partition columns and keys have different lengths");
    }
    auto movable = [](const qeh_column &c) {
        return (c.dtype == QEH_DT_INT64 || c.dtype == QEH_DT_FLOAT64) && (!c.validity || c.null_count == 0);
    };
    std::vector<int> mv, other;
    for (int c = 0; c < n_cols; ++c) (movable(cols[c]) ? mv : other).push_back(c);
    std::fill(counts, counts + n_parts, 0);
    std::vector<char> made(n_cols, 0);
    auto cleanup = [&]() {
        for (int c = 0; c < n_cols; ++c)
            if (made[c]) qeh_column_release(ctx, &out_cols[c]);
    };
    // one non-null, 16-B aligned Int64 key into at most kPsDig partitions: ids and per-segment
    // histograms in one pass (k_ids_hist_pred without terms), segments of whole 8192-row tiles
    const qeh_column &k0 = keys[0];
    const bool fused = n_keys == 1 && n_parts <= kPsDig && k0.dtype == QEH_DT_INT64 &&
                       (!k0.validity || k0.null_count == 0) &&
                       (((uintptr_t)k0.values + (uintptr_t)k0.offset * 8) & 15) == 0 && !std::getenv("QEH_PM_GENERIC");
    constexpr int64_t kFusedTile = (int64_t)kRsThreads * kFastR;
    int nblocks = (int)std::min<int64_t>(std::max<int64_t>((n + kPmTile - 1) / kPmTile, 1),
                                         (int64_t)ctx->props.multiProcessorCount);
    int64_t seg = (n + nblocks - 1) / nblocks;
    if (fused) {
        seg = std::max<int64_t>((seg + kFusedTile - 1) / kFusedTile * kFusedTile, kFusedTile);
        nblocks = (int)std::max<int64_t>((n + seg - 1) / seg, 1);
    }
    DevBuf ids, hist, offs;
    QEH_TRY(ids.alloc(ctx, (size_t)std::max<int64_t>(n, 1)));
    QEH_TRY(hist.alloc(ctx, (size_t)kRadix * nblocks * 4));
    QEH_TRY(offs.alloc(ctx, (size_t)kRadix * nblocks * 8));
    const int ndig = fused ? kPsDig : kRadix;  // digits the histogram holds (digit-major)
    std::vector<uint32_t> h((size_t)ndig * nblocks, 0);
    if (n > 0) {
        KernelTimer kt(ctx, "partition_move");
        if (fused) {
            FastIn fin{};
            fin.key = (const int64_t *)k0.values + k0.offset;
            hipLaunchKernelGGL(k_ids_hist_pred<0>, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, fin, PredTerms{}, n,
                               seg, (uint32_t)n_parts, ids.as<uint8_t>(), hist.as<uint32_t>(), nblocks);
        } else {
            if (n_keys == 1 && k0.dtype == QEH_DT_INT64 && (!k0.validity || k0.null_count == 0))
                hipLaunchKernelGGL(k_hash_ids8_i64, dim3(grid_for(ctx, (n + 7) / 8, kBlock, 8)), dim3(kBlock), 0,
                                   ctx->stream, (const int64_t *)k0.values + k0.offset, n, (uint32_t)n_parts,
                                   ids.as<uint8_t>());
            else
                hipLaunchKernelGGL(k_hash_ids8, dim3(grid_for(ctx, n, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream, hk, n,
                                   (uint32_t)n_parts, ids.as<uint8_t>());
            hipLaunchKernelGGL(k_rs_hist_u8, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, ids.as<uint8_t>(), n, seg,
                               hist.as<uint32_t>(), nblocks);  // ids are a byte stream: 16 per load
        }
        QEH_HIP(hipGetLastError());
        QEH_TRY(exclusive_scan_u32(ctx, hist.as<uint32_t>(), offs.as<uint64_t>(), (int64_t)ndig * nblocks, nullptr));
        QEH_TRY(read_small(ctx, h.data(), hist.p, h.size() * 4));
        for (int p = 0; p < n_parts; ++p)
            for (int b = 0; b < nblocks; ++b) counts[p] += h[(size_t)p * nblocks + b];
    }
    int s = QEH_OK;
    for (int c : mv) {
        if ((s = alloc_column(ctx, cols[c].dtype, n, false, &out_cols[c])) != QEH_OK) break;
        made[c] = 1;
    }
    const bool small = n_parts <= kPsDig && !std::getenv("QEH_PM_GENERIC");
    for (size_t g = 0; s == QEH_OK && g < mv.size() && n > 0; g += kPmMaxCols) {
        PmCols pc{};
        const int nc = (int)std::min<size_t>(kPmMaxCols, mv.size() - g);
        pc.n = nc;
        for (int q = 0; q < nc; ++q) {
            const qeh_column &src = cols[mv[g + q]];
            pc.src[q] = (const uint64_t *)src.values + src.offset;
            pc.dst[q] = (uint64_t *)out_cols[mv[g + q]].values;
        }
        KernelTimer kt(ctx, "partition_move");
#define QEH_PM(NCV, AT)                                                                                                       \
    do {                                                                                                               \
        if (small)                                                                                                     \
            hipLaunchKernelGGL((k_part_scatter_small<NCV, AT>), dim3(nblocks), dim3(kRsThreads), 0, ctx->stream,             \
                               ids.as<uint8_t>(), n, seg, offs.as<uint64_t>(), nblocks, pc, (uint32_t)kRadix);         \
        else                                                                                                           \
            hipLaunchKernelGGL((k_part_scatter<NCV, AT>), dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, ids.as<uint8_t>(), \
                               n, seg, offs.as<uint64_t>(), nblocks, pc, (uint32_t)kRadix);                            \
    } while (0)
        const bool ballot = rs_ballot(ctx);
        if (nc == 1) { if (ballot) QEH_PM(1, false); else QEH_PM(1, true); }
        else if (nc == 2) { if (ballot) QEH_PM(2, false); else QEH_PM(2, true); }
        else if (nc == 3) { if (ballot) QEH_PM(3, false); else QEH_PM(3, true); }
        else { if (ballot) QEH_PM(4, false); else QEH_PM(4, true); }
#undef QEH_PM
        if (hipGetLastError() != hipSuccess) s = fail(QEH_E_HIP, "partition move launch failed");
    }
    if (s == QEH_OK && !other.empty()) {  // permutation + gathers for the rest
        int64_t c2[kRadix];
        qeh_column perm{};
        s = qeh_partition_hash(ctx, keys, n_keys, n_parts, c2, &perm);
        for (size_t q = 0; s == QEH_OK && q < other.size(); ++q) {
            s = gather_column(ctx, cols[other[q]], (const uint32_t *)perm.values, n, &out_cols[other[q]]);
            if (s == QEH_OK) made[other[q]] = 1;
        }
        if (perm.owned) {
            (void)hipStreamSynchronize(ctx->stream);
            qeh_column_release(ctx, &perm);
        }
    }
    if (s == QEH_OK) {
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) s = fail(QEH_E_HIP, std::string("partition move: ") + hipGetErrorString(e));
    }
    if (s != QEH_OK) cleanup();
    return s;
}

// Filter + Exchange device side in two passes over the probe columns: partition ids of the
// qualifying rows (k_hash_ids8_pred), per-segment histograms, then the moved columns written
// partition-major with the rejected rows left out (k_part_scatter with a drop id).
extern "C" int qeh_filter_partition_hash_move(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *predicate,
                                              int key_idx, int n_parts, const int32_t *move_idx, int n_move,
                                              int64_t *counts, qeh_column *out_cols) {
    if (!ctx || !cols || n_cols < 1 || n_cols > kMaxCols || !predicate || key_idx < 0 || key_idx >= n_cols || !counts ||
        n_parts < 1 || n_parts >= kRadix || n_move < 1 || n_move > kPmMaxCols || !move_idx || !out_cols)
        return fail(QEH_E_INVALID, "qeh_filter_partition_hash_move: bad argument (1..255 partitions, 1..4 moved columns)");
    DeviceGuard dg(ctx->device);
    const int64_t n = cols[0].length;
    for (int c = 0; c < n_cols; ++c) {
        QEH_TRY(check_column(cols[c], "filter-partition column"));
        if (cols[c].length != n) return fail(QEH_E_INVALID, "filter-partition columns have different lengths");
    }
    const qeh_column &kc = cols[key_idx];
    if (kc.dtype != QEH_DT_INT64 && kc.dtype != QEH_DT_INT32)
        return fail(QEH_E_UNSUPPORTED, "qeh_filter_partition_hash_move: the key must be Int32 / Int64");
    for (int q = 0; q < n_move; ++q) {
        if (move_idx[q] < 0 || move_idx[q] >= n_cols) return fail(QEH_E_INVALID, "moved column index out of range");
        const qeh_column &c = cols[move_idx[q]];
        if ((c.dtype != QEH_DT_INT64 && c.dtype != QEH_DT_FLOAT64) || (c.validity && c.null_count != 0))
            return fail(QEH_E_UNSUPPORTED, "qeh_filter_partition_hash_move: moved columns must be non-null Int64 / Float64");
    }
    std::vector<int32_t> dts(n_cols);
    for (int i = 0; i < n_cols; ++i) dts[i] = cols[i].dtype;
    DevProgram prog;
    QEH_TRY(compile_expr(predicate, dts.data(), n_cols, &prog));
    if (prog.result_type != QEH_DT_BOOL) return fail(QEH_E_TYPE, "Filter predicate must return boolean");
    PredTerms terms{};
    if (!lower_to_terms(predicate, dts.data(), n_cols, &terms))
        return fail(QEH_E_UNSUPPORTED, "qeh_filter_partition_hash_move: predicate is not a list of column-literal comparisons");
    ColSet cs;
    QEH_TRY(make_colset(cols, n_cols, &cs));
    std::fill(counts, counts + n_parts, 0);
    // the fused id + histogram pass: fewer than kPsDig partitions, a non-null Int64 key and term
    // columns that are non-null 8-byte, 16-B aligned (FastTile's loads)
    auto fast_ok = [](const qeh_column &c) {
        return (c.dtype == QEH_DT_INT64 || c.dtype == QEH_DT_FLOAT64) && (!c.validity || c.null_count == 0) &&
               (((uintptr_t)c.values + (uintptr_t)c.offset * 8) & 15) == 0;
    };
    bool fused = n_parts < kPsDig && kc.dtype == QEH_DT_INT64 && fast_ok(kc) && terms.n <= 2 &&
                 !std::getenv("QEH_PM_GENERIC");
    FastIn fin{};
    if (fused) {
        fin.key = (const int64_t *)kc.values + kc.offset;
        for (int i = 0; i < terms.n; ++i) {
            const qeh_column &tc = cols[terms.t[i].col];
            if (!fast_ok(tc)) fused = false;
            fin.term[i] = (const int64_t *)tc.values + tc.offset;
            fin.term_dt[i] = tc.dtype;
        }
    }
    constexpr int64_t kFusedTile = (int64_t)kRsThreads * kFastR;
    int nblocks = (int)std::min<int64_t>(std::max<int64_t>((n + kPmTile - 1) / kPmTile, 1),
                                         (int64_t)ctx->props.multiProcessorCount);
    int64_t seg = (n + nblocks - 1) / nblocks;
    if (fused) {  // segments of whole 8192-row tiles (16-B aligned pairs in every segment)
        seg = std::max<int64_t>((seg + kFusedTile - 1) / kFusedTile * kFusedTile, kFusedTile);
        nblocks = (int)std::max<int64_t>((n + seg - 1) / seg, 1);
    }
    DevBuf ids, hist, offs;
    QEH_TRY(ids.alloc(ctx, (size_t)std::max<int64_t>(n, 1)));
    QEH_TRY(hist.alloc(ctx, (size_t)kRadix * nblocks * 4));
    QEH_TRY(offs.alloc(ctx, (size_t)kRadix * nblocks * 8));
    const int ndig = fused ? kPsDig : kRadix;  // digits the histogram holds (digit-major)
    std::vector<uint32_t> h((size_t)ndig * nblocks, 0);
    int64_t kept = 0;
    if (n > 0) {
        KernelTimer kt(ctx, "partition_move");
        if (fused) {
#define QEH_IH(NT)                                                                                                      \
    hipLaunchKernelGGL(k_ids_hist_pred<NT>, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, fin, terms, n, seg,      \
                       (uint32_t)n_parts, ids.as<uint8_t>(), hist.as<uint32_t>(), nblocks)
            if (terms.n == 0) QEH_IH(0);
            else if (terms.n == 1) QEH_IH(1);
            else QEH_IH(2);
#undef QEH_IH
        } else {
            hipLaunchKernelGGL(k_hash_ids8_pred, dim3(grid_for(ctx, n, kBlock * 4, 8)), dim3(kBlock), 0, ctx->stream,
                               make_colref(kc), cs, terms, n, (uint32_t)n_parts, ids.as<uint8_t>());
            hipLaunchKernelGGL(k_rs_hist_u8, dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, ids.as<uint8_t>(), n, seg,
                               hist.as<uint32_t>(), nblocks);  // ids are a byte stream: 16 per load
        }
        QEH_HIP(hipGetLastError());
        QEH_TRY(exclusive_scan_u32(ctx, hist.as<uint32_t>(), offs.as<uint64_t>(), (int64_t)ndig * nblocks, nullptr));
        QEH_TRY(read_small(ctx, h.data(), hist.p, h.size() * 4));
        for (int p = 0; p < n_parts; ++p)
            for (int b = 0; b < nblocks; ++b) counts[p] += h[(size_t)p * nblocks + b];
        for (int p = 0; p < n_parts; ++p) kept += counts[p];
    }
    int made = 0, s = QEH_OK;
    for (; made < n_move; ++made)
        if ((s = alloc_column(ctx, cols[move_idx[made]].dtype, kept, false, &out_cols[made])) != QEH_OK) break;
    if (s == QEH_OK && kept > 0) {
        PmCols pc{};
        pc.n = n_move;
        for (int q = 0; q < n_move; ++q) {
            const qeh_column &src = cols[move_idx[q]];
            pc.src[q] = (const uint64_t *)src.values + src.offset;
            pc.dst[q] = (uint64_t *)out_cols[q].values;
        }
        KernelTimer kt(ctx, "partition_move");
        const bool small = n_parts < kPsDig && !std::getenv("QEH_PM_GENERIC");  // ids 0..n_parts (the drop id)
#define QEH_FPM(NCV, AT)                                                                                                      \
    do {                                                                                                               \
        if (small)                                                                                                     \
            hipLaunchKernelGGL((k_part_scatter_small<NCV, AT>), dim3(nblocks), dim3(kRsThreads), 0, ctx->stream,             \
                               ids.as<uint8_t>(), n, seg, offs.as<uint64_t>(), nblocks, pc, (uint32_t)n_parts);        \
        else                                                                                                           \
            hipLaunchKernelGGL((k_part_scatter<NCV, AT>), dim3(nblocks), dim3(kRsThreads), 0, ctx->stream, ids.as<uint8_t>(), \
                               n, seg, offs.as<uint64_t>(), nblocks, pc, (uint32_t)n_parts);                           \
    } while (0)
        const bool ballot = rs_ballot(ctx);
        if (n_move == 1) { if (ballot) QEH_FPM(1, false); else QEH_FPM(1, true); }
        else if (n_move == 2) { if (ballot) QEH_FPM(2, false); else QEH_FPM(2, true); }
        else if (n_move == 3) { if (ballot) QEH_FPM(3, false); else QEH_FPM(3, true); }
        else { if (ballot) QEH_FPM(4, false); else QEH_FPM(4, true); }
#undef QEH_FPM
        if (hipGetLastError() != hipSuccess) s = fail(QEH_E_HIP, "filter-partition move launch failed");
    }
    if (s == QEH_OK) {
        const hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) s = fail(QEH_E_HIP, std::string("filter-partition move: ") + hipGetErrorString(e));
    }
    if (s != QEH_OK)
        for (int q = 0; q < made; ++q) qeh_column_release(ctx, &out_cols[q]);
    return s;
}

extern "C" int qeh_partition_range(qeh_ctx *ctx, const qeh_column *key, const int64_t *boundaries, int n_boundaries,
                                   int64_t *counts, qeh_column *out_perm) {
    if (!ctx || !key || !counts || !out_perm || n_boundaries < 0 || n_boundaries >= kRadix ||
        (n_boundaries > 0 && !boundaries))
        return fail(QEH_E_INVALID, "qeh_partition_range: bad argument (0..255 boundaries)");
    DeviceGuard dg(ctx->device);
    QEH_TRY(check_column(*key, "partition key"));
    const int64_t n = key->length;
    DevBuf bd;
    QEH_TRY(bd.alloc(ctx, (size_t)std::max(n_boundaries, 1) * 8));
    if (n_boundaries > 0)
        QEH_HIP(hipMemcpyAsync(bd.p, boundaries, (size_t)n_boundaries * 8, hipMemcpyHostToDevice, ctx->stream));
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    const ColRef kc = make_colref(*key);
    const int is_i64 = key->dtype == QEH_DT_INT64;
    return partition_perm(
        ctx, n, n_boundaries + 1,
        [&](uint64_t *ids, uint32_t *idx) {
            hipLaunchKernelGGL(k_range_ids_first_below, dim3(grid_for(ctx, n, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream,
                               kc, n, bd.as<int64_t>(), n_boundaries, is_i64, ids, idx);
        },
        "range_partition", counts, out_perm);
}

extern "C" int qeh_scatter(qeh_ctx *ctx, const qeh_column *col, const qeh_column *indices, qeh_column *out) {
    if (!ctx || !col || !indices || !out) return fail(QEH_E_INVALID, "qeh_scatter: bad argument");
    DeviceGuard dg(ctx->device);
    QEH_TRY(check_column(*col, "scatter"));
    if (indices->dtype != QEH_DT_UINT32 || indices->validity) return fail(QEH_E_INVALID, "scatter: indices must be non-null UInt32");
    if (indices->length != col->length) return fail(QEH_E_INVALID, "scatter: indices and column lengths differ");
    if (col->validity && col->null_count != 0) return fail(QEH_E_UNSUPPORTED, "scatter: nullable columns");
    int w = 0;
    switch (col->dtype) {
        case QEH_DT_INT64: case QEH_DT_FLOAT64: w = 8; break;
        case QEH_DT_INT32: case QEH_DT_FLOAT32: case QEH_DT_UINT32: w = 4; break;
        default: return fail(QEH_E_UNSUPPORTED, "scatter: fixed-width numeric columns only");
    }
    const int64_t m = col->length;
    QEH_TRY(alloc_column(ctx, col->dtype, m, false, out));
    if (m > 0) {
        KernelTimer kt(ctx, "scatter");
        const uint32_t *idx = (const uint32_t *)indices->values + indices->offset;
        const int grid = grid_for(ctx, m, kBlock * 8, 8);
        if (w == 8)
            hipLaunchKernelGGL(k_scatter<uint64_t>, dim3(grid), dim3(kBlock), 0, ctx->stream,
                               (const uint64_t *)col->values + col->offset, idx, m, (uint64_t *)out->values);
        else
            hipLaunchKernelGGL(k_scatter<uint32_t>, dim3(grid), dim3(kBlock), 0, ctx->stream,
                               (const uint32_t *)col->values + col->offset, idx, m, (uint32_t *)out->values);
    }
    QEH_HIP(hipGetLastError());
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    return QEH_OK;
}
