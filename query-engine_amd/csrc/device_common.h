// Device-side helpers shared by every qeh kernel (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qeh {

constexpr int kWave = 64;           // CDNA wavefront width
constexpr int kMaxCols = 12;        // columns visible to one kernel
constexpr int kBlock = 256;         // threads per workgroup for streaming kernels

// A column as a kernel sees it: base pointers already advanced by the Arrow
// element offset for values; validity keeps the bit offset separately.
struct ColRef {
    const void *values;
    const uint8_t *validity;  // nullptr = all valid
    int64_t vbit0;            // bit index of row 0 inside `validity`
    int32_t dtype;            // enum qeh_dtype
    int32_t _pad;
};

struct ColSet {
    ColRef c[kMaxCols];
    int32_t n;
};

__device__ __forceinline__ bool bit_at(const uint8_t *bm, int64_t bit) {
    return (bm[bit >> 3] >> (bit & 7)) & 1;
}

__device__ __forceinline__ bool col_valid(const ColRef &c, int64_t row) {
    return c.validity == nullptr || bit_at(c.validity, c.vbit0 + row);
}

// murmur3 fmix64 finaliser: the partition / table hash (the reference's
// SipHash choice is not observable).
__host__ __device__ __forceinline__ uint64_t hash64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

// IEEE-754 totalOrder as a signed-int order (arrow-rs compares floats with
// total_cmp: NaN largest, -0.0 < +0.0).
__host__ __device__ __forceinline__ int64_t f64_order_key(double d) {
    int64_t b = __builtin_bit_cast(int64_t, d);
    return b ^ (int64_t)(((uint64_t)(b >> 63)) >> 1);
}
__host__ __device__ __forceinline__ double f64_from_order_key(int64_t k) {
    int64_t b = k ^ (int64_t)(((uint64_t)(k >> 63)) >> 1);
    return __builtin_bit_cast(double, b);
}

// Read one element of a numeric column as 64-bit payload (ints sign-extended,
// float32 widened exactly to double bits).
__device__ __forceinline__ int64_t load_i64(const ColRef &c, int64_t row) {
    switch (c.dtype) {
        case 2: return (int64_t)((const int32_t *)c.values)[row];          // INT32
        case 7: return (int64_t)((const uint32_t *)c.values)[row];         // UINT32
        case 3: return ((const int64_t *)c.values)[row];                   // INT64
        case 4: return __builtin_bit_cast(int64_t, (double)((const float *)c.values)[row]);
        case 5: return ((const int64_t *)c.values)[row];                   // FLOAT64 bits
        case 1: return (int64_t)bit_at((const uint8_t *)c.values, c.vbit0 + row);  // BOOL (vbit0 reused)
        default: return 0;
    }
}

__device__ __forceinline__ double as_f64(int64_t bits) { return __builtin_bit_cast(double, bits); }
__device__ __forceinline__ int64_t f64_bits(double d) { return __builtin_bit_cast(int64_t, d); }

// wave helpers -----------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ unsigned popc64(uint64_t m) { return __popcll(m); }

// lanes below me in `mask`
__device__ __forceinline__ unsigned mbcnt(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// inclusive wave scan (add) of a 32-bit value
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (l >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// relaxed agent-scope atomics for cross-workgroup status words (L1-bypassing).
__device__ __forceinline__ uint64_t ld_agent(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace qeh
