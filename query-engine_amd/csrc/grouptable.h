// Group tables keyed by tuples of up to four columns (HashAggregate keys, and
// the build-side group keys of the fused join->aggregate pipeline).
#pragma once

#include "device_common.h"

namespace qeh {

constexpr int kMaxGroupKeys = 4;
constexpr uint32_t kGroupEmpty = 0xFFFFFFFFu;

struct KeyCols {
    ColRef c[kMaxGroupKeys];
    int32_t n;
};

// Hash of a key tuple; NULLs hash to a fixed marker (all NULLs of one key
// column form one group).
__device__ __forceinline__ uint64_t tuple_hash(const KeyCols &k, int64_t row) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < k.n; ++i) {
        bool v = col_valid(k.c[i], row);
        uint64_t x = v ? (uint64_t)load_i64(k.c[i], row) : 0x6E756C6Cull;
        h = hash64(h ^ (x + (v ? 0ull : 0x1234567ull) + (uint64_t)i * 0x632BE59BD9B4E019ull));
    }
    return h;
}

__device__ __forceinline__ bool tuple_eq(const KeyCols &k, int64_t a, int64_t b) {
    for (int i = 0; i < k.n; ++i) {
        bool va = col_valid(k.c[i], a), vb = col_valid(k.c[i], b);
        if (va != vb) return false;
        if (va && load_i64(k.c[i], a) != load_i64(k.c[i], b)) return false;
    }
    return true;
}

// Read-only lookup of a row's group slot in a finished table.
__device__ __forceinline__ uint64_t group_find(const KeyCols &k, int64_t row, const uint32_t *slots, uint64_t mask) {
    uint64_t h = tuple_hash(k, row) & mask;
    for (uint64_t p = 0; p <= mask; ++p) {
        uint32_t r = slots[h];
        if (r == kGroupEmpty || tuple_eq(k, r, row)) return h;
        h = (h + 1) & mask;
    }
    return h;
}

}  // namespace qeh
