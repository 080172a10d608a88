// Aggregate state machinery shared by HashAggregateExec and the fused
// join->aggregate pipeline.
//
// Semantics (operators.rs:745-848, evaluate_aggregate):
//   COUNT(x)  -> Int64 non-null count
//   SUM(x)    -> Int64 wrapping sum for Int64; Int32 is summed with i32 wrapping
//                then widened (compute::sum(Int32Array) as i64); Float64 sum;
//                Float32 -> Float64 (we accumulate in f64: documented deviation);
//                NULL when no non-null input
//   AVG(x)    -> Float64 (sum as f64) / count, NULL when count == 0
//   MIN/MAX   -> input type, NULL when no non-null input; floats by totalOrder
// States are 64-bit words: slot 0 = rows in the group; each aggregate owns a
// value slot and (unless its input has no nulls) a non-null-count slot.
#pragma once

#include "device_common.h"

namespace qeh {

enum AggKind : int32_t {
    AK_COUNT = 0,
    AK_SUM_I = 1,   // int64 wrapping add
    AK_SUM_F = 2,   // f64 add
    AK_MIN = 3,     // min over int64 keys (ints as-is, floats as totalOrder keys)
    AK_MAX = 4
};

constexpr int kMaxAggs = 8;

struct AggSpec {
    int32_t kind;      // AggKind
    int32_t func;      // qeh_agg_func (for finalize)
    int32_t col;       // input column index (kernel's ColSet)
    int32_t in_type;   // input dtype
    int32_t val_slot;  // -1 for COUNT
    int32_t cnt_slot;  // 0 = use the group row count (input has no nulls)
};

struct AggSpecs {
    int32_t n;
    int32_t n_slots;   // 1 + value slots + count slots
    int32_t shards;    // copies of the global states (>= 1), see shard_states
    int32_t _pad;
    AggSpec a[kMaxAggs];
};

__host__ __device__ __forceinline__ int64_t agg_init_value(int kind) {
    return kind == AK_MIN ? INT64_MAX : (kind == AK_MAX ? INT64_MIN : 0);
}

// Convert a loaded 64-bit payload (load_i64) into the aggregate's domain.
__device__ __forceinline__ int64_t agg_input(int kind, int in_type, int64_t x) {
    if ((kind == AK_MIN || kind == AK_MAX) && (in_type == 4 || in_type == 5)) return f64_order_key(as_f64(x));
    return x;
}

// Apply one non-null input to state words at `base` (slot s lives at base[s*stride]).
template <bool LDS>
__device__ __forceinline__ void agg_apply(int kind, uint64_t *val, int64_t x) {
    switch (kind) {
        case AK_SUM_I: atomicAdd((unsigned long long *)val, (unsigned long long)x); break;
        case AK_SUM_F:
            if (LDS) atomicAdd((double *)val, as_f64(x));
            else unsafeAtomicAdd((double *)val, as_f64(x));
            break;
        case AK_MIN: atomicMin((long long *)val, (long long)x); break;
        case AK_MAX: atomicMax((long long *)val, (long long)x); break;
        default: break;
    }
}

// Merge a partial state word into a global one.
__device__ __forceinline__ void agg_merge_global(int kind, uint64_t *dst, uint64_t v) {
    switch (kind) {
        case AK_SUM_I: atomicAdd((unsigned long long *)dst, (unsigned long long)v); break;
        case AK_SUM_F: unsafeAtomicAdd((double *)dst, __builtin_bit_cast(double, v)); break;
        case AK_MIN: atomicMin((long long *)dst, (long long)v); break;
        case AK_MAX: atomicMax((long long *)dst, (long long)v); break;
        default: atomicAdd((unsigned long long *)dst, (unsigned long long)v); break;  // counts
    }
}

}  // namespace qeh
