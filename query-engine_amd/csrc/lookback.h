// Decoupled look-back (single-pass order-preserving compaction) shared by the
// Filter and HashJoin kernels.  A tile publishes {flag, count} in one 8-byte
// status word with an agent-scope relaxed atomic store; successors read them
// with agent-scope relaxed atomic loads (L1-bypassing).  The word IS the
// handed-off data (MI355X_MICROARCH.md "R2 granule"), so no fence is needed.
// Tiles are claimed through an atomic ticket, so every predecessor of a tile
// is owned by a workgroup that is already running: the look-back cannot wait
// on an unscheduled workgroup.  Spins are bounded (kErrSpin on timeout).
#pragma once

#include "device_common.h"
#include "expr.h"

namespace qeh {

constexpr uint64_t kFlagAgg = 1ull << 62;    // tile count published
constexpr uint64_t kFlagIncl = 2ull << 62;   // inclusive prefix published
constexpr uint64_t kValMask = (1ull << 62) - 1;
constexpr uint64_t kSpinLimit = 1ull << 26;  // bounded look-back (protocol failure -> error)

__device__ __forceinline__ uint64_t lookback(uint64_t *status, int64_t tile, uint64_t total, uint32_t *err) {
    // one wave walks predecessors 64 at a time
    const int lane = threadIdx.x & 63;
    uint64_t excl = 0;
    int64_t look = tile - 1;
    uint64_t spins = 0;
    while (look >= 0) {
        const int64_t t = look - lane;
        uint64_t s = t >= 0 ? ld_agent(&status[t]) : kFlagIncl;
        // every lane needs a published word; otherwise retry this window
        const uint64_t not_ready = __ballot((s & ~kValMask) == 0);
        if (not_ready) {
            if (++spins > kSpinLimit) {
                if (lane == 0) atomicOr(err, kErrSpin);
                return 0;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        const uint64_t incl = __ballot((s & kFlagIncl) == kFlagIncl);
        // lanes up to (and including) the first inclusive word contribute
        const int first_incl = incl ? __builtin_ctzll(incl) : 64;
        uint64_t v = (lane <= first_incl && t >= 0) ? (s & kValMask) : 0;
        v = wave_sum_u64(v);
        excl += v;
        if (incl) break;
        look -= 64;
    }
    return excl;
}

}  // namespace qeh
