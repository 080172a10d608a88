// Join hash tables in HBM (build side of HashJoinExec).
//
// Three layouts, chosen per build from the build keys' min/max:
//   DIRECT  key range <= 4*n: uint32 (or uint16 when payloads < 65535) array indexed by
//           key-kmin, entry = payload+1
//           (a "perfect hash": one 4-B read per probe, table <= 16 B/build row)
//   PACKED  range < 2^(64-pbits): one uint64 per slot, entry = (key-kmin+1)<<pbits | payload,
//           linear probing, load <= 0.6 -> one 8-B read per probe (same line almost always)
//   WIDE    otherwise: 16-B slots {int64 key, uint64 payload+1 (0 = empty)}, linear probing,
//           load <= 0.6 -> one 16-B read per probe step (key and payload in one sector)
// Payload = build row id (materialising join) or dense group id (fused
// join->aggregate).  Tables are rebuilt per query (they live for one
// HashJoin execution, like the reference's per-query Vec<RecordBatch>).
#pragma once

#include "device_common.h"

namespace qeh {

enum TableKind : int32_t { TK_DIRECT = 0, TK_PACKED = 1, TK_WIDE = 2, TK_BUCKET = 3 };

struct HashTable {
    int32_t kind;
    int32_t pbits;       // PACKED: payload bits
    int32_t unique;      // every build key distinct -> stop at first match
    int32_t _pad;
    uint64_t mask;       // PACKED/WIDE: capacity - 1
    int64_t kmin;        // DIRECT/PACKED key base
    int64_t kmax;
    uint64_t range;      // DIRECT: entries
    uint64_t *slots;     // PACKED entries / WIDE slot pairs (key, payload+1)
    uint32_t *payload;   // DIRECT entries
    uint16_t *payload16; // DIRECT with payloads < 65535: 2-B entries (half the cache footprint)
    uint64_t nbkt;       // BUCKET: buckets (slots = nbkt 64-B lines)
};

// BUCKET (unique keys that neither DIRECT nor PACKED take -- sparse 64-bit keys): 64-B buckets, one cache
// line per probe: S keys (8 B each), then their payload + 1 (pbits 16: S = 6, u16; pbits 32: S = 5, u32),
// and in the last 4 bytes the bucket's insert count (attempts, so a count above S means some key moved
// on to the next bucket).  At 60 % load a table is ~10.7 (16-bit) or 12.8 B per key where WIDE's 16-B
// slots at 30-60 % load take 27-53 B: 1e7 keys fit the Infinity Cache instead of spilling to HBM.
__host__ __device__ __forceinline__ int bucket_slots(int pbits) { return pbits == 16 ? 6 : 5; }
__device__ __forceinline__ uint64_t bucket_home(const HashTable &t, uint64_t key) {
    return __umul64hi(hash64(key), t.nbkt);
}
// the payload (+1) of slot s of a bucket loaded as 8 words
__device__ __forceinline__ uint32_t bucket_payload(const uint64_t (&w)[8], int s, int pbits) {
    return pbits == 16 ? (uint32_t)((w[6 + s / 4] >> (16 * (s % 4))) & 0xFFFFu)
                       : (uint32_t)(w[5 + s / 2] >> (32 * (s % 2)));
}
__device__ __forceinline__ void bucket_load(const HashTable &t, uint64_t b, uint64_t (&w)[8]) {
    typedef unsigned long long v2u64b __attribute__((ext_vector_type(2)));
    const v2u64b *line = (const v2u64b *)(t.slots + b * 8);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const v2u64b x = line[q];
        w[2 * q] = x[0], w[2 * q + 1] = x[1];
    }
}

typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));

// one WIDE slot (key, payload+1) as a single 16-B load
__device__ __forceinline__ v2u64 wide_slot(const HashTable &t, uint64_t h) {
    return ((const v2u64 *)t.slots)[h];
}

// Probe `key`; calls f(payload) for every match (first match only when
// unique).  Returns number of matches.
template <class F>
__device__ __forceinline__ int table_probe(const HashTable &t, int64_t key, F &&f) {
    if (key < t.kmin || key > t.kmax) return 0;
    if (t.kind == TK_DIRECT) {
        const uint64_t i = (uint64_t)key - (uint64_t)t.kmin;
        uint32_t e = t.payload16 ? (uint32_t)t.payload16[i] : t.payload[i];
        if (e == 0) return 0;
        f(e - 1u);
        return 1;
    }
    int found = 0;
    if (t.kind == TK_BUCKET) {
        const int S = bucket_slots(t.pbits);
        uint64_t b = bucket_home(t, (uint64_t)key);
        for (uint64_t step = 0; step < t.nbkt; ++step) {
            uint64_t w[8];
            bucket_load(t, b, w);
            const uint32_t cnt = (uint32_t)(w[7] >> 32);
#pragma unroll
            for (int s = 0; s < 6; ++s)  // (constant register indices into w)
                if (s < S && s < (int)cnt && (int64_t)w[s] == key) {
                    f(bucket_payload(w, s, t.pbits) - 1u);
                    ++found;
                    if (t.unique) return found;
                }
            if (cnt <= (uint32_t)S) break;
            b = b + 1 == t.nbkt ? 0 : b + 1;
        }
        return found;
    }
    uint64_t h = hash64((uint64_t)key) & t.mask;
    if (t.kind == TK_PACKED) {
        const uint64_t want = (uint64_t)key - (uint64_t)t.kmin + 1ull;
        const uint64_t pm = (1ull << t.pbits) - 1ull;
        for (uint64_t i = 0; i <= t.mask; ++i) {
            uint64_t e = t.slots[h];
            if (e == 0) break;
            if ((e >> t.pbits) == want) {
                f((uint32_t)(e & pm));
                ++found;
                if (t.unique) break;
            }
            h = (h + 1) & t.mask;
        }
        return found;
    }
    for (uint64_t i = 0; i <= t.mask; ++i) {
        const v2u64 e = wide_slot(t, h);
        if (e[1] == 0) break;
        if ((int64_t)e[0] == key) {
            f((uint32_t)(e[1] - 1ull));
            ++found;
            if (t.unique) break;
        }
        h = (h + 1) & t.mask;
    }
    return found;
}

}  // namespace qeh
