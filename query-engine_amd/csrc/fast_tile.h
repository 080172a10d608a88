// Fast-path column tiles shared by the fused join-aggregate (k_aggregate.hip) and the fused
// filter + exchange pass (k_sort.hip): non-null 8-byte columns read as 16-B pairs, every load of a
// tile issued before the term predicate is evaluated.
#pragma once
#include "agg.h"
#include "device_common.h"
#include "expr_device.h"

namespace qeh {

constexpr int kFastPairs = 4;
constexpr int kFastR = 2 * kFastPairs;

typedef long long v2i64 __attribute__((ext_vector_type(2)));
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));

struct FastIn {
    const int64_t *key;
    const int64_t *term[2];
    int32_t term_dt[2];
    const int64_t *acol[2];
    int32_t agg_colslot[kMaxAggs];  // which acol an aggregate reads (-1: COUNT of a no-null column)
};

template <bool NT>
__device__ __forceinline__ v2i64 ld2(const int64_t *p) {
    if (NT) return __builtin_nontemporal_load((const v2i64 *)p);
    return *(const v2i64 *)p;
}

// One 2048-row tile of the fast-path columns: every load (16-B pairs) issued
// before the term predicate is evaluated.  Lane rows: base + j*128 + {0,1}.
// P: row pairs per lane (kFastPairs; the two-value-column slice pass uses 2).
template <int NTERMS, int NACOL, bool NT, int P = kFastPairs>
struct FastTile {
    static constexpr int R = 2 * P;
    v2i64 key[P], ac[NACOL > 0 ? NACOL : 1][P];
    v2i64 tc[NTERMS > 0 ? NTERMS : 1][P];
    uint32_t sel;
    __device__ __forceinline__ void load(const FastIn &in, const PredTerms &terms, int64_t base) {
        issue(in, base);
        eval(in, terms);
    }
    // issue every load of the tile (no use of the data: they stay in flight)
    __device__ __forceinline__ void issue(const FastIn &in, int64_t base) {
#pragma unroll
        for (int j = 0; j < P; ++j) key[j] = ld2<NT>(in.key + base + j * 128);
#pragma unroll
        for (int i = 0; i < NTERMS; ++i)
#pragma unroll
            for (int j = 0; j < P; ++j) tc[i][j] = ld2<NT>(in.term[i] + base + j * 128);
#pragma unroll
        for (int c = 0; c < NACOL; ++c)
#pragma unroll
            for (int j = 0; j < P; ++j) ac[c][j] = ld2<NT>(in.acol[c] + base + j * 128);
    }
    // a partial last tile: rows at and past `lim` are not read (8-B loads, zeros in their place);
    // the caller masks them out of `sel` after eval (tail_mask)
    __device__ __forceinline__ void issue_tail(const FastIn &in, int64_t base, int64_t lim) {
        auto ld1 = [&](const int64_t *p, int64_t r) -> int64_t { return r < lim ? p[r] : 0; };
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int64_t r = base + j * 128;
            key[j][0] = ld1(in.key, r), key[j][1] = ld1(in.key, r + 1);
#pragma unroll
            for (int i = 0; i < NTERMS; ++i) tc[i][j][0] = ld1(in.term[i], r), tc[i][j][1] = ld1(in.term[i], r + 1);
#pragma unroll
            for (int c = 0; c < NACOL; ++c) ac[c][j][0] = ld1(in.acol[c], r), ac[c][j][1] = ld1(in.acol[c], r + 1);
        }
    }
    // bit r set when row r of the lane (base + (r >> 1) * 128 + (r & 1)) is below `lim`
    __device__ __forceinline__ static uint32_t tail_mask(int64_t base, int64_t lim) {
        uint32_t m = 0;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (base + (r >> 1) * 128 + (r & 1) < lim) m |= 1u << r;
        return m;
    }
    // evaluate the term predicate into `sel`.  The comparison is branch-free: the (wave-uniform)
    // operator becomes a 3-bit truth table over {a < b, a == b, a > b}, so a row costs two 64-bit
    // compares and two selects instead of a scalar branch tree per row (the switch of cmp_i64 was
    // lowered into ~20 SALU per row inside the tile loop); the Float64 order-key conversion runs only
    // in the uniform branch of a float comparison.
    __device__ __forceinline__ static uint32_t term_bits(const int64_t (&v)[R], int64_t lit, uint32_t tt) {
        const uint32_t t_lt = tt & 1u, t_eq = (tt >> 1) & 1u, t_gt = tt >> 2;
        uint32_t tr = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t b = v[r] < lit ? t_lt : (v[r] > lit ? t_gt : t_eq);
            tr |= b << r;
        }
        return tr;
    }
    __device__ __forceinline__ void eval(const FastIn &in, const PredTerms &terms) {
        sel = (1u << R) - 1u;
#pragma unroll
        for (int i = 0; i < NTERMS; ++i) {
            const PredTerm pt = terms.t[i];
            const uint32_t tt = cmp_truth_table(pt.op);
            int64_t v[R];
#pragma unroll
            for (int r = 0; r < R; ++r) v[r] = tc[i][r >> 1][r & 1];
            if (pt.ctype == QEH_DT_FLOAT64) {  // uniform
                const bool fcol = in.term_dt[i] == QEH_DT_FLOAT64;
#pragma unroll
                for (int r = 0; r < R; ++r) v[r] = f64_order_key(fcol ? as_f64(v[r]) : (double)v[r]);
            }
            const uint32_t tr = term_bits(v, pt.lit, tt);
            if (NTERMS > 1 && terms.is_or) sel = (i == 0) ? tr : (sel | tr);
            else sel &= tr;
        }
    }
    __device__ __forceinline__ int64_t k(int r) const { return key[r >> 1][r & 1]; }
    // value of row r for aggregate input slot `cs` (0 or 1)
    // (a masked blend of the two registers: a select between two elements of ac became a select
    // between two addresses, which spilled ac to scratch every tile)
    __device__ __forceinline__ int64_t a(int cs, int r) const {
        const int64_t v0 = ac[0][r >> 1][r & 1];
        if constexpr (NACOL < 2) return v0;
        const int64_t v1 = ac[NACOL > 1 ? 1 : 0][r >> 1][r & 1];
        return v0 ^ ((v0 ^ v1) & -(int64_t)(cs == 1));
    }
};

}  // namespace qeh
