// Text rendering of cells the way the reference's pgwire result path does
// (crates/query-pgwire/src/result.rs:85-176 -> pgwire 0.28.0 ToSqlText, which
// writes Rust's Display of the value): integers in decimal, booleans "t"/"f",
// floats as Rust's `{}` = the shortest decimal that reads back to the same
// value, written positionally (no exponent: 1e21 -> "1000000000000000000000",
// 1e-7 -> "0.0000001", 1.0 -> "1", -0.0 -> "-0", NaN -> "NaN", inf -> "inf").
//
// Shortest digits: Schubfach (R. Giulietti, "The Schubfach way to render
// doubles", 2020): the rounding interval of v scaled by 10^-k with one
// 126-bit multiplication per bound (round to odd), then the one or two
// candidates of the coarser scale 10^(k+1) and of 10^k are tested for
// membership; ties go to the closer / even candidate.  The power table comes
// from tools/gen_schubfach_table.py.  Every function writes to `out` when it
// is non-null and returns the number of bytes either way (length pass + write
// pass share the code).
#pragma once

#include <cstdint>

#include "fmt_float_table.h"

namespace qeh {

struct FmtDec {
    uint64_t f;  // value = f * 10^e
    int e;
};

__device__ inline int fmt_flog10pow2(int q) { return (int)(((int64_t)q * 661971961083LL) >> 41); }
__device__ inline int fmt_flog10_3q_pow2(int q) { return (int)(((int64_t)q * 661971961083LL - 274743187321LL) >> 41); }
__device__ inline int fmt_flog2pow10(int e) { return (int)(((int64_t)e * 913124641741LL) >> 38); }

__device__ inline uint64_t fmt_mulhi(uint64_t a, uint64_t b) {
    return (uint64_t)(((unsigned __int128)a * (unsigned __int128)b) >> 64);
}

// floor(g * cp / 2^127), rounded to odd (sticky low bits), g = g1 * 2^63 + g0
__device__ inline uint64_t fmt_rop(uint64_t g1, uint64_t g0, uint64_t cp) {
    constexpr uint64_t kMask63 = (1ull << 63) - 1;
    const uint64_t x1 = fmt_mulhi(g0, cp);
    const uint64_t y0 = g1 * cp;
    const uint64_t y1 = fmt_mulhi(g1, cp);
    const uint64_t z = (y0 >> 1) + x1;
    const uint64_t vbp = y1 + (z >> 63);
    return vbp | (((z & kMask63) + kMask63) >> 63);
}

// v = c * 2^q (c_min: the smallest normal significand; q_min: the subnormal exponent)
__device__ inline FmtDec fmt_to_decimal(int q, uint64_t c, uint64_t c_min, int q_min) {
    const uint64_t out = c & 1u;
    const uint64_t cb = c << 2, cbr = cb + 2;
    uint64_t cbl;
    int k;
    if (c != c_min || q == q_min) {
        cbl = cb - 2;
        k = fmt_flog10pow2(q);
    } else {  // the interval below a power of two is half as wide
        cbl = cb - 1;
        k = fmt_flog10_3q_pow2(q);
    }
    const int h = q + fmt_flog2pow10(-k) + 2;
    const uint64_t g1 = kFmtG[2 * (k - kFmtKMin)], g0 = kFmtG[2 * (k - kFmtKMin) + 1];
    const uint64_t vb = fmt_rop(g1, g0, cb << h);
    const uint64_t vbl = fmt_rop(g1, g0, cbl << h);
    const uint64_t vbr = fmt_rop(g1, g0, cbr << h);
    const uint64_t s = vb >> 2;
    // one digit fewer: the multiple of 10 in the interval, if any (the interval is < 10 units
    // wide at this scale, so it is also the candidate with the most trailing zeros; s >= 10
    // rather than Java's s >= 100, which keeps two digits for the tiniest subnormals)
    if (s >= 10) {
        const uint64_t sp10 = 10 * (s / 10), tp10 = sp10 + 10;
        const bool upin = vbl + out <= (sp10 << 2);
        const bool wpin = (tp10 << 2) + out <= vbr;
        if (upin != wpin) return {upin ? sp10 : tp10, k};
    }
    const uint64_t t = s + 1;
    const bool uin = vbl + out <= (s << 2);
    const bool win = (t << 2) + out <= vbr;
    if (uin != win) return {uin ? s : t, k};
    const int64_t cmp = (int64_t)(vb - ((s + t) << 1));
    return {(cmp < 0 || (cmp == 0 && (s & 1u) == 0)) ? s : t, k};
}

__device__ inline int fmt_put(char *out, int n, const char *s) {
    int i = 0;
    for (; s[i]; ++i)
        if (out) out[n + i] = s[i];
    return n + i;
}

__device__ const uint64_t kFmtPow10[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull, 10000000ull,
                                          100000000ull, 1000000000ull, 10000000000ull, 100000000000ull,
                                          1000000000000ull, 10000000000000ull, 100000000000000ull,
                                          1000000000000000ull, 10000000000000000ull, 100000000000000000ull,
                                          1000000000000000000ull, 10000000000000000000ull};

// number of decimal digits: log10 from the bit length (1233 / 4096 ~ log10 2), one table compare
__device__ inline int fmt_u64_digits(uint64_t v) {
    const int bl = 64 - __builtin_clzll(v | 1);
    const int t = (bl * 1233) >> 12;
    return t + 1 - (v < kFmtPow10[t] && t > 0 ? 1 : 0);  // (v = 0: one digit)
}

// decimal digits of v at out[n .. n + digits), from the back: 8-digit pieces split off with one 64-bit
// division each, their digits in 32-bit arithmetic
__device__ inline int fmt_u64(char *out, int n, uint64_t v) {
    const int d = fmt_u64_digits(v);
    if (out) {
        int i = d;
        while (v >= 100000000ull) {
            const uint64_t q = v / 100000000ull;
            uint32_t r = (uint32_t)(v - q * 100000000ull);
            for (int j = 0; j < 8; ++j) {
                out[n + --i] = (char)('0' + r % 10u);
                r /= 10u;
            }
            v = q;
        }
        uint32_t r = (uint32_t)v;
        while (i > 0) {
            out[n + --i] = (char)('0' + r % 10u);
            r /= 10u;
        }
    }
    return n + d;
}

__device__ inline int fmt_i64(char *out, int64_t v) {
    int n = 0;
    uint64_t u = (uint64_t)v;
    if (v < 0) {
        if (out) out[0] = '-';
        n = 1;
        u = 0 - u;
    }
    return fmt_u64(out, n, u);
}

// f * 10^e positionally, trailing zeros of f removed first (Rust Display)
__device__ inline int fmt_positional(char *out, int n, FmtDec d) {
    while (d.f >= 10 && d.f % 10 == 0) {
        d.f /= 10;
        ++d.e;
    }
    const int nd = fmt_u64_digits(d.f);
    const int pt = d.e + nd;  // digits before the decimal point
    if (pt <= 0) {
        n = fmt_put(out, n, "0.");
        for (int i = 0; i < -pt; ++i)
            if (out) out[n + i] = '0';
        n += -pt;
        return fmt_u64(out, n, d.f);
    }
    if (pt >= nd) {
        n = fmt_u64(out, n, d.f);
        for (int i = 0; i < pt - nd; ++i)
            if (out) out[n + i] = '0';
        return n + (pt - nd);
    }
    // digits[0, pt) "." digits[pt, nd): all digits, then the fraction moved one place right
    if (out) {
        fmt_u64(out, n, d.f);
        for (int i = nd - 1; i >= pt; --i) out[n + i + 1] = out[n + i];
        out[n + pt] = '.';
    }
    return n + nd + 1;
}

__device__ inline int fmt_f64(char *out, double v) {
    uint64_t bits;
    __builtin_memcpy(&bits, &v, 8);
    const uint64_t t = bits & ((1ull << 52) - 1);
    const int bq = (int)((bits >> 52) & 0x7FF);
    if (bq == 0x7FF) return fmt_put(out, 0, t ? "NaN" : ((bits >> 63) ? "-inf" : "inf"));
    int n = 0;
    if (bits >> 63) n = fmt_put(out, 0, "-");
    if (bq == 0 && t == 0) return fmt_put(out, n, "0");
    constexpr uint64_t kCMin = 1ull << 52;
    constexpr int kQMin = -1074;
    FmtDec d;
    if (bq != 0) {
        const int mq = -kQMin + 1 - bq;
        const uint64_t c = kCMin | t;
        if (0 < mq && mq < 53 && ((c >> mq) << mq) == c) d = {c >> mq, 0};  // an integer below 2^53
        else d = fmt_to_decimal(-mq, c, kCMin, kQMin);
    } else {
        d = fmt_to_decimal(kQMin, t, kCMin, kQMin);
    }
    return fmt_positional(out, n, d);
}

__device__ inline int fmt_f32(char *out, float v) {
    uint32_t bits;
    __builtin_memcpy(&bits, &v, 4);
    const uint64_t t = bits & ((1u << 23) - 1);
    const int bq = (int)((bits >> 23) & 0xFF);
    if (bq == 0xFF) return fmt_put(out, 0, t ? "NaN" : ((bits >> 31) ? "-inf" : "inf"));
    int n = 0;
    if (bits >> 31) n = fmt_put(out, 0, "-");
    if (bq == 0 && t == 0) return fmt_put(out, n, "0");
    constexpr uint64_t kCMin = 1ull << 23;
    constexpr int kQMin = -149;
    FmtDec d;
    if (bq != 0) {
        const int mq = -kQMin + 1 - bq;
        const uint64_t c = kCMin | t;
        if (0 < mq && mq < 24 && ((c >> mq) << mq) == c) d = {c >> mq, 0};
        else d = fmt_to_decimal(-mq, c, kCMin, kQMin);
    } else {
        d = fmt_to_decimal(kQMin, t, kCMin, kQMin);
    }
    return fmt_positional(out, n, d);
}

}  // namespace qeh
