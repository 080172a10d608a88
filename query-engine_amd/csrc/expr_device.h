// Device interpreter for DevProgram / PredTerms (expr.h).
// Every lane evaluates R consecutive rows; the instruction stream is read
// from kernel arguments (scalar loads), so every branch on the opcode is
// wave-uniform and the per-row work is plain VALU.
#pragma once

#include "device_common.h"
#include "expr.h"

namespace qeh {

__device__ __forceinline__ bool add_ovf64(int64_t a, int64_t b, int64_t *r) { return __builtin_add_overflow(a, b, r); }
__device__ __forceinline__ bool sub_ovf64(int64_t a, int64_t b, int64_t *r) { return __builtin_sub_overflow(a, b, r); }
__device__ __forceinline__ bool mul_ovf64(int64_t a, int64_t b, int64_t *r) { return __builtin_mul_overflow(a, b, r); }

template <int R>
struct ExprRegs {
    int64_t v[kNS][R];
    uint32_t valid[kNS];  // bit r = row r valid
};

// Evaluate compare on int64 payloads (ints, bools or totalOrder keys).
// op (D_EQ..D_GE) as a truth table over the three outcomes: bit 0 = result when a < b, bit 1 when
// a == b, bit 2 when a > b
__host__ __device__ __forceinline__ uint32_t cmp_truth_table(int op) {
    switch (op) {
        case D_EQ: return 2u;
        case D_NE: return 5u;
        case D_LT: return 1u;
        case D_LE: return 3u;
        case D_GT: return 4u;
        case D_GE: return 6u;
        default: return 0u;  // (not a comparison: plan_predicate admits only compare ops to the fast tiles)
    }
}

__device__ __forceinline__ bool cmp_i64(int op, int64_t a, int64_t b) {
    switch (op) {
        case D_EQ: return a == b;
        case D_NE: return a != b;
        case D_LT: return a < b;
        case D_LE: return a <= b;
        case D_GT: return a > b;
        case D_GE: return a >= b;
        default: return false;  // (not a comparison: the host admits only compare ops here)
    }
}

// Slot accessors with a wave-uniform slot index: the switch compiles to
// scalar branches and every arm uses constant register indices.
template <int S, int R>
__device__ __forceinline__ void get_s(const ExprRegs<R> &X, int64_t (&out)[R], uint32_t &valid) {
#pragma unroll
    for (int r = 0; r < R; ++r) out[r] = X.v[S][r];
    valid = X.valid[S];
}
template <int S, int R>
__device__ __forceinline__ void put_s(ExprRegs<R> &X, const int64_t (&in)[R], uint32_t valid) {
#pragma unroll
    for (int r = 0; r < R; ++r) X.v[S][r] = in[r];
    X.valid[S] = valid;
}

template <int R>
__device__ __forceinline__ void get_slot(const ExprRegs<R> &X, int s, int64_t (&out)[R], uint32_t &valid) {
    switch (s) {
        case 0: get_s<0>(X, out, valid); break;
        case 1: get_s<1>(X, out, valid); break;
        case 2: get_s<2>(X, out, valid); break;
        case 3: get_s<3>(X, out, valid); break;
        case 4: get_s<4>(X, out, valid); break;
        case 5: get_s<5>(X, out, valid); break;
        case 6: get_s<6>(X, out, valid); break;
        default: get_s<7>(X, out, valid); break;
    }
}

template <int R>
__device__ __forceinline__ void put_slot(ExprRegs<R> &X, int s, const int64_t (&in)[R], uint32_t valid) {
    switch (s) {
        case 0: put_s<0>(X, in, valid); break;
        case 1: put_s<1>(X, in, valid); break;
        case 2: put_s<2>(X, in, valid); break;
        case 3: put_s<3>(X, in, valid); break;
        case 4: put_s<4>(X, in, valid); break;
        case 5: put_s<5>(X, in, valid); break;
        case 6: put_s<6>(X, in, valid); break;
        default: put_s<7>(X, in, valid); break;
    }
}

// Load rows row0 + r*stride (r < R) of column c; rows >= n are invalid.
// With stride = 64 and row0 = base + lane every load instruction of a wave
// reads one contiguous 64-element run (fully coalesced).
// The dtype switch sits outside the row loop: each arm issues its R loads back to back (a switch
// per row made the compiler wait for every load before the next).
template <int R, typename T>
__device__ __forceinline__ void load_rows_t(const void *p, int64_t row0, int64_t stride, int64_t n, T (&raw)[R]) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t row = row0 + r * stride;
        raw[r] = row < n ? ((const T *)p)[row] : T(0);
    }
}

template <int R>
__device__ __forceinline__ void load_rows(const ColRef &c, int64_t row0, int64_t stride, int64_t n,
                                          int64_t (&out)[R], uint32_t &valid) {
    switch (c.dtype) {
        case 3:    // INT64
        case 5: {  // FLOAT64 bits
            load_rows_t<R, int64_t>(c.values, row0, stride, n, out);
            break;
        }
        case 2: {  // INT32
            int32_t t[R];
            load_rows_t<R, int32_t>(c.values, row0, stride, n, t);
#pragma unroll
            for (int r = 0; r < R; ++r) out[r] = (int64_t)t[r];
            break;
        }
        case 7: {  // UINT32
            uint32_t t[R];
            load_rows_t<R, uint32_t>(c.values, row0, stride, n, t);
#pragma unroll
            for (int r = 0; r < R; ++r) out[r] = (int64_t)t[r];
            break;
        }
        case 4: {  // FLOAT32, widened exactly
            float t[R];
            load_rows_t<R, float>(c.values, row0, stride, n, t);
#pragma unroll
            for (int r = 0; r < R; ++r) out[r] = __builtin_bit_cast(int64_t, (double)t[r]);
            break;
        }
        default: {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int64_t row = row0 + r * stride;
                out[r] = row < n ? load_i64(c, row) : 0;
            }
        }
    }
    valid = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t row = row0 + r * stride;
        if (row < n && col_valid(c, row)) valid |= 1u << r;
    }
}

// Run a full program over R rows; result in slot 0.  `err` collects kErr* bits.
template <int R>
__device__ void run_program(const DevProgram &P, const ColSet &cols, int64_t row0, int64_t stride,
                            int64_t n, ExprRegs<R> &X, uint32_t &err) {
    for (int pc = 0; pc < P.n; ++pc) {
        const DevInstr in = P.ins[pc];
        int64_t a[R], b[R], o[R];
        uint32_t va = 0, vb = 0, vo = 0;
        switch (in.op) {
            case D_LOAD:
                load_rows<R>(cols.c[in.a], row0, stride, n, o, vo);
                break;
            case D_LIT:
#pragma unroll
                for (int r = 0; r < R; ++r) o[r] = in.imm;
                vo = in.flag ? 0u : ((1u << R) - 1u);
                break;
            case D_TOF64:
                get_slot<R>(X, in.a, a, va);
#pragma unroll
                for (int r = 0; r < R; ++r) o[r] = f64_bits((double)a[r]);
                vo = va;
                break;
            case D_NOT:
                get_slot<R>(X, in.a, a, va);
#pragma unroll
                for (int r = 0; r < R; ++r) o[r] = a[r] ^ 1;
                vo = va;
                break;
            case D_NEG:
                get_slot<R>(X, in.a, a, va);
                if (in.t == QEH_DT_FLOAT64 || in.t == QEH_DT_FLOAT32) {
#pragma unroll
                    for (int r = 0; r < R; ++r) o[r] = f64_bits(-as_f64(a[r]));
                } else if (in.t == QEH_DT_INT32) {
#pragma unroll
                    for (int r = 0; r < R; ++r) o[r] = (int64_t)(int32_t)(0u - (uint32_t)a[r]);
                } else {
#pragma unroll
                    for (int r = 0; r < R; ++r) o[r] = (int64_t)(0ull - (uint64_t)a[r]);
                }
                vo = va;
                break;
            default: {
                get_slot<R>(X, in.a, a, va);
                get_slot<R>(X, in.b, b, vb);
                vo = va & vb;
                const int t = in.t;
                if (in.op >= D_EQ && in.op <= D_GE) {
                    if (t == QEH_DT_FLOAT64) {
#pragma unroll
                        for (int r = 0; r < R; ++r)
                            o[r] = cmp_i64(in.op, f64_order_key(as_f64(a[r])), f64_order_key(as_f64(b[r])));
                    } else {
#pragma unroll
                        for (int r = 0; r < R; ++r) o[r] = cmp_i64(in.op, a[r], b[r]);
                    }
                } else if (in.op == D_AND) {
#pragma unroll
                    for (int r = 0; r < R; ++r) o[r] = a[r] & b[r];
                } else if (in.op == D_OR) {
#pragma unroll
                    for (int r = 0; r < R; ++r) o[r] = a[r] | b[r];
                } else if (t == QEH_DT_FLOAT64 || t == QEH_DT_FLOAT32) {
                    const bool f32 = t == QEH_DT_FLOAT32;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        double x = as_f64(a[r]), y = as_f64(b[r]), z;
                        if (f32) {
                            float xf = (float)x, yf = (float)y, zf;
                            switch (in.op) {
                                case D_ADD: zf = xf + yf; break;
                                case D_SUB: zf = xf - yf; break;
                                case D_MUL: zf = xf * yf; break;
                                default: zf = xf / yf; break;
                            }
                            z = (double)zf;
                        } else {
                            switch (in.op) {
                                case D_ADD: z = x + y; break;
                                case D_SUB: z = x - y; break;
                                case D_MUL: z = x * y; break;
                                default: z = x / y; break;
                            }
                        }
                        o[r] = f64_bits(z);
                    }
                } else {
                    // checked integer arithmetic; errors only on valid rows (arrow try_binary)
                    const bool i32 = t == QEH_DT_INT32;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const bool live = (vo >> r) & 1;
                        int64_t x = a[r], y = b[r], z = 0;
                        bool ov = false;
                        switch (in.op) {
                            case D_ADD: ov = add_ovf64(x, y, &z); break;
                            case D_SUB: ov = sub_ovf64(x, y, &z); break;
                            case D_MUL: ov = mul_ovf64(x, y, &z); break;
                            case D_DIV:
                                if (y == 0) { if (live) err |= kErrDiv0; z = 0; }
                                else if (y == -1 && x == (i32 ? (int64_t)INT32_MIN : INT64_MIN)) { ov = true; z = 0; }
                                else z = x / y;
                                break;
                            default:  // D_MOD: r == 0 -> NULL (operators.rs:711-743)
                                if (y == 0) { vo &= ~(1u << r); z = 0; }
                                else if (y == -1 && x == (i32 ? (int64_t)INT32_MIN : INT64_MIN)) {
                                    if (live) err |= kErrModOverflow;
                                    z = 0;
                                } else z = x % y;
                                break;
                        }
                        if (i32 && (z < INT32_MIN || z > INT32_MAX)) ov = true;
                        if (ov && live) err |= kErrOverflow;
                        o[r] = z;
                    }
                }
                break;
            }
        }
        put_slot<R>(X, in.dst, o, vo);
    }
}

// Fast predicate: returns the R-bit mask of rows whose predicate is TRUE.
template <int R>
__device__ __forceinline__ uint32_t eval_terms(const PredTerms &T, const ColSet &cols, int64_t row0,
                                               int64_t stride, int64_t n) {
    uint32_t live = 0;
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (row0 + r * stride < n) live |= 1u << r;
    if (T.n == 0) return live;
    uint32_t all_valid = live, any_true = 0, all_true = live;
    for (int i = 0; i < T.n; ++i) {
        const PredTerm t = T.t[i];
        const ColRef c = cols.c[t.col];
        int64_t v[R];
        uint32_t vv;
        load_rows<R>(c, row0, stride, n, v, vv);
        uint32_t tr = 0;
        if (t.ctype == QEH_DT_FLOAT64) {
            const bool isf = c.dtype == QEH_DT_FLOAT64 || c.dtype == QEH_DT_FLOAT32;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                double d = isf ? as_f64(v[r]) : (double)v[r];
                if (cmp_i64(t.op, f64_order_key(d), t.lit)) tr |= 1u << r;
            }
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (cmp_i64(t.op, v[r], t.lit)) tr |= 1u << r;
        }
        all_valid &= vv;
        any_true |= tr;
        all_true &= tr;
    }
    return T.is_or ? (all_valid & any_true) : (all_valid & all_true);
}

// Boolean mask of rows where a full program's BOOL result is TRUE.
template <int R>
__device__ __forceinline__ uint32_t program_true_mask(const ExprRegs<R> &X) {
    uint32_t m = 0;
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (X.v[0][r] & 1) m |= 1u << r;
    return m & X.valid[0];
}

}  // namespace qeh
