// FilterExec and ProjectionExec expressions.
//
// Reference: execute_filter (crates/query-executor/src/executor.rs:131-155)
// evaluates the predicate with evaluate_expr (operators.rs:13-62) and calls
// arrow's filter_record_batch (NULL -> dropped, order preserved) on every
// column; execute_projection (executor.rs:93-129) evaluates each expression
// (column references are Arc clones, operators.rs:15-23).
//
// Filter on the device is ONE pass: every workgroup takes a 2048-row tile in
// dispatch order (atomic ticket), evaluates the predicate (wave-uniform
// interpreter, expr_device.h), ranks the surviving rows with ballot+mbcnt,
// publishes its count, learns the rows before it by a decoupled look-back
// over 8-byte {flag, value} status words (agent-scope relaxed atomics: the
// status word is the only data handed between workgroups), and writes the
// selected rows of every output column to their final, order-preserving
// positions.  Inputs are read once, outputs written once.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "expr_device.h"
#include "lookback.h"
#include "ops.h"

namespace qeh {

constexpr int kFR = 8;                       // rows per thread
constexpr int kFTile = kBlock * kFR;         // 2048 rows per tile
struct OutSpec {
    const void *src_values;     // ColRef.values of the source column
    const uint8_t *src_valid;
    int64_t src_vbit0;
    int32_t dtype;
    int32_t _pad;
    void *dst_values;
    uint32_t *dst_valid;        // nullptr when the source has no validity
};
struct OutSpecs {
    OutSpec o[kMaxCols];
    int32_t n;
};

template <int PM>
__global__ __launch_bounds__(kBlock) void k_filter(ColSet cols, int64_t n, int64_t n_tiles, PredTerms terms,
                                                   DevProgram prog, OutSpecs outs, uint64_t *__restrict__ status,
                                                   unsigned long long *__restrict__ ticket, uint32_t *__restrict__ errp,
                                                   uint64_t *__restrict__ total_out, uint64_t cap, uint64_t exit_at,
                                                   uint64_t *__restrict__ done) {
    __shared__ uint32_t wave_cnt[kFR][kBlock / 64];
    __shared__ uint32_t wave_off[kFR][kBlock / 64];
    __shared__ int64_t s_tile;
    __shared__ uint64_t s_prefix;
    __shared__ uint32_t s_total;
    __shared__ uint32_t vbits[kMaxCols + 1][kFTile / 32 + 2];  // row kMaxCols: validity staging
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t err = 0;
    for (;;) {
        if (threadIdx.x == 0) {
            int64_t t = (int64_t)atomicAdd(ticket, 1ull);
            if (exit_at != kValMask && t < n_tiles && ld_agent(done)) {
                // the first `cap` rows are already placed: publish a prefix >= cap so that a
                // successor that started before `done` was raised still completes its look-back
                st_agent(&status[t], kFlagIncl | cap);
                t = n_tiles;
            }
            s_tile = t;
        }
        __syncthreads();
        const int64_t tile = s_tile;
        if (tile >= n_tiles) break;
        const int64_t row0 = tile * kFTile + threadIdx.x;  // rows row0 + r*256
        uint32_t sel;
        if (PM == 1) {
            sel = eval_terms<kFR>(terms, cols, row0, kBlock, n);
        } else {
            ExprRegs<kFR> X;
            run_program<kFR>(prog, cols, row0, kBlock, n, X, err);
            sel = program_true_mask<kFR>(X);
        }
        uint32_t rank[kFR];
#pragma unroll
        for (int r = 0; r < kFR; ++r) {
            const uint64_t b = __ballot((sel >> r) & 1);
            rank[r] = mbcnt(b);
            if (lane == 0) wave_cnt[r][wave] = (uint32_t)popc64(b);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            for (int r = 0; r < kFR; ++r)
                for (int w = 0; w < kBlock / 64; ++w) {
                    wave_off[r][w] = acc;
                    acc += wave_cnt[r][w];
                }
            s_total = acc;
        }
        __syncthreads();
        const uint32_t total = s_total;
        if (wave == 0) {
            uint64_t prefix = 0;
            if (tile == 0) {
                if (lane == 0) st_agent(&status[0], kFlagIncl | total);
            } else {
                if (lane == 0) st_agent(&status[tile], kFlagAgg | total);
                prefix = lookback(status, tile, total, errp);
                if (lane == 0) st_agent(&status[tile], kFlagIncl | (prefix + total));
            }
            if (lane == 0) {
                s_prefix = prefix;
                if (tile == n_tiles - 1) *total_out = prefix + total;
                if (prefix + total >= exit_at) st_agent(done, 1ull);
            }
        }
        // stage validity / boolean bits of this tile's output range in LDS
        for (int i = threadIdx.x; i < outs.n * (kFTile / 32 + 2); i += blockDim.x) (&vbits[0][0])[i] = 0;
        __syncthreads();
        const uint64_t prefix = s_prefix;
        const uint32_t lim = prefix >= cap ? 0u : (uint32_t)std::min<uint64_t>(total, cap - prefix);  // rows kept
        const uint32_t shift = (uint32_t)(prefix & 31);  // bit offset of the tile's first row in its word
#pragma unroll
        for (int r = 0; r < kFR; ++r) {
            if (!((sel >> r) & 1)) continue;
            const int64_t row = row0 + (int64_t)r * kBlock;
            const uint32_t local = wave_off[r][wave] + rank[r];
            if (local >= lim) continue;
            const uint64_t pos = prefix + local;
            for (int c = 0; c < outs.n; ++c) {
                const OutSpec &o = outs.o[c];
                switch (o.dtype) {
                    case QEH_DT_BOOL: {
                        if (bit_at((const uint8_t *)o.src_values, o.src_vbit0 + row)) {
                            const uint32_t b = local + shift;
                            atomicOr(&vbits[c][b >> 5], 1u << (b & 31));
                        }
                        break;
                    }
                    case QEH_DT_INT32: case QEH_DT_FLOAT32: case QEH_DT_UINT32:
                        ((uint32_t *)o.dst_values)[pos] = ((const uint32_t *)o.src_values)[row];
                        break;
                    default:
                        ((uint64_t *)o.dst_values)[pos] = ((const uint64_t *)o.src_values)[row];
                        break;
                }
            }
        }
        __syncthreads();
        // validity (and boolean values) words: interior words are owned by this
        // tile; the first and last word may be shared with neighbours -> atomicOr
        const uint32_t nwords = lim ? (shift + lim + 31) / 32 : 0;
        for (int c = 0; c < outs.n; ++c) {
            const OutSpec &o = outs.o[c];
            const bool bool_vals = o.dtype == QEH_DT_BOOL;
            if (!o.dst_valid && !bool_vals) continue;
            // validity bits need their own staging pass
            if (o.dst_valid) {
                __syncthreads();
                for (int i = threadIdx.x; i < kFTile / 32 + 2; i += blockDim.x) vbits[kMaxCols][i] = 0;
                __syncthreads();
#pragma unroll
                for (int r = 0; r < kFR; ++r) {
                    if (!((sel >> r) & 1)) continue;
                    const int64_t row = row0 + (int64_t)r * kBlock;
                    if (wave_off[r][wave] + rank[r] >= lim) continue;
                    if (!o.src_valid || bit_at(o.src_valid, o.src_vbit0 + row)) {
                        const uint32_t b = wave_off[r][wave] + rank[r] + shift;
                        atomicOr(&vbits[kMaxCols][b >> 5], 1u << (b & 31));
                    }
                }
                __syncthreads();
                for (uint32_t w = threadIdx.x; w < nwords; w += blockDim.x) {
                    uint32_t *dst = &o.dst_valid[(prefix >> 5) + w];
                    const uint32_t v = vbits[kMaxCols][w];
                    if (w == 0 || w == nwords - 1) atomicOr(dst, v);
                    else *dst = v;
                }
            }
            if (bool_vals) {
                for (uint32_t w = threadIdx.x; w < nwords; w += blockDim.x) {
                    uint32_t *dst = &((uint32_t *)o.dst_values)[(prefix >> 5) + w];
                    const uint32_t v = vbits[c][w];
                    if (w == 0 || w == nwords - 1) atomicOr(dst, v);
                    else *dst = v;
                }
            }
        }
        __syncthreads();
    }
    if (err) atomicOr(errp, err);
}

// ---- fast filter: non-null 8-byte columns, <= 2 terms ---------------------------------------
// Every column the tile needs (outputs first, then predicate-only columns) is
// loaded once as 16-byte pairs before anything else, the selected rows are
// ranked with ballots, the tile's output offset comes from the same decoupled
// look-back, and each output column leaves through LDS as one contiguous run
// (full-line writes instead of one scattered 8-byte store per selected row).
constexpr int kFFMaxCols = 4;
constexpr int kFFPairs = 4, kFFR = 2 * kFFPairs;
static_assert(kFFR * kBlock == kFTile, "fast filter tiles match the generic filter's");
typedef long long v2i64f __attribute__((ext_vector_type(2)));

struct FastFilterIn {
    const int64_t *col[kFFMaxCols];   // slots: outputs first, then predicate-only columns
    int64_t *out[kFFMaxCols];
    int32_t n_out;
    int32_t term_slot[2];
    int32_t term_dt[2];
    int32_t _pad;
    int64_t n;
};

__device__ __forceinline__ v2i64f ff_pair(const int64_t *p, int64_t row, int64_t n) {
    if (row + 1 < n) return __builtin_nontemporal_load((const v2i64f *)(p + row));
    v2i64f v = {0, 0};
    if (row < n) v[0] = p[row];
    return v;
}

template <int NTERMS, int NC>
__global__ __launch_bounds__(kBlock) void k_filter_fast(FastFilterIn in, int64_t n_tiles, PredTerms terms,
                                                        uint64_t *__restrict__ status, unsigned long long *__restrict__ ticket,
                                                        uint32_t *__restrict__ errp, uint64_t *__restrict__ total_out,
                                                        uint64_t cap, uint64_t exit_at, uint64_t *__restrict__ done) {
    constexpr int W = kBlock / 64;
    __shared__ int64_t stage[kFTile];
    __shared__ uint32_t cnt[W][kFFPairs], offs[W][kFFPairs];
    __shared__ int64_t s_tile;
    __shared__ uint64_t s_prefix;
    __shared__ uint32_t s_total;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (;;) {
        if (threadIdx.x == 0) {
            int64_t t = (int64_t)atomicAdd(ticket, 1ull);
            if (exit_at != kValMask && t < n_tiles && ld_agent(done)) {
                // the first `cap` rows are already placed: publish a prefix >= cap so that a
                // successor that started before `done` was raised still completes its look-back
                st_agent(&status[t], kFlagIncl | cap);
                t = n_tiles;
            }
            s_tile = t;
        }
        __syncthreads();
        const int64_t tile = s_tile;
        if (tile >= n_tiles) break;
        const int64_t base = tile * kFTile + (int64_t)wave * (64 * kFFR) + 2 * lane;
        v2i64f cv[NC][kFFPairs];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int j = 0; j < kFFPairs; ++j) cv[c][j] = ff_pair(in.col[c], base + j * 128, in.n);
        uint32_t live = 0;
#pragma unroll
        for (int r = 0; r < kFFR; ++r)
            if (base + (r >> 1) * 128 + (r & 1) < in.n) live |= 1u << r;
        uint32_t acc = live;
#pragma unroll
        for (int i = 0; i < NTERMS; ++i) {
            const PredTerm pt = terms.t[i];
            const int slot = in.term_slot[i];
            const bool fcol = in.term_dt[i] == QEH_DT_FLOAT64;
            uint32_t tr = 0;
#pragma unroll
            for (int r = 0; r < kFFR; ++r) {
                int64_t v = 0;
#pragma unroll
                for (int c = 0; c < NC; ++c)  // wave-uniform select, constant register indices
                    if (c == slot) v = cv[c][r >> 1][r & 1];
                if (pt.ctype == QEH_DT_FLOAT64) v = f64_order_key(fcol ? as_f64(v) : (double)v);
                if (cmp_i64(pt.op, v, pt.lit)) tr |= 1u << r;
            }
            if (NTERMS > 1 && terms.is_or) acc = (i == 0) ? tr : (acc | tr);
            else acc &= tr;
        }
        const uint32_t sel = acc & live;
        uint32_t rank[kFFR];
#pragma unroll
        for (int j = 0; j < kFFPairs; ++j) {
            const uint64_t m0 = __ballot((sel >> (2 * j)) & 1), m1 = __ballot((sel >> (2 * j + 1)) & 1);
            const uint32_t below = mbcnt(m0) + mbcnt(m1);
            rank[2 * j] = below;
            rank[2 * j + 1] = below + ((sel >> (2 * j)) & 1);
            if (lane == 0) cnt[wave][j] = (uint32_t)(popc64(m0) + popc64(m1));
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            for (int w = 0; w < W; ++w)
                for (int j = 0; j < kFFPairs; ++j) {
                    offs[w][j] = acc;
                    acc += cnt[w][j];
                }
            s_total = acc;
        }
        __syncthreads();
        const uint32_t total = s_total;
        if (wave == 0) {
            uint64_t prefix = 0;
            if (tile == 0) {
                if (lane == 0) st_agent(&status[0], kFlagIncl | total);
            } else {
                if (lane == 0) st_agent(&status[tile], kFlagAgg | total);
                prefix = lookback(status, tile, total, errp);
                if (lane == 0) st_agent(&status[tile], kFlagIncl | (prefix + total));
            }
            if (lane == 0) {
                s_prefix = prefix;
                if (tile == n_tiles - 1) *total_out = prefix + total;
                if (prefix + total >= exit_at) st_agent(done, 1ull);
            }
        }
        __syncthreads();
        const uint64_t prefix = s_prefix;
        const uint32_t lim = prefix >= cap ? 0u : (uint32_t)std::min<uint64_t>(total, cap - prefix);  // rows kept
        auto emit = [&](auto cc) {
            constexpr int c = decltype(cc)::value;
            if constexpr (c < NC) {
                if (c < in.n_out) {  // wave-uniform
#pragma unroll
                    for (int r = 0; r < kFFR; ++r)
                        if ((sel >> r) & 1) stage[offs[wave][r >> 1] + rank[r]] = cv[c][r >> 1][r & 1];
                    __syncthreads();
                    int64_t *dst = in.out[c] + prefix;
                    for (uint32_t i = threadIdx.x; i < lim; i += kBlock) __builtin_nontemporal_store(stage[i], &dst[i]);
                    __syncthreads();
                }
            }
        };
        emit(std::integral_constant<int, 0>{});
        emit(std::integral_constant<int, 1>{});
        emit(std::integral_constant<int, 2>{});
        emit(std::integral_constant<int, 3>{});
    }
}

// ---- projection expression -------------------------------------------------------------
constexpr int kER = 4;
template <int RT>  // result dtype class: 0 = 8-byte, 1 = 4-byte int, 2 = float32, 3 = bool
__global__ __launch_bounds__(kBlock) void k_eval(ColSet cols, int64_t n, DevProgram prog, void *__restrict__ out,
                                                 uint64_t *__restrict__ out_valid, uint32_t *__restrict__ errp) {
    const int lane = threadIdx.x & 63;
    uint32_t err = 0;
    const int64_t nchunks = (n + 64 * kER - 1) / (64 * kER);
    const int64_t wstride = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t w = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); w < nchunks; w += wstride) {
        const int64_t base = w * 64 * kER;
        ExprRegs<kER> X;
        run_program<kER>(prog, cols, base + lane, 64, n, X, err);
#pragma unroll
        for (int r = 0; r < kER; ++r) {
            const int64_t row = base + r * 64 + lane;
            const bool live = row < n;
            const bool valid = live && ((X.valid[0] >> r) & 1);
            const uint64_t vb = __ballot(valid);
            if (RT == 3) {
                const uint64_t bb = __ballot(live && (X.v[0][r] & 1));
                if (lane == 0) ((uint64_t *)out)[(base + r * 64) >> 6] = bb;
            } else if (live) {
                if (RT == 0) ((int64_t *)out)[row] = X.v[0][r];
                else if (RT == 1) ((int32_t *)out)[row] = (int32_t)X.v[0][r];
                else ((float *)out)[row] = (float)as_f64(X.v[0][r]);
            }
            if (lane == 0) out_valid[(base + r * 64) >> 6] = vb;
        }
    }
    if (err) atomicOr(errp, err);
}

}  // namespace qeh

using namespace qeh;

__global__ void k_iota_u32(uint32_t *out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (uint32_t)i;
}

static int filter_impl(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *predicate,
                       const int32_t *out_idx, int n_out, int64_t max_rows, qeh_column *out, int64_t *out_rows) {
    if (!ctx || !out_rows || (n_out > 0 && (!out || !out_idx))) return fail(QEH_E_INVALID, "qeh_filter: bad argument");
    *out_rows = 0;
    DeviceGuard dg(ctx->device);
    for (int j = 0; j < n_out; ++j)
        if (out_idx[j] < 0 || out_idx[j] >= n_cols) return fail(QEH_E_INVALID, "filter output column index out of range");
    // Utf8 comparisons become BOOL columns appended after the inputs (k_utf8.hip)
    Utf8Rewrite uw;
    QEH_TRY(rewrite_utf8_compares(ctx, cols, n_cols, predicate, &uw));
    if (uw.changed) {
        cols = uw.cols.data();
        n_cols = (int)uw.cols.size();
        predicate = &uw.expr;
    }
    ColSet cs;
    QEH_TRY(make_colset(cols, n_cols, &cs));
    const int64_t n = n_cols > 0 ? cols[0].length : 0;
    for (int i = 0; i < n_cols; ++i)
        if (cols[i].length != n) return fail(QEH_E_INVALID, "filter columns have different lengths");
    // LIMIT pushed into the filter: rows past `cap` are neither written nor allocated, and tiles
    // claimed after the first `cap` selected rows are placed are not read at all
    const uint64_t cap = max_rows < 0 ? kValMask : std::min<uint64_t>((uint64_t)max_rows, kValMask);
    const int64_t n_alloc = (int64_t)std::min<uint64_t>((uint64_t)n, cap);
    uint64_t exit_at = kValMask;  // set below for predicates that cannot raise
    std::vector<int32_t> dts(n_cols);
    for (int i = 0; i < n_cols; ++i) dts[i] = cols[i].dtype;
    DevProgram prog;
    QEH_TRY(compile_expr(predicate, dts.data(), n_cols, &prog));
    if (prog.result_type != QEH_DT_BOOL) return fail(QEH_E_TYPE, "Filter predicate must return boolean");
    PredTerms terms{};
    const bool fast = lower_to_terms(predicate, dts.data(), n_cols, &terms);
    // comparisons of columns with literals cannot raise, so tiles past the cap may go unread;
    // a general predicate (arithmetic may overflow) is evaluated on every row, as the reference does
    if (fast) exit_at = cap;
    for (int j = 0; j < n_out; ++j)
        if (out_idx[j] < 0 || out_idx[j] >= n_cols) return fail(QEH_E_INVALID, "filter output column index out of range");
    // fixed-width outputs are compacted by the kernel; Utf8 outputs are
    // gathered afterwards through the selected-row ids (an extra UINT32 output)
    std::vector<int> fixed, utf8;
    for (int j = 0; j < n_out; ++j) (cols[out_idx[j]].dtype == QEH_DT_UTF8 ? utf8 : fixed).push_back(j);
    const int n_kernel_out = (int)fixed.size() + (utf8.empty() ? 0 : 1);
    if (n_kernel_out > kMaxCols) return fail(QEH_E_UNSUPPORTED, "too many output columns for one filter (max 12)");
    std::vector<char> made(n_out, 0);
    auto cleanup = [&]() {
        for (int j = 0; j < n_out; ++j)
            if (made[j]) qeh_column_release(ctx, &out[j]);
    };
    OutSpecs os{};
    os.n = n_kernel_out;
    DevBuf iota, rowids;
    for (size_t q = 0; q < fixed.size(); ++q) {
        const int j = fixed[q];
        const qeh_column &src = cols[out_idx[j]];
        int s = alloc_column(ctx, src.dtype, n_alloc, src.validity != nullptr, &out[j]);
        if (s != QEH_OK) {
            cleanup();
            return s;
        }
        made[j] = 1;
        const size_t words = ((size_t)(n_alloc + 63) / 64) * 8;
        if (src.validity) QEH_HIP(hipMemsetAsync(out[j].validity, 0, words ? words : 8, ctx->stream));
        if (src.dtype == QEH_DT_BOOL) QEH_HIP(hipMemsetAsync(out[j].values, 0, words ? words : 8, ctx->stream));
        const ColRef cr = make_colref(src);
        OutSpec &o = os.o[q];
        o.src_values = cr.values;
        o.src_valid = cr.validity;
        o.src_vbit0 = cr.vbit0;
        o.dtype = src.dtype;
        o.dst_values = out[j].values;
        o.dst_valid = (uint32_t *)out[j].validity;
    }
    if (!utf8.empty()) {
        int s = iota.alloc(ctx, (size_t)std::max<int64_t>(n, 1) * 4);
        if (s == QEH_OK) s = rowids.alloc(ctx, (size_t)std::max<int64_t>(n_alloc, 1) * 4);
        if (s != QEH_OK) {
            cleanup();
            return s;
        }
        if (n > 0)
            hipLaunchKernelGGL(k_iota_u32, dim3(grid_for(ctx, n, kBlock * 8, 8)), dim3(kBlock), 0, ctx->stream,
                               iota.as<uint32_t>(), n);
        OutSpec &o = os.o[fixed.size()];
        o.src_values = iota.p;
        o.dtype = QEH_DT_UINT32;
        o.dst_values = rowids.p;
    }
    // fast path: every referenced column non-null 8-byte and 16-byte aligned, <= 2 terms,
    // distinct output columns, <= 4 columns in all
    FastFilterIn ffi{};
    int ff_nc = 0;
    bool ff = fast && terms.n <= 2 && utf8.empty() && !std::getenv("QEH_NO_FAST_FILTER");
    auto ff_ok = [&](const qeh_column &c) {
        return (c.dtype == QEH_DT_INT64 || c.dtype == QEH_DT_FLOAT64) && (!c.validity || c.null_count == 0) &&
               ((uintptr_t)((const int64_t *)c.values + c.offset) & 15) == 0;
    };
    std::vector<int> slot_col;  // slot -> input column
    for (int j = 0; ff && j < n_out; ++j) {
        const int ci = out_idx[j];
        if (!ff_ok(cols[ci]) || std::find(slot_col.begin(), slot_col.end(), ci) != slot_col.end()) ff = false;
        else slot_col.push_back(ci);
    }
    for (int i = 0; ff && i < terms.n; ++i) {
        const int ci = terms.t[i].col;
        if (!ff_ok(cols[ci]) || (terms.t[i].ctype != QEH_DT_INT64 && terms.t[i].ctype != QEH_DT_FLOAT64)) ff = false;
        auto it = std::find(slot_col.begin(), slot_col.end(), ci);
        if (ff && it == slot_col.end()) slot_col.push_back(ci);
    }
    if (ff && ((int)slot_col.size() > kFFMaxCols || slot_col.empty())) ff = false;
    if (ff) {
        ff_nc = (int)slot_col.size();
        for (int c = 0; c < ff_nc; ++c) ffi.col[c] = (const int64_t *)cols[slot_col[c]].values + cols[slot_col[c]].offset;
        for (int j = 0; j < n_out; ++j) ffi.out[j] = (int64_t *)out[j].values;
        ffi.n_out = n_out;
        for (int i = 0; i < terms.n; ++i) {
            ffi.term_slot[i] = (int)(std::find(slot_col.begin(), slot_col.end(), terms.t[i].col) - slot_col.begin());
            ffi.term_dt[i] = cols[terms.t[i].col].dtype;
        }
        ffi.n = n;
    }
    const int64_t n_tiles = (n + kFTile - 1) / kFTile;
    uint64_t total = 0;
    if (n_tiles > 0) {
        void *scr = nullptr;
        const size_t hdr = 256;  // ticket/err/total in one line, `done` in its own (away from the ticket atomics)
        int s = scratch_zeroed(ctx, hdr + (size_t)n_tiles * 8, &scr);
        if (s != QEH_OK) {
            cleanup();
            return s;
        }
        unsigned long long *ticket = (unsigned long long *)scr;
        uint32_t *err = (uint32_t *)((char *)scr + 8);
        uint64_t *tot = (uint64_t *)((char *)scr + 16);
        uint64_t *done = (uint64_t *)((char *)scr + 128);
        uint64_t *status = (uint64_t *)((char *)scr + hdr);
        const int grid = grid_for(ctx, n, kFTile, 4);
        {
            KernelTimer kt(ctx, "filter");
            if (ff) {
#define QEH_FF(NTV, NCV) \
    hipLaunchKernelGGL((k_filter_fast<NTV, NCV>), dim3(grid), dim3(kBlock), 0, ctx->stream, ffi, n_tiles, terms, status, ticket, err, tot, cap, exit_at, done)
#define QEH_FF_NC(NTV)                                    \
    if (ff_nc == 1) QEH_FF(NTV, 1);                       \
    else if (ff_nc == 2) QEH_FF(NTV, 2);                  \
    else if (ff_nc == 3) QEH_FF(NTV, 3);                  \
    else QEH_FF(NTV, 4);
                if (terms.n == 0) { QEH_FF_NC(0) } else if (terms.n == 1) { QEH_FF_NC(1) } else { QEH_FF_NC(2) }
#undef QEH_FF_NC
#undef QEH_FF
            } else if (fast)
                hipLaunchKernelGGL(k_filter<1>, dim3(grid), dim3(kBlock), 0, ctx->stream, cs, n, n_tiles, terms, prog, os,
                                   status, ticket, err, tot, cap, exit_at, done);
            else
                hipLaunchKernelGGL(k_filter<2>, dim3(grid), dim3(kBlock), 0, ctx->stream, cs, n, n_tiles, terms, prog, os,
                                   status, ticket, err, tot, cap, exit_at, done);
        }
        QEH_HIP(hipGetLastError());
        uint64_t hdrv[17];
        s = read_small(ctx, hdrv, scr, 136);
        if (s == QEH_OK) s = kernel_error_status((uint32_t)hdrv[1], "filter");
        if (s != QEH_OK) {
            cleanup();
            return s;
        }
        total = hdrv[16] ? cap : std::min<uint64_t>(hdrv[2], cap);  // done: at least `cap` rows qualified
    }
    for (int j : utf8) {
        int s = gather_column(ctx, cols[out_idx[j]], rowids.as<uint32_t>(), (int64_t)total, &out[j]);
        if (s != QEH_OK) {
            cleanup();
            return s;
        }
        made[j] = 1;
    }
    if (!utf8.empty()) QEH_HIP(hipStreamSynchronize(ctx->stream));
    for (int j = 0; j < n_out; ++j) {
        out[j].length = (int64_t)total;
        if (out[j].dtype != QEH_DT_UTF8) out[j].null_count = out[j].validity ? -1 : 0;
    }
    *out_rows = (int64_t)total;
    return QEH_OK;
}

extern "C" int qeh_filter(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *predicate,
                          const int32_t *out_idx, int n_out, qeh_column *out, int64_t *out_rows) {
    return filter_impl(ctx, cols, n_cols, predicate, out_idx, n_out, -1, out, out_rows);
}

extern "C" int qeh_filter_limit(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *predicate,
                                const int32_t *out_idx, int n_out, int64_t max_rows, qeh_column *out,
                                int64_t *out_rows) {
    return filter_impl(ctx, cols, n_cols, predicate, out_idx, n_out, max_rows, out, out_rows);
}

extern "C" int qeh_eval(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *expr, int64_t n_rows,
                        qeh_column *out) {
    if (!ctx || !out || !expr) return fail(QEH_E_INVALID, "qeh_eval: bad argument");
    std::memset(out, 0, sizeof(*out));
    DeviceGuard dg(ctx->device);
    for (int i = 0; i < n_cols; ++i)
        if (cols[i].length != n_rows) return fail(QEH_E_INVALID, "eval columns have different lengths");
    Utf8Rewrite uw;  // Utf8 comparisons become BOOL columns appended after the inputs (k_utf8.hip)
    QEH_TRY(rewrite_utf8_compares(ctx, cols, n_cols, expr, &uw));
    const int n_in = n_cols;
    if (uw.changed) {
        cols = uw.cols.data();
        n_cols = (int)uw.cols.size();
        expr = &uw.expr;
    }
    const int ci = expr_as_column(expr);
    if (ci >= n_in) {  // the whole expression was one Utf8 comparison: hand its column over
        *out = cols[ci];
        uw.temps.erase(uw.temps.begin() + (ci - n_in));
        return QEH_OK;
    }
    if (ci >= 0) {  // zero-copy column reference (operators.rs:15-23)
        if (ci >= n_cols) return fail(QEH_E_INVALID, "Column index " + std::to_string(ci) + " out of bounds");
        *out = cols[ci];
        out->owned = 0;
        return QEH_OK;
    }
    ColSet cs;
    QEH_TRY(make_colset(cols, n_cols, &cs));
    std::vector<int32_t> dts(n_cols);
    for (int i = 0; i < n_cols; ++i) dts[i] = cols[i].dtype;
    DevProgram prog;
    QEH_TRY(compile_expr(expr, dts.data(), n_cols, &prog));
    int rt = prog.result_type;
    if (rt == QEH_DT_NULL) rt = QEH_DT_INT64;  // NullArray: all-null column, typed Int64 here
    QEH_TRY(alloc_column(ctx, rt, n_rows, true, out));
    if (n_rows == 0) return QEH_OK;
    void *scr = nullptr;
    int s = scratch_zeroed(ctx, 64, &scr);
    if (s != QEH_OK) {
        qeh_column_release(ctx, out);
        return s;
    }
    const int grid = grid_for(ctx, n_rows, kBlock * kER, 8);
    {
        KernelTimer kt(ctx, "eval");
        uint32_t *err = (uint32_t *)scr;
        uint64_t *ov = (uint64_t *)out->validity;
        switch (rt) {
            case QEH_DT_BOOL:
                hipLaunchKernelGGL(k_eval<3>, dim3(grid), dim3(kBlock), 0, ctx->stream, cs, n_rows, prog, out->values, ov, err);
                break;
            case QEH_DT_INT32:
                hipLaunchKernelGGL(k_eval<1>, dim3(grid), dim3(kBlock), 0, ctx->stream, cs, n_rows, prog, out->values, ov, err);
                break;
            case QEH_DT_FLOAT32:
                hipLaunchKernelGGL(k_eval<2>, dim3(grid), dim3(kBlock), 0, ctx->stream, cs, n_rows, prog, out->values, ov, err);
                break;
            default:
                hipLaunchKernelGGL(k_eval<0>, dim3(grid), dim3(kBlock), 0, ctx->stream, cs, n_rows, prog, out->values, ov, err);
                break;
        }
    }
    QEH_HIP(hipGetLastError());
    uint32_t e = 0;
    s = read_small(ctx, &e, scr, 4);
    if (s == QEH_OK) s = kernel_error_status(e, "eval");
    if (s != QEH_OK) {
        qeh_column_release(ctx, out);
        return s;
    }
    out->null_count = -1;
    return QEH_OK;
}
