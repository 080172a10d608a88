// Utf8 comparisons in predicates and projections.
//
// Reference: evaluate_binary_op's comparison arms (crates/query-executor/src/
// operators.rs:509-538) coerce numeric types only, so Utf8 = Utf8 (a string
// column against a Utf8 literal broadcast by create_literal_array, :322-347, or
// against another string column) reaches arrow's eq / neq / lt / lt_eq / gt /
// gt_eq on StringArray: byte-wise lexicographic order, NULL in -> NULL out.  A
// Utf8 side against any other type is arrow's "Invalid comparison operation"
// error.
//
// On the device the register interpreter (expr_device.h) carries 64-bit
// values, not strings, so every comparison whose two operands are leaves
// (column / literal) with a Utf8 side is evaluated first by k_utf8_cmp into a
// bit-packed BOOL column appended to the operator's inputs, and the expression
// is rewritten to read that column.  The rest of the predicate (AND / OR / NOT,
// numeric terms) then runs unchanged.
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "device_common.h"
#include "ops.h"

namespace qeh {

struct StrSide {
    ColRef valid;            // validity only (column side)
    const int32_t *offs;     // column side: offsets advanced by the column offset
    const uint8_t *data;     // column bytes, or the literal's bytes
    int32_t lit_len;
    int32_t is_lit;
};

__device__ inline int str_cmp(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb) {
    const int32_t m = la < lb ? la : lb;
    for (int32_t i = 0; i < m; ++i)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

__global__ void k_utf8_cmp(StrSide a, StrSide b, int op, int64_t n, uint64_t *__restrict__ out_bits,
                           uint64_t *__restrict__ out_valid) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t w = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); w * 64 < n; w += nw) {
        const int64_t i = w * 64 + lane;
        bool r = false, v = false;
        if (i < n) {
            v = (a.is_lit || col_valid(a.valid, i)) && (b.is_lit || col_valid(b.valid, i));
            if (v) {
                const uint8_t *pa = a.is_lit ? a.data : a.data + a.offs[i];
                const uint8_t *pb = b.is_lit ? b.data : b.data + b.offs[i];
                const int32_t la = a.is_lit ? a.lit_len : a.offs[i + 1] - a.offs[i];
                const int32_t lb = b.is_lit ? b.lit_len : b.offs[i + 1] - b.offs[i];
                const int c = str_cmp(pa, la, pb, lb);
                switch (op) {
                    case QEH_OP_EQ: r = c == 0; break;
                    case QEH_OP_NEQ: r = c != 0; break;
                    case QEH_OP_LT: r = c < 0; break;
                    case QEH_OP_LTE: r = c <= 0; break;
                    case QEH_OP_GT: r = c > 0; break;
                    default: r = c >= 0; break;
                }
            }
        }
        const uint64_t rb = __ballot(r && v), vb = __ballot(v);
        if (lane == 0) {
            out_bits[w] = rb;
            if (out_valid) out_valid[w] = vb;
        }
    }
}

static bool is_cmp(int op) { return op >= QEH_OP_EQ && op <= QEH_OP_GTE; }

static const char *op_text(int op) {  // arrow-rs cmp Op display
    switch (op) {
        case QEH_OP_EQ: return "==";
        case QEH_OP_NEQ: return "!=";
        case QEH_OP_LT: return "<";
        case QEH_OP_LTE: return "<=";
        case QEH_OP_GT: return ">";
        default: return ">=";
    }
}

static const char *arrow_type_name(int dt) {
    switch (dt) {
        case QEH_DT_NULL: return "Null";
        case QEH_DT_BOOL: return "Boolean";
        case QEH_DT_INT32: return "Int32";
        case QEH_DT_INT64: return "Int64";
        case QEH_DT_FLOAT32: return "Float32";
        case QEH_DT_FLOAT64: return "Float64";
        case QEH_DT_UTF8: return "Utf8";
        case QEH_DT_UINT32: return "UInt32";
        default: return "?";
    }
}

Utf8Rewrite::~Utf8Rewrite() {
    if (!ctx) return;
    (void)hipStreamSynchronize(ctx->stream);
    for (auto &c : temps) qeh_column_release(ctx, &c);
}

bool expr_has_utf8(const qeh_expr *e, const int32_t *dtypes, int n_cols) {
    if (!e) return false;
    for (int i = 0; i < e->n_nodes; ++i) {
        const qeh_expr_node &nd = e->nodes[i];
        if (nd.kind == QEH_EX_COLUMN && nd.index >= 0 && nd.index < n_cols && dtypes[nd.index] == QEH_DT_UTF8) return true;
        if (nd.kind == QEH_EX_LITERAL && !nd.lit_is_null && nd.lit_dtype == QEH_DT_UTF8) return true;
    }
    return false;
}

int rewrite_utf8_compares(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *e, Utf8Rewrite *out) {
    out->ctx = ctx;
    out->cols.assign(cols, cols + n_cols);
    out->nodes.clear();
    out->changed = false;
    if (!e) return QEH_OK;
    const int64_t n = n_cols > 0 ? cols[0].length : 0;
    auto leaf_type = [&](const qeh_expr_node &nd) -> int {
        if (nd.kind == QEH_EX_COLUMN)
            return (nd.index >= 0 && nd.index < (int)out->cols.size()) ? out->cols[nd.index].dtype : -1;
        if (nd.kind == QEH_EX_LITERAL) return nd.lit_is_null ? QEH_DT_NULL : nd.lit_dtype;
        return -1;
    };
    auto is_leaf = [](const qeh_expr_node &nd) { return nd.kind == QEH_EX_COLUMN || nd.kind == QEH_EX_LITERAL; };
    for (int i = 0; i < e->n_nodes; ++i) {
        const qeh_expr_node &nd = e->nodes[i];
        const size_t m = out->nodes.size();
        if (nd.kind == QEH_EX_BINARY && is_cmp(nd.op) && m >= 2 && is_leaf(out->nodes[m - 2]) && is_leaf(out->nodes[m - 1])) {
            const qeh_expr_node l = out->nodes[m - 2], r = out->nodes[m - 1];
            const int lt = leaf_type(l), rt = leaf_type(r);
            if (lt == QEH_DT_UTF8 || rt == QEH_DT_UTF8) {
                if (lt != rt)
                    return fail(QEH_E_TYPE, std::string("Invalid argument error: Invalid comparison operation: ") +
                                                arrow_type_name(lt) + " " + op_text(nd.op) + " " + arrow_type_name(rt));
                StrSide side[2];
                bool any_valid = false;
                for (int s = 0; s < 2; ++s) {
                    const qeh_expr_node &x = s == 0 ? l : r;
                    StrSide &sd = side[s];
                    sd = StrSide{};
                    if (x.kind == QEH_EX_LITERAL) {
                        const int32_t len = x.index;
                        if (len < 0 || (len > 0 && x.lit_i64 == 0)) return fail(QEH_E_INVALID, "Utf8 literal without bytes");
                        out->bufs.push_back(std::make_unique<DevBuf>());
                        DevBuf &buf = *out->bufs.back();
                        QEH_TRY(buf.alloc(ctx, (size_t)std::max(len, 1)));
                        if (len > 0)
                            QEH_HIP(hipMemcpyAsync(buf.p, (const void *)(uintptr_t)x.lit_i64, (size_t)len,
                                                   hipMemcpyHostToDevice, ctx->stream));
                        sd.data = buf.as<uint8_t>();
                        sd.lit_len = len;
                        sd.is_lit = 1;
                    } else {
                        const qeh_column &c = out->cols[x.index];
                        QEH_TRY(check_column(c, "Utf8 comparison"));
                        sd.valid = make_colref(c);
                        sd.offs = c.offsets + c.offset;
                        sd.data = (const uint8_t *)c.values;
                        if (c.validity && c.null_count != 0) any_valid = true;
                    }
                }
                qeh_column res{};
                QEH_TRY(alloc_column(ctx, QEH_DT_BOOL, n, any_valid, &res));
                out->temps.push_back(res);
                if (n > 0) {
                    KernelTimer kt(ctx, "utf8_compare");
                    hipLaunchKernelGGL(k_utf8_cmp, dim3(grid_for(ctx, (n + 63) / 64, kBlock / 64, 8)), dim3(kBlock), 0,
                                       ctx->stream, side[0], side[1], nd.op, n, (uint64_t *)res.values,
                                       (uint64_t *)res.validity);
                    QEH_HIP(hipGetLastError());
                }
                res.null_count = any_valid ? -1 : 0;
                out->temps.back() = res;
                out->cols.push_back(res);
                qeh_expr_node c{};
                c.kind = QEH_EX_COLUMN;
                c.index = (int32_t)out->cols.size() - 1;
                out->nodes.resize(m - 2);
                out->nodes.push_back(c);
                out->changed = true;
                continue;
            }
        }
        out->nodes.push_back(nd);
    }
    if (out->changed) QEH_HIP(hipStreamSynchronize(ctx->stream));  // literal host bytes are the caller's
    out->expr.nodes = out->nodes.data();
    out->expr.n_nodes = (int32_t)out->nodes.size();
    return QEH_OK;
}

}  // namespace qeh
