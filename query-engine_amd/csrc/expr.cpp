// Host compiler: postfix PhysicalExpr -> typed register program / term list.
//
// Typing mirrors crates/query-executor/src/operators.rs:
//   Column        -> column type; index >= n_cols -> "Column index {} out of bounds" (:15-23)
//   Literal       -> literal type; typed None / Null -> NullArray (:322-347)
//   NOT           -> Boolean only, "NOT operator requires boolean array" (:351-359)
//   unary minus   -> Int64/Float64/Int32/Float32, "Unsupported type for negation" (:360-378)
//   + - * /       -> identical operand types among Int64/Int32/Float64/Float32, no coercion,
//                    "Unsupported types for addition|subtraction|multiplication|division" (:384-507)
//   %             -> Int64/Int64 or Int32/Int32, "Modulo operation requires integer arrays" (:711-743)
//   comparisons   -> coerce_numeric_types (:616-675) then arrow cmp on equal types
//   AND / OR      -> Boolean only, "AND requires boolean arrays" / "OR ..." (:540-571)
#include <string>
#include <vector>

#include "expr.h"
#include "qeh_internal.h"

namespace qeh {

static const char *dt_name(int t) {
    switch (t) {
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

static bool is_int(int t) { return t == QEH_DT_INT32 || t == QEH_DT_INT64; }
static bool is_num(int t) {
    return t == QEH_DT_INT32 || t == QEH_DT_INT64 || t == QEH_DT_FLOAT32 || t == QEH_DT_FLOAT64;
}

static const char *cmp_sym(int op) {
    switch (op) {
        case QEH_OP_EQ: return "==";
        case QEH_OP_NEQ: return "!=";
        case QEH_OP_LT: return "<";
        case QEH_OP_LTE: return "<=";
        case QEH_OP_GT: return ">";
        default: return ">=";
    }
}

// coerce_numeric_types (operators.rs:616-675): returns the (left, right) types
// after coercion; `castl/castr` say whether an int->f64 cast is inserted.
static void coerce(int lt, int rt, int *olt, int *ort) {
    *olt = lt;
    *ort = rt;
    if (lt == rt) return;
    if (lt == QEH_DT_FLOAT64 && is_int(rt)) { *ort = QEH_DT_FLOAT64; return; }
    if (rt == QEH_DT_FLOAT64 && is_int(lt)) { *olt = QEH_DT_FLOAT64; return; }
    if (lt == QEH_DT_FLOAT32 || rt == QEH_DT_FLOAT32) {
        // cast_to_float64 (:678-709): Float32/Int64/Int32 -> Float64, others unchanged
        if (is_num(lt)) *olt = QEH_DT_FLOAT64;
        if (is_num(rt)) *ort = QEH_DT_FLOAT64;
        return;
    }
    if (lt == QEH_DT_INT64 && rt == QEH_DT_INT32) { *ort = QEH_DT_INT64; return; }
    if (rt == QEH_DT_INT64 && lt == QEH_DT_INT32) { *olt = QEH_DT_INT64; return; }
}

int expr_as_column(const qeh_expr *e) {
    if (e && e->n_nodes == 1 && e->nodes[0].kind == QEH_EX_COLUMN) return e->nodes[0].index;
    return -1;
}

uint64_t expr_columns(const qeh_expr *e) {
    uint64_t m = 0;
    if (!e) return 0;
    for (int i = 0; i < e->n_nodes; ++i)
        if (e->nodes[i].kind == QEH_EX_COLUMN && e->nodes[i].index >= 0 && e->nodes[i].index < 64)
            m |= 1ull << e->nodes[i].index;
    return m;
}

int compile_expr(const qeh_expr *e, const int32_t *dtypes, int n_cols, DevProgram *out) {
    if (!e || e->n_nodes <= 0 || !e->nodes) return fail(QEH_E_INVALID, "empty expression");
    out->n = 0;
    std::vector<int> ty;  // type stack (slot = depth)
    auto emit = [&](DevInstr in) -> int {
        if (out->n >= kMaxInstr)
            return fail(QEH_E_UNSUPPORTED, "expression too large for the device program (max " +
                                               std::to_string(kMaxInstr) + " instructions)");
        out->ins[out->n++] = in;
        return QEH_OK;
    };
    for (int i = 0; i < e->n_nodes; ++i) {
        const qeh_expr_node &nd = e->nodes[i];
        DevInstr in{};
        switch (nd.kind) {
            case QEH_EX_COLUMN: {
                if (nd.index < 0 || nd.index >= n_cols)
                    return fail(QEH_E_INVALID,
                                "Column index " + std::to_string(nd.index) + " out of bounds");
                int t = dtypes[nd.index];
                if (t == QEH_DT_UTF8)
                    return fail(QEH_E_UNSUPPORTED, "Utf8 expressions are not evaluated on the device");
                if ((int)ty.size() >= kNS) return fail(QEH_E_UNSUPPORTED, "expression too deep");
                in.op = D_LOAD;
                in.t = (uint8_t)t;
                in.dst = (uint8_t)ty.size();
                in.a = (uint8_t)nd.index;
                QEH_TRY(emit(in));
                ty.push_back(t);
                break;
            }
            case QEH_EX_LITERAL: {
                int t = nd.lit_is_null ? QEH_DT_NULL : nd.lit_dtype;
                if (t == QEH_DT_UTF8)
                    return fail(QEH_E_UNSUPPORTED, "Utf8 literals are not evaluated on the device");
                if ((int)ty.size() >= kNS) return fail(QEH_E_UNSUPPORTED, "expression too deep");
                in.op = D_LIT;
                in.t = (uint8_t)t;
                in.dst = (uint8_t)ty.size();
                in.flag = t == QEH_DT_NULL;
                if (t == QEH_DT_FLOAT64 || t == QEH_DT_FLOAT32) {
                    double d = nd.lit_f64;
                    if (t == QEH_DT_FLOAT32) d = (double)(float)d;
                    in.imm = __builtin_bit_cast(int64_t, d);
                } else if (t == QEH_DT_INT32) {
                    in.imm = (int64_t)(int32_t)nd.lit_i64;
                } else if (t == QEH_DT_BOOL) {
                    in.imm = nd.lit_i64 != 0;
                } else {
                    in.imm = nd.lit_i64;
                }
                QEH_TRY(emit(in));
                ty.push_back(t);
                break;
            }
            case QEH_EX_UNARY: {
                if (ty.empty()) return fail(QEH_E_INVALID, "malformed expression (unary)");
                int t = ty.back();
                int d = (int)ty.size() - 1;
                if (nd.op == QEH_UOP_NOT) {
                    if (t != QEH_DT_BOOL)
                        return fail(QEH_E_TYPE, "NOT operator requires boolean array");
                    in.op = D_NOT;
                } else if (nd.op == QEH_UOP_MINUS) {
                    if (!is_num(t)) return fail(QEH_E_TYPE, "Unsupported type for negation");
                    in.op = D_NEG;
                } else {
                    return fail(QEH_E_INVALID, "unknown unary operator");
                }
                in.t = (uint8_t)t;
                in.dst = (uint8_t)d;
                in.a = (uint8_t)d;
                QEH_TRY(emit(in));
                break;
            }
            case QEH_EX_BINARY: {
                if (ty.size() < 2) return fail(QEH_E_INVALID, "malformed expression (binary)");
                int rt = ty.back();
                int lt = ty[ty.size() - 2];
                int dl = (int)ty.size() - 2, dr = (int)ty.size() - 1;
                in.dst = (uint8_t)dl;
                in.a = (uint8_t)dl;
                in.b = (uint8_t)dr;
                int res;
                switch (nd.op) {
                    case QEH_OP_ADD: case QEH_OP_SUB: case QEH_OP_MUL: case QEH_OP_DIV: {
                        static const char *nm[] = {"addition", "subtraction", "multiplication", "division"};
                        if (lt != rt || !is_num(lt))
                            return fail(QEH_E_TYPE, std::string("Unsupported types for ") + nm[nd.op]);
                        in.op = (uint8_t)(D_ADD + nd.op);
                        in.t = (uint8_t)lt;
                        res = lt;
                        break;
                    }
                    case QEH_OP_MOD: {
                        if (lt != rt || !is_int(lt))
                            return fail(QEH_E_TYPE, "Modulo operation requires integer arrays");
                        in.op = D_MOD;
                        in.t = (uint8_t)lt;
                        res = lt;
                        break;
                    }
                    case QEH_OP_EQ: case QEH_OP_NEQ: case QEH_OP_LT: case QEH_OP_LTE:
                    case QEH_OP_GT: case QEH_OP_GTE: {
                        int cl, cr;
                        coerce(lt, rt, &cl, &cr);
                        if (cl != cr || cl == QEH_DT_NULL)
                            return fail(QEH_E_TYPE, std::string("Invalid argument error: Invalid comparison operation: ") +
                                                        dt_name(cl) + " " + cmp_sym(nd.op) + " " + dt_name(cr));
                        if (cl == QEH_DT_FLOAT64 && lt != QEH_DT_FLOAT64 && lt != QEH_DT_FLOAT32) {
                            DevInstr c{};
                            c.op = D_TOF64; c.t = (uint8_t)lt; c.dst = (uint8_t)dl; c.a = (uint8_t)dl;
                            QEH_TRY(emit(c));
                        }
                        if (cr == QEH_DT_FLOAT64 && rt != QEH_DT_FLOAT64 && rt != QEH_DT_FLOAT32) {
                            DevInstr c{};
                            c.op = D_TOF64; c.t = (uint8_t)rt; c.dst = (uint8_t)dr; c.a = (uint8_t)dr;
                            QEH_TRY(emit(c));
                        }
                        in.op = (uint8_t)(D_EQ + (nd.op - QEH_OP_EQ));
                        // Float32 stays Float32 only when both sides are Float32; slots hold
                        // exact doubles, so compare as Float64 either way.
                        int ct = cl == QEH_DT_FLOAT32 ? QEH_DT_FLOAT64 : cl;
                        in.t = (uint8_t)ct;
                        res = QEH_DT_BOOL;
                        break;
                    }
                    case QEH_OP_AND: case QEH_OP_OR: {
                        if (lt != QEH_DT_BOOL || rt != QEH_DT_BOOL)
                            return fail(QEH_E_TYPE, nd.op == QEH_OP_AND ? "AND requires boolean arrays"
                                                                         : "OR requires boolean arrays");
                        in.op = nd.op == QEH_OP_AND ? D_AND : D_OR;
                        in.t = QEH_DT_BOOL;
                        res = QEH_DT_BOOL;
                        break;
                    }
                    default:
                        return fail(QEH_E_UNSUPPORTED, "binary operator not supported on the device");
                }
                QEH_TRY(emit(in));
                ty.pop_back();
                ty.back() = res;
                break;
            }
            default:
                return fail(QEH_E_UNSUPPORTED, "expression node kind not supported on the device");
        }
    }
    if (ty.size() != 1) return fail(QEH_E_INVALID, "malformed expression (stack)");
    out->result_type = ty[0];
    return QEH_OK;
}

// Leaf `Column cmp Literal` (or `Literal cmp Column`) starting at node range
// [lo, hi); returns true and fills `t`.
static bool leaf_term(const qeh_expr_node *nd, int cnt, const int32_t *dtypes, int n_cols, PredTerm *t) {
    if (cnt != 3 || nd[2].kind != QEH_EX_BINARY) return false;
    int op = nd[2].op;
    if (op < QEH_OP_EQ || op > QEH_OP_GTE) return false;
    const qeh_expr_node *c, *l;
    bool flipped;
    if (nd[0].kind == QEH_EX_COLUMN && nd[1].kind == QEH_EX_LITERAL) { c = &nd[0]; l = &nd[1]; flipped = false; }
    else if (nd[1].kind == QEH_EX_COLUMN && nd[0].kind == QEH_EX_LITERAL) { c = &nd[1]; l = &nd[0]; flipped = true; }
    else return false;
    if (c->index < 0 || c->index >= n_cols) return false;
    if (l->lit_is_null) return false;
    int ct = dtypes[c->index], ltp = l->lit_dtype;
    int cl, cr;
    coerce(flipped ? ltp : ct, flipped ? ct : ltp, &cl, &cr);
    if (cl != cr) return false;
    int cmpt = cl == QEH_DT_FLOAT32 ? QEH_DT_FLOAT64 : cl;
    if (cmpt != QEH_DT_INT64 && cmpt != QEH_DT_FLOAT64 && cmpt != QEH_DT_INT32 && cmpt != QEH_DT_BOOL) return false;
    if (cmpt == QEH_DT_INT32) cmpt = QEH_DT_INT64;  // int32 vs int32: sign-extended compare is identical
    int dop = D_EQ + (op - QEH_OP_EQ);
    if (flipped) {  // lit OP col  ==  col OP' lit
        switch (dop) {
            case D_LT: dop = D_GT; break;
            case D_LE: dop = D_GE; break;
            case D_GT: dop = D_LT; break;
            case D_GE: dop = D_LE; break;
            default: break;
        }
    }
    t->col = c->index;
    t->ctype = cmpt;
    t->op = dop;
    if (cmpt == QEH_DT_FLOAT64) {
        double d = (ltp == QEH_DT_FLOAT64 || ltp == QEH_DT_FLOAT32) ? l->lit_f64 : (double)l->lit_i64;
        if (ltp == QEH_DT_FLOAT32) d = (double)(float)d;
        t->lit = f64_order_key(d);
    } else if (cmpt == QEH_DT_BOOL) {
        t->lit = l->lit_i64 != 0;
    } else {
        t->lit = ltp == QEH_DT_INT32 ? (int64_t)(int32_t)l->lit_i64 : l->lit_i64;
    }
    return true;
}

bool lower_to_terms(const qeh_expr *e, const int32_t *dtypes, int n_cols, PredTerms *out) {
    out->n = 0;
    out->is_or = 0;
    if (!e || e->n_nodes <= 0) return false;
    // Split the postfix sequence into 3-node leaves joined by one kind of
    // connective.  Left-deep ((a AND b) AND c) and right-deep forms both occur;
    // walk the postfix with a stack of (start,len) fragments.
    struct Frag { int lo, len; bool leaf; };
    std::vector<Frag> st;
    std::vector<PredTerm> terms;
    int conn = -1;
    for (int i = 0; i < e->n_nodes; ++i) {
        const qeh_expr_node &nd = e->nodes[i];
        if (nd.kind == QEH_EX_COLUMN || nd.kind == QEH_EX_LITERAL) {
            st.push_back({i, 1, false});
        } else if (nd.kind == QEH_EX_BINARY && nd.op >= QEH_OP_EQ && nd.op <= QEH_OP_GTE) {
            if (st.size() < 2) return false;
            Frag r = st.back(); st.pop_back();
            Frag l = st.back(); st.pop_back();
            if (l.len != 1 || r.len != 1 || l.leaf || r.leaf) return false;
            PredTerm t;
            if (!leaf_term(&e->nodes[l.lo], 3, dtypes, n_cols, &t)) return false;
            if ((int)terms.size() >= kMaxTerms) return false;
            terms.push_back(t);
            st.push_back({l.lo, 3, true});
        } else if (nd.kind == QEH_EX_BINARY && (nd.op == QEH_OP_AND || nd.op == QEH_OP_OR)) {
            if (st.size() < 2) return false;
            int c = nd.op == QEH_OP_AND ? 0 : 1;
            if (conn >= 0 && conn != c) return false;
            conn = c;
            Frag r = st.back(); st.pop_back();
            Frag l = st.back(); st.pop_back();
            if (!l.leaf || !r.leaf) return false;
            st.push_back({l.lo, l.len + r.len + 1, true});
        } else {
            return false;
        }
    }
    if (st.size() != 1 || !st[0].leaf || terms.empty()) return false;
    out->n = (int)terms.size();
    out->is_or = conn == 1;
    for (size_t i = 0; i < terms.size(); ++i) out->t[i] = terms[i];
    return true;
}

}  // namespace qeh

extern "C" int qeh_expr_type(const int32_t *col_dtypes, int n_cols, const qeh_expr *expr,
                             int32_t *out_dtype) {
    qeh::DevProgram p;
    int s = qeh::compile_expr(expr, col_dtypes, n_cols, &p);
    if (s != QEH_OK) return s;
    if (out_dtype) *out_dtype = p.result_type;
    return QEH_OK;
}
