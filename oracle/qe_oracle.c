/*
 * qe_oracle.c — CPU ORACLE for the qeh hot path.  TEST INFRASTRUCTURE ONLY:
 * loaded by tests/ (checker), __graft_entry__.smoke() (checker) and bench.py's
 * cpu_baseline leg.  Nothing in query-engine_amd/ links or calls it.
 *
 * Restates crates/query-executor/src/{executor.rs,operators.rs} of
 * AarambhDevHub/query-engine column-at-a-time, the way the reference
 * evaluates (each expression node materialises a full array):
 *   evaluate_expr            operators.rs:13-62        -> qo_eval
 *   create_literal_array     operators.rs:322-347      -> lit_array
 *   evaluate_unary_op        operators.rs:349-380      -> unary
 *   evaluate_binary_op       operators.rs:382-612      -> binary
 *   coerce_numeric_types     operators.rs:616-675      -> coerce
 *   cast_to_float64          operators.rs:678-709      -> to_f64
 *   modulo_op                operators.rs:711-743      -> binary (MOD)
 *   evaluate_aggregate       operators.rs:745-848      -> finish_group
 *   execute_filter           executor.rs:131-155       -> qo_filter
 *   execute_aggregate        executor.rs:157-190       -> qo_hash_aggregate (global part)
 * and the intended semantics of SURVEY.md §8.0 for the stubbed operators:
 *   GROUP BY (executor.rs:189 returns nothing)        -> qo_hash_aggregate (grouped)
 *   INNER JOIN (executor.rs:363-381, `on` ignored)    -> qo_hash_join_inner
 *   Sort (identity, executor.rs:290-297)              -> qo_sort_indices
 *   ROW_NUMBER (docs/WINDOW_FUNCTIONS.md:44-65)       -> qo_row_number
 *   RANK ... LAST_VALUE (docs/WINDOW_FUNCTIONS.md:67-205) -> qo_window
 * arrow-rs library semantics restated: cmp kernels are null-propagating and
 * compare floats by IEEE totalOrder; and/or are the non-Kleene variants (NULL
 * if either side is NULL); integer add/sub/mul/div are checked (error on
 * overflow / division by zero, only for valid slots); float arithmetic is IEEE;
 * filter drops NULL predicate rows; sum wraps for integers.
 */
#define _GNU_SOURCE
#include "qe_oracle.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static __thread char g_err[512];

static int err(int status, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return status;
}

const char *qo_last_error(void) { return g_err; }
void qo_free(void *p) { free(p); }
void qo_col_free(qo_col *c) {
    if (!c) return;
    free(c->values);
    free(c->valid);
    memset(c, 0, sizeof *c);
}

/* ---- synthetic data (must equal query-engine_amd/csrc/k_datagen.hip) ------ */
static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void qo_generate(int kind, uint64_t seed, uint64_t col_id, int64_t row0, int64_t n, int64_t modulus,
                 int64_t lo, void *out) {
    const uint64_t base = seed ^ (col_id << 56);
#pragma omp parallel for schedule(static, 1 << 16) if (n > (1 << 22))
    for (int64_t i = 0; i < n; ++i) {
        uint64_t row = (uint64_t)(row0 + i);
        if (kind == QEH_GEN_UNIFORM_MOD)
            ((int64_t *)out)[i] = (int64_t)(splitmix64(base + row) % (uint64_t)modulus) + lo;
        else if (kind == QEH_GEN_UNIT_F64)
            ((double *)out)[i] = (double)(splitmix64(base + row) >> 11) * 0x1.0p-53;
        else if (kind == QEH_GEN_SPARSE_KEY)
            ((int64_t *)out)[i] = (int64_t)splitmix64((modulus > 0 ? splitmix64(base + row) % (uint64_t)modulus : row) ^
                                                      (seed * 0xD6E8FEB86659FD93ull));
        else
            ((int64_t *)out)[i] = (int64_t)((row * 0x9E3779B1ull + col_id) % (uint64_t)modulus) + lo;
    }
}

/* ---- arrays ---------------------------------------------------------------- */
typedef struct {
    int t;        /* dtype */
    int64_t n;
    int64_t *i;   /* BOOL/INT32/INT64/UINT32 (ints sign-extended) */
    double *f;    /* FLOAT32/FLOAT64 (float32 values exact) */
    uint8_t *v;   /* validity, always materialised */
} arr;

static void arr_free(arr *a) {
    free(a->i);
    free(a->f);
    free(a->v);
    memset(a, 0, sizeof *a);
}

static int is_float(int t) { return t == QEH_DT_FLOAT32 || t == QEH_DT_FLOAT64; }
static int is_intt(int t) { return t == QEH_DT_INT32 || t == QEH_DT_INT64; }
static int is_num(int t) { return is_float(t) || is_intt(t); }

static const char *dt_name(int t) {
    switch (t) {
        case QEH_DT_NULL: return "Null";
        case QEH_DT_BOOL: return "Boolean";
        case QEH_DT_INT32: return "Int32";
        case QEH_DT_INT64: return "Int64";
        case QEH_DT_FLOAT32: return "Float32";
        case QEH_DT_FLOAT64: return "Float64";
        case QEH_DT_UTF8: return "Utf8";
        default: return "UInt32";
    }
}

static int arr_alloc(arr *a, int t, int64_t n) {
    memset(a, 0, sizeof *a);
    a->t = t;
    a->n = n;
    size_t m = (size_t)(n > 0 ? n : 1);
    a->v = calloc(m, 1);
    if (is_float(t)) a->f = calloc(m, sizeof(double));
    else a->i = calloc(m, sizeof(int64_t));
    return QEH_OK;
}

static int col_to_arr(const qo_col *c, arr *a) {
    arr_alloc(a, c->dtype, c->length);
    for (int64_t r = 0; r < c->length; ++r) {
        a->v[r] = c->valid ? c->valid[r] : 1;
        switch (c->dtype) {
            case QEH_DT_BOOL: a->i[r] = ((const uint8_t *)c->values)[r] != 0; break;
            case QEH_DT_INT32: a->i[r] = ((const int32_t *)c->values)[r]; break;
            case QEH_DT_UINT32: a->i[r] = ((const uint32_t *)c->values)[r]; break;
            case QEH_DT_INT64: a->i[r] = ((const int64_t *)c->values)[r]; break;
            case QEH_DT_FLOAT32: a->f[r] = ((const float *)c->values)[r]; break;
            case QEH_DT_FLOAT64: a->f[r] = ((const double *)c->values)[r]; break;
            default: arr_free(a); return err(QEH_E_UNSUPPORTED, "oracle: unsupported column type %s", dt_name(c->dtype));
        }
    }
    return QEH_OK;
}

static size_t esize(int t) {
    switch (t) {
        case QEH_DT_BOOL: return 1;
        case QEH_DT_INT32: case QEH_DT_FLOAT32: case QEH_DT_UINT32: return 4;
        default: return 8;
    }
}

/* take ownership of nothing; writes a fresh qo_col with rows `idx` (or all) */
static void arr_to_col(const arr *a, const int64_t *idx, int64_t m, qo_col *out) {
    memset(out, 0, sizeof *out);
    out->dtype = a->t == QEH_DT_NULL ? QEH_DT_INT64 : a->t;
    out->length = m;
    size_t es = esize(out->dtype);
    out->values = calloc((size_t)(m > 0 ? m : 1), es);
    out->valid = calloc((size_t)(m > 0 ? m : 1), 1);
    for (int64_t k = 0; k < m; ++k) {
        int64_t r = idx ? idx[k] : k;
        if (r < 0) continue; /* outer-join filler row: NULL */
        out->valid[k] = a->v[r];
        switch (out->dtype) {
            case QEH_DT_BOOL: ((uint8_t *)out->values)[k] = (uint8_t)(a->i[r] & 1); break;
            case QEH_DT_INT32: ((int32_t *)out->values)[k] = (int32_t)a->i[r]; break;
            case QEH_DT_UINT32: ((uint32_t *)out->values)[k] = (uint32_t)a->i[r]; break;
            case QEH_DT_INT64: ((int64_t *)out->values)[k] = a->i[r]; break;
            case QEH_DT_FLOAT32: ((float *)out->values)[k] = (float)a->f[r]; break;
            default: ((double *)out->values)[k] = a->f[r]; break;
        }
    }
}

/* create_literal_array (operators.rs:322-347): broadcast to n rows; typed
 * None and Null become a NullArray. */
static void lit_array(const qeh_expr_node *nd, int64_t n, arr *a) {
    int t = nd->lit_is_null ? QEH_DT_NULL : nd->lit_dtype;
    arr_alloc(a, t, n);
    for (int64_t r = 0; r < n; ++r) {
        if (t == QEH_DT_NULL) continue;
        a->v[r] = 1;
        if (t == QEH_DT_FLOAT64) a->f[r] = nd->lit_f64;
        else if (t == QEH_DT_FLOAT32) a->f[r] = (float)nd->lit_f64;
        else if (t == QEH_DT_INT32) a->i[r] = (int32_t)nd->lit_i64;
        else if (t == QEH_DT_BOOL) a->i[r] = nd->lit_i64 != 0;
        else a->i[r] = nd->lit_i64;
    }
}

/* cast_to_float64 (operators.rs:678-709) and the int->f64 casts of coerce */
static void to_f64(arr *a) {
    if (a->t == QEH_DT_FLOAT64) return;
    if (a->t == QEH_DT_FLOAT32) { a->t = QEH_DT_FLOAT64; return; }
    if (!is_intt(a->t)) return;
    a->f = calloc((size_t)(a->n > 0 ? a->n : 1), sizeof(double));
    for (int64_t r = 0; r < a->n; ++r) a->f[r] = (double)a->i[r];
    free(a->i);
    a->i = NULL;
    a->t = QEH_DT_FLOAT64;
}

/* coerce_numeric_types (operators.rs:616-675) */
static void coerce(arr *l, arr *r) {
    if (l->t == r->t) return;
    if (l->t == QEH_DT_FLOAT64 && is_intt(r->t)) { to_f64(r); return; }
    if (r->t == QEH_DT_FLOAT64 && is_intt(l->t)) { to_f64(l); return; }
    if (l->t == QEH_DT_FLOAT32 || r->t == QEH_DT_FLOAT32) { to_f64(l); to_f64(r); return; }
    if (l->t == QEH_DT_INT64 && r->t == QEH_DT_INT32) { r->t = QEH_DT_INT64; return; }
    if (r->t == QEH_DT_INT64 && l->t == QEH_DT_INT32) { l->t = QEH_DT_INT64; return; }
}

/* IEEE totalOrder as signed order (arrow-rs float comparisons) */
static int64_t tkey(double d) {
    int64_t b;
    memcpy(&b, &d, 8);
    return b ^ (int64_t)(((uint64_t)(b >> 63)) >> 1);
}

static int cmp_res(int op, int c) { /* c = sign(a - b) */
    switch (op) {
        case QEH_OP_EQ: return c == 0;
        case QEH_OP_NEQ: return c != 0;
        case QEH_OP_LT: return c < 0;
        case QEH_OP_LTE: return c <= 0;
        case QEH_OP_GT: return c > 0;
        default: return c >= 0;
    }
}

static const char *cmp_sym(int op) {
    static const char *s[] = {"==", "!=", "<", "<=", ">", ">="};
    return s[op - QEH_OP_EQ];
}

static int unary(int op, arr *a) {
    if (op == QEH_UOP_NOT) {
        if (a->t != QEH_DT_BOOL) return err(QEH_E_TYPE, "NOT operator requires boolean array");
        for (int64_t r = 0; r < a->n; ++r) a->i[r] = !a->i[r];
        return QEH_OK;
    }
    if (!is_num(a->t)) return err(QEH_E_TYPE, "Unsupported type for negation");
    for (int64_t r = 0; r < a->n; ++r) {
        if (is_float(a->t)) a->f[r] = -a->f[r];
        else if (a->t == QEH_DT_INT32) a->i[r] = (int32_t)(0u - (uint32_t)a->i[r]); /* release-mode wrap */
        else a->i[r] = (int64_t)(0ull - (uint64_t)a->i[r]);
    }
    return QEH_OK;
}

/* evaluate_binary_op (operators.rs:382-612); result replaces *l */
static int binary(int op, arr *l, arr *r) {
    const int64_t n = l->n;
    if (op <= QEH_OP_DIV) {
        static const char *nm[] = {"addition", "subtraction", "multiplication", "division"};
        if (l->t != r->t || !is_num(l->t)) return err(QEH_E_TYPE, "Unsupported types for %s", nm[op]);
        for (int64_t k = 0; k < n; ++k) {
            int valid = l->v[k] && r->v[k];
            l->v[k] = (uint8_t)valid;
            if (is_float(l->t)) {
                double a = l->f[k], b = r->f[k], z;
                if (l->t == QEH_DT_FLOAT32) {
                    float af = (float)a, bf = (float)b, zf;
                    zf = op == QEH_OP_ADD ? af + bf : op == QEH_OP_SUB ? af - bf : op == QEH_OP_MUL ? af * bf : af / bf;
                    z = zf;
                } else {
                    z = op == QEH_OP_ADD ? a + b : op == QEH_OP_SUB ? a - b : op == QEH_OP_MUL ? a * b : a / b;
                }
                l->f[k] = z;
                continue;
            }
            int64_t a = l->i[k], b = r->i[k], z = 0;
            int ovf = 0;
            const int i32 = l->t == QEH_DT_INT32;
            const int64_t mn = i32 ? INT32_MIN : INT64_MIN;
            if (op == QEH_OP_ADD) ovf = __builtin_add_overflow(a, b, &z);
            else if (op == QEH_OP_SUB) ovf = __builtin_sub_overflow(a, b, &z);
            else if (op == QEH_OP_MUL) ovf = __builtin_mul_overflow(a, b, &z);
            else {
                if (b == 0) {
                    if (valid) return err(QEH_E_DIV0, "Arrow error: Divide by zero error");
                } else if (b == -1 && a == mn) ovf = 1;
                else z = a / b;
            }
            if (i32 && (z < INT32_MIN || z > INT32_MAX)) ovf = 1;
            if (ovf && valid) return err(QEH_E_OVERFLOW, "Arrow error: Arithmetic overflow");
            l->i[k] = z;
        }
        return QEH_OK;
    }
    if (op == QEH_OP_MOD) {
        if (l->t != r->t || !is_intt(l->t)) return err(QEH_E_TYPE, "Modulo operation requires integer arrays");
        const int64_t mn = l->t == QEH_DT_INT32 ? INT32_MIN : INT64_MIN;
        for (int64_t k = 0; k < n; ++k) {
            int valid = l->v[k] && r->v[k] && r->i[k] != 0;
            l->v[k] = (uint8_t)valid;
            if (!valid) { l->i[k] = 0; continue; }
            if (r->i[k] == -1 && l->i[k] == mn)
                return err(QEH_E_OVERFLOW, "attempt to calculate the remainder with overflow (the reference aborts here, operators.rs:720)");
            l->i[k] = l->i[k] % r->i[k];
        }
        return QEH_OK;
    }
    if (op >= QEH_OP_EQ && op <= QEH_OP_GTE) {
        coerce(l, r);
        if (l->t != r->t || l->t == QEH_DT_NULL)
            return err(QEH_E_TYPE, "Invalid argument error: Invalid comparison operation: %s %s %s", dt_name(l->t),
                       cmp_sym(op), dt_name(r->t));
        int64_t *res = calloc((size_t)(n > 0 ? n : 1), sizeof(int64_t));
        for (int64_t k = 0; k < n; ++k) {
            l->v[k] = l->v[k] && r->v[k];
            int c;
            if (is_float(l->t)) {
                int64_t a = tkey(l->f[k]), b = tkey(r->f[k]);
                c = (a > b) - (a < b);
            } else {
                int64_t a = l->i[k], b = r->i[k];
                c = (a > b) - (a < b);
            }
            res[k] = cmp_res(op, c);
        }
        free(l->i);
        free(l->f);
        l->f = NULL;
        l->i = res;
        l->t = QEH_DT_BOOL;
        return QEH_OK;
    }
    if (op == QEH_OP_AND || op == QEH_OP_OR) {
        if (l->t != QEH_DT_BOOL || r->t != QEH_DT_BOOL)
            return err(QEH_E_TYPE, op == QEH_OP_AND ? "AND requires boolean arrays" : "OR requires boolean arrays");
        for (int64_t k = 0; k < n; ++k) {
            l->v[k] = l->v[k] && r->v[k]; /* arrow compute::and / or: NULL if either side NULL */
            l->i[k] = op == QEH_OP_AND ? (l->i[k] & r->i[k]) : (l->i[k] | r->i[k]);
        }
        return QEH_OK;
    }
    return err(QEH_E_UNSUPPORTED, "oracle: unsupported binary operator %d", op);
}

static int eval_arr(const qo_col *cols, int n_cols, int64_t n_rows, const qeh_expr_node *nodes, int n_nodes, arr *out) {
    arr *st = calloc((size_t)(n_nodes > 0 ? n_nodes : 1), sizeof(arr));
    int sp = 0, s = QEH_OK;
    for (int i = 0; i < n_nodes && s == QEH_OK; ++i) {
        const qeh_expr_node *nd = &nodes[i];
        switch (nd->kind) {
            case QEH_EX_COLUMN:
                if (nd->index < 0 || nd->index >= n_cols) {
                    s = err(QEH_E_INVALID, "Column index %d out of bounds", nd->index);
                    break;
                }
                s = col_to_arr(&cols[nd->index], &st[sp]);
                if (s == QEH_OK) ++sp;
                break;
            case QEH_EX_LITERAL: lit_array(nd, n_rows, &st[sp++]); break;
            case QEH_EX_UNARY:
                if (sp < 1) { s = err(QEH_E_INVALID, "malformed expression"); break; }
                s = unary(nd->op, &st[sp - 1]);
                break;
            case QEH_EX_BINARY:
                if (sp < 2) { s = err(QEH_E_INVALID, "malformed expression"); break; }
                s = binary(nd->op, &st[sp - 2], &st[sp - 1]);
                arr_free(&st[sp - 1]);
                --sp;
                break;
            default: s = err(QEH_E_UNSUPPORTED, "oracle: unsupported node kind"); break;
        }
    }
    if (s == QEH_OK && sp != 1) s = err(QEH_E_INVALID, "malformed expression");
    if (s == QEH_OK) {
        *out = st[0];
        sp = 0;
    }
    for (int k = 0; k < sp; ++k) arr_free(&st[k]);
    free(st);
    return s;
}

int qo_eval(const qo_col *cols, int n_cols, int64_t n_rows, const qeh_expr_node *nodes, int n_nodes, qo_col *out) {
    arr a;
    int s = eval_arr(cols, n_cols, n_rows, nodes, n_nodes, &a);
    if (s != QEH_OK) return s;
    arr_to_col(&a, NULL, a.n, out);
    arr_free(&a);
    return QEH_OK;
}

/* execute_filter (executor.rs:131-155) + arrow filter_record_batch */
int qo_filter(const qo_col *cols, int n_cols, const qeh_expr_node *nodes, int n_nodes, const int32_t *out_idx,
              int n_out, qo_col *out, int64_t *out_rows) {
    int64_t n = n_cols > 0 ? cols[0].length : 0;
    arr p;
    int s = eval_arr(cols, n_cols, n, nodes, n_nodes, &p);
    if (s != QEH_OK) return s;
    if (p.t != QEH_DT_BOOL) {
        arr_free(&p);
        return err(QEH_E_TYPE, "Filter predicate must return boolean");
    }
    int64_t *idx = malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    int64_t m = 0;
    for (int64_t r = 0; r < n; ++r)
        if (p.v[r] && p.i[r]) idx[m++] = r; /* NULL -> dropped */
    arr_free(&p);
    for (int j = 0; j < n_out; ++j) {
        arr a;
        s = col_to_arr(&cols[out_idx[j]], &a);
        if (s != QEH_OK) break;
        arr_to_col(&a, idx, m, &out[j]);
        arr_free(&a);
    }
    free(idx);
    *out_rows = m;
    return s;
}

/* ---- hashing of key tuples ----------------------------------------------- */
static uint64_t mix(uint64_t k);

/* partition.rs:151-212: per row, compute_row_hash (:292-316, NULL cells skip the hasher) and push
 * the row onto partition (hash % n); the partitions are then taken in order (partition-major,
 * input order inside each).  Hash: the device's (k_hash_ids_multi in k_sort.hip). */
int qo_partition_hash(const qo_col *keys, int n_keys, int n_parts, int64_t *counts, uint32_t *out_perm) {
    if (n_keys < 1 || n_parts < 1) return err(QEH_E_INVALID, "qo_partition_hash: bad argument");
    const int64_t n = keys[0].length;
    for (int j = 0; j < n_keys; ++j)
        if (keys[j].dtype != QEH_DT_INT64 && keys[j].dtype != QEH_DT_INT32)
            return err(QEH_E_UNSUPPORTED, "qo_partition_hash: Int32 / Int64 keys only");
    uint32_t *part = malloc((size_t)(n > 0 ? n : 1) * sizeof(uint32_t));
    for (int p = 0; p < n_parts; ++p) counts[p] = 0;
    for (int64_t r = 0; r < n; ++r) {
        uint64_t h = 0x9E3779B97F4A7C15ull;
        for (int j = 0; j < n_keys; ++j) {
            const qo_col *c = &keys[j];
            if (c->valid && !c->valid[r]) continue;
            uint64_t v = c->dtype == QEH_DT_INT64 ? (uint64_t)((const int64_t *)c->values)[r]
                                                  : (uint64_t)(int64_t)((const int32_t *)c->values)[r];
            h = mix(h ^ (mix(v) + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2)));
        }
        part[r] = (uint32_t)(h % (uint64_t)n_parts);
        counts[part[r]]++;
    }
    int64_t *next = malloc((size_t)n_parts * sizeof(int64_t));
    int64_t acc = 0;
    for (int p = 0; p < n_parts; ++p) next[p] = acc, acc += counts[p];
    for (int64_t r = 0; r < n; ++r) out_perm[next[part[r]]++] = (uint32_t)r;
    free(next);
    free(part);
    return QEH_OK;
}

static uint64_t mix(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

static int64_t key_bits(const arr *a, int64_t r) {
    if (is_float(a->t)) return tkey(a->f[r]); /* equality of bits == equality of totalOrder keys */
    return a->i[r];
}

static uint64_t tuple_hash(const arr *k, int nk, int64_t r) {
    uint64_t h = 0x12345;
    for (int j = 0; j < nk; ++j) h = mix(h ^ (uint64_t)(k[j].v[r] ? key_bits(&k[j], r) : 0x6E756C6C) ^ ((uint64_t)k[j].v[r] << 40));
    return h;
}

static int tuple_eq(const arr *ka, int64_t a, const arr *kb, int64_t b, int nk) {
    for (int j = 0; j < nk; ++j) {
        if (ka[j].v[a] != kb[j].v[b]) return 0;
        if (ka[j].v[a] && key_bits(&ka[j], a) != key_bits(&kb[j], b)) return 0;
    }
    return 1;
}

typedef struct {
    uint64_t cap;
    int64_t *slot;  /* group index or -1 */
} gmap;

/* ---- aggregate states (evaluate_aggregate, operators.rs:745-848) --------- */
typedef struct {
    uint64_t isum;  /* wrapping */
    double fsum;
    float f32sum;   /* compute::sum(Float32Array) accumulates in f32 */
    int64_t cnt;    /* non-null */
    int64_t imin, imax;
    double fmin, fmax;
} astate;

static void agg_update(astate *s, const arr *in, int64_t r) {
    if (!in->v[r]) return;
    s->cnt++;
    if (is_float(in->t)) {
        double x = in->f[r];
        s->fsum += x;
        s->f32sum += (float)x;
        if (s->cnt == 1 || tkey(x) < tkey(s->fmin)) s->fmin = x;
        if (s->cnt == 1 || tkey(x) > tkey(s->fmax)) s->fmax = x;
    } else {
        int64_t x = in->i[r];
        s->isum += (uint64_t)x;
        if (s->cnt == 1 || x < s->imin) s->imin = x;
        if (s->cnt == 1 || x > s->imax) s->imax = x;
    }
}

static int agg_out_type(int func, int t) {
    if (func == QEH_AGG_COUNT) return QEH_DT_INT64;
    if (func == QEH_AGG_AVG) return QEH_DT_FLOAT64;
    if (func == QEH_AGG_SUM) return is_float(t) ? QEH_DT_FLOAT64 : QEH_DT_INT64;
    return t;
}

static void finish_group(const astate *s, int func, int t, arr *out, int64_t g) {
    if (func == QEH_AGG_COUNT) { out->v[g] = 1; out->i[g] = s->cnt; return; }
    out->v[g] = s->cnt > 0;
    if (!out->v[g]) return;
    switch (func) {
        case QEH_AGG_SUM:
            if (t == QEH_DT_FLOAT64) out->f[g] = s->fsum;
            else if (t == QEH_DT_FLOAT32) out->f[g] = (double)s->f32sum;
            else if (t == QEH_DT_INT32) out->i[g] = (int64_t)(int32_t)(uint32_t)s->isum;
            else out->i[g] = (int64_t)s->isum;
            break;
        case QEH_AGG_AVG: {
            double sum = t == QEH_DT_FLOAT64 ? s->fsum : t == QEH_DT_FLOAT32 ? (double)s->f32sum
                       : t == QEH_DT_INT32 ? (double)(int32_t)(uint32_t)s->isum : (double)(int64_t)s->isum;
            out->f[g] = sum / (double)s->cnt;
            break;
        }
        case QEH_AGG_MIN:
            if (is_float(t)) out->f[g] = s->fmin; else out->i[g] = s->imin;
            break;
        default:
            if (is_float(t)) out->f[g] = s->fmax; else out->i[g] = s->imax;
            break;
    }
}

/* Group rows by `keys` (first-appearance order). rows_sel: optional mask. */
typedef struct {
    int64_t groups;
    int64_t *rep;      /* representative row per group */
    int64_t *gid;      /* per row, -1 if not selected */
} grouping;

static void group_rows(const arr *keys, int nk, int64_t n, const uint8_t *sel, grouping *g) {
    uint64_t cap = 1024;
    while (cap < (uint64_t)n * 2) cap <<= 1;
    int64_t *slot = malloc(cap * sizeof(int64_t));
    for (uint64_t i = 0; i < cap; ++i) slot[i] = -1;
    g->groups = 0;
    g->rep = malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    g->gid = malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    for (int64_t r = 0; r < n; ++r) {
        if (sel && !sel[r]) { g->gid[r] = -1; continue; }
        uint64_t h = tuple_hash(keys, nk, r) & (cap - 1);
        for (;;) {
            if (slot[h] < 0) {
                slot[h] = g->groups;
                g->rep[g->groups] = r;
                g->gid[r] = g->groups++;
                break;
            }
            if (tuple_eq(keys, g->rep[slot[h]], keys, r, nk)) { g->gid[r] = slot[h]; break; }
            h = (h + 1) & (cap - 1);
        }
    }
    free(slot);
}

static int emit_groups(const arr *keys, int nk, const arr *inputs, const qeh_agg *aggs, int n_aggs, int64_t G,
                       const int64_t *rep, const astate *st, qo_col *out_keys, qo_col *out_aggs) {
    for (int j = 0; j < nk; ++j) arr_to_col(&keys[j], rep, G, &out_keys[j]);
    for (int a = 0; a < n_aggs; ++a) {
        int t = inputs[aggs[a].column].t;
        arr o;
        arr_alloc(&o, agg_out_type(aggs[a].func, t), G);
        for (int64_t g = 0; g < G; ++g) finish_group(&st[g * n_aggs + a], aggs[a].func, t, &o, g);
        arr_to_col(&o, NULL, G, &out_aggs[a]);
        arr_free(&o);
    }
    return QEH_OK;
}

static int check_agg_types(const arr *inputs, int n_inputs, const qeh_agg *aggs, int n_aggs) {
    static const char *nm[] = {"COUNT", "SUM", "AVG", "MIN", "MAX"};
    for (int a = 0; a < n_aggs; ++a) {
        if (aggs[a].column < 0 || aggs[a].column >= n_inputs) return err(QEH_E_INVALID, "aggregate input index out of range");
        if (aggs[a].func != QEH_AGG_COUNT && !is_num(inputs[aggs[a].column].t))
            return err(QEH_E_TYPE, "Unsupported type for %s", nm[aggs[a].func]);
    }
    return QEH_OK;
}

/* execute_aggregate (executor.rs:157-190): global part literal; GROUP BY intended */
int qo_hash_aggregate(const qo_col *keys, int n_keys, const qo_col *inputs, int n_inputs, const qeh_agg *aggs,
                      int n_aggs, int64_t input_batches, qo_col *out_keys, qo_col *out_aggs, int64_t *out_groups) {
    *out_groups = 0;
    if (n_aggs == 0) return QEH_OK;                       /* executor.rs:163-165 */
    if (n_keys == 0 && input_batches == 0) return QEH_OK; /* executor.rs:178-186 */
    int64_t n = n_inputs > 0 ? inputs[0].length : (n_keys > 0 ? keys[0].length : 0);
    arr *ka = calloc((size_t)n_keys + 1, sizeof(arr));
    arr *ia = calloc((size_t)n_inputs + 1, sizeof(arr));
    int s = QEH_OK;
    for (int j = 0; j < n_keys && s == QEH_OK; ++j) s = col_to_arr(&keys[j], &ka[j]);
    for (int j = 0; j < n_inputs && s == QEH_OK; ++j) s = col_to_arr(&inputs[j], &ia[j]);
    if (s == QEH_OK) s = check_agg_types(ia, n_inputs, aggs, n_aggs);
    if (s == QEH_OK) {
        grouping g = {0};
        if (n_keys > 0) {
            group_rows(ka, n_keys, n, NULL, &g);
        } else {
            g.groups = 1;
            g.rep = calloc(1, sizeof(int64_t));
            g.gid = calloc((size_t)(n > 0 ? n : 1), sizeof(int64_t));
        }
        astate *st = calloc((size_t)(g.groups > 0 ? g.groups : 1) * (size_t)n_aggs, sizeof(astate));
        for (int64_t r = 0; r < n; ++r)
            for (int a = 0; a < n_aggs; ++a) agg_update(&st[g.gid[r] * n_aggs + a], &ia[aggs[a].column], r);
        emit_groups(ka, n_keys, ia, aggs, n_aggs, g.groups, g.rep, st, out_keys, out_aggs);
        *out_groups = g.groups;
        free(st);
        free(g.rep);
        free(g.gid);
    }
    for (int j = 0; j < n_keys; ++j) arr_free(&ka[j]);
    for (int j = 0; j < n_inputs; ++j) arr_free(&ia[j]);
    free(ka);
    free(ia);
    return s;
}

/* ---- join ------------------------------------------------------------------ */
typedef struct {
    uint64_t cap;
    int64_t *head; /* first build row per slot chain, by key */
    int64_t *hkey;
    int64_t *next; /* next build row with the same key, increasing row order */
} jmap;

static void jmap_build(const arr *bk, jmap *m) {
    int64_t n = bk->n;
    m->cap = 1024;
    while (m->cap < (uint64_t)n * 2) m->cap <<= 1;
    m->head = malloc(m->cap * sizeof(int64_t));
    m->hkey = malloc(m->cap * sizeof(int64_t));
    m->next = malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    for (uint64_t i = 0; i < m->cap; ++i) m->head[i] = -1;
    for (int64_t r = n - 1; r >= 0; --r) { /* reverse so chains iterate in build order */
        m->next[r] = -1;
        if (!bk->v[r]) continue; /* NULL keys never match */
        int64_t k = bk->i[r];
        uint64_t h = mix((uint64_t)k) & (m->cap - 1);
        while (m->head[h] >= 0 && m->hkey[h] != k) h = (h + 1) & (m->cap - 1);
        if (m->head[h] >= 0) m->next[r] = m->head[h];
        m->head[h] = r;
        m->hkey[h] = k;
    }
}

static int64_t jmap_first(const jmap *m, int64_t k) {
    uint64_t h = mix((uint64_t)k) & (m->cap - 1);
    while (m->head[h] >= 0) {
        if (m->hkey[h] == k) return m->head[h];
        h = (h + 1) & (m->cap - 1);
    }
    return -1;
}

static void jmap_free(jmap *m) {
    free(m->head);
    free(m->hkey);
    free(m->next);
}

static int join_key_arr(const qo_col *c, arr *a) {
    if (c->dtype != QEH_DT_INT64 && c->dtype != QEH_DT_INT32)
        return err(QEH_E_UNSUPPORTED, "oracle: join keys must be Int32/Int64");
    return col_to_arr(c, a);
}

/* INNER equi-join: the pairs of join_batches' Cartesian product
 * (executor.rs:500-540, left row-major) on which `probe.key = build.key` is TRUE */
int qo_hash_join_inner(const qo_col *probe_key, const qo_col *probe_cols, int n_probe, const qo_col *build_key,
                       const qo_col *build_cols, int n_build, qo_col *out_probe, qo_col *out_build, int64_t *out_rows) {
    arr pk, bk;
    int s = join_key_arr(probe_key, &pk);
    if (s != QEH_OK) return s;
    s = join_key_arr(build_key, &bk);
    if (s != QEH_OK) { arr_free(&pk); return s; }
    jmap m;
    jmap_build(&bk, &m);
    int64_t cap = pk.n > 0 ? pk.n : 1, cnt = 0;
    int64_t *pi = malloc((size_t)cap * sizeof(int64_t)), *bi = malloc((size_t)cap * sizeof(int64_t));
    for (int64_t r = 0; r < pk.n; ++r) {
        if (!pk.v[r]) continue;
        for (int64_t b = jmap_first(&m, pk.i[r]); b >= 0; b = m.next[b]) {
            if (cnt == cap) {
                cap *= 2;
                pi = realloc(pi, (size_t)cap * sizeof(int64_t));
                bi = realloc(bi, (size_t)cap * sizeof(int64_t));
            }
            pi[cnt] = r;
            bi[cnt++] = b;
        }
    }
    for (int j = 0; j < n_probe && s == QEH_OK; ++j) {
        arr a;
        s = col_to_arr(&probe_cols[j], &a);
        if (s == QEH_OK) { arr_to_col(&a, pi, cnt, &out_probe[j]); arr_free(&a); }
    }
    for (int j = 0; j < n_build && s == QEH_OK; ++j) {
        arr a;
        s = col_to_arr(&build_cols[j], &a);
        if (s == QEH_OK) { arr_to_col(&a, bi, cnt, &out_build[j]); arr_free(&a); }
    }
    *out_rows = cnt;
    free(pi);
    free(bi);
    jmap_free(&m);
    arr_free(&pk);
    arr_free(&bk);
    return s;
}

/* LEFT / RIGHT / FULL equi-join.  The reference routes these
 * through the same Cartesian join_batches as INNER (executor.rs:383-435); the
 * intended semantics extend the INNER contract: every matching (left, right)
 * pair, plus each left row without a match (LEFT, FULL) with the right columns
 * NULL, plus each right row without a match (RIGHT, FULL) with the left
 * columns NULL.  NULL keys never match.  Row order: LEFT and FULL in left-row
 * order (matches of one row in build order), the unmatched right rows of FULL
 * after them in right-row order; RIGHT in right-row order. */
static void pairs_push(int64_t **a, int64_t **b, int64_t *cnt, int64_t *cap, int64_t x, int64_t y) {
    if (*cnt == *cap) {
        *cap *= 2;
        *a = realloc(*a, (size_t)*cap * sizeof(int64_t));
        *b = realloc(*b, (size_t)*cap * sizeof(int64_t));
    }
    (*a)[*cnt] = x;
    (*b)[(*cnt)++] = y;
}

int qo_hash_join_outer(int join_type, const qo_col *left_key, const qo_col *left_cols, int n_left,
                       const qo_col *right_key, const qo_col *right_cols, int n_right, qo_col *out_left,
                       qo_col *out_right, int64_t *out_rows) {
    if (join_type < 1 || join_type > 3) return err(QEH_E_INVALID, "outer join type must be LEFT, RIGHT or FULL");
    const int right_outer = join_type == 2;
    /* RIGHT probes with the right side and builds on the left */
    const qo_col *pkc = right_outer ? right_key : left_key, *bkc = right_outer ? left_key : right_key;
    arr pk, bk;
    int s = join_key_arr(pkc, &pk);
    if (s != QEH_OK) return s;
    s = join_key_arr(bkc, &bk);
    if (s != QEH_OK) { arr_free(&pk); return s; }
    jmap m;
    jmap_build(&bk, &m);
    int64_t cap = pk.n + bk.n + 1, cnt = 0;
    int64_t *pi = malloc((size_t)cap * sizeof(int64_t)), *bi = malloc((size_t)cap * sizeof(int64_t));
    uint8_t *hit = calloc((size_t)bk.n + 1, 1);
    for (int64_t r = 0; r < pk.n; ++r) {
        int any = 0;
        if (pk.v[r])
            for (int64_t b = jmap_first(&m, pk.i[r]); b >= 0; b = m.next[b]) {
                pairs_push(&pi, &bi, &cnt, &cap, r, b);
                hit[b] = 1;
                any = 1;
            }
        if (!any) pairs_push(&pi, &bi, &cnt, &cap, r, -1);
    }
    if (join_type == 3)
        for (int64_t b = 0; b < bk.n; ++b)
            if (!hit[b]) pairs_push(&pi, &bi, &cnt, &cap, -1, b);
    const int64_t *li = right_outer ? bi : pi, *ri = right_outer ? pi : bi;
    for (int j = 0; j < n_left && s == QEH_OK; ++j) {
        arr a;
        s = col_to_arr(&left_cols[j], &a);
        if (s == QEH_OK) { arr_to_col(&a, li, cnt, &out_left[j]); arr_free(&a); }
    }
    for (int j = 0; j < n_right && s == QEH_OK; ++j) {
        arr a;
        s = col_to_arr(&right_cols[j], &a);
        if (s == QEH_OK) { arr_to_col(&a, ri, cnt, &out_right[j]); arr_free(&a); }
    }
    *out_rows = cnt;
    free(pi);
    free(bi);
    free(hit);
    jmap_free(&m);
    arr_free(&pk);
    arr_free(&bk);
    return s;
}

/* HashAggregate(Filter(HashJoin(probe, build))) with the filter over probe
 * columns and group keys from the build side, evaluated row by row in the
 * join's output order (no materialisation of the joined batch). */
int qo_join_filter_aggregate(const qo_col *probe_cols, int n_probe, int probe_key_idx, const qeh_expr_node *pred,
                             int n_pred, const qo_col *build_key, const qo_col *build_group_keys, int n_group_keys,
                             const qeh_agg *aggs, int n_aggs, qo_col *out_keys, qo_col *out_aggs, int64_t *out_groups) {
    *out_groups = 0;
    if (n_aggs == 0) return QEH_OK;
    int64_t n = n_probe > 0 ? probe_cols[0].length : 0;
    int s = QEH_OK;
    arr pmask;
    int have_pred = pred && n_pred > 0;
    if (have_pred) {
        s = eval_arr(probe_cols, n_probe, n, pred, n_pred, &pmask);
        if (s != QEH_OK) return s;
        if (pmask.t != QEH_DT_BOOL) { arr_free(&pmask); return err(QEH_E_TYPE, "Filter predicate must return boolean"); }
    }
    arr pk, bk;
    arr *ia = calloc((size_t)n_probe + 1, sizeof(arr));
    arr *gk = calloc((size_t)n_group_keys + 1, sizeof(arr));
    s = join_key_arr(&probe_cols[probe_key_idx], &pk);
    if (s == QEH_OK) s = join_key_arr(build_key, &bk);
    for (int j = 0; j < n_probe && s == QEH_OK; ++j) s = col_to_arr(&probe_cols[j], &ia[j]);
    for (int j = 0; j < n_group_keys && s == QEH_OK; ++j) s = col_to_arr(&build_group_keys[j], &gk[j]);
    if (s == QEH_OK) s = check_agg_types(ia, n_probe, aggs, n_aggs);
    if (s == QEH_OK) {
        jmap m;
        jmap_build(&bk, &m);
        grouping g;
        group_rows(gk, n_group_keys, bk.n, NULL, &g); /* gid per build row */
        astate *st = calloc((size_t)(g.groups > 0 ? g.groups : 1) * (size_t)n_aggs, sizeof(astate));
        int64_t *rows = calloc((size_t)(g.groups > 0 ? g.groups : 1), sizeof(int64_t));
        for (int64_t r = 0; r < n; ++r) {
            if (!pk.v[r]) continue;
            if (have_pred && !(pmask.v[r] && pmask.i[r])) continue;
            for (int64_t b = jmap_first(&m, pk.i[r]); b >= 0; b = m.next[b]) {
                int64_t grp = g.gid[b];
                rows[grp]++;
                for (int a = 0; a < n_aggs; ++a) agg_update(&st[grp * n_aggs + a], &ia[aggs[a].column], r);
            }
        }
        /* groups that received no joined row do not exist in the result */
        int64_t G = 0;
        int64_t *rep = malloc((size_t)(g.groups > 0 ? g.groups : 1) * sizeof(int64_t));
        astate *st2 = calloc((size_t)(g.groups > 0 ? g.groups : 1) * (size_t)n_aggs, sizeof(astate));
        for (int64_t q = 0; q < g.groups; ++q) {
            if (!rows[q]) continue;
            rep[G] = g.rep[q];
            memcpy(&st2[G * n_aggs], &st[q * n_aggs], (size_t)n_aggs * sizeof(astate));
            ++G;
        }
        emit_groups(gk, n_group_keys, ia, aggs, n_aggs, G, rep, st2, out_keys, out_aggs);
        *out_groups = G;
        free(rep);
        free(st2);
        free(st);
        free(rows);
        free(g.rep);
        free(g.gid);
        jmap_free(&m);
    }
    if (have_pred) arr_free(&pmask);
    arr_free(&pk);
    arr_free(&bk);
    for (int j = 0; j < n_probe; ++j) arr_free(&ia[j]);
    for (int j = 0; j < n_group_keys; ++j) arr_free(&gk[j]);
    free(ia);
    free(gk);
    return s;
}

/* ---- literal Cartesian joins and joins on an arbitrary `on` ------------------------- */
static int gather_side(const qo_col *cols, int n, const int64_t *idx, int64_t m, qo_col *out) {
    int s = QEH_OK;
    for (int j = 0; j < n && s == QEH_OK; ++j) {
        arr a;
        s = col_to_arr(&cols[j], &a);
        if (s == QEH_OK) { arr_to_col(&a, idx, m, &out[j]); arr_free(&a); }
    }
    return s;
}

/* join_batches (executor.rs:500-540), the reference's INNER / LEFT / RIGHT / FULL join
 * (executor.rs:363-435, `on` unused): left row li is repeated right_rows times
 * (left row-major), right rows cycle; schema = left fields ++ right fields.  An empty side
 * yields no batch at all (executor.rs:350-352): *out_rows = -1 then. */
int qo_join_batches(const qo_col *left, int nl, const qo_col *right, int nr, qo_col *out, int64_t *out_rows) {
    const int64_t L = nl > 0 ? left[0].length : 0, R = nr > 0 ? right[0].length : 0;
    if (L == 0 || R == 0) { *out_rows = -1; return QEH_OK; }
    const int64_t m = L * R;
    int64_t *li = malloc((size_t)m * sizeof(int64_t)), *ri = malloc((size_t)m * sizeof(int64_t));
    for (int64_t l = 0, k = 0; l < L; ++l)      /* executor.rs:509-513 */
        for (int64_t r = 0; r < R; ++r, ++k) li[k] = l;
    for (int64_t l = 0, k = 0; l < L; ++l)      /* executor.rs:522-526 */
        for (int64_t r = 0; r < R; ++r, ++k) ri[k] = r;
    int s = gather_side(left, nl, li, m, out);
    if (s == QEH_OK) s = gather_side(right, nr, ri, m, out + nl);
    free(li);
    free(ri);
    *out_rows = m;
    return s;
}

/* execute_cross_join (executor.rs:437-498): the left index cycles fastest (for each right
 * row, every left row: executor.rs:455-459, 470-474), i.e. right row-major. */
int qo_cross_join(const qo_col *left, int nl, const qo_col *right, int nr, qo_col *out, int64_t *out_rows) {
    const int64_t L = nl > 0 ? left[0].length : 0, R = nr > 0 ? right[0].length : 0;
    if (L == 0 || R == 0) { *out_rows = -1; return QEH_OK; }
    const int64_t m = L * R;
    int64_t *li = malloc((size_t)m * sizeof(int64_t)), *ri = malloc((size_t)m * sizeof(int64_t));
    for (int64_t r = 0, k = 0; r < R; ++r)
        for (int64_t l = 0; l < L; ++l, ++k) { li[k] = l; ri[k] = r; }
    int s = gather_side(left, nl, li, m, out);
    if (s == QEH_OK) s = gather_side(right, nr, ri, m, out + nl);
    free(li);
    free(ri);
    *out_rows = m;
    return s;
}

/* Join on an arbitrary boolean `on` over the concatenated schema (planner.rs:148-157 resolves
 * its column indices there) — the intended semantics of SURVEY.md §8.0 generalised from the
 * equi-join: the pairs of join_batches' Cartesian product (left row-major) on which `on` is
 * TRUE (NULL = not a match); LEFT / FULL add each left row without a match (right side NULL)
 * at its place in left-row order, FULL then the unmatched right rows in right-row order;
 * RIGHT is the mirror image (right-row order).  `on` is evaluated literally, column at a
 * time, over blocks of the Cartesian product (O(L*R): small inputs only). */
int qo_join_on(int join_type, const qo_col *left, int nl, const qo_col *right, int nr, const qeh_expr_node *on,
               int n_on, qo_col *out_left, qo_col *out_right, int64_t *out_rows) {
    if (join_type < 0 || join_type > 3) return err(QEH_E_INVALID, "join type must be INNER, LEFT, RIGHT or FULL");
    const int64_t L = nl > 0 ? left[0].length : 0, R = nr > 0 ? right[0].length : 0;
    int s = QEH_OK;
    arr *la = calloc((size_t)nl + 1, sizeof(arr)), *ra = calloc((size_t)nr + 1, sizeof(arr));
    for (int j = 0; j < nl && s == QEH_OK; ++j) s = col_to_arr(&left[j], &la[j]);
    for (int j = 0; j < nr && s == QEH_OK; ++j) s = col_to_arr(&right[j], &ra[j]);
    /* match[l * R + r] for the TRUE pairs, evaluated over blocks of left rows */
    uint8_t *match = calloc((size_t)(L * R > 0 ? L * R : 1), 1);
    const int64_t blk = R > 0 ? (((int64_t)1 << 20) / R > 0 ? ((int64_t)1 << 20) / R : 1) : 1;
    qo_col *tmp = calloc((size_t)(nl + nr) + 1, sizeof(qo_col));
    int64_t *li = malloc((size_t)(blk * R > 0 ? blk * R : 1) * sizeof(int64_t));
    int64_t *ri = malloc((size_t)(blk * R > 0 ? blk * R : 1) * sizeof(int64_t));
    for (int64_t l0 = 0; l0 < L && R > 0 && s == QEH_OK; l0 += blk) {
        const int64_t l1 = l0 + blk < L ? l0 + blk : L, m = (l1 - l0) * R;
        for (int64_t l = l0, k = 0; l < l1; ++l)
            for (int64_t r = 0; r < R; ++r, ++k) { li[k] = l; ri[k] = r; }
        for (int j = 0; j < nl; ++j) arr_to_col(&la[j], li, m, &tmp[j]);
        for (int j = 0; j < nr; ++j) arr_to_col(&ra[j], ri, m, &tmp[nl + j]);
        arr p;
        s = eval_arr(tmp, nl + nr, m, on, n_on, &p);
        for (int j = 0; j < nl + nr; ++j) qo_col_free(&tmp[j]);
        if (s != QEH_OK) break;
        if (p.t != QEH_DT_BOOL) { arr_free(&p); s = err(QEH_E_TYPE, "join condition must return boolean"); break; }
        for (int64_t k = 0; k < m; ++k) match[l0 * R + k] = p.v[k] && p.i[k];
        arr_free(&p);
    }
    free(tmp);
    free(li);
    free(ri);
    if (s == QEH_OK) {
        int64_t cap = L + R + 16, cnt = 0;
        int64_t *pl = malloc((size_t)cap * sizeof(int64_t)), *pr = malloc((size_t)cap * sizeof(int64_t));
        if (join_type == 2) { /* RIGHT: right-row order */
            for (int64_t r = 0; r < R; ++r) {
                int any = 0;
                for (int64_t l = 0; l < L; ++l)
                    if (match[l * R + r]) { pairs_push(&pl, &pr, &cnt, &cap, l, r); any = 1; }
                if (!any) pairs_push(&pl, &pr, &cnt, &cap, -1, r);
            }
        } else {
            uint8_t *hit = calloc((size_t)R + 1, 1);
            for (int64_t l = 0; l < L; ++l) {
                int any = 0;
                for (int64_t r = 0; r < R; ++r)
                    if (match[l * R + r]) { pairs_push(&pl, &pr, &cnt, &cap, l, r); hit[r] = 1; any = 1; }
                if (!any && join_type != 0) pairs_push(&pl, &pr, &cnt, &cap, l, -1);
            }
            if (join_type == 3)
                for (int64_t r = 0; r < R; ++r)
                    if (!hit[r]) pairs_push(&pl, &pr, &cnt, &cap, -1, r);
            free(hit);
        }
        for (int j = 0; j < nl; ++j) arr_to_col(&la[j], pl, cnt, &out_left[j]);
        for (int j = 0; j < nr; ++j) arr_to_col(&ra[j], pr, cnt, &out_right[j]);
        *out_rows = cnt;
        free(pl);
        free(pr);
    }
    free(match);
    for (int j = 0; j < nl; ++j) arr_free(&la[j]);
    for (int j = 0; j < nr; ++j) arr_free(&ra[j]);
    free(la);
    free(ra);
    return s;
}

/* ---- all-cores CPU baseline of the metric query ----------------------------------------
 * Same semantics as qo_join_filter_aggregate (HashAggregate(Filter(HashJoin)) with the
 * filter over probe columns and group keys from the build side), restructured for T host
 * threads (OpenMP): the build side is grouped and inserted into shared open-addressing
 * tables with CAS (group ids then renumbered in build-row order of first appearance), the
 * probe side is split into chunks of rows, each chunk's predicate evaluated over column
 * slices, and every thread aggregates into its own state table; the states are merged in
 * thread order.  Float sums therefore add in a different order (within the 1e-6 bound).
 * The reference executor itself is single-threaded (rayon unused, Cargo.toml:18): this is a
 * baseline for the host's cores, not a restatement of its execution order. */
static void agg_merge(astate *d, const astate *s, int is_f) {
    if (!s->cnt) return;
    if (!d->cnt) { *d = *s; return; }
    d->isum += s->isum;
    d->fsum += s->fsum;
    d->f32sum += s->f32sum;
    if (is_f) {
        if (tkey(s->fmin) < tkey(d->fmin)) d->fmin = s->fmin;
        if (tkey(s->fmax) > tkey(d->fmax)) d->fmax = s->fmax;
    } else {
        if (s->imin < d->imin) d->imin = s->imin;
        if (s->imax > d->imax) d->imax = s->imax;
    }
    d->cnt += s->cnt;
}

static int cmp_i64(const void *x, const void *y) {
    const int64_t p = *(const int64_t *)x, q = *(const int64_t *)y;
    return p < q ? -1 : p > q;
}

static qo_col col_slice(const qo_col *c, int64_t r0, int64_t n) {
    qo_col o = *c;
    o.length = n;
    o.values = (char *)c->values + (size_t)r0 * esize(c->dtype);
    if (c->valid) o.valid = c->valid + r0;
    return o;
}

int qo_join_filter_aggregate_mt(const qo_col *probe_cols, int n_probe, int probe_key_idx, const qeh_expr_node *pred,
                                int n_pred, const qo_col *build_key, const qo_col *build_group_keys, int n_group_keys,
                                const qeh_agg *aggs, int n_aggs, int threads, qo_col *out_keys, qo_col *out_aggs,
                                int64_t *out_groups) {
    *out_groups = 0;
    if (n_aggs == 0) return QEH_OK;
    if (threads < 1) threads = 1;
    const int64_t n = n_probe > 0 ? probe_cols[0].length : 0, nb = build_key->length;
    int s = QEH_OK;
    arr bk;
    arr *gk = calloc((size_t)n_group_keys + 1, sizeof(arr));
    s = join_key_arr(build_key, &bk);
    for (int j = 0; j < n_group_keys && s == QEH_OK; ++j) s = col_to_arr(&build_group_keys[j], &gk[j]);
    if (probe_cols[probe_key_idx].dtype != QEH_DT_INT64 && probe_cols[probe_key_idx].dtype != QEH_DT_INT32)
        s = err(QEH_E_UNSUPPORTED, "oracle: join keys must be Int32/Int64");
    for (int a = 0; a < n_aggs && s == QEH_OK; ++a) {
        if (aggs[a].column < 0 || aggs[a].column >= n_probe) s = err(QEH_E_INVALID, "aggregate input index out of range");
        else if (aggs[a].func != QEH_AGG_COUNT && !is_num(probe_cols[aggs[a].column].dtype))
            s = err(QEH_E_TYPE, "Unsupported type for aggregate");
    }
    if (s != QEH_OK) {
        arr_free(&bk);
        for (int j = 0; j < n_group_keys; ++j) arr_free(&gk[j]);
        free(gk);
        return s;
    }
    /* build: group slots (CAS on representative row + 1), then dense ids in build-row order */
    uint64_t gcap = 1024, jcap = 1024;
    while (gcap < (uint64_t)nb * 2) gcap <<= 1;
    while (jcap < (uint64_t)nb * 2) jcap <<= 1;
    int64_t *gslot = calloc(gcap, sizeof(int64_t));     /* 0 = empty, else rep row + 1 */
    int64_t *gid = malloc((size_t)(nb > 0 ? nb : 1) * sizeof(int64_t));
    int64_t *jhead = malloc(jcap * sizeof(int64_t));   /* -1 = empty */
    int64_t *jkey = malloc(jcap * sizeof(int64_t));
    int64_t *jnext = malloc((size_t)(nb > 0 ? nb : 1) * sizeof(int64_t));
#pragma omp parallel for num_threads(threads) schedule(static)
    for (uint64_t i = 0; i < jcap; ++i) jhead[i] = -1;
#pragma omp parallel for num_threads(threads) schedule(static, 65536)
    for (int64_t r = 0; r < nb; ++r) {
        uint64_t h = tuple_hash(gk, n_group_keys, r) & (gcap - 1);
        for (;;) {
            int64_t cur = __atomic_load_n(&gslot[h], __ATOMIC_ACQUIRE);
            if (cur == 0) {
                int64_t want = 0;
                if (__atomic_compare_exchange_n(&gslot[h], &want, r + 1, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
                    gid[r] = (int64_t)h;
                    break;
                }
                cur = want;
            }
            if (tuple_eq(gk, cur - 1, gk, r, n_group_keys)) { gid[r] = (int64_t)h; break; }
            h = (h + 1) & (gcap - 1);
        }
        /* join table: key slot by CAS on the head (key written before publication) */
        jnext[r] = -1;
        if (!bk.v[r]) continue;
        const int64_t k = bk.i[r];
        uint64_t q = mix((uint64_t)k) & (jcap - 1);
        for (;;) {
            int64_t hd = __atomic_load_n(&jhead[q], __ATOMIC_ACQUIRE);
            if (hd == -1) { /* claim the empty slot (-2 = key being written), then publish */
                int64_t want = -1;
                if (__atomic_compare_exchange_n(&jhead[q], &want, -2, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
                    jkey[q] = k;
                    __atomic_store_n(&jhead[q], r, __ATOMIC_RELEASE);
                    break;
                }
                hd = want;
            }
            while (hd == -2) hd = __atomic_load_n(&jhead[q], __ATOMIC_ACQUIRE); /* slot being published */
            if (jkey[q] == k) { /* push onto the chain */
                int64_t old = __atomic_load_n(&jhead[q], __ATOMIC_ACQUIRE);
                do { jnext[r] = old; } while (!__atomic_compare_exchange_n(&jhead[q], &old, r, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE));
                break;
            }
            q = (q + 1) & (jcap - 1);
        }
    }
    /* dense group ids: slots ordered by their representative row (first appearance) */
    int64_t G0 = 0;
    for (uint64_t i = 0; i < gcap; ++i) if (gslot[i]) ++G0;
    int64_t *slot_rep = malloc((size_t)(G0 > 0 ? G0 : 1) * sizeof(int64_t));
    int64_t *dense = malloc(gcap * sizeof(int64_t));
    for (uint64_t i = 0, g = 0; i < gcap; ++i) if (gslot[i]) slot_rep[g++] = gslot[i] - 1;
    qsort(slot_rep, (size_t)G0, sizeof(int64_t), cmp_i64);
    for (int64_t g = 0; g < G0; ++g) {
        const int64_t r = slot_rep[g];
        dense[gid[r]] = g;
    }
#pragma omp parallel for num_threads(threads) schedule(static, 65536)
    for (int64_t r = 0; r < nb; ++r) gid[r] = dense[gid[r]];
    /* probe: chunks of rows, thread-private states */
    const int64_t chunk = 1 << 16;
    const int64_t nchunks = (n + chunk - 1) / chunk;
    astate *st = calloc((size_t)threads * (size_t)(G0 > 0 ? G0 : 1) * (size_t)n_aggs, sizeof(astate));
    int64_t *rows = calloc((size_t)threads * (size_t)(G0 > 0 ? G0 : 1), sizeof(int64_t));
    int fail_s = QEH_OK;
#pragma omp parallel num_threads(threads)
    {
        int t = 0;
#ifdef _OPENMP
        t = omp_get_thread_num();
#endif
        astate *my = st + (size_t)t * (size_t)(G0 > 0 ? G0 : 1) * (size_t)n_aggs;
        int64_t *myrows = rows + (size_t)t * (size_t)(G0 > 0 ? G0 : 1);
        qo_col *sl = calloc((size_t)n_probe + 1, sizeof(qo_col));
        arr *ia = calloc((size_t)n_probe + 1, sizeof(arr));
#pragma omp for schedule(dynamic, 1)
        for (int64_t c = 0; c < nchunks; ++c) {
            const int64_t r0 = c * chunk, m = r0 + chunk < n ? chunk : n - r0;
            for (int j = 0; j < n_probe; ++j) sl[j] = col_slice(&probe_cols[j], r0, m);
            arr pm;
            int ls = QEH_OK, have = pred && n_pred > 0;
            if (have) {
                ls = eval_arr(sl, n_probe, m, pred, n_pred, &pm);
                if (ls == QEH_OK && pm.t != QEH_DT_BOOL) { arr_free(&pm); ls = QEH_E_TYPE; }
            }
            if (ls != QEH_OK) { fail_s = ls; continue; }
            for (int j = 0; j < n_probe; ++j) col_to_arr(&sl[j], &ia[j]);
            const arr *pk = &ia[probe_key_idx];
            for (int64_t r = 0; r < m; ++r) {
                if (!pk->v[r]) continue;
                if (have && !(pm.v[r] && pm.i[r])) continue;
                const int64_t k = pk->i[r];
                uint64_t q = mix((uint64_t)k) & (jcap - 1);
                int64_t b = -1;
                while (jhead[q] >= 0) {
                    if (jkey[q] == k) { b = jhead[q]; break; }
                    q = (q + 1) & (jcap - 1);
                }
                for (; b >= 0; b = jnext[b]) {
                    const int64_t g = gid[b];
                    myrows[g]++;
                    for (int a = 0; a < n_aggs; ++a) agg_update(&my[g * n_aggs + a], &ia[aggs[a].column], r);
                }
            }
            for (int j = 0; j < n_probe; ++j) arr_free(&ia[j]);
            if (have) arr_free(&pm);
        }
        free(sl);
        free(ia);
    }
    if (fail_s != QEH_OK) {
        s = fail_s == QEH_E_TYPE ? err(QEH_E_TYPE, "Filter predicate must return boolean") : fail_s;
    } else {
        /* merge in thread order; groups without a joined row do not exist in the result */
        astate *fin = calloc((size_t)(G0 > 0 ? G0 : 1) * (size_t)n_aggs, sizeof(astate));
        int64_t *rep = malloc((size_t)(G0 > 0 ? G0 : 1) * sizeof(int64_t));
        int64_t G = 0;
        arr *ia = calloc((size_t)n_probe + 1, sizeof(arr));
        for (int j = 0; j < n_probe; ++j) ia[j].t = probe_cols[j].dtype;
        for (int64_t g = 0; g < G0; ++g) {
            int64_t cnt = 0;
            for (int t = 0; t < threads; ++t) cnt += rows[(size_t)t * (size_t)G0 + g];
            if (!cnt) continue;
            for (int a = 0; a < n_aggs; ++a)
                for (int t = 0; t < threads; ++t)
                    agg_merge(&fin[G * n_aggs + a], &st[((size_t)t * (size_t)G0 + g) * n_aggs + a],
                              is_float(probe_cols[aggs[a].column].dtype));
            rep[G++] = slot_rep[g];
        }
        emit_groups(gk, n_group_keys, ia, aggs, n_aggs, G, rep, fin, out_keys, out_aggs);
        *out_groups = G;
        free(ia);
        free(fin);
        free(rep);
    }
    free(st);
    free(rows);
    free(slot_rep);
    free(dense);
    free(gslot);
    free(gid);
    free(jhead);
    free(jkey);
    free(jnext);
    arr_free(&bk);
    for (int j = 0; j < n_group_keys; ++j) arr_free(&gk[j]);
    free(gk);
    return s;
}

/* ---- sort / row_number ------------------------------------------------------ */
typedef struct {
    const arr *k;
    int nk;
    const int8_t *asc;
    const int8_t *nulls_first; /* NULL: all first */
} sort_ctx;

/* arrow SortOptions default nulls_first = true (distributed/operators.rs:97-104); Merge::sorted
 * passes it per column (operators.rs:163-172) */
static int row_cmp(const sort_ctx *c, int64_t a, int64_t b) {
    for (int j = 0; j < c->nk; ++j) {
        const arr *k = &c->k[j];
        int va = k->v[a], vb = k->v[b];
        if (va != vb) {
            const int nf = c->nulls_first ? c->nulls_first[j] != 0 : 1;
            return (va ? 1 : -1) * (nf ? 1 : -1);
        }
        if (!va) continue;
        int64_t x = key_bits(k, a), y = key_bits(k, b);
        int r = (x > y) - (x < y);
        if (!c->asc[j]) r = -r;
        if (r) return r;
    }
    return 0;
}

static void msort(const sort_ctx *c, int64_t *idx, int64_t *tmp, int64_t n) {
    if (n < 2) return;
    int64_t h = n / 2;
    msort(c, idx, tmp, h);
    msort(c, idx + h, tmp, n - h);
    int64_t i = 0, j = h, k = 0;
    while (i < h && j < n) tmp[k++] = row_cmp(c, idx[j], idx[i]) < 0 ? idx[j++] : idx[i++]; /* stable */
    while (i < h) tmp[k++] = idx[i++];
    while (j < n) tmp[k++] = idx[j++];
    memcpy(idx, tmp, (size_t)n * sizeof(int64_t));
}

static int sorted_perm_nulls(const qo_col *keys, int n_keys, const int8_t *asc, const int8_t *nulls_first, int64_t n,
                             int64_t **perm_out, arr **ka_out);
static int sorted_perm(const qo_col *keys, int n_keys, const int8_t *asc, int64_t n, int64_t **perm_out, arr **ka_out) {
    return sorted_perm_nulls(keys, n_keys, asc, NULL, n, perm_out, ka_out);
}

static int sorted_perm_nulls(const qo_col *keys, int n_keys, const int8_t *asc, const int8_t *nulls_first, int64_t n,
                             int64_t **perm_out, arr **ka_out) {
    arr *ka = calloc((size_t)n_keys + 1, sizeof(arr));
    int s = QEH_OK;
    for (int j = 0; j < n_keys && s == QEH_OK; ++j) s = col_to_arr(&keys[j], &ka[j]);
    int64_t *perm = malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    int64_t *tmp = malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    for (int64_t r = 0; r < n; ++r) perm[r] = r;
    if (s == QEH_OK) {
        sort_ctx c = {ka, n_keys, asc, nulls_first};
        msort(&c, perm, tmp, n);
    }
    free(tmp);
    *perm_out = perm;
    *ka_out = ka;
    return s;
}

int qo_sort_indices(const qo_col *keys, int n_keys, const int8_t *ascending, int64_t n_rows, uint32_t *out_perm) {
    int64_t *perm;
    arr *ka;
    int s = sorted_perm(keys, n_keys, ascending, n_rows, &perm, &ka);
    if (s == QEH_OK)
        for (int64_t r = 0; r < n_rows; ++r) out_perm[r] = (uint32_t)perm[r];
    for (int j = 0; j < n_keys; ++j) arr_free(&ka[j]);
    free(ka);
    free(perm);
    return s;
}

/* Window functions of `WindowFunctionType` (physical_plan.rs:160-170) over the ROW_NUMBER order
 * (partition keys ascending, then the ORDER BY keys, ties by input position).  Semantics from
 * docs/WINDOW_FUNCTIONS.md (the reference executor passes Window through, executor.rs:76-80):
 *   RANK (:67-89) = 1 + rows of the partition ordered strictly before the row's peers;
 *   DENSE_RANK (:91-113) = 1 + distinct ORDER BY tuples before it; NTILE(n) (:115-137) = SQL
 *   buckets (the first size % n buckets hold one row more); LAG/LEAD(col, n) (:139-175) = col
 *   n rows before/after inside the partition, else dflt (NULL when dflt is NULL);
 *   FIRST_VALUE / LAST_VALUE (:177-205) = col at the partition's first / last row (the
 *   WindowExpr carries no frame; the doc's LAST_VALUE example spans the whole partition).
 * out_bits holds Int64 results, or the argument's raw element bits (4-byte types zero-extended);
 * out_valid one byte per row. */
int qo_window(int func, const qo_col *part, int n_part, const qo_col *order, int n_order, const int8_t *ascending,
              const qo_col *arg, int64_t param, const int64_t *dflt, int64_t n_rows, int64_t *out_bits,
              uint8_t *out_valid) {
    int nk = n_part + n_order;
    qo_col *all = calloc((size_t)nk + 1, sizeof(qo_col));
    int8_t *asc = calloc((size_t)nk + 1, 1);
    for (int j = 0; j < n_part; ++j) { all[j] = part[j]; asc[j] = 1; }
    for (int j = 0; j < n_order; ++j) { all[n_part + j] = order[j]; asc[n_part + j] = ascending ? ascending[j] : 1; }
    int64_t *perm;
    arr *ka;
    int s = sorted_perm(all, nk, asc, n_rows, &perm, &ka);
    const int value_fn = func >= 4;
    int esz = 8;
    if (s == QEH_OK && value_fn) {
        if (!arg) s = err(QEH_E_INVALID, "oracle: window value function needs an argument");
        else if (arg->dtype == QEH_DT_INT32 || arg->dtype == QEH_DT_FLOAT32) esz = 4;
        else if (arg->dtype != QEH_DT_INT64 && arg->dtype != QEH_DT_FLOAT64)
            s = err(QEH_E_UNSUPPORTED, "oracle: window argument type %s", dt_name(arg->dtype));
    }
    if (s == QEH_OK && func == 3 && param < 1) s = err(QEH_E_INVALID, "oracle: NTILE needs n >= 1");
    if (s == QEH_OK && (func == 4 || func == 5) && param < 0) s = err(QEH_E_INVALID, "oracle: negative offset");
    for (int64_t a = 0; s == QEH_OK && a < n_rows;) {
        int64_t b = a + 1;  /* partition [a, b) in sorted order */
        while (b < n_rows && tuple_eq(ka, perm[b - 1], ka, perm[b], n_part)) ++b;
        int64_t peer = a, dense = 0;
        for (int64_t i = a; i < b; ++i) {
            if (i == a || !tuple_eq(ka, perm[i - 1], ka, perm[i], nk)) { peer = i; ++dense; }
            const int64_t r0 = i - a, size = b - a, row = perm[i];
            int64_t v = 0, src = -1;
            uint8_t ok = 1;
            switch (func) {
                case 0: v = r0 + 1; break;
                case 1: v = peer - a + 1; break;
                case 2: v = dense; break;
                case 3: {
                    const int64_t q = size / param, r = size % param;
                    v = r0 < r * (q + 1) ? r0 / (q + 1) + 1 : r + (r0 - r * (q + 1)) / q + 1;
                    break;
                }
                case 4: src = i - param >= a ? perm[i - param] : -2; break;
                case 5: src = i + param < b ? perm[i + param] : -2; break;
                case 6: src = perm[a]; break;
                case 7: src = perm[b - 1]; break;
                default: s = err(QEH_E_UNSUPPORTED, "oracle: window function %d", func);
            }
            if (src == -2) {
                ok = dflt != NULL;
                v = dflt ? *dflt : 0;
            } else if (src >= 0) {
                ok = arg->valid ? arg->valid[src] != 0 : 1;
                v = esz == 8 ? ((const int64_t *)arg->values)[src] : (int64_t)((const uint32_t *)arg->values)[src];
                if (!ok) v = 0;
            }
            out_bits[row] = v;
            out_valid[row] = ok;
        }
        a = b;
    }
    for (int j = 0; j < nk; ++j) arr_free(&ka[j]);
    free(ka);
    free(perm);
    free(all);
    free(asc);
    return s;
}

/* Merge::sorted's lexsort (operators.rs:163-186) with per-key nulls_first, stable. */
int qo_sort_indices_nulls(const qo_col *keys, int n_keys, const int8_t *ascending, const int8_t *nulls_first,
                          int64_t n_rows, uint32_t *out_perm) {
    int64_t *perm;
    arr *ka;
    int s = sorted_perm_nulls(keys, n_keys, ascending, nulls_first, n_rows, &perm, &ka);
    if (s == QEH_OK)
        for (int64_t r = 0; r < n_rows; ++r) out_perm[r] = (uint32_t)perm[r];
    for (int j = 0; j < n_keys; ++j) arr_free(&ka[j]);
    free(ka);
    free(perm);
    return s;
}

int qo_row_number(const qo_col *part, int n_part, const qo_col *order, int n_order, const int8_t *ascending,
                  int64_t n_rows, int64_t *out_rn) {
    int nk = n_part + n_order;
    qo_col *all = calloc((size_t)nk + 1, sizeof(qo_col));
    int8_t *asc = calloc((size_t)nk + 1, 1);
    for (int j = 0; j < n_part; ++j) { all[j] = part[j]; asc[j] = 1; }
    for (int j = 0; j < n_order; ++j) { all[n_part + j] = order[j]; asc[n_part + j] = ascending ? ascending[j] : 1; }
    int64_t *perm;
    arr *ka;
    int s = sorted_perm(all, nk, asc, n_rows, &perm, &ka);
    if (s == QEH_OK) {
        int64_t rn = 0;
        for (int64_t i = 0; i < n_rows; ++i) {
            if (i == 0 || !tuple_eq(ka, perm[i - 1], ka, perm[i], n_part)) rn = 0;
            out_rn[perm[i]] = ++rn;
        }
    }
    for (int j = 0; j < nk; ++j) arr_free(&ka[j]);
    free(ka);
    free(perm);
    free(all);
    free(asc);
    return s;
}
