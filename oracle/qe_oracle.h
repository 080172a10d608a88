/*
 * qe_oracle.h — CPU ORACLE (test infrastructure only; never linked into the
 * product).  A plain-C restatement of the reference executor's semantics for
 * the hot path, used by tests/ as the checker and by bench.py as the timed
 * CPU baseline ("port").  See qe_oracle.c for per-function citations.
 *
 * Parity pinning (DESIGN.md "Oracle"): the reference cannot be built here (no
 * cargo/rustc, arrow-rs 53.4.1 not vendored) and its own tests pin almost
 * nothing on this path, so this oracle is pinned by (a) the reference's known
 * answers (config 1 on data/employees.csv, the sorted-merge and partition-
 * conservation tests) and (b) golden vectors produced in the build container
 * by Arrow C++ (pyarrow 25) for the arrow-rs kernel semantics the reference
 * calls (tests/golden/, tools/gen_golden.py).  Join / group-by / sort /
 * ROW_NUMBER follow the intended semantics of SURVEY.md §8.0 because the
 * reference's implementations are stubs: for those, parity is against this
 * restatement, not against reference output.
 */
#ifndef QE_ORACLE_H
#define QE_ORACLE_H
#include <stdint.h>

/* dtypes and expression nodes share the numbering of include/qeh.h */
#include "../include/qeh.h"

#ifdef __cplusplus
extern "C" {
#endif

/* host column: booleans/validity one byte per row (1 = true / valid) */
typedef struct qo_col {
    int32_t dtype;
    int32_t _pad;
    int64_t length;
    void *values;   /* int32/int64/float/double/uint8(bool)/uint32 */
    uint8_t *valid; /* NULL = all valid */
} qo_col;

const char *qo_last_error(void);
void qo_free(void *p);
void qo_col_free(qo_col *c);

void qo_generate(int kind, uint64_t seed, uint64_t col_id, int64_t row0, int64_t n, int64_t modulus,
                 int64_t lo, void *out);

int qo_eval(const qo_col *cols, int n_cols, int64_t n_rows, const qeh_expr_node *nodes, int n_nodes,
            qo_col *out);
int qo_filter(const qo_col *cols, int n_cols, const qeh_expr_node *nodes, int n_nodes,
              const int32_t *out_idx, int n_out, qo_col *out, int64_t *out_rows);
int qo_hash_aggregate(const qo_col *keys, int n_keys, const qo_col *inputs, int n_inputs,
                      const qeh_agg *aggs, int n_aggs, int64_t input_batches, qo_col *out_keys,
                      qo_col *out_aggs, int64_t *out_groups);
int qo_hash_join_inner(const qo_col *probe_key, const qo_col *probe_cols, int n_probe,
                       const qo_col *build_key, const qo_col *build_cols, int n_build,
                       qo_col *out_probe, qo_col *out_build, int64_t *out_rows);
/* LEFT (1) / RIGHT (2) / FULL (3) equi-join, values of qeh_join_type (qeh_plan.h). */
int qo_hash_join_outer(int join_type, const qo_col *left_key, const qo_col *left_cols, int n_left,
                       const qo_col *right_key, const qo_col *right_cols, int n_right, qo_col *out_left,
                       qo_col *out_right, int64_t *out_rows);
int qo_join_filter_aggregate(const qo_col *probe_cols, int n_probe, int probe_key_idx,
                             const qeh_expr_node *pred, int n_pred, const qo_col *build_key,
                             const qo_col *build_group_keys, int n_group_keys, const qeh_agg *aggs,
                             int n_aggs, qo_col *out_keys, qo_col *out_aggs, int64_t *out_groups);
/* literal Cartesian joins: join_batches (executor.rs:500-540, left row-major; the reference's
 * INNER/LEFT/RIGHT/FULL) and execute_cross_join (executor.rs:437-498, right row-major).
 * out = left columns then right columns; *out_rows = -1 when a side is empty (no batch). */
int qo_join_batches(const qo_col *left, int nl, const qo_col *right, int nr, qo_col *out, int64_t *out_rows);
int qo_cross_join(const qo_col *left, int nl, const qo_col *right, int nr, qo_col *out, int64_t *out_rows);
/* join on an arbitrary boolean `on` over left ++ right columns; join_type 0 INNER, 1 LEFT,
 * 2 RIGHT, 3 FULL (the intended semantics) */
int qo_join_on(int join_type, const qo_col *left, int nl, const qo_col *right, int nr, const qeh_expr_node *on,
               int n_on, qo_col *out_left, qo_col *out_right, int64_t *out_rows);
/* all-cores CPU baseline of qo_join_filter_aggregate (OpenMP, `threads` threads) */
int qo_join_filter_aggregate_mt(const qo_col *probe_cols, int n_probe, int probe_key_idx,
                                const qeh_expr_node *pred, int n_pred, const qo_col *build_key,
                                const qo_col *build_group_keys, int n_group_keys, const qeh_agg *aggs,
                                int n_aggs, int threads, qo_col *out_keys, qo_col *out_aggs,
                                int64_t *out_groups);
/* Partitioner::partition_by_hash (query-distributed/src/partition.rs:151-212, compute_row_hash
 * :292-316) over Int32 / Int64 key columns: every row goes to hash(row) % n_parts, rows keep input
 * order inside a partition; out_perm = the partition-major row order, counts[p] = rows of p.
 * The row hash is the device's (murmur3 fmix64 combine, NULL cells skipped), not SipHash: the
 * hash is not observable in any query result. */
int qo_partition_hash(const qo_col *keys, int n_keys, int n_parts, int64_t *counts, uint32_t *out_perm);
int qo_sort_indices(const qo_col *keys, int n_keys, const int8_t *ascending, int64_t n_rows,
                    uint32_t *out_perm);
int qo_sort_indices_nulls(const qo_col *keys, int n_keys, const int8_t *ascending, const int8_t *nulls_first,
                          int64_t n_rows, uint32_t *out_perm);
int qo_row_number(const qo_col *part, int n_part, const qo_col *order, int n_order,
                  const int8_t *ascending, int64_t n_rows, int64_t *out_rn);
int qo_window(int func, const qo_col *part, int n_part, const qo_col *order, int n_order, const int8_t *ascending,
              const qo_col *arg, int64_t param, const int64_t *dflt, int64_t n_rows, int64_t *out_bits,
              uint8_t *out_valid);

#ifdef __cplusplus
}
#endif
#endif
