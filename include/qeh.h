/*
 * qeh.h — C ABI of the MI355X (gfx950) physical-execution backend for
 * AarambhDevHub/query-engine's `crates/query-executor`.
 *
 * Boundary (SURVEY.md §8 row b): the reference executes a closed enum
 *   `PhysicalPlan` (crates/query-executor/src/physical_plan.rs:13-72) through
 *   `QueryExecutor::execute(&self, &PhysicalPlan) -> Result<Vec<RecordBatch>>`
 *   (crates/query-executor/src/executor.rs:19-21).  There is no operator trait,
 *   so the drop-in is "same enum, same signature": a Rust `HipQueryExecutor`
 *    walks the enum and calls the operator entry points
 *   below, or hands the whole plan to `qeh_execute_plan`.
 *
 * Conventions
 *   - Every function returns an `int` status (enum qeh_status).  On failure the
 *     calling thread's message is available from qeh_last_error(); status codes
 *     map onto `query_core::QueryError` (crates/query-core/src/error.rs:4-57):
 *     QEH_E_OVERFLOW / QEH_E_DIV0 -> QueryError::ArrowError (arrow's
 *     ArithmeticOverflow / DivideByZero), everything else -> ExecutionError.
 *   - Column buffers passed to operator entry points are DEVICE pointers
 *     (HBM-resident).  qeh_column mirrors an Arrow primitive array:
 *     values + optional LSB-first validity bitmap + element offset.  Booleans
 *     are bit-packed exactly as in Arrow.
 *   - Output columns are allocated by the library from its device pool; the
 *     caller releases them with qeh_column_release().  Input buffers are never
 *     written or retained.
 *   - A context is bound to one device and one HIP stream; all work is
 *     enqueued on that stream.  Use one context per host thread.
 */
#ifndef QEH_H
#define QEH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QEH_ABI_VERSION 1

/* ---- status -------------------------------------------------------------- */
enum qeh_status {
    QEH_OK = 0,
    QEH_E_INVALID = 1,     /* bad argument / shape                          */
    QEH_E_OVERFLOW = 2,    /* checked integer arithmetic overflow           */
    QEH_E_DIV0 = 3,        /* integer division by zero                      */
    QEH_E_OOM = 4,         /* device allocation failed                      */
    QEH_E_UNSUPPORTED = 5, /* operator / type not implemented on device     */
    QEH_E_HIP = 6,         /* HIP runtime error                              */
    QEH_E_TYPE = 7,        /* expression type error (reference error text)  */
    QEH_E_INTERNAL = 8     /* kernel-side protocol failure (bounded spin)   */
};

/* ---- data types (subset of query_core::DataType, types.rs:5-40) ---------- */
enum qeh_dtype {
    QEH_DT_NULL = 0,
    QEH_DT_BOOL = 1,
    QEH_DT_INT32 = 2,
    QEH_DT_INT64 = 3,
    QEH_DT_FLOAT32 = 4,
    QEH_DT_FLOAT64 = 5,
    QEH_DT_UTF8 = 6,   /* values = byte buffer, offsets = int32[length+1] */
    QEH_DT_UINT32 = 7  /* internal: row indices / permutations          */
};

/* An Arrow-layout column.  All pointers are device pointers. */
typedef struct qeh_column {
    int32_t dtype;            /* enum qeh_dtype                               */
    int32_t owned;            /* 1 if allocated by the library (release it)   */
    int64_t length;           /* logical rows                                 */
    int64_t offset;           /* element offset into values/validity (Arrow)  */
    int64_t null_count;       /* -1 = unknown                                 */
    void *values;             /* element buffer (bit-packed for BOOL)         */
    uint8_t *validity;        /* LSB-first bitmap, NULL = all valid           */
    int32_t *offsets;         /* UTF8 only                                    */
    int64_t values_bytes;     /* UTF8 only: size of the byte buffer           */
} qeh_column;

/* ---- expressions: postfix encoding of PhysicalExpr ------------------------
 * physical_plan.rs:74-142.  Only the variants the converters emit
 * (crates/query-pgwire/src/backend.rs:727-756) are representable:
 * Column{index}, Literal(ScalarValue), BinaryExpr, UnaryExpr.  Children come
 * before parents (post-order); the last node is the root.  Type coercion is
 * NOT encoded: the library applies the reference's rules
 * (operators.rs:616-709) itself.                                             */
enum qeh_expr_kind {
    QEH_EX_COLUMN = 1,
    QEH_EX_LITERAL = 2,
    QEH_EX_BINARY = 3,
    QEH_EX_UNARY = 4
};
/* Same order as `BinaryOp` (physical_plan.rs:119-136; TsMatch excluded). */
enum qeh_binop {
    QEH_OP_ADD = 0, QEH_OP_SUB = 1, QEH_OP_MUL = 2, QEH_OP_DIV = 3, QEH_OP_MOD = 4,
    QEH_OP_EQ = 5, QEH_OP_NEQ = 6, QEH_OP_LT = 7, QEH_OP_LTE = 8, QEH_OP_GT = 9,
    QEH_OP_GTE = 10, QEH_OP_AND = 11, QEH_OP_OR = 12
};
/* `UnaryOp` (physical_plan.rs:138-142). */
enum qeh_unop { QEH_UOP_NOT = 0, QEH_UOP_MINUS = 1 };

typedef struct qeh_expr_node {
    int32_t kind;        /* enum qeh_expr_kind                              */
    int32_t op;          /* qeh_binop / qeh_unop                            */
    int32_t index;       /* COLUMN: input column index; UTF8 LITERAL: byte length */
    int32_t lit_dtype;   /* LITERAL: enum qeh_dtype (NULL = ScalarValue::Null) */
    int32_t lit_is_null; /* LITERAL: typed None (e.g. Int64(None))         */
    int32_t _pad;
    int64_t lit_i64;     /* BOOL/INT32/INT64 literal; UTF8 LITERAL: host address of
                            its bytes (read during the call only).  Utf8 operands
                            appear only in comparisons of two leaves (column /
                            literal), evaluated by byte-wise lexicographic order,
                            operators.rs:509-538 on StringArray             */
    double lit_f64;      /* FLOAT32/FLOAT64 literal                         */
} qeh_expr_node;

typedef struct qeh_expr {
    const qeh_expr_node *nodes;
    int32_t n_nodes;
} qeh_expr;

/* ---- aggregates: `AggregateFunction` (physical_plan.rs:150-157) ---------- */
enum qeh_agg_func {
    QEH_AGG_COUNT = 0, QEH_AGG_SUM = 1, QEH_AGG_AVG = 2, QEH_AGG_MIN = 3, QEH_AGG_MAX = 4
};
typedef struct qeh_agg {
    int32_t func;        /* enum qeh_agg_func                                */
    int32_t column;      /* index into the aggregate-input column list       */
} qeh_agg;

/* ---- context / runtime --------------------------------------------------- */
typedef struct qeh_ctx qeh_ctx;

int qeh_abi_version(void);
/* Thread-local message for the last failing call on this thread. */
const char *qeh_last_error(void);

int qeh_init(int device, qeh_ctx **out);
/* 1 when the device serves the lanes of one returning LDS atomic in lane order (the stable tile
 * ranking of the sort, exchange and window passes relies on it; checked once per process by a
 * self-test kernel, else those passes rank by ballot matching), 0 otherwise. */
int qeh_lds_atomic_rank_ok(qeh_ctx *ctx);
int qeh_shutdown(qeh_ctx *ctx);
/* Run on a caller-owned hipStream_t (e.g. torch's current stream); NULL =
 * the context's own stream. */
int qeh_set_stream(qeh_ctx *ctx, void *hip_stream);
void *qeh_get_stream(qeh_ctx *ctx);
int qeh_synchronize(qeh_ctx *ctx);

/* Device memory through the context's caching pool (no hipMalloc on the hot
 * path after warm-up). */
int qeh_device_alloc(qeh_ctx *ctx, size_t bytes, void **out);
int qeh_device_free(qeh_ctx *ctx, void *ptr);
/* Return every cached block to the driver. */
int qeh_pool_trim(qeh_ctx *ctx);
int qeh_memcpy_h2d(qeh_ctx *ctx, void *dst, const void *src, size_t bytes);
int qeh_memcpy_d2h(qeh_ctx *ctx, void *dst, const void *src, size_t bytes);
int qeh_memcpy_d2d(qeh_ctx *ctx, void *dst, const void *src, size_t bytes); /* async */
int qeh_memset(qeh_ctx *ctx, void *dst, int value, size_t bytes);
int qeh_column_release(qeh_ctx *ctx, qeh_column *col);

/* Per-kernel device timing (HIP events on the context stream).  When enabled
 * every launch is bracketed by events; qeh_kernel_time() synchronises and
 * returns total milliseconds and launch count for kernels whose name equals
 * `name` since the last qeh_timing_reset(). */
int qeh_timing_enable(qeh_ctx *ctx, int enable);
int qeh_timing_reset(qeh_ctx *ctx);
int qeh_kernel_time(qeh_ctx *ctx, const char *name, double *total_ms, int64_t *launches);

/* ---- synthetic data (counter-based; identical on host: oracle/qe_oracle.c)
 * value(row) = splitmix64((seed ^ (col_id << 56)) + row), then per kind:
 *   UNIFORM_MOD : (int64)(u % modulus) + lo
 *   UNIT_F64    : (double)(u >> 11) * 2^-53            in [0,1)
 *   PERMUTATION : (row * 0x9E3779B1 + col_id) % modulus  (bijection when
 *                 gcd(0x9E3779B1, modulus) == 1)                            */
/* QEH_GEN_SPARSE_KEY: a 64-bit key H(x) = splitmix64(x ^ seed-derived salt), a bijection of x,
 * with x = the row (modulus == 0: distinct dimension keys) or x = uniform(row) % modulus
 * (modulus > 0: fact keys drawn from the same key set). */
enum qeh_gen_kind { QEH_GEN_UNIFORM_MOD = 0, QEH_GEN_UNIT_F64 = 1, QEH_GEN_PERMUTATION = 2, QEH_GEN_SPARSE_KEY = 3 };
int qeh_generate(qeh_ctx *ctx, int kind, uint64_t seed, uint64_t col_id, int64_t row0,
                 int64_t n, int64_t modulus, int64_t lo, void *out_values);

/* ---- operators (each cites the reference operator it replaces) ----------- */

/* Filter: executor.rs:131-155 (+ arrow filter_record_batch).  Evaluates
 * `predicate` over `cols`, keeps rows where it is TRUE (NULL -> dropped),
 * order-preserving, and gathers columns `out_idx[0..n_out)` into `out`.
 * Non-boolean predicate -> QEH_E_TYPE "Filter predicate must return boolean". */
int qeh_filter(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *predicate,
               const int32_t *out_idx, int n_out, qeh_column *out, int64_t *out_rows);

/* Filter followed by LimitExec (executor.rs:299-341): the first `max_rows` rows that qualify
 * (order-preserving; max_rows < 0: all) — the same rows as qeh_filter then a slice, but
 * outputs are sized to max_rows and input tiles past the cap are not read. */
int qeh_filter_limit(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *predicate,
                     const int32_t *out_idx, int n_out, int64_t max_rows, qeh_column *out, int64_t *out_rows);

/* Projection expression: operators.rs:13-62 evaluate_expr over one input.
 * Column references are returned zero-copy (owned = 0). */
int qeh_eval(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *expr,
             int64_t n_rows, qeh_column *out);

/* Result type of `expr` over inputs of the given dtypes (no device work).
 * Mirrors the reference's typing; errors with the reference's message. */
int qeh_expr_type(const int32_t *col_dtypes, int n_cols, const qeh_expr *expr, int32_t *out_dtype);

/* HashAggregate: executor.rs:157-190, operators.rs:745-848.
 * n_keys == 0: global aggregate -> one row (or zero rows when `input_batches`
 * is 0, matching the reference's "no batches -> no row" quirk, executor.rs:178).
 * n_keys >= 1: one row per distinct key tuple (NULL keys form one group);
 * out_keys[n_keys], out_aggs[n_aggs] are filled; row order unspecified.
 * Result types follow operators.rs:745-848 (COUNT Int64; SUM int->Int64,
 * float->Float64; AVG Float64; MIN/MAX keep the input type).              */
int qeh_hash_aggregate(qeh_ctx *ctx, const qeh_column *keys, int n_keys,
                       const qeh_column *agg_inputs, int n_inputs, const qeh_agg *aggs,
                       int n_aggs, int64_t input_batches, qeh_column *out_keys,
                       qeh_column *out_aggs, int64_t *out_groups);

/* Fused HashAggregate(Filter(input)): executor.rs:38-49 composed without
 * materialising the filtered batch.  `predicate` (may be NULL) and the key /
 * aggregate column indexes all refer to `cols`.  Output as qeh_hash_aggregate. */
int qeh_filter_aggregate(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *predicate,
                         const int32_t *key_idx, int n_keys, const qeh_agg *aggs, int n_aggs,
                         int64_t input_batches, qeh_column *out_keys, qeh_column *out_aggs,
                         int64_t *out_groups);

/* Inner equi-join: the intended semantics of executor.rs:363-381 (the
 * reference ignores `on`).  Builds a hash table on
 * `build_key`, probes with `probe_key` (NULL keys never match), and emits the
 * matching (probe row, build row) pairs with probe payload columns first
 * (left ++ right, executor.rs:532-537).  Row order unspecified.              */
int qeh_hash_join_inner(qeh_ctx *ctx, const qeh_column *probe_key, const qeh_column *probe_cols,
                        int n_probe_cols, const qeh_column *build_key,
                        const qeh_column *build_cols, int n_build_cols, qeh_column *out_probe,
                        qeh_column *out_build, int64_t *out_rows);

/* LEFT / RIGHT / FULL equi-join on one Int32/Int64 key.  The reference sends
 * these through the same Cartesian join_batches as INNER (executor.rs:383-435); the intended
 * semantics extend the INNER contract: every matching (left, right) pair, plus each unmatched left
 * row (LEFT, FULL) with NULL right columns, plus each unmatched right row (RIGHT, FULL) with NULL
 * left columns; NULL keys never match.  join_type: qeh_join_type values (qeh_plan.h) 1 LEFT,
 * 2 RIGHT, 3 FULL (0 = INNER, forwarded to qeh_hash_join_inner with the left side probing).
 * Row order: preserved side's row order, FULL's unmatched right rows last (compare as multisets).
 * LEFT / RIGHT over a unique Int-keyed build side whose payloads are non-null 8-byte columns
 * return the preserved side's columns as views of the inputs (owned = 0, like arrow's column
 * clones): keep the inputs alive while using them; every other output is owned. */
int qeh_hash_join_outer(qeh_ctx *ctx, int join_type, const qeh_column *left_key, const qeh_column *left_cols,
                        int n_left_cols, const qeh_column *right_key, const qeh_column *right_cols, int n_right_cols,
                        qeh_column *out_left, qeh_column *out_right, int64_t *out_rows);

/* Fused filter -> hash-join -> group-by (the BASELINE metric path):
 *   SELECT <build group keys>, AGG(probe cols)... FROM probe JOIN build
 *   ON probe.key = build.key WHERE <predicate over probe cols> GROUP BY <build keys>
 * = HashAggregate(Filter(HashJoin(Scan probe, Scan build))) with the filter
 * referring only to probe-side columns (physical_plan.rs:28-39; the planner's
 * operator order, planner.rs:114-166).  `predicate` may be NULL.
 * Group keys are build-side columns; aggregate inputs are probe-side columns.
 * Output exactly as qeh_hash_aggregate over the joined+filtered rows.     */
int qeh_join_filter_aggregate(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols,
                              int probe_key_idx, const qeh_expr *predicate,
                              const qeh_column *build_key, const qeh_column *build_group_keys,
                              int n_group_keys, const qeh_agg *aggs, int n_aggs,
                              qeh_column *out_keys, qeh_column *out_aggs, int64_t *out_groups);

/* Phase A of qeh_join_filter_aggregate ahead of its build side (a distributed broadcast join:
 * the build shards are still arriving over RCCL).  build_key_range / group_key_range = [min, max,
 * non-null count] of the full build key / the single build group key.  The next
 * qeh_join_filter_aggregate with the same probe columns, key and predicate adopts the launched
 * work when its build columns have exactly these ranges, and discards it otherwise -- results
 * never depend on the hint.  Not launching (shape outside the LDS-slice path) is not an error. */
int qeh_join_filter_aggregate_prelaunch(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols,
                                        int probe_key_idx, const qeh_expr *predicate, const qeh_agg *aggs,
                                        int n_aggs, const int64_t *build_key_range, const int64_t *group_key_range);

/* qeh_join_filter_aggregate_prelaunch with the build ranges still in device memory: `stats` = the
 * ranks' qeh_broadcast_stats rows ([world][row_len], row_len >= 6, column 5 = has-bitmap) as an
 * RCCL all-gather left them.  A plan kernel reduces them to the job-wide ranges and phase A reads its
 * shape from that plan, so the host does not wait for the gather before phase A starts; the adopting
 * call reads the plan back.  Launches nothing when the shape is outside the LDS-slice path. */
int qeh_join_filter_aggregate_prelaunch_stats(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols,
                                              int probe_key_idx, const qeh_expr *predicate, const qeh_agg *aggs,
                                              int n_aggs, const int64_t *stats, int world, int row_len);

/* Broadcast join in table form (the distributed metric path at N > 1; the partial/final stage
 * shape of distributed/planner.rs:200-249): instead of all-gathering the dimension and building the
 * whole join table on every rank, each rank inserts its dimension shard into a DIRECT u16 table
 * over the job-wide key range, the ranks sum their tables (RCCL all-reduce: keys are unique, so
 * every entry has one writer), and the fused probe runs against the summed table.
 *   qeh_direct_group_table_insert: table[key - key_min] = (group key - group_min) + 1 for every row
 *     of this shard; `table` is caller-owned device memory of key_range u16 entries, zeroed by the
 *     caller; keys must lie in [key_min, key_min + key_range) and group keys in
 *     [group_min, group_min + 65534) (QEH_E_INVALID otherwise, nothing written out of range).
 *   qeh_u16_count_nonzero: non-empty entries of such a table (the duplicate check after the sum:
 *     fewer than the job's build rows means a key repeats, and the caller falls back).
 *   qeh_join_filter_aggregate_table: qeh_join_filter_aggregate with that table as the join table;
 *     group g = entry - 1 has key group_min + g (group_dtype Int64 / Int32); only non-empty groups
 *     are returned.  Adopts a phase A prelaunched (qeh_join_filter_aggregate_prelaunch) for the
 *     same probe columns, predicate, aggregates and key range. */
int qeh_direct_group_table_insert(qeh_ctx *ctx, const qeh_column *build_key, const qeh_column *group_key,
                                  int64_t key_min, uint64_t key_range, int64_t group_min, uint16_t *table);
/* The same insert without the range check's host wait: rows outside the ranges are skipped (not an
 * error), which the caller's non-empty count (qeh_u16_count_nonzero_dev) then shows as missing rows.
 * The distributed step queues it while phase A runs. */
int qeh_direct_group_table_insert_async(qeh_ctx *ctx, const qeh_column *build_key, const qeh_column *group_key,
                                        int64_t key_min, uint64_t key_range, int64_t group_min, uint16_t *table);
int qeh_u16_count_nonzero(qeh_ctx *ctx, const uint16_t *table, uint64_t n, int64_t *out);
/* The same count into device memory (*dev_out, 8 B, overwritten), no host wait: the distributed step
 * reads it with its final results instead of stalling the queue between the table sum and the probe. */
int qeh_u16_count_nonzero_dev(qeh_ctx *ctx, const uint16_t *table, uint64_t n, uint64_t *dev_out);
/* The no-wait duplicate check of the summed table: *dev_out = entries in [1, max_entry] (8 B,
 * overwritten), and every entry above max_entry is cleared in place, so a probe queued behind it reads
 * such a key as a miss instead of indexing group state max_entry or beyond.  A build key held by two
 * ranks sums to a larger entry (or to a wrong one); either way the count falls below the job's build
 * rows and the caller discards the probe's result.  max_entry = the group slots G (1..65535). */
int qeh_u16_table_check_dev(qeh_ctx *ctx, uint16_t *table, uint64_t n, uint32_t max_entry, uint64_t *dev_out);
/* [min, max, non-null count] of each Int32 / Int64 column (out[3 i .. 3 i + 2]; an all-NULL or empty
 * column gives min > max), one synchronous read for all of them -- the job-wide build ranges of a
 * distributed broadcast join are gathered from these. */
int qeh_columns_minmax(qeh_ctx *ctx, const qeh_column *cols, int n_cols, int64_t *out);
/* The dense final stage of a distributed broadcast join whose single group key is a bounded
 * integer (the reference's partial/final aggregate, distributed/planner.rs:200-249): this rank's
 * partial states (group keys + n_vals non-null value columns) scattered into f64 lanes
 * [1 + n_vals][range] at key - key_min (lane 0 = 1.0 presence; values exact below 2^53), into
 * caller-zeroed `out`; the caller sums the ranks' lanes (one RCCL all-reduce), then
 * qeh_dense_states_take returns the groups this rank owns ((key - key_min) % world == rank) that
 * are present, in key order, as key_dtype keys and out_dtypes[j] (Int64 / Float64) values. */
int qeh_dense_states_f64(qeh_ctx *ctx, const qeh_column *keys, const qeh_column *vals, int n_vals, int64_t key_min,
                         int64_t range, double *out);
int qeh_dense_states_take(qeh_ctx *ctx, const double *in, int n_vals, int64_t key_min, int64_t range, int world,
                          int rank, int32_t key_dtype, const int32_t *out_dtypes, qeh_column *out_keys,
                          qeh_column *out_vals, int64_t *out_groups);
int qeh_join_filter_aggregate_table(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols, int probe_key_idx,
                                    const qeh_expr *predicate, const uint16_t *table, int64_t key_min,
                                    uint64_t key_range, int64_t group_min, int64_t n_groups, int32_t group_dtype,
                                    const qeh_agg *aggs, int n_aggs, qeh_column *out_keys, qeh_column *out_aggs,
                                    int64_t *out_groups);
/* The same fused operator with the dense final stage's input as its output: instead of compacted
 * group columns, f64 lanes [1 + n_aggs][n_groups] in caller-owned device memory (every entry
 * written): lane 0 = the group's row count (> 0: present), lane 1 + j = aggregate j's partial state
 * (COUNT, or SUM of a non-null Float64 column; QEH_E_UNSUPPORTED for others).  Summed over the
 * ranks (RCCL all-reduce) they are qeh_dense_states_take's input -- the partial/final aggregate of
 * distributed/planner.rs:200-249 without compacting, finalizing and re-scattering the partials. */
int qeh_join_filter_aggregate_table_lanes(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols,
                                          int probe_key_idx, const qeh_expr *predicate, const uint16_t *table,
                                          int64_t key_min, uint64_t key_range, int64_t n_groups, const qeh_agg *aggs,
                                          int n_aggs, double *lanes);
/* ..._lanes without a host wait: the operator's status words go to dev_status[0..3] (device memory;
 * [0] kernel error bits, [1] a slice region overflowed -- then the lanes are incomplete), and one more
 * lane after the (1 + n_aggs) * n_groups ones, lanes[(1 + n_aggs) * n_groups] = 1.0 when either is set
 * (else 0.0; `lanes` holds (1 + n_aggs) * n_groups + 1 doubles), so an all-reduce of the lanes carries
 * every rank's flag.  The call returns as soon as its kernels are queued; the caller reads the flag
 * with its final results and, when it is set, runs qeh_join_filter_aggregate_table_lanes (which
 * recovers) instead. */
int qeh_join_filter_aggregate_table_lanes_async(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols,
                                                int probe_key_idx, const qeh_expr *predicate, const uint16_t *table,
                                                int64_t key_min, uint64_t key_range, int64_t n_groups,
                                                const qeh_agg *aggs, int n_aggs, double *lanes, uint32_t *dev_status);
/* This dimension shard's broadcast-join statistics into device memory, no host wait:
 * dev_out[0..4] = [rows, build key min, max, group key min, max] (min > max for an empty or all-NULL
 * shard), dev_out[5 + i] = extra[i] (n_extra <= 16: flags the caller gathers with them).  The ranks
 * all-gather these rows (RCCL) and read them back once, instead of a min/max read plus a gather. */
int qeh_broadcast_stats(qeh_ctx *ctx, const qeh_column *build_key, const qeh_column *group_key, const int64_t *extra,
                        int n_extra, int64_t *dev_out);

/* The items form of the distributed broadcast join (the BASELINE metric at N > 1; replaces the
 * table form's all-reduced 2-B-per-key table).  Distributed HashJoinExec + HashAggregateExec
 * (query-distributed/src/planner.rs:200-249 over query-executor/src/executor.rs:157-190, 363-381):
 *   qeh_fused_items_begin: plans the fused pipeline from the gathered qeh_broadcast_stats rows
 *     (stats_dev[world][row_len], device memory) and queues phase A over this rank's fact shard
 *     (probe_cols) -- no host wait; *handle is opaque.  COUNT and non-null Float64 SUM aggregates over
 *     at most one aggregate column, a column-literal predicate list (QEH_E_UNSUPPORTED otherwise).
 *   qeh_fused_items_build: this rank's dimension rows (one non-null Int64 key, one non-null integer
 *     group key) grouped by 2^16-key slice by n_blocks workgroups, each into its own span of `span` u32
 *     (span >= ceil(rows / n_blocks) + 640, a multiple of 4; items: caller-owned device memory of
 *     n_blocks * span u32): span w's slice b has offs[w * 322 + 161 + b] items from
 *     items[w * span + offs[w * 322 + b]] (a multiple of 4); offs holds n_blocks * 322 u32.
 *   (caller: all-gather items and offs over the ranks, rank-major; every rank uses the same n_blocks
 *     and span)
 *   qeh_fused_items_finish: phase B over the n_regions = world * n_blocks gathered spans (region r at
 *     items + r * span, its offs at offs + r * 322; n_regions <= 512) and the dense final stage's
 *     lanes as qeh_join_filter_aggregate_table_lanes_async writes them for group keys
 *     group_min + [0, n_groups) ((1 + n_aggs) * n_groups + 1 doubles; the last = 1.0 when the plan
 *     declined the shape, a key lies outside the gathered ranges, a key repeats -- on any rank -- or a
 *     kernel failed: the caller then takes another form).  Frees the handle.
 *   qeh_fused_items_abort: waits for the queued work and frees the handle (a rank that does not finish). */
int qeh_fused_items_begin(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols, int probe_key_idx,
                          const qeh_expr *predicate, const qeh_agg *aggs, int n_aggs, const int64_t *stats_dev, int world,
                          int row_len, void **handle);
int qeh_fused_items_build(qeh_ctx *ctx, void *handle, const qeh_column *build_key, const qeh_column *group_key,
                          int n_blocks, uint64_t span, uint32_t *items, uint32_t *offs);
int qeh_fused_items_finish(qeh_ctx *ctx, void *handle, const uint32_t *items, uint64_t span, const uint32_t *offs,
                           int n_regions, int64_t n_groups, double *lanes);
int qeh_fused_items_abort(qeh_ctx *ctx, void *handle);
/* The items form of the shuffle join (BASELINE config 4, hash-partitioned join + aggregate; replaces
 * the two-pass filter + exchange and the receiving rank's own pipeline over (key, value) rows for the
 * shapes qeh_fused_items_check accepts).  The partition function: a fact or dimension row with join
 * key k goes to rank ((k - kmin) >> 16) % world, kmin = the job-wide dimension key minimum -- a
 * modulo hash of the key's 2^16-key slice, so both sides of every key meet on one rank.
 *   qeh_shuffle_items_begin: as qeh_fused_items_begin (plan from the gathered stats rows, phase A
 *     queued over this rank's fact shard, no host wait), with the regions laid out per destination.
 *   qeh_fused_items_build: this rank's dimension items, all-gathered by the caller as for the
 *     broadcast items form (phase B takes each of its slices' rows from every rank's spans).
 *   qeh_shuffle_items_pack: waits for phase A; *ok = 0 (nothing allocated) when the plan declined, a
 *     region filled up or a kernel failed -- every rank must then learn it (the caller gathers the flag)
 *     and take the two-pass path.  Else packs each destination q's regions into one block: keys
 *     (*keys)[q * blockcap ..] and values (*vals)[q * blockcap ..], totals[q] items (region counts
 *     rounded up to 2), and the block's region counts (*counts)[q * block_regions .. + block_regions],
 *     all library-owned until qeh_shuffle_items_finish returns.  This rank's own block is not packed
 *     (its keys / values stay in phase A's regions, read there by finish): totals[rank] is its size.
 *   (caller: all-to-all of the totals[q] keys and values of block q to rank q, source-major on the
 *   receiver, nothing to or from itself; all-to-all of the block_regions counts, its own included)
 *   qeh_shuffle_items_finish: phase B over the received blocks (keys / vals / counts as the
 *     all-to-all left them, source q's items from src_offsets[q], world entries, host memory; the
 *     entry of this rank unused) and this rank's own regions in place, with
 *     this rank's slices built from the gathered dimension items (n_regions spans of `span`, as
 *     qeh_fused_items_finish), then the dense final stage's lanes ((1 + n_aggs) * n_groups + 1
 *     doubles, the last = the status lane: a key on two ranks, an overflow); frees the handle.
 *   qeh_fused_items_abort frees a handle that does not finish. */
int qeh_shuffle_items_begin(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols, int probe_key_idx,
                            const qeh_expr *predicate, const qeh_agg *aggs, int n_aggs, const int64_t *stats_dev,
                            int world, int rank, int row_len, void **handle);
int qeh_shuffle_items_pack(qeh_ctx *ctx, void *handle, uint16_t **keys, int64_t **vals, uint32_t **counts,
                           uint64_t *blockcap, int64_t *block_regions, int64_t *totals, int *ok);
int qeh_shuffle_items_finish(qeh_ctx *ctx, void *handle, const uint16_t *keys, const int64_t *vals,
                             const uint32_t *counts, const int64_t *src_offsets, const uint32_t *items, uint64_t span,
                             const uint32_t *offs, int n_regions, int64_t n_groups, double *lanes);
/* qeh_dense_states_take that also returns the status lane after the (1 + n_vals) * range lanes (the
 * no-wait forms' flag) in *status, from the same host read as the group count. */
int qeh_dense_states_take_status(qeh_ctx *ctx, const double *in, int n_vals, int64_t key_min, int64_t range,
                                 int world, int rank, int32_t key_dtype, const int32_t *out_dtypes,
                                 qeh_column *out_keys, qeh_column *out_vals, int64_t *out_groups, double *status);
/* qeh_fused_items_begin's shape checks only (QEH_OK or QEH_E_UNSUPPORTED; nothing queued): the flag
 * every rank contributes to the gathered stats before any rank's choice of collectives depends on it. */
int qeh_fused_items_check(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols, int probe_key_idx,
                          const qeh_expr *predicate, const qeh_agg *aggs, int n_aggs);

/* Stable lexicographic sort -> permutation (UINT32 row ids) of the input.
 * Intended semantics of `Sort` (physical_plan.rs:40-44; executor.rs:290-297
 * is the identity): per-key ascending flag, NULLs first, floats totalOrder. */
int qeh_sort_indices(qeh_ctx *ctx, const qeh_column *keys, int n_keys, const int8_t *ascending,
                     qeh_column *out_perm);

/* qeh_sort_indices with arrow SortOptions.nulls_first per key (nulls_first NULL: all first),
 * as Merge::sorted passes it (crates/query-distributed/src/operators.rs:97-104,163-172). */
int qeh_sort_indices_nulls(qeh_ctx *ctx, const qeh_column *keys, int n_keys, const int8_t *ascending,
                           const int8_t *nulls_first, qeh_column *out_perm);

/* arrow concat of one column's parts (same dtype), as concat_batches does per column
 * (operators.rs:206-216, executor.rs:176-181). */
int qeh_concat(qeh_ctx *ctx, const qeh_column *parts, int n_parts, qeh_column *out);

/* Merge::execute with MergeStrategy::SortedMerge (operators.rs:143-193): concatenate the
 * partitions' columns (`parts` = [n_parts][n_cols], partition-major) and sort the rows by
 * columns key_idx[0..n_keys) (ascending / nulls_first per key); n_keys == 0 returns the
 * concatenation, as the reference does when no sort column name resolves.  Outputs n_cols
 * owned columns. */
int qeh_merge_sorted(qeh_ctx *ctx, const qeh_column *parts, int n_parts, int n_cols, const int32_t *key_idx,
                     const int8_t *ascending, const int8_t *nulls_first, int n_keys, qeh_column *out,
                     int64_t *out_rows);

/* Gather rows `indices` (UINT32 or INT64 device column) of `col`. */
int qeh_take(qeh_ctx *ctx, const qeh_column *col, const qeh_column *indices, qeh_column *out);

/* ROW_NUMBER() OVER (PARTITION BY part_keys ORDER BY order_keys): Int64 column
 * aligned to input order; 1-based within each partition, ties broken by input
 * position (docs/WINDOW_FUNCTIONS.md:44-65; `WindowFunctionType::RowNumber`,
 * physical_plan.rs:160-179). */
int qeh_row_number(qeh_ctx *ctx, const qeh_column *part_keys, int n_part,
                   const qeh_column *order_keys, int n_order, const int8_t *ascending,
                   qeh_column *out_rn);

/* The other `WindowFunctionType`s (physical_plan.rs:160-170; semantics of
 * docs/WINDOW_FUNCTIONS.md:67-205, the reference executor passes Window through,
 * executor.rs:76-80) over the ROW_NUMBER order (PARTITION BY keys, then ORDER BY keys, ties by
 * input position).  func = enum qeh_window_func (qeh_plan.h):
 *   ROW_NUMBER / RANK / DENSE_RANK / NTILE(param >= 1) -> Int64, no NULLs;
 *   LAG / LEAD(arg, param >= 0 rows) / FIRST_VALUE / LAST_VALUE(arg) -> arg's type
 *   (Int32/Int64/Float32/Float64), NULL where arg is NULL or the offset leaves the partition
 *   (then *dflt, the value's bit pattern, when dflt != NULL).  LAST_VALUE spans the whole
 *   partition (WindowExpr carries no frame).  Peers compare keys by value bits (NULLs equal).
 * With no keys (OVER ()), `arg` must be given and supplies the row count. */
int qeh_window(qeh_ctx *ctx, int32_t func, const qeh_column *part_keys, int n_part,
               const qeh_column *order_keys, int n_order, const int8_t *ascending,
               const qeh_column *arg, int64_t param, const int64_t *dflt, qeh_column *out);

/* Hash partitioning for multi-GPU exchange (model: Partitioner::partition_by_hash,
 * crates/query-distributed/src/partition.rs:151-212; the hash function is not
 * observable in results, §8 row a15).  Writes `counts[n_parts]` and a
 * partition-major permutation (UINT32) so that rows of partition p are
 * perm[offsets[p] .. offsets[p]+counts[p]), stable within a partition.
 * NULL keys go to partition 0 (reference skips them when hashing,
 * partition.rs:292-316, i.e. they hash like an empty key). */
int qeh_hash_partition(qeh_ctx *ctx, const qeh_column *key, int n_parts, int64_t *counts,
                       qeh_column *out_perm);

/* Range partition for distributed Sort / ORDER BY (SURVEY.md §8 row e):
 * partition p holds the rows whose order key lies between splitters p-1 and p
 * (`splitters` = host array of ascending order keys: the Int value itself, the
 * IEEE totalOrder key of Float64 bits, Float32 widened to Float64 first);
 * equal keys share a partition, NULLs go to partition 0 (NULLs first, as in
 * qeh_sort_indices); `ascending` = 0 reverses the partition order.  Same
 * counts / stable partition-major `out_perm` contract as qeh_hash_partition. */
int qeh_range_partition(qeh_ctx *ctx, const qeh_column *key, int ascending, const int64_t *splitters,
                        int n_splitters, int64_t *counts, qeh_column *out_perm);

/* Partitioner::partition_by_hash over several key columns (distributed/partition.rs:151-212):
 * a partition-major permutation, stable within a partition, with per-partition row counts.
 * Int32 / Int64 / Utf8 keys; NULL cells are skipped when hashing, as compute_row_hash does
 * (partition.rs:292-316).  The hash differs from the reference's SipHash: which partition a
 * key lands in is not observable in query results; rows with equal keys always share one. */
int qeh_partition_hash(qeh_ctx *ctx, const qeh_column *keys, int n_keys, int n_parts, int64_t *counts,
                       qeh_column *out_perm);

/* qeh_partition_hash + the gathers in one go: `cols` leave in partition-major order (stable)
 * as owned columns out_cols[0 .. n_cols), with per-partition counts.  Non-null Int64 / Float64
 * columns are moved by a single tile-ranked pass; other columns through the permutation. */
int qeh_partition_hash_move(qeh_ctx *ctx, const qeh_column *keys, int n_keys, int n_parts, const qeh_column *cols,
                            int n_cols, int64_t *counts, qeh_column *out_cols);
/* The reverse of qeh_partition_hash_move over one non-null Int64 key into at most 16 partitions:
 * out_cols[c][i] = moved[c][p(i)], p(i) = row i's position in the stable partition-major order the
 * move produces (rows of lower partitions, then the rows of its own partition before it) -- results
 * computed on moved rows (a distributed window function's numbers, returned by the reverse
 * all-to-all) back into input order in one streaming pass.  1..2 non-null Int64 / Float64 columns of
 * the key's length. */
int qeh_partition_hash_unmove(qeh_ctx *ctx, const qeh_column *key, int n_parts, const qeh_column *moved, int n_cols,
                              qeh_column *out_cols);

/* FilterExec followed by the hash Exchange of a shuffle stage (executor.rs:131-155, then
 * partition.rs:151-212 / operators.rs:15-73; config 4's probe side), fused: rows of `cols` whose
 * `predicate` is TRUE are hash-partitioned by cols[key_idx] (same partition function as
 * qeh_partition_hash), and columns move_idx[0 .. n_move) leave partition-major (stable) in
 * out_cols, with per-partition counts.  The predicate must be an AND / OR list of column-literal
 * comparisons; the key Int32 / Int64; moved columns non-null Int64 / Float64 (1..4) -- otherwise
 * QEH_E_UNSUPPORTED and the caller runs qeh_filter + qeh_partition_hash_move. */
int qeh_filter_partition_hash_move(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *predicate,
                                   int key_idx, int n_parts, const int32_t *move_idx, int n_move, int64_t *counts,
                                   qeh_column *out_cols);

/* Partitioner::partition_by_range (partition.rs:259-341): row -> the first i with
 * value < boundaries[i], else n_boundaries; NULL -> 0; a non-Int64 key puts every row in
 * partition 0, as the reference does.  Same output as qeh_partition_hash. */
int qeh_partition_range(qeh_ctx *ctx, const qeh_column *key, const int64_t *boundaries, int n_boundaries,
                        int64_t *counts, qeh_column *out_perm);

/* out[indices[i]] = col[i] (inverse of qeh_take for a permutation): returns
 * per-row results to their original positions after an exchange.  Non-null
 * fixed-width columns; `indices` UINT32 of the same length. */
int qeh_scatter(qeh_ctx *ctx, const qeh_column *col, const qeh_column *indices, qeh_column *out);

/* Result encoding: PostgreSQL DataRow messages in text format, one per row,
 * as crates/query-pgwire/src/result.rs:56-176 builds them through pgwire 0.28.0 (NULL -> length
 * -1, booleans "t"/"f", integers in decimal, floats as Rust's Display: shortest round-trip
 * digits without exponent, Utf8 bytes).  `out` is an owned Utf8 column whose string i is row
 * i's complete message ('D', Int32 length, Int16 field count, fields), ready to be sent.
 * Types: BOOL, INT32, INT64, UINT32 (as Int64), FLOAT32, FLOAT64, UTF8; <= 32 columns;
 * QEH_E_UNSUPPORTED when the messages exceed 2 GiB (encode the batch in slices). */
int qeh_encode_pg_datarows(qeh_ctx *ctx, const qeh_column *cols, int n_cols, qeh_column *out);

/* Arrow IPC stream of one batch (schema message, record batch message, end-of-stream), as
 * SerializedBatch::from_batch writes it with arrow-rs's StreamWriter
 * (crates/query-distributed/src/network.rs:56-72): fields nullable, named `names[i]`, body
 * buffers 64-byte aligned.  Device columns are normalised to offset 0 on the device and copied
 * into a host buffer the library allocates; free it with qeh_host_free. */
int qeh_encode_arrow_ipc(qeh_ctx *ctx, const qeh_column *cols, const char *const *names, int n_cols,
                         uint8_t **out_bytes, int64_t *out_size);
void qeh_host_free(void *p);

/* The first record batch of an Arrow IPC stream, as SerializedBatch::to_batch reads it
 * (network.rs:75-90), uploaded into owned device columns out_cols[0 .. *out_n_cols); the field
 * names come back NUL-separated in *out_names (free with qeh_host_free; may be NULL).  Int32 /
 * Int64 / UInt32 / Float32 / Float64 / Utf8 / Bool fields; dictionaries, nesting and body
 * compression -> QEH_E_UNSUPPORTED; malformed or truncated input -> QEH_E_INVALID. */
int qeh_decode_arrow_ipc(qeh_ctx *ctx, const uint8_t *bytes, int64_t size, qeh_column *out_cols, int max_cols,
                         int *out_n_cols, char **out_names, int64_t *out_rows);

/* Validity bitmap <-> one byte per row (1 = valid), for moving nullable
 * columns through byte-addressed collectives (RCCL all-to-all splits are
 * row counts, not bit offsets).  Buffers are device pointers. */
int qeh_validity_to_bytes(qeh_ctx *ctx, const qeh_column *col, uint8_t *out_bytes);
int qeh_bytes_to_validity(qeh_ctx *ctx, const uint8_t *bytes, int64_t n, uint8_t *out_bitmap);

#ifdef __cplusplus
}
#endif
#endif /* QEH_H */
