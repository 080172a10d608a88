/*
 * qeh_plan.h — plan-level C ABI: QueryExecutor::execute(&PhysicalPlan).
 *
 * Reference interface replaced: `QueryExecutor::execute(&self, plan:
 * &PhysicalPlan) -> query_core::Result<Vec<RecordBatch>>`
 * (crates/query-executor/src/executor.rs:19-21, dispatch :23-91) over the
 * closed enum `PhysicalPlan` (crates/query-executor/src/physical_plan.rs:13-72).
 *
 * The enum crosses the boundary as a flat array of nodes in any order with
 * child indices (a Rust binding emits it post-order while walking the enum,
 * INTEGRATION.md).  `DataSource::scan()` results (physical_plan.rs:8-11) enter
 * as Arrow C Data Interface record batches (struct arrays), borrowed for the
 * duration of the call; the result leaves as ONE exported record batch (or
 * none, when the reference would return `vec![]`), owned by the caller and
 * freed through its `release` callbacks — exactly what arrow-rs's
 * `arrow::ffi::{FFI_ArrowArray, FFI_ArrowSchema}` import.  Batch boundaries
 * are not semantically visible in the reference except through its
 * "no batches" quirks, which the executor tracks.
 */
#ifndef QEH_PLAN_H
#define QEH_PLAN_H

#include "qeh.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Arrow C Data Interface (Arrow format spec, stable ABI) ------------- */
#ifndef ARROW_C_DATA_INTERFACE
#define ARROW_C_DATA_INTERFACE
#define ARROW_FLAG_DICTIONARY_ORDERED 1
#define ARROW_FLAG_NULLABLE 2
#define ARROW_FLAG_MAP_KEYS_SORTED 4
struct ArrowSchema {
    const char *format;
    const char *name;
    const char *metadata;
    int64_t flags;
    int64_t n_children;
    struct ArrowSchema **children;
    struct ArrowSchema *dictionary;
    void (*release)(struct ArrowSchema *);
    void *private_data;
};
struct ArrowArray {
    int64_t length;
    int64_t null_count;
    int64_t offset;
    int64_t n_buffers;
    int64_t n_children;
    const void **buffers;
    struct ArrowArray **children;
    struct ArrowArray *dictionary;
    void (*release)(struct ArrowArray *);
    void *private_data;
};
#endif

/* `PhysicalPlan` variants, physical_plan.rs:13-72 (declaration order) */
enum qeh_plan_kind {
    QEH_PLAN_SCAN = 0,
    QEH_PLAN_PROJECTION = 1,
    QEH_PLAN_FILTER = 2,
    QEH_PLAN_HASH_JOIN = 3,
    QEH_PLAN_HASH_AGGREGATE = 4,
    QEH_PLAN_SORT = 5,
    QEH_PLAN_LIMIT = 6,
    QEH_PLAN_SUBQUERY_SCAN = 7,
    QEH_PLAN_WINDOW = 8,
    QEH_PLAN_INDEX_SCAN = 9
};

/* `query_parser::JoinType` */
enum qeh_join_type { QEH_JOIN_INNER = 0, QEH_JOIN_LEFT = 1, QEH_JOIN_RIGHT = 2, QEH_JOIN_FULL = 3, QEH_JOIN_CROSS = 4 };

/* `WindowFunctionType`, physical_plan.rs:160-170 */
enum qeh_window_func {
    QEH_WIN_ROW_NUMBER = 0, QEH_WIN_RANK = 1, QEH_WIN_DENSE_RANK = 2, QEH_WIN_NTILE = 3,
    QEH_WIN_LAG = 4, QEH_WIN_LEAD = 5, QEH_WIN_FIRST_VALUE = 6, QEH_WIN_LAST_VALUE = 7
};

/* `AggregateExpr { func, expr }`, physical_plan.rs:144-148 */
typedef struct qeh_agg_expr {
    int32_t func; /* enum qeh_agg_func */
    int32_t _pad;
    qeh_expr expr;
} qeh_agg_expr;

/* `WindowExpr { func, args, partition_by, order_by }`, physical_plan.rs:172-179 */
typedef struct qeh_window_expr {
    int32_t func; /* enum qeh_window_func */
    int32_t n_args;
    const qeh_expr *args;
    int32_t n_partition;
    int32_t n_order;
    const qeh_expr *partition_by;
    const qeh_expr *order_by;
} qeh_window_expr;

typedef struct qeh_plan_node {
    int32_t kind;             /* enum qeh_plan_kind                                   */
    int32_t input;            /* child (Projection/Filter/Aggregate/Sort/Limit/Window/SubqueryScan) */
    int32_t left, right;      /* HASH_JOIN children                                   */
    int32_t source;           /* SCAN / INDEX_SCAN: index into the sources array      */
    int32_t join_type;        /* HASH_JOIN: enum qeh_join_type                        */
    int32_t has_predicate;    /* FILTER: 1; HASH_JOIN: `on` is Some                   */
    int32_t n_exprs;          /* PROJECTION exprs / SORT exprs / AGGREGATE group exprs */
    qeh_expr predicate;       /* FILTER predicate / HASH_JOIN on                      */
    const qeh_expr *exprs;
    const int8_t *ascending;  /* SORT: one flag per expr                              */
    const qeh_agg_expr *aggs; /* HASH_AGGREGATE aggr_exprs                            */
    const qeh_window_expr *window;
    int32_t n_aggs;
    int32_t n_window;
    int64_t skip;             /* LIMIT                                                */
    int64_t fetch;            /* LIMIT: -1 = None                                     */
    int32_t n_fields;         /* output schema names (PROJECTION / WINDOW), Schema::to_arrow */
    int32_t _pad;
    const char *const *field_names;
} qeh_plan_node;

typedef struct qeh_plan {
    const qeh_plan_node *nodes;
    int32_t n_nodes;
    int32_t root;
} qeh_plan;

/* `DataSource::scan()` result for one Scan / IndexScan source (borrowed).
 * cache_key != 0: the caller promises that every source passed with this key
 * holds identical data (e.g. a MemoryDataSource's table id + version, memory.rs
 * scan() returns clones of the same Arc'd batches); the device copy made by the
 * first query is kept on the context and reused without touching the batches
 * until qeh_source_cache_evict.  0: import on every call (the reference's
 * per-query Vec<RecordBatch>). */
typedef struct qeh_source {
    struct ArrowSchema *schema;        /* struct schema of the batches          */
    struct ArrowArray *const *batches; /* struct arrays, one per RecordBatch    */
    int64_t n_batches;
    uint64_t cache_key;
} qeh_source;

/* Drop the cached device copy of `cache_key` (0: every entry). */
int qeh_source_cache_evict(qeh_ctx *ctx, uint64_t cache_key);
/* Cache occupancy and counters since the context was created. */
int qeh_source_cache_stats(qeh_ctx *ctx, int64_t *entries, int64_t *bytes, int64_t *hits, int64_t *misses);
/* Device bytes the cache may hold before it drops its oldest entries (default 64 GiB). */
int qeh_source_cache_budget(qeh_ctx *ctx, int64_t bytes);

/* Execute `plan` on the device.  On success *out_n_batches is 0 (the
 * reference returns no batches; out_* untouched, release == NULL) or 1
 * (out_schema / out_batch hold one exported record batch, caller releases).
 * Errors: reference messages through qeh_last_error(), status as qeh.h. */
int qeh_execute_plan(qeh_ctx *ctx, const qeh_plan *plan, const qeh_source *sources, int n_sources,
                     struct ArrowSchema *out_schema, struct ArrowArray *out_batch, int64_t *out_n_batches);

#ifdef __cplusplus
}
#endif
#endif /* QEH_PLAN_H */
