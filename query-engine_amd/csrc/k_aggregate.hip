// HashAggregateExec and the fused Filter -> HashJoin -> HashAggregate pipeline.
//
// Reference: execute_aggregate (crates/query-executor/src/executor.rs:157-190)
// computes global aggregates by concatenating every batch of the argument and
// calling evaluate_aggregate (operators.rs:745-848); GROUP BY returns no rows
// (:189).  The intended grouped semantics are SURVEY.md §8.0: one row per
// distinct key tuple, NULL keys form one group, key columns then aggregates.
//
// Device design: each row resolves a dense group id (0 for a global
// aggregate, a read-only group-table probe for GROUP BY, a join-table probe
// whose payload IS the group id for the fused pipeline), then updates 64-bit
// state words with LDS atomics (per-workgroup partials, flushed once per
// workgroup with global atomics) or directly with global atomics when the
// states do not fit the LDS budget.  A finalize pass compacts non-empty
// groups and converts states to the reference's result types.
#include <algorithm>
#include <cstring>
#include <string>

#include "agg.h"
#include "expr_device.h"
#include "ops.h"

namespace qeh {

constexpr int kAggR = 4;                           // rows per lane
constexpr int kAggTile = kBlock * kAggR;           // rows per workgroup iteration
constexpr size_t kLdsStateBudget = 48 * 1024;      // bytes of LDS state per workgroup

enum GidMode { GM_ZERO = 0, GM_JOIN = 1, GM_GROUP = 2 };
enum PredMode { PM_NONE = 0, PM_TERMS = 1, PM_PROG = 2 };

struct GidSource {
    HashTable jt;            // GM_JOIN
    int32_t key_col;         // GM_JOIN: probe key column in the ColSet
    int32_t _pad;
    KeyCols gk;              // GM_GROUP: key columns (absolute ColRefs)
    const uint32_t *gslots;  // GM_GROUP
    uint64_t gmask;
    const uint64_t *gdense;
};

template <int GM, int PM, bool LDS>
__global__ __launch_bounds__(kBlock) void k_agg_rows(ColSet cols, int64_t n, PredTerms terms, DevProgram prog,
                                                     GidSource src, AggSpecs specs, int64_t G,
                                                     uint64_t *__restrict__ gstates, uint32_t *__restrict__ errp) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    uint64_t *st = LDS ? lds : gstates;
    const int64_t stride_slot = G;
    if (LDS) {
        const int64_t words = (int64_t)specs.n_slots * G;
        for (int64_t i = threadIdx.x; i < words; i += blockDim.x) lds[i] = 0;
        __syncthreads();
        for (int a = 0; a < specs.n; ++a) {
            const AggSpec sp = specs.a[a];
            if (sp.kind == AK_MIN || sp.kind == AK_MAX)
                for (int64_t g = threadIdx.x; g < G; g += blockDim.x)
                    lds[(int64_t)sp.val_slot * stride_slot + g] = (uint64_t)agg_init_value(sp.kind);
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t err = 0;
    const int64_t ntiles = (n + kAggTile - 1) / kAggTile;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t row0 = tile * kAggTile + (int64_t)wave * 64 * kAggR + lane;
        uint32_t sel;
        if (PM == PM_TERMS) {
            sel = eval_terms<kAggR>(terms, cols, row0, 64, n);
        } else if (PM == PM_PROG) {
            ExprRegs<kAggR> X;
            run_program<kAggR>(prog, cols, row0, 64, n, X, err);
            sel = program_true_mask<kAggR>(X);
        } else {
            sel = 0;
#pragma unroll
            for (int r = 0; r < kAggR; ++r)
                if (row0 + r * 64 < n) sel |= 1u << r;
        }
        int64_t kv[kAggR];
        uint32_t kvalid = 0;
        if (GM == GM_JOIN) load_rows<kAggR>(cols.c[src.key_col], row0, 64, n, kv, kvalid);
#pragma unroll
        for (int r = 0; r < kAggR; ++r) {
            if (!((sel >> r) & 1)) continue;
            const int64_t row = row0 + r * 64;
            auto apply = [&](uint32_t g) {
                atomicAdd((unsigned long long *)&st[g], 1ull);
                for (int a = 0; a < specs.n; ++a) {
                    const AggSpec sp = specs.a[a];
                    const ColRef &c = cols.c[sp.col];
                    if (!col_valid(c, row)) continue;
                    if (sp.cnt_slot) atomicAdd((unsigned long long *)&st[(int64_t)sp.cnt_slot * stride_slot + g], 1ull);
                    if (sp.kind != AK_COUNT) {
                        int64_t x = agg_input(sp.kind, sp.in_type, load_i64(c, row));
                        agg_apply<LDS>(sp.kind, &st[(int64_t)sp.val_slot * stride_slot + g], x);
                    }
                }
            };
            if (GM == GM_ZERO) {
                apply(0u);
            } else if (GM == GM_JOIN) {
                if ((kvalid >> r) & 1) table_probe(src.jt, kv[r], apply);
            } else {
                uint64_t s = group_find(src.gk, row, src.gslots, src.gmask);
                apply((uint32_t)src.gdense[s]);
            }
        }
    }
    if (err) atomicOr(errp, err);
    if (LDS) {
        __syncthreads();
        for (int64_t g = threadIdx.x; g < G; g += blockDim.x) {
            uint64_t rows = lds[g];
            if (!rows) continue;
            atomicAdd((unsigned long long *)&gstates[g], (unsigned long long)rows);
            for (int a = 0; a < specs.n; ++a) {
                const AggSpec sp = specs.a[a];
                if (sp.cnt_slot) {
                    uint64_t c = lds[(int64_t)sp.cnt_slot * stride_slot + g];
                    if (c) atomicAdd((unsigned long long *)&gstates[(int64_t)sp.cnt_slot * stride_slot + g], (unsigned long long)c);
                }
                if (sp.kind != AK_COUNT)
                    agg_merge_global(sp.kind, &gstates[(int64_t)sp.val_slot * stride_slot + g],
                                     lds[(int64_t)sp.val_slot * stride_slot + g]);
            }
        }
    }
}

__global__ void k_states_init(uint64_t *states, int64_t G, AggSpecs specs) {
    const int64_t words = (int64_t)specs.n_slots * G;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t slot = i / G;
        uint64_t v = 0;
        for (int a = 0; a < specs.n; ++a)
            if (specs.a[a].val_slot == slot) v = (uint64_t)agg_init_value(specs.a[a].kind);
        states[i] = v;
    }
}

// ---- finalize ------------------------------------------------------------------------
__global__ void k_group_nonempty(const uint64_t *states, int64_t G, uint32_t *flags) {
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (int64_t)gridDim.x * blockDim.x)
        flags[g] = states[g] != 0;
}

struct OutCol {
    void *values;
    uint32_t *validity;  // nullptr when never null
    int32_t dtype;
    int32_t _pad;
};
struct OutCols {
    OutCol c[kMaxGroupKeys + kMaxAggs];
};

__device__ __forceinline__ void write_value(const OutCol &o, int64_t p, int64_t payload, bool valid) {
    if (o.validity && valid) atomicOr(&o.validity[p >> 5], 1u << (p & 31));
    switch (o.dtype) {
        case QEH_DT_BOOL:
            if (payload & 1) atomicOr(&((uint32_t *)o.values)[p >> 5], 1u << (p & 31));
            break;
        case QEH_DT_INT32: ((int32_t *)o.values)[p] = (int32_t)payload; break;
        case QEH_DT_FLOAT32: ((float *)o.values)[p] = (float)as_f64(payload); break;
        default: ((int64_t *)o.values)[p] = payload; break;  // INT64, FLOAT64 bits
    }
}

__global__ void k_finalize(const uint64_t *__restrict__ states, int64_t G, const uint64_t *__restrict__ pos,
                           KeyCols keys, const uint32_t *__restrict__ rep_row, AggSpecs specs, OutCols outs) {
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t rows = states[g];
        int64_t p;
        if (pos) {
            if (!rows) continue;
            p = (int64_t)pos[g];
        } else {
            p = g;
        }
        for (int k = 0; k < keys.n; ++k) {
            const int64_t r = rep_row[g];
            write_value(outs.c[k], p, load_i64(keys.c[k], r), col_valid(keys.c[k], r));
        }
        for (int a = 0; a < specs.n; ++a) {
            const AggSpec sp = specs.a[a];
            const uint64_t cnt = sp.cnt_slot ? states[(int64_t)sp.cnt_slot * G + g] : rows;
            const int64_t v = sp.kind == AK_COUNT ? 0 : (int64_t)states[(int64_t)sp.val_slot * G + g];
            const OutCol &o = outs.c[keys.n + a];
            const bool i32 = sp.in_type == QEH_DT_INT32;
            const bool flt = sp.in_type == QEH_DT_FLOAT32 || sp.in_type == QEH_DT_FLOAT64;
            switch (sp.func) {
                case QEH_AGG_COUNT: write_value(o, p, (int64_t)cnt, true); break;
                case QEH_AGG_SUM:
                    // Int32 sums wrap at 32 bits before widening (compute::sum(Int32Array) as i64)
                    write_value(o, p, i32 ? (int64_t)(int32_t)v : v, cnt != 0);
                    break;
                case QEH_AGG_AVG: {
                    double s = flt ? as_f64(v) : (double)(i32 ? (int64_t)(int32_t)v : v);
                    write_value(o, p, f64_bits(cnt ? s / (double)cnt : 0.0), cnt != 0);
                    break;
                }
                default: {  // MIN / MAX keep the input type
                    int64_t out = flt ? f64_bits(f64_from_order_key(v)) : v;
                    write_value(o, p, out, cnt != 0);
                    break;
                }
            }
        }
    }
}

// ---- host helpers ----------------------------------------------------------------------
static int agg_output_type(int func, int in_type) {
    switch (func) {
        case QEH_AGG_COUNT: return QEH_DT_INT64;
        case QEH_AGG_SUM: return (in_type == QEH_DT_FLOAT32 || in_type == QEH_DT_FLOAT64) ? QEH_DT_FLOAT64 : QEH_DT_INT64;
        case QEH_AGG_AVG: return QEH_DT_FLOAT64;
        default: return in_type;
    }
}

// `cols` are the kernel's columns; aggs[i].column indexes `agg_cols[]`, which
// maps to ColSet indexes through `colset_index`.
static int plan_aggs(const qeh_agg *aggs, int n_aggs, const qeh_column *inputs, int n_inputs,
                     const int *colset_index, AggSpecs *out) {
    if (n_aggs > kMaxAggs) return fail(QEH_E_UNSUPPORTED, "too many aggregates for one device operator (max 8)");
    std::memset(out, 0, sizeof(*out));
    out->n = n_aggs;
    int slot = 1;
    for (int i = 0; i < n_aggs; ++i) {
        const qeh_agg &a = aggs[i];
        if (a.column < 0 || a.column >= n_inputs) return fail(QEH_E_INVALID, "aggregate input index out of range");
        const qeh_column &c = inputs[a.column];
        int t = c.dtype;
        AggSpec &s = out->a[i];
        s.func = a.func;
        s.col = colset_index[a.column];
        s.in_type = t;
        const bool numeric = t == QEH_DT_INT32 || t == QEH_DT_INT64 || t == QEH_DT_FLOAT32 || t == QEH_DT_FLOAT64;
        const bool flt = t == QEH_DT_FLOAT32 || t == QEH_DT_FLOAT64;
        switch (a.func) {
            case QEH_AGG_COUNT: s.kind = AK_COUNT; break;
            case QEH_AGG_SUM:
                if (!numeric) return fail(QEH_E_TYPE, "Unsupported type for SUM");
                s.kind = flt ? AK_SUM_F : AK_SUM_I;
                break;
            case QEH_AGG_AVG:
                if (!numeric) return fail(QEH_E_TYPE, "Unsupported type for AVG");
                s.kind = flt ? AK_SUM_F : AK_SUM_I;
                break;
            case QEH_AGG_MIN:
                if (!numeric) return fail(QEH_E_TYPE, "Unsupported type for MIN");
                s.kind = AK_MIN;
                break;
            case QEH_AGG_MAX:
                if (!numeric) return fail(QEH_E_TYPE, "Unsupported type for MAX");
                s.kind = AK_MAX;
                break;
            default: return fail(QEH_E_INVALID, "unknown aggregate function");
        }
        s.val_slot = s.kind == AK_COUNT ? -1 : slot++;
        const bool has_nulls = c.validity != nullptr && c.null_count != 0;
        s.cnt_slot = has_nulls ? slot++ : 0;
    }
    out->n_slots = slot;
    return QEH_OK;
}

struct PredPlan {
    int mode = PM_NONE;
    PredTerms terms{};
    DevProgram prog{};
};

static int plan_predicate(const qeh_expr *pred, const int32_t *dtypes, int n_cols, PredPlan *pp) {
    pp->mode = PM_NONE;
    if (!pred || pred->n_nodes == 0) return QEH_OK;
    QEH_TRY(compile_expr(pred, dtypes, n_cols, &pp->prog));
    if (pp->prog.result_type != QEH_DT_BOOL)
        return fail(QEH_E_TYPE, "Filter predicate must return boolean");
    pp->mode = lower_to_terms(pred, dtypes, n_cols, &pp->terms) ? PM_TERMS : PM_PROG;
    return QEH_OK;
}

template <int GM>
static void launch_agg_rows(qeh_ctx *ctx, int pm, bool lds, int grid, size_t shmem, const ColSet &cols, int64_t n,
                            const PredPlan &pp, const GidSource &src, const AggSpecs &specs, int64_t G,
                            uint64_t *states, uint32_t *err) {
#define QEH_LAUNCH(PMV, LDSV)                                                                                  \
    hipLaunchKernelGGL((k_agg_rows<GM, PMV, LDSV>), dim3(grid), dim3(kBlock), shmem, ctx->stream, cols, n, pp.terms, \
                       pp.prog, src, specs, G, states, err)
    if (pm == PM_NONE) { if (lds) QEH_LAUNCH(PM_NONE, true); else QEH_LAUNCH(PM_NONE, false); }
    else if (pm == PM_TERMS) { if (lds) QEH_LAUNCH(PM_TERMS, true); else QEH_LAUNCH(PM_TERMS, false); }
    else { if (lds) QEH_LAUNCH(PM_PROG, true); else QEH_LAUNCH(PM_PROG, false); }
#undef QEH_LAUNCH
}

// Run the row-aggregation kernel and finalize into owned output columns.
static int aggregate_rows(qeh_ctx *ctx, int gm, const ColSet &cols, int64_t n, const PredPlan &pp,
                          const GidSource &src, const AggSpecs &specs, int64_t G, const KeyCols &out_keys_src,
                          const int32_t *key_dtypes, const uint32_t *rep_row, bool drop_empty, const char *kname,
                          qeh_column *out_keys, qeh_column *out_aggs, int64_t *out_groups) {
    DevBuf states, errw;
    const int64_t Gs = std::max<int64_t>(G, 1);
    QEH_TRY(states.alloc(ctx, (size_t)specs.n_slots * Gs * 8));
    QEH_TRY(errw.alloc(ctx, 8));
    QEH_HIP(hipMemsetAsync(errw.p, 0, 8, ctx->stream));
    hipLaunchKernelGGL(k_states_init, dim3(grid_for(ctx, specs.n_slots * Gs, kBlock * 4, 8)), dim3(kBlock), 0, ctx->stream,
                       states.as<uint64_t>(), Gs, specs);
    const size_t lds_bytes = (size_t)specs.n_slots * Gs * 8;
    const bool lds = lds_bytes <= kLdsStateBudget;
    if (n > 0 && G > 0) {
        // LDS partials: ~3-6 workgroups per CU; fewer per CU when the state is large
        int per_cu = lds ? (int)std::max<size_t>(1, std::min<size_t>(8, (160 * 1024) / std::max<size_t>(lds_bytes, 1))) : 8;
        per_cu = std::min(per_cu, 8);
        int grid = grid_for(ctx, n, kAggTile, per_cu);
        KernelTimer kt(ctx, kname);
        if (gm == GM_ZERO) launch_agg_rows<GM_ZERO>(ctx, pp.mode, lds, grid, lds ? lds_bytes : 0, cols, n, pp, src, specs, Gs, states.as<uint64_t>(), errw.as<uint32_t>());
        else if (gm == GM_JOIN) launch_agg_rows<GM_JOIN>(ctx, pp.mode, lds, grid, lds ? lds_bytes : 0, cols, n, pp, src, specs, Gs, states.as<uint64_t>(), errw.as<uint32_t>());
        else launch_agg_rows<GM_GROUP>(ctx, pp.mode, lds, grid, lds ? lds_bytes : 0, cols, n, pp, src, specs, Gs, states.as<uint64_t>(), errw.as<uint32_t>());
    }
    QEH_HIP(hipGetLastError());

    // compact non-empty groups
    DevBuf flags, pos;
    uint64_t out_n = (uint64_t)G;
    const uint64_t *posp = nullptr;
    if (drop_empty && G > 0) {
        QEH_TRY(flags.alloc(ctx, Gs * 4));
        QEH_TRY(pos.alloc(ctx, Gs * 8));
        hipLaunchKernelGGL(k_group_nonempty, dim3(grid_for(ctx, Gs, kBlock, 8)), dim3(kBlock), 0, ctx->stream,
                           states.as<uint64_t>(), Gs, flags.as<uint32_t>());
        QEH_TRY(exclusive_scan_u32(ctx, flags.as<uint32_t>(), pos.as<uint64_t>(), G, &out_n));
        posp = pos.as<uint64_t>();
    } else {
        uint32_t e = 0;
        QEH_TRY(read_small(ctx, &e, errw.p, 4));
        QEH_TRY(kernel_error_status(e, "aggregate"));
    }
    uint32_t e = 0;
    QEH_TRY(read_small(ctx, &e, errw.p, 4));
    QEH_TRY(kernel_error_status(e, "aggregate"));

    OutCols oc{};
    const int nk = out_keys_src.n;
    int made = 0;
    auto cleanup = [&]() {
        for (int i = 0; i < made; ++i) {
            qeh_column *c = i < nk ? &out_keys[i] : &out_aggs[i - nk];
            qeh_column_release(ctx, c);
        }
    };
    for (int i = 0; i < nk + specs.n; ++i) {
        qeh_column *c = i < nk ? &out_keys[i] : &out_aggs[i - nk];
        int dt;
        bool nullable;
        if (i < nk) {
            dt = key_dtypes[i];
            nullable = out_keys_src.c[i].validity != nullptr;
        } else {
            const AggSpec &sp = specs.a[i - nk];
            dt = agg_output_type(sp.func, sp.in_type);
            nullable = sp.func != QEH_AGG_COUNT;
        }
        int s = alloc_column(ctx, dt, (int64_t)out_n, nullable, c);
        if (s != QEH_OK) {
            cleanup();
            return s;
        }
        ++made;
        if (nullable) QEH_HIP(hipMemsetAsync(c->validity, 0, ((out_n + 63) / 64) * 8, ctx->stream));
        if (dt == QEH_DT_BOOL) QEH_HIP(hipMemsetAsync(c->values, 0, ((out_n + 63) / 64) * 8, ctx->stream));
        oc.c[i].values = c->values;
        oc.c[i].validity = (uint32_t *)c->validity;
        oc.c[i].dtype = dt;
    }
    if (G > 0 && out_n > 0) {
        KernelTimer kt(ctx, "aggregate_finalize");
        hipLaunchKernelGGL(k_finalize, dim3(grid_for(ctx, Gs, kBlock, 8)), dim3(kBlock), 0, ctx->stream,
                           states.as<uint64_t>(), Gs, posp, out_keys_src, rep_row, specs, oc);
    }
    QEH_HIP(hipGetLastError());
    QEH_HIP(hipStreamSynchronize(ctx->stream));
    for (int i = 0; i < nk + specs.n; ++i) {
        qeh_column *c = i < nk ? &out_keys[i] : &out_aggs[i - nk];
        c->null_count = c->validity ? -1 : 0;
    }
    *out_groups = (int64_t)out_n;
    return QEH_OK;
}

// Internal entry shared by qeh_hash_aggregate and the executor's fused
// Aggregate(Filter(..)) path: `cols` = key columns then aggregate inputs.
int hash_aggregate_filtered(qeh_ctx *ctx, const qeh_column *keys, int n_keys, const qeh_column *agg_inputs,
                            int n_inputs, const qeh_agg *aggs, int n_aggs, const qeh_column *pred_cols,
                            int n_pred_cols, const qeh_expr *predicate, int64_t input_batches,
                            qeh_column *out_keys, qeh_column *out_aggs, int64_t *out_groups) {
    if (!out_groups) return fail(QEH_E_INVALID, "qeh_hash_aggregate: out_groups is NULL");
    *out_groups = 0;
    if (n_aggs == 0) return QEH_OK;  // executor.rs:163-165: no aggregates -> no batches
    int64_t n = -1;
    auto take_len = [&](const qeh_column &c) -> int {
        if (n < 0) n = c.length;
        else if (c.length != n) return fail(QEH_E_INVALID, "aggregate columns have different lengths");
        return QEH_OK;
    };
    for (int i = 0; i < n_keys; ++i) QEH_TRY(take_len(keys[i]));
    for (int i = 0; i < n_inputs; ++i) QEH_TRY(take_len(agg_inputs[i]));
    for (int i = 0; i < n_pred_cols; ++i) QEH_TRY(take_len(pred_cols[i]));
    if (n < 0) n = 0;
    // kernel ColSet = predicate columns, then aggregate inputs (keys are read through KeyCols)
    std::vector<qeh_column> all;
    for (int i = 0; i < n_pred_cols; ++i) all.push_back(pred_cols[i]);
    std::vector<int> idx(n_inputs);
    for (int i = 0; i < n_inputs; ++i) {
        idx[i] = (int)all.size();
        all.push_back(agg_inputs[i]);
    }
    ColSet cols;
    QEH_TRY(make_colset(all.data(), (int)all.size(), &cols));
    std::vector<int32_t> dts(all.size());
    for (size_t i = 0; i < all.size(); ++i) dts[i] = all[i].dtype;
    PredPlan pp;
    QEH_TRY(plan_predicate(predicate, dts.data(), n_pred_cols, &pp));
    AggSpecs specs;
    QEH_TRY(plan_aggs(aggs, n_aggs, agg_inputs, n_inputs, idx.data(), &specs));
    DeviceGuard dg(ctx->device);
    GidSource src{};
    std::vector<int32_t> kd(n_keys);
    for (int i = 0; i < n_keys; ++i) kd[i] = keys[i].dtype;
    if (n_keys == 0) {
        if (input_batches == 0) return QEH_OK;  // executor.rs:178-186: no batches -> no row
        KeyCols none{};
        return aggregate_rows(ctx, GM_ZERO, cols, n, pp, src, specs, 1, none, nullptr, nullptr, false,
                              "aggregate_rows", out_keys, out_aggs, out_groups);
    }
    GroupTable gt;
    QEH_TRY(build_group_table(ctx, keys, n_keys, n, &gt, nullptr));
    src.gk = gt.keys;
    src.gslots = gt.slots.as<uint32_t>();
    src.gmask = gt.cap - 1;
    src.gdense = gt.dense.as<uint64_t>();
    return aggregate_rows(ctx, GM_GROUP, cols, n, pp, src, specs, gt.groups, gt.keys, kd.data(),
                          gt.rep_row.as<uint32_t>(), true, "aggregate_rows", out_keys, out_aggs, out_groups);
}

}  // namespace qeh

using namespace qeh;

extern "C" int qeh_hash_aggregate(qeh_ctx *ctx, const qeh_column *keys, int n_keys, const qeh_column *agg_inputs,
                                  int n_inputs, const qeh_agg *aggs, int n_aggs, int64_t input_batches,
                                  qeh_column *out_keys, qeh_column *out_aggs, int64_t *out_groups) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    return hash_aggregate_filtered(ctx, keys, n_keys, agg_inputs, n_inputs, aggs, n_aggs, nullptr, 0, nullptr,
                                   input_batches, out_keys, out_aggs, out_groups);
}

extern "C" int qeh_filter_aggregate(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *predicate,
                                    const int32_t *key_idx, int n_keys, const qeh_agg *aggs, int n_aggs,
                                    int64_t input_batches, qeh_column *out_keys, qeh_column *out_aggs,
                                    int64_t *out_groups) {
    if (!ctx) return fail(QEH_E_INVALID, "null context");
    if (n_keys > kMaxGroupKeys) return fail(QEH_E_UNSUPPORTED, "1..4 group keys supported on the device");
    std::vector<qeh_column> keys(n_keys);
    for (int i = 0; i < n_keys; ++i) {
        if (key_idx[i] < 0 || key_idx[i] >= n_cols) return fail(QEH_E_INVALID, "group key index out of range");
        keys[i] = cols[key_idx[i]];
    }
    return hash_aggregate_filtered(ctx, keys.data(), n_keys, cols, n_cols, aggs, n_aggs, cols, n_cols, predicate,
                                   input_batches, out_keys, out_aggs, out_groups);
}

extern "C" int qeh_join_filter_aggregate(qeh_ctx *ctx, const qeh_column *probe_cols, int n_probe_cols,
                                         int probe_key_idx, const qeh_expr *predicate, const qeh_column *build_key,
                                         const qeh_column *build_group_keys, int n_group_keys, const qeh_agg *aggs,
                                         int n_aggs, qeh_column *out_keys, qeh_column *out_aggs,
                                         int64_t *out_groups) {
    if (!ctx || !out_groups || !build_key) return fail(QEH_E_INVALID, "qeh_join_filter_aggregate: bad argument");
    *out_groups = 0;
    if (n_aggs == 0) return QEH_OK;
    if (probe_key_idx < 0 || probe_key_idx >= n_probe_cols) return fail(QEH_E_INVALID, "probe key index out of range");
    if (n_group_keys < 1) return fail(QEH_E_UNSUPPORTED, "fused join-aggregate needs at least one build-side group key");
    const int64_t n = probe_cols[0].length;
    for (int i = 0; i < n_probe_cols; ++i)
        if (probe_cols[i].length != n) return fail(QEH_E_INVALID, "probe columns have different lengths");
    for (int i = 0; i < n_group_keys; ++i)
        if (build_group_keys[i].length != build_key->length) return fail(QEH_E_INVALID, "build columns have different lengths");
    DeviceGuard dg(ctx->device);
    ColSet cols;
    QEH_TRY(make_colset(probe_cols, n_probe_cols, &cols));
    std::vector<int32_t> dts(n_probe_cols);
    std::vector<int> idx(n_probe_cols);
    for (int i = 0; i < n_probe_cols; ++i) {
        dts[i] = probe_cols[i].dtype;
        idx[i] = i;
    }
    PredPlan pp;
    QEH_TRY(plan_predicate(predicate, dts.data(), n_probe_cols, &pp));
    AggSpecs specs;
    QEH_TRY(plan_aggs(aggs, n_aggs, probe_cols, n_probe_cols, idx.data(), &specs));
    if (probe_cols[probe_key_idx].dtype != QEH_DT_INT64 && probe_cols[probe_key_idx].dtype != QEH_DT_INT32)
        return fail(QEH_E_UNSUPPORTED, "hash join keys must be Int32/Int64 on the device");

    // build side: dense group ids of the build rows, then the join table with gid payloads
    GroupTable gt;
    DevBuf gid_of_row;
    QEH_TRY(assign_group_ids(ctx, build_group_keys, n_group_keys, build_key->length, &gt, &gid_of_row));
    BuiltTable bt;
    QEH_TRY(build_join_table(ctx, *build_key, gid_of_row.as<uint32_t>(),
                             (uint64_t)std::max<int64_t>(gt.groups - 1, 0), &bt));
    GidSource src{};
    src.jt = bt.t;
    src.key_col = probe_key_idx;
    std::vector<int32_t> kd(n_group_keys);
    for (int i = 0; i < n_group_keys; ++i) kd[i] = build_group_keys[i].dtype;
    return aggregate_rows(ctx, GM_JOIN, cols, n, pp, src, specs, gt.groups, gt.keys, kd.data(),
                          gt.rep_row.as<uint32_t>(), true, "join_filter_aggregate", out_keys, out_aggs, out_groups);
}
