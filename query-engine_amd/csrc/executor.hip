// QueryExecutor on the device: walks the reference's PhysicalPlan enum
// (crates/query-executor/src/physical_plan.rs:13-72, flattened by
// include/qeh_plan.h) the way QueryExecutor::execute_plan does
// (crates/query-executor/src/executor.rs:23-91): post-order, every child
// fully materialised — but the materialised tables stay in HBM, and the
// patterns the reference's planner emits for the hot path are fused:
//   HashAggregate(Filter(HashJoin(L, R)))  -> qeh_join_filter_aggregate
//   HashAggregate(HashJoin(L, R))          -> qeh_join_filter_aggregate (no predicate)
//   HashAggregate(Filter(X)), grouped      -> qeh_filter_aggregate
// Semantics per node: Scan uploads DataSource batches;
// Filter drops NULL-predicate rows and empty batches (executor.rs:131-155);
// Projection uses the planner schema's names (executor.rs:93-129); global
// aggregates keep the "no input batch -> no row" quirk (executor.rs:157-190);
// GROUP BY, INNER equi-join, Sort and ROW_NUMBER follow the intended
// semantics; Limit slices (executor.rs:299-341); SubqueryScan and IndexScan
// behave as in the reference (executor.rs:72-88).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/qeh_plan.h"
#include "ops.h"

namespace qeh {
int hash_aggregate_filtered(qeh_ctx *ctx, const qeh_column *keys, int n_keys, const qeh_column *agg_inputs,
                            int n_inputs, const qeh_agg *aggs, int n_aggs, const qeh_column *pred_cols,
                            int n_pred_cols, const qeh_expr *predicate, int64_t input_batches,
                            qeh_column *out_keys, qeh_column *out_aggs, int64_t *out_groups);
}

namespace {

using namespace qeh;

struct Holder {
    qeh_ctx *ctx = nullptr;
    qeh_column c{};
    ~Holder() {
        if (c.owned) qeh_column_release(ctx, &c);
    }
};

struct Col {
    qeh_column c{};                  // view (offset/length may differ from the owner's)
    std::shared_ptr<Holder> owner;   // keeps the buffers alive
};

struct Field {
    std::string name;
    int dtype;
    bool nullable;
};

struct Table {
    std::vector<Field> fields;
    std::vector<Col> cols;
    int64_t rows = 0;
    int64_t batches = 0;  // >0 iff the reference would hold at least one batch here
};

Col own(qeh_ctx *ctx, const qeh_column &c) {
    Col r;
    r.c = c;
    auto h = std::make_shared<Holder>();  // constructed in place: exactly one releasing owner
    h->ctx = ctx;
    h->c = c;
    r.owner = h;
    return r;
}

// ---- Arrow import ----------------------------------------------------------------------
int dtype_of_format(const char *f, int *dt) {
    if (!f) return fail(QEH_E_INVALID, "arrow schema without format");
    if (!std::strcmp(f, "l")) *dt = QEH_DT_INT64;
    else if (!std::strcmp(f, "i")) *dt = QEH_DT_INT32;
    else if (!std::strcmp(f, "g")) *dt = QEH_DT_FLOAT64;
    else if (!std::strcmp(f, "f")) *dt = QEH_DT_FLOAT32;
    else if (!std::strcmp(f, "b")) *dt = QEH_DT_BOOL;
    else if (!std::strcmp(f, "u")) *dt = QEH_DT_UTF8;
    else return fail(QEH_E_UNSUPPORTED, std::string("arrow type '") + f + "' is not supported on the device");
    return QEH_OK;
}

const char *format_of_dtype(int dt) {
    switch (dt) {
        case QEH_DT_INT64: return "l";
        case QEH_DT_INT32: return "i";
        case QEH_DT_FLOAT64: return "g";
        case QEH_DT_FLOAT32: return "f";
        case QEH_DT_BOOL: return "b";
        case QEH_DT_UTF8: return "u";
        case QEH_DT_UINT32: return "I";
        default: return "n";
    }
}

inline bool get_bit(const uint8_t *b, int64_t i) { return (b[i >> 3] >> (i & 7)) & 1; }
inline void set_bit(uint8_t *b, int64_t i, bool v) {
    if (v) b[i >> 3] |= (uint8_t)(1u << (i & 7));
    else b[i >> 3] &= (uint8_t)~(1u << (i & 7));
}

int upload_host(qeh_ctx *ctx, void **dst, const void *src, size_t bytes) {
    QEH_TRY(ctx->pool->alloc(bytes ? bytes : 8, dst));
    if (bytes) QEH_HIP(hipMemcpyAsync(*dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    return QEH_OK;
}

// Concatenate column `ci` of every batch into one device column.
int import_column(qeh_ctx *ctx, const qeh_source &src, int ci, int dt, Col *out) {
    int64_t total = 0;
    bool any_nulls = false;
    for (int64_t b = 0; b < src.n_batches; ++b) {
        const ArrowArray *batch = src.batches[b];
        if (ci >= batch->n_children) return fail(QEH_E_INVALID, "record batch has fewer columns than its schema");
        const ArrowArray *ch = batch->children[ci];
        total += batch->length;
        if (ch->null_count != 0 && ch->buffers[0]) any_nulls = true;
    }
    qeh_column c{};
    c.dtype = dt;
    c.owned = 1;
    c.length = total;
    c.null_count = 0;
    const size_t es0 = dtype_size(dt);
    if (!any_nulls && dt != QEH_DT_BOOL && dt != QEH_DT_UTF8 && es0) {
        // no nulls, fixed width: each batch's value buffer goes straight to its
        // place in the device column (no host staging, no per-row loop)
        void *p = nullptr;
        QEH_TRY(ctx->pool->alloc(total ? (size_t)total * es0 : 8, &p));
        int64_t pos = 0;
        for (int64_t b = 0; b < src.n_batches; ++b) {
            const ArrowArray *batch = src.batches[b];
            const ArrowArray *ch = batch->children[ci];
            const int64_t len = batch->length, off = batch->offset + ch->offset;
            if (len)
                QEH_HIP(hipMemcpyAsync((char *)p + (size_t)pos * es0, (const uint8_t *)ch->buffers[1] + (size_t)off * es0,
                                       (size_t)len * es0, hipMemcpyHostToDevice, ctx->stream));
            pos += len;
        }
        c.values = p;
        QEH_HIP(hipStreamSynchronize(ctx->stream));  // the batches are borrowed for this call only
        *out = own(ctx, c);
        return QEH_OK;
    }
    const size_t vbytes = (size_t)((total + 63) / 64) * 8 + 8;
    std::vector<uint8_t> valid;
    if (any_nulls) valid.assign(vbytes, 0);
    std::vector<uint8_t> vals;
    std::vector<int32_t> offs;
    std::vector<uint8_t> data;
    const size_t es = dtype_size(dt);
    if (dt == QEH_DT_BOOL) vals.assign(vbytes, 0);
    else if (dt == QEH_DT_UTF8) offs.assign((size_t)total + 1, 0);
    else vals.resize((size_t)total * es);
    int64_t pos = 0;
    int64_t nulls = 0;
    for (int64_t b = 0; b < src.n_batches; ++b) {
        const ArrowArray *batch = src.batches[b];
        const ArrowArray *ch = batch->children[ci];
        const int64_t len = batch->length, off = batch->offset + ch->offset;
        const uint8_t *vb = (const uint8_t *)ch->buffers[0];
        for (int64_t i = 0; i < len; ++i) {
            const bool v = !(ch->null_count != 0 && vb) || get_bit(vb, off + i);
            if (any_nulls) set_bit(valid.data(), pos + i, v);
            nulls += !v;
        }
        if (dt == QEH_DT_BOOL) {
            const uint8_t *bits = (const uint8_t *)ch->buffers[1];
            for (int64_t i = 0; i < len; ++i) set_bit(vals.data(), pos + i, get_bit(bits, off + i));
        } else if (dt == QEH_DT_UTF8) {
            const int32_t *so = (const int32_t *)ch->buffers[1];
            const uint8_t *sd = (const uint8_t *)ch->buffers[2];
            const int32_t base = (int32_t)data.size();
            data.insert(data.end(), sd + so[off], sd + so[off + len]);
            for (int64_t i = 0; i < len; ++i) offs[(size_t)(pos + i + 1)] = base + (so[off + i + 1] - so[off]);
        } else if (len) {
            std::memcpy(vals.data() + (size_t)pos * es, (const uint8_t *)ch->buffers[1] + (size_t)off * es, (size_t)len * es);
        }
        pos += len;
    }
    c.null_count = nulls;
    void *p = nullptr;
    if (dt == QEH_DT_UTF8) {
        QEH_TRY(upload_host(ctx, &p, offs.data(), offs.size() * 4));
        c.offsets = (int32_t *)p;
        QEH_TRY(upload_host(ctx, &p, data.data(), data.size()));
        c.values = p;
        c.values_bytes = (int64_t)data.size();
    } else {
        QEH_TRY(upload_host(ctx, &p, vals.data(), vals.size()));
        c.values = p;
    }
    if (any_nulls && nulls > 0) {
        QEH_TRY(upload_host(ctx, &p, valid.data(), valid.size()));
        c.validity = (uint8_t *)p;
    }
    QEH_HIP(hipStreamSynchronize(ctx->stream));  // host staging buffers die here
    *out = own(ctx, c);
    return QEH_OK;
}

int import_source_uncached(qeh_ctx *ctx, const qeh_source &src, Table *t);

size_t table_device_bytes(const Table &t) {
    size_t b = 0;
    for (const Col &c : t.cols) {
        const size_t es = dtype_size(c.c.dtype);
        if (c.c.dtype == QEH_DT_UTF8) b += (size_t)c.c.values_bytes + (size_t)(c.c.length + 1) * 4;
        else if (c.c.dtype == QEH_DT_BOOL) b += (size_t)(c.c.length + 7) / 8;
        else b += (size_t)c.c.length * es;
        if (c.c.validity) b += (size_t)(c.c.length + 7) / 8;
    }
    return b;
}

}  // namespace

namespace qeh {
struct SourceCache {
    std::mutex mu;
    struct Entry {
        std::shared_ptr<void> table;  // Table (shared column owners)
        size_t bytes = 0;
        uint64_t stamp = 0;
    };
    std::map<uint64_t, Entry> entries;
    uint64_t clock = 0;
    size_t bytes = 0;
    size_t budget = size_t(64) << 30;
    int64_t hits = 0, misses = 0;
    void evict_oldest_until(size_t limit) {
        while (bytes > limit && !entries.empty()) {
            auto victim = entries.begin();
            for (auto it = entries.begin(); it != entries.end(); ++it)
                if (it->second.stamp < victim->second.stamp) victim = it;
            bytes -= victim->second.bytes;
            entries.erase(victim);
        }
    }
};
}  // namespace qeh

namespace {

SourceCache &source_cache(qeh_ctx *ctx) {
    if (!ctx->source_cache) ctx->source_cache = std::make_shared<SourceCache>();
    return *ctx->source_cache;
}

// Scan input: the cached device copy for a non-zero cache_key, else an import.
int import_source(qeh_ctx *ctx, const qeh_source &src, Table *t) {
    if (src.cache_key == 0) return import_source_uncached(ctx, src, t);
    SourceCache &sc = source_cache(ctx);
    {
        std::lock_guard<std::mutex> g(sc.mu);
        auto it = sc.entries.find(src.cache_key);
        if (it != sc.entries.end()) {
            *t = *std::static_pointer_cast<Table>(it->second.table);
            it->second.stamp = ++sc.clock;
            ++sc.hits;
            return QEH_OK;
        }
    }
    QEH_TRY(import_source_uncached(ctx, src, t));
    auto keep = std::make_shared<Table>(*t);
    const size_t bytes = table_device_bytes(*t);
    std::lock_guard<std::mutex> g(sc.mu);
    ++sc.misses;
    if (bytes <= sc.budget) {
        sc.evict_oldest_until(sc.budget - bytes);
        auto &e = sc.entries[src.cache_key];
        sc.bytes -= e.bytes;  // 0 unless another thread inserted the same key meanwhile
        e.table = keep;
        e.bytes = bytes;
        e.stamp = ++sc.clock;
        sc.bytes += bytes;
    }
    return QEH_OK;
}

int import_source_uncached(qeh_ctx *ctx, const qeh_source &src, Table *t) {
    if (!src.schema) return fail(QEH_E_INVALID, "source without schema");
    t->fields.clear();
    t->cols.clear();
    for (int64_t i = 0; i < src.schema->n_children; ++i) {
        const ArrowSchema *f = src.schema->children[i];
        int dt;
        QEH_TRY(dtype_of_format(f->format, &dt));
        t->fields.push_back({f->name ? f->name : "", dt, (f->flags & ARROW_FLAG_NULLABLE) != 0});
        Col c;
        QEH_TRY(import_column(ctx, src, (int)i, dt, &c));
        t->cols.push_back(c);
    }
    t->rows = 0;
    for (int64_t b = 0; b < src.n_batches; ++b) t->rows += src.batches[b]->length;
    t->batches = src.n_batches;
    return QEH_OK;
}

// ---- Arrow export ----------------------------------------------------------------------
struct ExportArray {
    std::vector<std::vector<uint8_t>> bufs;
    std::vector<const void *> ptrs;
    std::vector<ArrowArray *> children;
};
struct ExportSchema {
    std::string format, name;
    std::vector<ArrowSchema *> children;
};

void release_array(ArrowArray *a) {
    if (!a || !a->release) return;
    for (int64_t i = 0; i < a->n_children; ++i) {
        if (a->children[i]->release) a->children[i]->release(a->children[i]);
        delete a->children[i];
    }
    delete (ExportArray *)a->private_data;
    a->release = nullptr;
}

void release_schema(ArrowSchema *s) {
    if (!s || !s->release) return;
    for (int64_t i = 0; i < s->n_children; ++i) {
        if (s->children[i]->release) s->children[i]->release(s->children[i]);
        delete s->children[i];
    }
    delete (ExportSchema *)s->private_data;
    s->release = nullptr;
}

int download(qeh_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!bytes) return QEH_OK;
    QEH_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    return QEH_OK;
}

int export_column(qeh_ctx *ctx, const Col &col, ArrowArray *out) {
    const qeh_column &c = col.c;
    const int64_t n = c.length, off = c.offset;
    auto *ex = new ExportArray();
    ex->bufs.resize(3);
    std::vector<uint8_t> tmp;
    const size_t bitbytes = (size_t)(n + 7) / 8 + 8;
    int64_t nulls = 0;
    int s = QEH_OK;
    if (c.validity) {
        const size_t src_bytes = (size_t)(off + n + 7) / 8;
        tmp.resize(src_bytes + 8);
        s = download(ctx, tmp.data(), c.validity, src_bytes);
    }
    std::vector<uint8_t> raw;
    if (s == QEH_OK) {
        if (c.dtype == QEH_DT_BOOL) {
            raw.resize((size_t)(off + n + 7) / 8 + 8);
            s = download(ctx, raw.data(), c.values, (size_t)(off + n + 7) / 8);
        } else if (c.dtype == QEH_DT_UTF8) {
            ex->bufs[1].resize((size_t)(n + 1) * 4);
            s = download(ctx, ex->bufs[1].data(), c.offsets + off, (size_t)(n + 1) * 4);
        } else {
            const size_t es = dtype_size(c.dtype);
            ex->bufs[1].resize((size_t)n * es + 8);
            s = download(ctx, ex->bufs[1].data(), (const char *)c.values + (size_t)off * es, (size_t)n * es);
        }
    }
    if (s == QEH_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) s = fail(QEH_E_HIP, "export: stream sync failed");
    if (s != QEH_OK) {
        delete ex;
        return s;
    }
    if (c.validity) {
        ex->bufs[0].assign(bitbytes, 0);
        for (int64_t i = 0; i < n; ++i) {
            const bool v = get_bit(tmp.data(), off + i);
            set_bit(ex->bufs[0].data(), i, v);
            nulls += !v;
        }
    }
    if (c.dtype == QEH_DT_BOOL) {
        ex->bufs[1].assign(bitbytes, 0);
        for (int64_t i = 0; i < n; ++i) set_bit(ex->bufs[1].data(), i, get_bit(raw.data(), off + i));
    }
    int nbuf = 2;
    if (c.dtype == QEH_DT_UTF8) {
        int32_t *o = (int32_t *)ex->bufs[1].data();
        const int32_t b0 = o[0];
        const int32_t b1 = o[n];
        ex->bufs[2].resize((size_t)(b1 - b0) + 8);
        if (b1 > b0) {
            if (download(ctx, ex->bufs[2].data(), (const uint8_t *)c.values + b0, (size_t)(b1 - b0)) != QEH_OK ||
                hipStreamSynchronize(ctx->stream) != hipSuccess) {
                delete ex;
                return fail(QEH_E_HIP, "export: utf8 download failed");
            }
        }
        for (int64_t i = 0; i <= n; ++i) o[i] -= b0;
        nbuf = 3;
    }
    ex->ptrs.resize(nbuf);
    ex->ptrs[0] = c.validity ? ex->bufs[0].data() : nullptr;
    for (int i = 1; i < nbuf; ++i) ex->ptrs[i] = ex->bufs[i].data();
    std::memset(out, 0, sizeof(*out));
    out->length = n;
    out->null_count = nulls;
    out->offset = 0;
    out->n_buffers = nbuf;
    out->buffers = ex->ptrs.data();
    out->release = release_array;
    out->private_data = ex;
    return QEH_OK;
}

int export_table(qeh_ctx *ctx, const Table &t, ArrowSchema *os, ArrowArray *oa) {
    auto *ea = new ExportArray();
    auto *es = new ExportSchema();
    es->format = "+s";
    std::memset(oa, 0, sizeof(*oa));
    std::memset(os, 0, sizeof(*os));
    oa->length = t.rows;
    oa->n_buffers = 1;
    ea->ptrs.push_back(nullptr);
    oa->buffers = ea->ptrs.data();
    oa->release = release_array;
    oa->private_data = ea;
    os->format = es->format.c_str();
    os->name = "";
    os->release = release_schema;
    os->private_data = es;
    for (size_t i = 0; i < t.cols.size(); ++i) {
        auto *ca = new ArrowArray();
        int s = export_column(ctx, t.cols[i], ca);
        if (s != QEH_OK) {
            delete ca;
            oa->n_children = (int64_t)ea->children.size();
            oa->children = ea->children.data();
            release_array(oa);
            os->n_children = (int64_t)es->children.size();
            os->children = es->children.data();
            release_schema(os);
            return s;
        }
        ea->children.push_back(ca);
        auto *cs = new ArrowSchema();
        auto *ces = new ExportSchema();
        ces->format = format_of_dtype(t.fields[i].dtype);
        ces->name = t.fields[i].name;
        std::memset(cs, 0, sizeof(*cs));
        cs->format = ces->format.c_str();
        cs->name = ces->name.c_str();
        cs->flags = t.fields[i].nullable ? ARROW_FLAG_NULLABLE : 0;
        cs->release = release_schema;
        cs->private_data = ces;
        es->children.push_back(cs);
    }
    oa->n_children = (int64_t)ea->children.size();
    oa->children = ea->children.data();
    os->n_children = (int64_t)es->children.size();
    os->children = es->children.data();
    return QEH_OK;
}

// ---- Cartesian index generation -------------------------------------------------------
// left row-major = join_batches (executor.rs:500-540, the reference's INNER/LEFT/RIGHT/FULL);
// right row-major = execute_cross_join (executor.rs:437-498: the left index cycles fastest)
__global__ void k_cross_indices(int64_t nl, int64_t nr, uint32_t *li, uint32_t *ri, int right_major) {
    const int64_t m = nl * nr;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        li[i] = right_major ? (uint32_t)(i % nl) : (uint32_t)(i / nr);
        ri[i] = right_major ? (uint32_t)(i / nl) : (uint32_t)(i % nr);
    }
}

// ---- joins on a general `on` ------------------------------------------------------------
// Several equi conjuncts: one Int64 key per side; exact bit-packing of (key - min) when the
// spans fit 63 bits, else a 64-bit hash of the tuple (the full `on` is then re-checked).
struct PackSpec {
    uint64_t mn[kMaxGroupKeys];
    int32_t shift[kMaxGroupKeys];
    int32_t n;
    int32_t hash;
};

__global__ void k_pack_keys(KeyCols keys, PackSpec ps, int64_t n, int64_t *__restrict__ out, uint64_t *__restrict__ vwords) {
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x - lane); base < n; base += stride) {
        const int64_t i = base + lane;
        bool ok = i < n;
        uint64_t v = ps.hash ? 0x9E3779B97F4A7C15ull : 0ull;
        for (int c = 0; c < ps.n; ++c) {
            if (!ok) break;
            if (!col_valid(keys.c[c], i)) {
                ok = false;  // a NULL component: the tuple never matches (NULL = x is not TRUE)
                break;
            }
            const uint64_t x = (uint64_t)load_i64(keys.c[c], i) - ps.mn[c];
            v = ps.hash ? hash64(v ^ (hash64(x) + 0x9E3779B97F4A7C15ull + (v << 6) + (v >> 2))) : (v | (x << ps.shift[c]));
        }
        if (i < n) out[i] = ok ? (int64_t)v : 0;
        const uint64_t m = __ballot(ok);
        if (lane == 0) vwords[base >> 6] = m;
    }
}

__global__ void k_iota_u32(uint32_t *out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (uint32_t)i;
}

__global__ void k_fill_u32(uint32_t *out, int64_t n, uint32_t v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) out[i] = v;
}

// flags[idx[i]] = 1 (plain stores: idempotent)
__global__ void k_mark_rows(const uint32_t *__restrict__ idx, int64_t m, int32_t *__restrict__ flags) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        flags[idx[i]] = 1;
}

// ---- the executor ------------------------------------------------------------------------
class Executor {
  public:
    Executor(qeh_ctx *ctx, const qeh_plan *plan, const qeh_source *src, int n_src)
        : ctx_(ctx), plan_(plan), src_(src), n_src_(n_src) {}

    int run(int node, Table *out, int depth = 0) {
        if (node < 0 || node >= plan_->n_nodes) return fail(QEH_E_INVALID, "plan node index out of range");
        if (depth > 256) return fail(QEH_E_INVALID, "plan too deep (cycle?)");
        const qeh_plan_node &nd = plan_->nodes[node];
        switch (nd.kind) {
            case QEH_PLAN_SCAN:
            case QEH_PLAN_INDEX_SCAN:  // executor.rs:81-88: IndexScan falls back to a full scan
                if (nd.source < 0 || nd.source >= n_src_) return fail(QEH_E_INVALID, "scan source index out of range");
                return import_source(ctx_, src_[nd.source], out);
            case QEH_PLAN_SUBQUERY_SCAN: return run(nd.input, out, depth + 1);
            case QEH_PLAN_FILTER: return filter(nd, out, depth);
            case QEH_PLAN_PROJECTION: return projection(nd, out, depth);
            case QEH_PLAN_HASH_AGGREGATE: return aggregate(nd, out, depth);
            case QEH_PLAN_HASH_JOIN: return join(nd, out, depth);
            case QEH_PLAN_SORT: return sort(nd, out, depth);
            case QEH_PLAN_LIMIT: return limit(nd, out, depth);
            case QEH_PLAN_WINDOW: return window(nd, out, depth);
            default: return fail(QEH_E_INVALID, "unknown plan node kind");
        }
    }

  private:
    qeh_ctx *ctx_;
    const qeh_plan *plan_;
    const qeh_source *src_;
    int n_src_;

    static std::vector<qeh_column> raw(const Table &t) {
        std::vector<qeh_column> v;
        for (auto &c : t.cols) v.push_back(c.c);
        return v;
    }

    int eval(const Table &t, const qeh_expr &e, Col *out) {
        const int ci = expr_as_column(&e);
        if (ci >= 0) {
            if (ci >= (int)t.cols.size())
                return fail(QEH_E_INVALID, "Column index " + std::to_string(ci) + " out of bounds");
            *out = t.cols[ci];
            return QEH_OK;
        }
        auto cols = raw(t);
        qeh_column r{};
        QEH_TRY(qeh_eval(ctx_, cols.data(), (int)cols.size(), &e, t.rows, &r));
        *out = own(ctx_, r);
        return QEH_OK;
    }

    int filter(const qeh_plan_node &nd, Table *out, int depth) {
        Table in;
        QEH_TRY(run(nd.input, &in, depth + 1));
        return filter_table(in, nd.predicate, out);
    }

    int filter_table(const Table &in, const qeh_expr &pred, Table *out) {
        std::vector<int32_t> idx(in.cols.size());
        for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int32_t)i;
        return filter_columns(in, pred, idx, -1, out);
    }

    // Filter keeping only columns `idx` of `in` (in that order) and at most `cap` rows (< 0: all).
    int filter_columns(const Table &in, const qeh_expr &pred, const std::vector<int32_t> &idx, int64_t cap, Table *out) {
        out->fields.clear();
        out->cols.clear();
        for (int32_t i : idx) out->fields.push_back(in.fields[i]);
        auto cols = raw(in);
        std::vector<qeh_column> res(std::max<size_t>(idx.size(), 1));
        int64_t rows = 0;
        if (cols.empty()) return fail(QEH_E_UNSUPPORTED, "filter over a batch without columns");
        QEH_TRY(qeh_filter_limit(ctx_, cols.data(), (int)cols.size(), &pred, idx.data(), (int)idx.size(), cap, res.data(),
                                 &rows));
        for (size_t i = 0; i < idx.size(); ++i) out->cols.push_back(own(ctx_, res[i]));
        out->rows = rows;
        out->batches = (in.batches > 0 && rows > 0) ? 1 : 0;  // empty batches are dropped (executor.rs:149-151)
        return QEH_OK;
    }

    // Projection(Filter(X)) [under Limit]: the filter gathers only the columns the projection
    // reads, and with `cap` >= 0 only the first `cap` qualifying rows (the Limit's skip + fetch).
    // Expressions are re-indexed onto the gathered columns; the result equals the unfused
    // Filter -> Projection -> Limit chain (the cap is only passed for pure column projections,
    // so no expression error on a row past the limit can go unseen).
    int filter_project(const qeh_plan_node &proj, int64_t cap, Table *out, int depth) {
        const qeh_plan_node &fn = plan_->nodes[proj.input];
        Table in;
        QEH_TRY(run(fn.input, &in, depth + 2));
        std::vector<int32_t> remap(in.cols.size(), -1), idx;
        for (int i = 0; i < proj.n_exprs; ++i)
            for (int k = 0; k < proj.exprs[i].n_nodes; ++k) {
                const qeh_expr_node &x = proj.exprs[i].nodes[k];
                if (x.kind != QEH_EX_COLUMN) continue;
                if (x.index < 0 || x.index >= (int)in.cols.size())
                    return fail(QEH_E_INVALID, "Column index " + std::to_string(x.index) + " out of bounds");
                if (remap[x.index] < 0) {
                    remap[x.index] = (int32_t)idx.size();
                    idx.push_back(x.index);
                }
            }
        std::sort(idx.begin(), idx.end());
        for (size_t j = 0; j < idx.size(); ++j) remap[idx[j]] = (int32_t)j;
        Table f;
        QEH_TRY(filter_columns(in, fn.predicate, idx, cap, &f));
        out->fields.clear();
        out->cols.clear();
        for (int i = 0; i < proj.n_exprs; ++i) {
            std::vector<qeh_expr_node> nodes(proj.exprs[i].nodes, proj.exprs[i].nodes + proj.exprs[i].n_nodes);
            for (auto &x : nodes)
                if (x.kind == QEH_EX_COLUMN) x.index = remap[x.index];
            qeh_expr e = proj.exprs[i];
            e.nodes = nodes.data();
            Col c;
            QEH_TRY(eval(f, e, &c));
            std::string name = (proj.field_names && i < proj.n_fields && proj.field_names[i])
                                   ? proj.field_names[i]
                                   : "col_" + std::to_string(i);
            out->fields.push_back({name, c.c.dtype, true});
            out->cols.push_back(c);
        }
        out->rows = f.rows;
        out->batches = proj.n_exprs == 0 ? 0 : f.batches;  // executor.rs:109-111
        return QEH_OK;
    }

    bool fusable_filter_projection(const qeh_plan_node &proj) const {
        return proj.kind == QEH_PLAN_PROJECTION && plan_->nodes[proj.input].kind == QEH_PLAN_FILTER &&
               !std::getenv("QEH_NO_FUSION");
    }

    int projection(const qeh_plan_node &nd, Table *out, int depth) {
        if (fusable_filter_projection(nd)) return filter_project(nd, -1, out, depth);
        Table in;
        QEH_TRY(run(nd.input, &in, depth + 1));
        out->fields.clear();
        out->cols.clear();
        for (int i = 0; i < nd.n_exprs; ++i) {
            Col c;
            QEH_TRY(eval(in, nd.exprs[i], &c));
            std::string name = (nd.field_names && i < nd.n_fields && nd.field_names[i]) ? nd.field_names[i]
                                                                                        : "col_" + std::to_string(i);
            out->fields.push_back({name, c.c.dtype, true});
            out->cols.push_back(c);
        }
        out->rows = in.rows;
        out->batches = nd.n_exprs == 0 ? 0 : in.batches;  // executor.rs:109-111
        return QEH_OK;
    }

    // `on` = Column(a) = Column(b) with one side in each input
    static bool equi_keys(const qeh_expr &on, int n_left, int *lk, int *rk) {
        if (on.n_nodes != 3) return false;
        const qeh_expr_node *n = on.nodes;
        if (n[0].kind != QEH_EX_COLUMN || n[1].kind != QEH_EX_COLUMN || n[2].kind != QEH_EX_BINARY || n[2].op != QEH_OP_EQ)
            return false;
        int a = n[0].index, b = n[1].index;
        if (a >= n_left && b < n_left) std::swap(a, b);
        if (!(a < n_left && b >= n_left)) return false;
        *lk = a;
        *rk = b - n_left;
        return true;
    }

    int join(const qeh_plan_node &nd, Table *out, int depth) {
        Table l, r;
        QEH_TRY(run(nd.left, &l, depth + 1));
        QEH_TRY(run(nd.right, &r, depth + 1));
        return join_tables(nd, l, r, out);
    }

    int join_tables(const qeh_plan_node &nd, const Table &l, const Table &r, Table *out) {
        out->fields = l.fields;
        out->fields.insert(out->fields.end(), r.fields.begin(), r.fields.end());
        out->cols.clear();
        out->rows = 0;
        out->batches = 0;
        if (l.batches == 0 || r.batches == 0) {  // executor.rs:350-352
            for (auto &f : out->fields) {
                qeh_column c{};
                QEH_TRY(alloc_column(ctx_, f.dtype == QEH_DT_UTF8 ? QEH_DT_INT64 : f.dtype, 0, false, &c));
                c.dtype = f.dtype;
                out->cols.push_back(own(ctx_, c));
            }
            return QEH_OK;
        }
        std::vector<qeh_column> lo(l.cols.size()), ro(r.cols.size());
        int64_t rows = 0;
        auto lc = raw(l), rc = raw(r);
        if (nd.join_type == QEH_JOIN_CROSS || (nd.join_type == QEH_JOIN_INNER && !nd.has_predicate)) {
            const int64_t m = l.rows * r.rows;
            if (m >= (int64_t)0xFFFFFFFF) return fail(QEH_E_UNSUPPORTED, "cross join output beyond 2^32 rows");
            DevBuf li, ri;
            QEH_TRY(li.alloc(ctx_, (size_t)std::max<int64_t>(m, 1) * 4));
            QEH_TRY(ri.alloc(ctx_, (size_t)std::max<int64_t>(m, 1) * 4));
            if (m > 0)
                hipLaunchKernelGGL(k_cross_indices, dim3(grid_for(ctx_, m, kBlock * 4, 8)), dim3(kBlock), 0, ctx_->stream,
                                   l.rows, r.rows, li.as<uint32_t>(), ri.as<uint32_t>(),
                                   nd.join_type == QEH_JOIN_CROSS ? 1 : 0);
            for (size_t i = 0; i < lc.size(); ++i) {
                QEH_TRY(gather_column(ctx_, lc[i], li.as<uint32_t>(), m, &lo[i]));
                out->cols.push_back(own(ctx_, lo[i]));
            }
            for (size_t i = 0; i < rc.size(); ++i) {
                QEH_TRY(gather_column(ctx_, rc[i], ri.as<uint32_t>(), m, &ro[i]));
                out->cols.push_back(own(ctx_, ro[i]));
            }
            QEH_HIP(hipStreamSynchronize(ctx_->stream));
            rows = m;
        } else {
            int lk, rk;
            if (!equi_keys(nd.predicate, (int)l.cols.size(), &lk, &rk) || !int_key(lc[lk]) || !int_key(rc[rk]))
                return join_general(nd, l, r, out);
            if (nd.join_type == QEH_JOIN_INNER)
                QEH_TRY(qeh_hash_join_inner(ctx_, &lc[lk], lc.data(), (int)lc.size(), &rc[rk], rc.data(), (int)rc.size(),
                                            lo.data(), ro.data(), &rows));
            else  // LEFT / RIGHT / FULL
                QEH_TRY(qeh_hash_join_outer(ctx_, nd.join_type, &lc[lk], lc.data(), (int)lc.size(), &rc[rk], rc.data(),
                                            (int)rc.size(), lo.data(), ro.data(), &rows));
            // a column returned as a view (owned = 0: an outer join's preserved side) keeps the
            // input's owner alive
            for (size_t i = 0; i < lo.size(); ++i) out->cols.push_back(lo[i].owned ? own(ctx_, lo[i]) : l.cols[i]);
            for (size_t i = 0; i < ro.size(); ++i) out->cols.push_back(ro[i].owned ? own(ctx_, ro[i]) : r.cols[i]);
        }
        out->rows = rows;
        out->batches = rows > 0 ? 1 : 0;  // executor.rs:374-376 keeps non-empty joins only
        return QEH_OK;
    }

    static bool int_key(const qeh_column &c) { return c.dtype == QEH_DT_INT64 || c.dtype == QEH_DT_INT32; }

    // Postfix ranges [b, e) of the AND-ed conjuncts of `e` (nested ANDs flattened).  A malformed
    // expression yields itself as the only conjunct (its evaluation reports the error).
    static void split_conjuncts(const qeh_expr &e, std::vector<std::pair<int, int>> *out) {
        const int n = e.n_nodes;
        std::vector<int> start(std::max(n, 1), 0);
        bool ok = n > 0;
        for (int i = 0; i < n && ok; ++i) {
            const qeh_expr_node &x = e.nodes[i];
            if (x.kind == QEH_EX_BINARY) {
                ok = i >= 2 && start[i - 1] >= 1;
                if (ok) start[i] = start[start[i - 1] - 1];
            } else if (x.kind == QEH_EX_UNARY) {
                ok = i >= 1;
                if (ok) start[i] = start[i - 1];
            } else {
                start[i] = i;
            }
        }
        if (!ok || start[n - 1] != 0) {
            out->push_back({0, n});
            return;
        }
        std::vector<int> stack{n - 1};
        std::vector<std::pair<int, int>> found;
        while (!stack.empty()) {
            const int root = stack.back();
            stack.pop_back();
            const qeh_expr_node &x = e.nodes[root];
            if (x.kind == QEH_EX_BINARY && x.op == QEH_OP_AND) {
                const int right = root - 1, left = start[right] - 1;
                stack.push_back(right);  // left conjunct first
                stack.push_back(left);
            } else {
                found.push_back({start[root], root + 1});
            }
        }
        *out = found;
    }

    // One conjunct `Column(a) = Column(b)` with one side in each input and integer keys.
    static bool equi_conjunct(const qeh_expr_node *x, int len, int nl, const std::vector<qeh_column> &lc,
                              const std::vector<qeh_column> &rc, int *lk, int *rk) {
        if (len != 3 || x[0].kind != QEH_EX_COLUMN || x[1].kind != QEH_EX_COLUMN || x[2].kind != QEH_EX_BINARY ||
            x[2].op != QEH_OP_EQ)
            return false;
        int a = x[0].index, b = x[1].index;
        if (a >= nl && b < nl) std::swap(a, b);
        if (!(a >= 0 && a < nl && b >= nl && b - nl < (int)rc.size())) return false;
        if (!int_key(lc[a]) || !int_key(rc[b - nl])) return false;
        *lk = a;
        *rk = b - nl;
        return true;
    }

    // Pack several key columns of each side into one Int64 key column per side (k_pack_keys).
    int pack_keys(const std::vector<qeh_column> &lc, const std::vector<int> &lk, const std::vector<qeh_column> &rc,
                  const std::vector<int> &rk, Col *lkey, Col *rkey, bool *hashed) {
        const int nk = (int)lk.size();
        PackSpec ps{};
        ps.n = nk;
        int bits = 0;
        for (int j = 0; j < nk; ++j) {
            const qeh_column pair[2] = {lc[lk[j]], rc[rk[j]]};
            int64_t mn[2], mx[2], cnt[2];
            QEH_TRY(columns_minmax(ctx_, pair, 2, mn, mx, cnt));
            int64_t lo = INT64_MAX, hi = INT64_MIN;
            for (int q = 0; q < 2; ++q)
                if (cnt[q]) lo = std::min(lo, mn[q]), hi = std::max(hi, mx[q]);
            if (lo > hi) lo = hi = 0;
            ps.mn[j] = (uint64_t)lo;
            const uint64_t span = (uint64_t)hi - (uint64_t)lo;
            int w = 0;
            while (w < 64 && (span >> w)) ++w;
            ps.shift[j] = bits;
            bits += w;
        }
        ps.hash = bits > 63 ? 1 : 0;
        *hashed = ps.hash != 0;
        for (int side = 0; side < 2; ++side) {
            const auto &cols = side == 0 ? lc : rc;
            const auto &ks = side == 0 ? lk : rk;
            KeyCols kc{};
            kc.n = nk;
            int64_t n = 0;
            for (int j = 0; j < nk; ++j) kc.c[j] = make_colref(cols[ks[j]]), n = cols[ks[j]].length;
            qeh_column c{};
            QEH_TRY(alloc_column(ctx_, QEH_DT_INT64, n, true, &c));
            Col held = own(ctx_, c);
            if (n > 0)
                hipLaunchKernelGGL(k_pack_keys, dim3(grid_for(ctx_, n, kBlock, 8)), dim3(kBlock), 0, ctx_->stream, kc, ps, n,
                                   (int64_t *)c.values, (uint64_t *)c.validity);
            QEH_HIP(hipGetLastError());
            *(side == 0 ? lkey : rkey) = held;
        }
        return QEH_OK;
    }

    int iota_column(int64_t n, Col *out) {
        qeh_column c{};
        QEH_TRY(alloc_column(ctx_, QEH_DT_UINT32, n, false, &c));
        *out = own(ctx_, c);
        if (n > 0)
            hipLaunchKernelGGL(k_iota_u32, dim3(grid_for(ctx_, n, kBlock * 4, 8)), dim3(kBlock), 0, ctx_->stream,
                               (uint32_t *)c.values, n);
        QEH_HIP(hipGetLastError());
        return QEH_OK;
    }

    // Rows of a side that no surviving pair references: their indices (UInt32 column).
    int unmatched_rows(const Col &pairs_idx, int64_t m, int64_t n, Col *out, int64_t *count) {
        qeh_column fl{};
        QEH_TRY(alloc_column(ctx_, QEH_DT_INT32, n, false, &fl));
        Col flags = own(ctx_, fl);
        QEH_HIP(hipMemsetAsync(fl.values, 0, (size_t)std::max<int64_t>(n, 1) * 4, ctx_->stream));
        if (m > 0)
            hipLaunchKernelGGL(k_mark_rows, dim3(grid_for(ctx_, m, kBlock * 4, 8)), dim3(kBlock), 0, ctx_->stream,
                               (const uint32_t *)pairs_idx.c.values + pairs_idx.c.offset, m, (int32_t *)fl.values);
        QEH_HIP(hipGetLastError());
        Col ids;
        QEH_TRY(iota_column(n, &ids));
        Table t;
        t.fields = {{"flag", QEH_DT_INT32, false}, {"row", QEH_DT_UINT32, false}};
        t.cols = {flags, ids};
        t.rows = n;
        t.batches = 1;
        const qeh_expr_node nodes[3] = {
            {QEH_EX_COLUMN, 0, 0}, {QEH_EX_LITERAL, 0, 0}, {QEH_EX_BINARY, QEH_OP_EQ, 0}};
        std::vector<qeh_expr_node> nv(nodes, nodes + 3);
        nv[1].lit_dtype = QEH_DT_INT64;
        nv[1].lit_i64 = 0;
        qeh_expr pred{nv.data(), 3};
        Table f;
        QEH_TRY(filter_columns(t, pred, {1}, -1, &f));
        *out = f.cols[0];
        *count = f.rows;
        return QEH_OK;
    }

    // Join whose `on` is not a single integer equi-key: AND-ed equi conjuncts become the hash key
    // (packed when there are several), everything else is checked by evaluating the whole `on`
    // over the candidate pairs; with no equi conjunct the candidates are the Cartesian product
    // (left row-major, as join_batches builds it).  LEFT / RIGHT / FULL add the rows no
    // surviving pair references, the other side NULL.  Output row order: the matching pairs,
    // then unmatched left rows, then unmatched right rows (the join contract is a multiset).
    int join_general(const qeh_plan_node &nd, const Table &l, const Table &r, Table *out) {
        const int nl = (int)l.cols.size(), nr = (int)r.cols.size();
        auto lc = raw(l), rc = raw(r);
        std::vector<std::pair<int, int>> conj;
        split_conjuncts(nd.predicate, &conj);
        std::vector<int> lks, rks;
        bool need_check = false;
        for (auto &bc : conj) {
            int a, b;
            if ((int)lks.size() < kMaxGroupKeys &&
                equi_conjunct(nd.predicate.nodes + bc.first, bc.second - bc.first, nl, lc, rc, &a, &b)) {
                lks.push_back(a);
                rks.push_back(b);
            } else {
                need_check = true;
            }
        }
        if (l.rows >= (int64_t)0xFFFFFFFF || r.rows >= (int64_t)0xFFFFFFFF)
            return fail(QEH_E_UNSUPPORTED, "join input beyond 2^32 rows");
        Col pl, pr;  // candidate pairs: UInt32 row indices into l and r
        int64_t m = 0;
        if (lks.empty()) {
            m = l.rows * r.rows;
            if (m >= (int64_t)0xFFFFFFFF)
                return fail(QEH_E_UNSUPPORTED, "join without an equi-key conjunct: Cartesian product beyond 2^32 rows");
            qeh_column a{}, b{};
            QEH_TRY(alloc_column(ctx_, QEH_DT_UINT32, m, false, &a));
            pl = own(ctx_, a);
            QEH_TRY(alloc_column(ctx_, QEH_DT_UINT32, m, false, &b));
            pr = own(ctx_, b);
            if (m > 0)
                hipLaunchKernelGGL(k_cross_indices, dim3(grid_for(ctx_, m, kBlock * 4, 8)), dim3(kBlock), 0, ctx_->stream,
                                   l.rows, r.rows, (uint32_t *)a.values, (uint32_t *)b.values, 0);
            QEH_HIP(hipGetLastError());
            need_check = true;
        } else {
            Col lkey, rkey;
            if (lks.size() == 1) {
                lkey.c = lc[lks[0]];
                rkey.c = rc[rks[0]];
            } else {
                bool hashed = false;
                QEH_TRY(pack_keys(lc, lks, rc, rks, &lkey, &rkey, &hashed));
                need_check = need_check || hashed;
            }
            Col lid, rid;
            QEH_TRY(iota_column(l.rows, &lid));
            QEH_TRY(iota_column(r.rows, &rid));
            qeh_column po{}, bo{};
            QEH_TRY(qeh_hash_join_inner(ctx_, &lkey.c, &lid.c, 1, &rkey.c, &rid.c, 1, &po, &bo, &m));
            pl = po.owned ? own(ctx_, po) : lid;
            pr = bo.owned ? own(ctx_, bo) : rid;
            if (!po.owned) pl.c = po;
            if (!bo.owned) pr.c = bo;
        }
        if (need_check && m > 0) {
            // gather the columns `on` reads for every candidate pair, evaluate it, keep the pairs
            const uint64_t used = (nl + nr) <= 64 ? expr_columns(&nd.predicate) : ~0ull;
            Table t;
            std::vector<int32_t> pos(nl + nr, -1);
            for (int i = 0; i < nl + nr; ++i) {
                if (i < 64 && !((used >> i) & 1)) continue;
                const bool left = i < nl;
                qeh_column g{};
                QEH_TRY(gather_column(ctx_, left ? lc[i] : rc[i - nl], (const uint32_t *)(left ? pl : pr).c.values +
                                      (left ? pl : pr).c.offset, m, &g));
                pos[i] = (int32_t)t.cols.size();
                t.cols.push_back(own(ctx_, g));
                t.fields.push_back({"", g.dtype, true});
            }
            const int32_t ipl = (int32_t)t.cols.size();
            t.cols.push_back(pl);
            t.cols.push_back(pr);
            t.fields.push_back({"l", QEH_DT_UINT32, false});
            t.fields.push_back({"r", QEH_DT_UINT32, false});
            t.rows = m;
            t.batches = 1;
            std::vector<qeh_expr_node> nodes(nd.predicate.nodes, nd.predicate.nodes + nd.predicate.n_nodes);
            for (auto &x : nodes)
                if (x.kind == QEH_EX_COLUMN) {
                    if (x.index < 0 || x.index >= nl + nr)
                        return fail(QEH_E_INVALID, "Column index " + std::to_string(x.index) + " out of bounds");
                    x.index = pos[x.index];
                }
            qeh_expr on{nodes.data(), (int32_t)nodes.size()};
            Table f;
            QEH_TRY(filter_columns(t, on, {ipl, ipl + 1}, -1, &f));
            pl = f.cols[0];
            pr = f.cols[1];
            m = f.rows;
        }
        // outer joins: the rows no surviving pair references, other side NULL (kNullRow)
        const bool keep_left = nd.join_type == QEH_JOIN_LEFT || nd.join_type == QEH_JOIN_FULL;
        const bool keep_right = nd.join_type == QEH_JOIN_RIGHT || nd.join_type == QEH_JOIN_FULL;
        Col ul, ur;
        int64_t nul = 0, nur = 0;
        if (keep_left) QEH_TRY(unmatched_rows(pl, m, l.rows, &ul, &nul));
        if (keep_right) QEH_TRY(unmatched_rows(pr, m, r.rows, &ur, &nur));
        const int64_t total = m + nul + nur;
        DevBuf li, ri;
        QEH_TRY(li.alloc(ctx_, (size_t)std::max<int64_t>(total, 1) * 4));
        QEH_TRY(ri.alloc(ctx_, (size_t)std::max<int64_t>(total, 1) * 4));
        auto copy_idx = [&](uint32_t *dst, const Col &src, int64_t n) -> int {
            if (n > 0)
                QEH_HIP(hipMemcpyAsync(dst, (const uint32_t *)src.c.values + src.c.offset, (size_t)n * 4,
                                       hipMemcpyDeviceToDevice, ctx_->stream));
            return QEH_OK;
        };
        auto fill_null = [&](uint32_t *dst, int64_t n) -> int {
            if (n > 0)
                hipLaunchKernelGGL(k_fill_u32, dim3(grid_for(ctx_, n, kBlock * 4, 8)), dim3(kBlock), 0, ctx_->stream, dst, n,
                                   kNullRow);
            QEH_HIP(hipGetLastError());
            return QEH_OK;
        };
        QEH_TRY(copy_idx(li.as<uint32_t>(), pl, m));
        QEH_TRY(copy_idx(ri.as<uint32_t>(), pr, m));
        QEH_TRY(copy_idx(li.as<uint32_t>() + m, ul, nul));
        QEH_TRY(fill_null(ri.as<uint32_t>() + m, nul));
        QEH_TRY(fill_null(li.as<uint32_t>() + m + nul, nur));
        QEH_TRY(copy_idx(ri.as<uint32_t>() + m + nul, ur, nur));
        const bool outer = nd.join_type != QEH_JOIN_INNER;
        for (int i = 0; i < nl; ++i) {
            qeh_column g{};
            QEH_TRY(gather_column(ctx_, lc[i], li.as<uint32_t>(), total, &g, outer));
            out->cols.push_back(own(ctx_, g));
        }
        for (int i = 0; i < nr; ++i) {
            qeh_column g{};
            QEH_TRY(gather_column(ctx_, rc[i], ri.as<uint32_t>(), total, &g, outer));
            out->cols.push_back(own(ctx_, g));
        }
        QEH_HIP(hipStreamSynchronize(ctx_->stream));
        out->rows = total;
        out->batches = total > 0 ? 1 : 0;
        return QEH_OK;
    }

    static bool all_column_exprs(const qeh_plan_node &proj) {
        for (int i = 0; i < proj.n_exprs; ++i)
            if (expr_as_column(&proj.exprs[i]) < 0) return false;
        return true;
    }

    static bool all_columns(const qeh_expr *e, int n, int lo, int hi) {
        for (int i = 0; i < n; ++i) {
            int c = expr_as_column(&e[i]);
            if (c < lo || c >= hi) return false;
        }
        return true;
    }

    int aggregate(const qeh_plan_node &nd, Table *out, int depth) {
        out->fields.clear();
        out->cols.clear();
        out->rows = 0;
        out->batches = 0;
        if (nd.n_aggs == 0) {  // executor.rs:163-165
            Table in;
            QEH_TRY(run(nd.input, &in, depth + 1));
            return QEH_OK;
        }
        const qeh_plan_node &child = plan_->nodes[nd.input];
        const bool grouped = nd.n_exprs > 0;
        std::vector<qeh_agg_expr> aggs(nd.aggs, nd.aggs + nd.n_aggs);
        std::vector<qeh_expr> aexprs(nd.n_aggs);
        for (int i = 0; i < nd.n_aggs; ++i) aexprs[i] = aggs[i].expr;

        // fused: HashAggregate([Filter](HashJoin(L, R) on L.k = R.k)), grouped by R columns, aggregating L columns
        const qeh_plan_node *jn = nullptr;
        const qeh_expr *pred = nullptr;
        if (grouped && !std::getenv("QEH_NO_FUSION")) {
            if (child.kind == QEH_PLAN_HASH_JOIN) jn = &child;
            else if (child.kind == QEH_PLAN_FILTER && plan_->nodes[child.input].kind == QEH_PLAN_HASH_JOIN) {
                jn = &plan_->nodes[child.input];
                pred = &child.predicate;
            }
            if (jn && !(jn->join_type == QEH_JOIN_INNER && jn->has_predicate)) jn = nullptr;
        }
        if (jn) {
            Table l, r;
            QEH_TRY(run(jn->left, &l, depth + 2));
            QEH_TRY(run(jn->right, &r, depth + 2));
            const int nl = (int)l.cols.size(), nr = (int)r.cols.size();
            int lk, rk;
            const bool keys_ok = equi_keys(jn->predicate, nl, &lk, &rk);
            const bool pred_left = !pred || (expr_columns(pred) >> nl) == 0;
            if (keys_ok && pred_left && all_columns(nd.exprs, nd.n_exprs, nl, nl + nr) &&
                all_columns(aexprs.data(), nd.n_aggs, 0, nl) && l.batches > 0 && r.batches > 0) {
                auto lc = raw(l), rc = raw(r);
                std::vector<qeh_column> gk;
                for (int i = 0; i < nd.n_exprs; ++i) gk.push_back(rc[expr_as_column(&nd.exprs[i]) - nl]);
                std::vector<qeh_agg> qa(nd.n_aggs);
                for (int i = 0; i < nd.n_aggs; ++i) qa[i] = {aggs[i].func, expr_as_column(&aexprs[i])};
                std::vector<qeh_column> ok(gk.size()), oa(qa.size());
                int64_t g = 0;
                QEH_TRY(qeh_join_filter_aggregate(ctx_, lc.data(), nl, lk, pred, &rc[rk], gk.data(), (int)gk.size(),
                                                  qa.data(), (int)qa.size(), ok.data(), oa.data(), &g));
                for (int i = 0; i < nd.n_exprs; ++i) {
                    const Field &f = r.fields[expr_as_column(&nd.exprs[i]) - nl];
                    out->fields.push_back({f.name, f.dtype, true});
                    out->cols.push_back(own(ctx_, ok[i]));
                }
                for (int i = 0; i < nd.n_aggs; ++i) {
                    out->fields.push_back({"col_" + std::to_string(i), oa[i].dtype, true});
                    out->cols.push_back(own(ctx_, oa[i]));
                }
                out->rows = g;
                out->batches = g > 0 ? 1 : 0;
                return QEH_OK;
            }
            // not fusable: materialise join (and filter) then aggregate
            Table joined;
            QEH_TRY(join_tables(*jn, l, r, &joined));
            if (pred) {
                Table f;
                QEH_TRY(filter_table(joined, *pred, &f));
                return aggregate_table(nd, f, out);
            }
            return aggregate_table(nd, joined, out);
        }
        // fused HashAggregate(Filter(X)) for GROUP BY
        if (grouped && child.kind == QEH_PLAN_FILTER && !std::getenv("QEH_NO_FUSION")) {
            Table in;
            QEH_TRY(run(child.input, &in, depth + 2));
            const int n = (int)in.cols.size();
            if (n <= 11 && all_columns(nd.exprs, nd.n_exprs, 0, n) && all_columns(aexprs.data(), nd.n_aggs, 0, n) &&
                in.batches > 0) {
                auto cols = raw(in);
                std::vector<qeh_column> keys;
                for (int i = 0; i < nd.n_exprs; ++i) keys.push_back(cols[expr_as_column(&nd.exprs[i])]);
                std::vector<qeh_agg> qa(nd.n_aggs);
                for (int i = 0; i < nd.n_aggs; ++i) qa[i] = {aggs[i].func, expr_as_column(&aexprs[i])};
                std::vector<qeh_column> ok(keys.size()), oa(qa.size());
                int64_t g = 0;
                QEH_TRY(hash_aggregate_filtered(ctx_, keys.data(), (int)keys.size(), cols.data(), n, qa.data(),
                                                (int)qa.size(), cols.data(), n, &child.predicate, in.batches, ok.data(),
                                                oa.data(), &g));
                for (int i = 0; i < nd.n_exprs; ++i) {
                    const Field &f = in.fields[expr_as_column(&nd.exprs[i])];
                    out->fields.push_back({f.name, f.dtype, true});
                    out->cols.push_back(own(ctx_, ok[i]));
                }
                for (int i = 0; i < nd.n_aggs; ++i) {
                    out->fields.push_back({"col_" + std::to_string(i), oa[i].dtype, true});
                    out->cols.push_back(own(ctx_, oa[i]));
                }
                out->rows = g;
                out->batches = g > 0 ? 1 : 0;
                return QEH_OK;
            }
            Table f;
            QEH_TRY(filter_table(in, child.predicate, &f));
            return aggregate_table(nd, f, out);
        }
        Table in;
        QEH_TRY(run(nd.input, &in, depth + 1));
        return aggregate_table(nd, in, out);
    }

    int aggregate_table(const qeh_plan_node &nd, const Table &in, Table *out) {
        out->fields.clear();
        out->cols.clear();
        std::vector<Col> keys, inputs;
        for (int i = 0; i < nd.n_exprs; ++i) {
            Col c;
            QEH_TRY(eval(in, nd.exprs[i], &c));
            keys.push_back(c);
        }
        for (int i = 0; i < nd.n_aggs; ++i) {
            Col c;
            QEH_TRY(eval(in, nd.aggs[i].expr, &c));
            inputs.push_back(c);
        }
        std::vector<qeh_column> kc, ic;
        for (auto &c : keys) kc.push_back(c.c);
        for (auto &c : inputs) ic.push_back(c.c);
        std::vector<qeh_agg> qa(nd.n_aggs);
        for (int i = 0; i < nd.n_aggs; ++i) qa[i] = {nd.aggs[i].func, i};
        std::vector<qeh_column> ok(std::max<size_t>(kc.size(), 1)), oa(qa.size());
        int64_t g = 0;
        QEH_TRY(qeh_hash_aggregate(ctx_, kc.data(), (int)kc.size(), ic.data(), (int)ic.size(), qa.data(), (int)qa.size(),
                                   in.batches, ok.data(), oa.data(), &g));
        if (nd.n_exprs == 0 && in.batches == 0) {  // executor.rs:178-186 / 196-198
            out->rows = 0;
            out->batches = 0;
            return QEH_OK;
        }
        for (int i = 0; i < nd.n_exprs; ++i) {
            const int ci = expr_as_column(&nd.exprs[i]);
            std::string name = ci >= 0 ? in.fields[ci].name : "group_" + std::to_string(i);
            out->fields.push_back({name, ok[i].dtype, true});
            out->cols.push_back(own(ctx_, ok[i]));
        }
        for (int i = 0; i < nd.n_aggs; ++i) {
            out->fields.push_back({"col_" + std::to_string(i), oa[i].dtype, true});  // executor.rs:203-207
            out->cols.push_back(own(ctx_, oa[i]));
        }
        out->rows = g;
        out->batches = g > 0 || nd.n_exprs == 0 ? 1 : 0;
        return QEH_OK;
    }

    int sort(const qeh_plan_node &nd, Table *out, int depth) {
        Table in;
        QEH_TRY(run(nd.input, &in, depth + 1));
        if (nd.n_exprs == 0 || in.rows == 0) {
            *out = in;
            return QEH_OK;
        }
        const int kj = nd.n_exprs == 1 && in.cols.size() == 2 ? expr_as_column(&nd.exprs[0]) : -1;
        if (kj == 0 || kj == 1) {
            // a key column and one 8-byte payload: the payload rides through the radix passes (no
            // permutation, no gathers); NULL keys first, as qeh_sort_indices
            qeh_column ok{}, ov{};
            const int ps = sort_pairs_payload(ctx_, in.cols[kj].c, in.cols[1 - kj].c,
                                              nd.ascending ? nd.ascending[0] != 0 : true, true, &ok, &ov);
            if (ps != kPayloadSortNotEligible) {
                QEH_TRY(ps);
                Col k = own(ctx_, ok), v = own(ctx_, ov);
                out->fields = in.fields;
                out->cols.assign(2, Col{});
                out->cols[kj] = k;
                out->cols[1 - kj] = v;
                out->rows = in.rows;
                out->batches = in.batches;
                return QEH_OK;
            }
        }
        std::vector<Col> keys;
        for (int i = 0; i < nd.n_exprs; ++i) {
            Col c;
            QEH_TRY(eval(in, nd.exprs[i], &c));
            keys.push_back(c);
        }
        std::vector<qeh_column> kc;
        for (auto &c : keys) kc.push_back(c.c);
        std::vector<int8_t> asc(nd.n_exprs, 1);
        for (int i = 0; i < nd.n_exprs; ++i)
            if (nd.ascending) asc[i] = nd.ascending[i];
        qeh_column perm{};
        QEH_TRY(qeh_sort_indices(ctx_, kc.data(), (int)kc.size(), asc.data(), &perm));
        Col p = own(ctx_, perm);
        out->fields = in.fields;
        out->cols.clear();
        for (auto &c : in.cols) {
            qeh_column g{};
            QEH_TRY(qeh_take(ctx_, &c.c, &p.c, &g));
            out->cols.push_back(own(ctx_, g));
        }
        out->rows = in.rows;
        out->batches = in.batches;
        return QEH_OK;
    }

    int limit(const qeh_plan_node &nd, Table *out, int depth) {
        Table in;
        const qeh_plan_node &child = plan_->nodes[nd.input];
        const int64_t cap = nd.fetch >= 0 && !std::getenv("QEH_NO_FUSION")
                                ? std::max<int64_t>(nd.skip, 0) + nd.fetch : -1;
        if (cap >= 0 && child.kind == QEH_PLAN_FILTER) {  // Limit(Filter(X)): stop at skip + fetch rows
            Table x;
            QEH_TRY(run(child.input, &x, depth + 2));
            std::vector<int32_t> idx(x.cols.size());
            for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int32_t)i;
            QEH_TRY(filter_columns(x, child.predicate, idx, cap, &in));
        } else if (cap >= 0 && fusable_filter_projection(child) && all_column_exprs(child)) {
            QEH_TRY(filter_project(child, cap, &in, depth + 1));
        } else {
            QEH_TRY(run(nd.input, &in, depth + 1));
        }
        const int64_t start = std::min<int64_t>(std::max<int64_t>(nd.skip, 0), in.rows);
        int64_t end = in.rows;
        if (nd.fetch >= 0) end = std::min<int64_t>(end, start + nd.fetch);
        *out = in;
        for (auto &c : out->cols) {  // zero-copy slice (RecordBatch::slice)
            c.c.offset += start;
            c.c.length = end - start;
            c.c.null_count = c.c.validity ? -1 : 0;
        }
        out->rows = end - start;
        out->batches = (in.batches > 0 && out->rows > 0) ? 1 : 0;
        return QEH_OK;
    }

    // integer literal argument of a window function (NTILE(n), LAG/LEAD offsets)
    static bool lit_int(const qeh_expr &e, int64_t *v) {
        if (e.n_nodes != 1 || e.nodes[0].kind != QEH_EX_LITERAL || e.nodes[0].lit_is_null) return false;
        const int dt = e.nodes[0].lit_dtype;
        if (dt != QEH_DT_INT32 && dt != QEH_DT_INT64) return false;
        *v = e.nodes[0].lit_i64;
        return true;
    }

    // RANK / DENSE_RANK / NTILE(n) / LAG / LEAD(col[, n[, default]]) / FIRST_VALUE / LAST_VALUE(col)
    // (WindowFunctionType, physical_plan.rs:160-170) through qeh_window
    int window_fn(const qeh_plan_node &nd, const qeh_window_expr &we, const Table &in, Table *out) {
        std::vector<Col> pk, okc;
        for (int i = 0; i < we.n_partition; ++i) {
            Col c;
            QEH_TRY(eval(in, we.partition_by[i], &c));
            pk.push_back(c);
        }
        for (int i = 0; i < we.n_order; ++i) {
            Col c;
            QEH_TRY(eval(in, we.order_by[i], &c));
            okc.push_back(c);
        }
        std::vector<qeh_column> pc, oc;
        for (auto &c : pk) pc.push_back(c.c);
        for (auto &c : okc) oc.push_back(c.c);
        std::vector<int8_t> asc(std::max(we.n_order, 1), 1);
        const bool value_fn = we.func >= QEH_WIN_LAG;
        int64_t param = 0, dflt = 0;
        bool has_dflt = false;
        Col argc;
        bool have_arg = false;
        if (we.func == QEH_WIN_NTILE) {
            if (we.n_args < 1 || !lit_int(we.args[0], &param))
                return fail(QEH_E_UNSUPPORTED, "NTILE needs an integer literal bucket count");
        } else if (value_fn) {
            if (we.n_args < 1) return fail(QEH_E_INVALID, "window value function without an argument");
            QEH_TRY(eval(in, we.args[0], &argc));
            have_arg = true;
            if (we.func == QEH_WIN_LAG || we.func == QEH_WIN_LEAD) {
                param = 1;  // LAG(col) = LAG(col, 1)
                if (we.n_args >= 2 && !lit_int(we.args[1], &param))
                    return fail(QEH_E_UNSUPPORTED, "LAG/LEAD offset must be an integer literal");
                if (we.n_args >= 3) {
                    const qeh_expr &d = we.args[2];
                    if (d.n_nodes != 1 || d.nodes[0].kind != QEH_EX_LITERAL)
                        return fail(QEH_E_UNSUPPORTED, "LAG/LEAD default must be a literal");
                    const qeh_expr_node &ln = d.nodes[0];
                    if (!ln.lit_is_null && ln.lit_dtype != QEH_DT_NULL) {
                        has_dflt = true;
                        const int adt = argc.c.dtype;
                        const bool lit_f = ln.lit_dtype == QEH_DT_FLOAT32 || ln.lit_dtype == QEH_DT_FLOAT64;
                        if (adt == QEH_DT_FLOAT64) {
                            const double x = lit_f ? ln.lit_f64 : (double)ln.lit_i64;
                            std::memcpy(&dflt, &x, 8);
                        } else if (adt == QEH_DT_FLOAT32) {
                            const float x = (float)(lit_f ? ln.lit_f64 : (double)ln.lit_i64);
                            uint32_t b;
                            std::memcpy(&b, &x, 4);
                            dflt = (int64_t)b;
                        } else if (lit_f) {
                            return fail(QEH_E_UNSUPPORTED, "LAG/LEAD float default for an integer column");
                        } else {
                            dflt = adt == QEH_DT_INT32 ? (int64_t)(uint32_t)(int32_t)ln.lit_i64 : ln.lit_i64;
                        }
                    }
                }
            }
        } else if (pc.empty() && oc.empty() && !in.cols.empty()) {
            argc = in.cols[0];  // OVER (): any input column carries the row count
            have_arg = true;
        }
        qeh_column res{};
        QEH_TRY(qeh_window(ctx_, we.func, pc.data(), (int)pc.size(), oc.data(), (int)oc.size(), asc.data(),
                           have_arg ? &argc.c : nullptr, param, has_dflt ? &dflt : nullptr, &res));
        static const char *names[] = {"row_number", "rank", "dense_rank", "ntile", "lag", "lead", "first_value", "last_value"};
        const size_t idx = out->cols.size();
        std::string name = (nd.field_names && (int)idx < nd.n_fields && nd.field_names[idx]) ? nd.field_names[idx]
                                                                                            : names[we.func];
        out->fields.push_back({name, res.dtype, true});
        out->cols.push_back(own(ctx_, res));
        return QEH_OK;
    }

    int window(const qeh_plan_node &nd, Table *out, int depth) {
        Table in;
        QEH_TRY(run(nd.input, &in, depth + 1));
        *out = in;
        for (int w = 0; w < nd.n_window; ++w) {
            const qeh_window_expr &we = nd.window[w];
            if (we.func != QEH_WIN_ROW_NUMBER) {
                QEH_TRY(window_fn(nd, we, in, out));
                continue;
            }
            std::vector<Col> pk, okc;
            for (int i = 0; i < we.n_partition; ++i) {
                Col c;
                QEH_TRY(eval(in, we.partition_by[i], &c));
                pk.push_back(c);
            }
            for (int i = 0; i < we.n_order; ++i) {
                Col c;
                QEH_TRY(eval(in, we.order_by[i], &c));
                okc.push_back(c);
            }
            std::vector<qeh_column> pc, oc;
            for (auto &c : pk) pc.push_back(c.c);
            for (auto &c : okc) oc.push_back(c.c);
            std::vector<int8_t> asc(std::max(we.n_order, 1), 1);
            qeh_column rn{};
            if (pc.empty() && oc.empty()) {
                // ROW_NUMBER() OVER (): 1..n in input order
                qeh_column iota{};
                QEH_TRY(alloc_column(ctx_, QEH_DT_INT64, in.rows, false, &iota));
                std::vector<int64_t> h((size_t)in.rows);
                for (int64_t i = 0; i < in.rows; ++i) h[(size_t)i] = i + 1;
                QEH_HIP(hipMemcpyAsync(iota.values, h.data(), h.size() * 8, hipMemcpyHostToDevice, ctx_->stream));
                QEH_HIP(hipStreamSynchronize(ctx_->stream));
                rn = iota;
            } else {
                QEH_TRY(qeh_row_number(ctx_, pc.data(), (int)pc.size(), oc.data(), (int)oc.size(), asc.data(), &rn));
            }
            const size_t idx = out->cols.size();
            std::string name = (nd.field_names && (int)idx < nd.n_fields && nd.field_names[idx]) ? nd.field_names[idx]
                                                                                                : "row_number";
            out->fields.push_back({name, QEH_DT_INT64, true});  // planner.rs:767-770 types it Int64
            out->cols.push_back(own(ctx_, rn));
        }
        return QEH_OK;
    }
};

}  // namespace

extern "C" int qeh_execute_plan(qeh_ctx *ctx, const qeh_plan *plan, const qeh_source *sources, int n_sources,
                                ArrowSchema *out_schema, ArrowArray *out_batch, int64_t *out_n_batches) {
    if (!ctx || !plan || !out_n_batches || !out_schema || !out_batch)
        return fail(QEH_E_INVALID, "qeh_execute_plan: bad argument");
    *out_n_batches = 0;
    DeviceGuard dg(ctx->device);
    Executor ex(ctx, plan, sources, n_sources);
    Table t;
    QEH_TRY(ex.run(plan->root, &t));
    if (t.batches == 0) return QEH_OK;
    QEH_TRY(export_table(ctx, t, out_schema, out_batch));
    *out_n_batches = 1;
    return QEH_OK;
}

extern "C" int qeh_source_cache_evict(qeh_ctx *ctx, uint64_t cache_key) {
    if (!ctx) return qeh::fail(QEH_E_INVALID, "null context");
    if (!ctx->source_cache) return QEH_OK;
    qeh::DeviceGuard dg(ctx->device);
    qeh::SourceCache &sc = *ctx->source_cache;
    std::lock_guard<std::mutex> g(sc.mu);
    if (cache_key == 0) {
        sc.entries.clear();
        sc.bytes = 0;
        return QEH_OK;
    }
    auto it = sc.entries.find(cache_key);
    if (it != sc.entries.end()) {
        sc.bytes -= it->second.bytes;
        sc.entries.erase(it);
    }
    return QEH_OK;
}

extern "C" int qeh_source_cache_stats(qeh_ctx *ctx, int64_t *entries, int64_t *bytes, int64_t *hits, int64_t *misses) {
    if (!ctx) return qeh::fail(QEH_E_INVALID, "null context");
    int64_t e = 0, b = 0, h = 0, m = 0;
    if (ctx->source_cache) {
        qeh::SourceCache &sc = *ctx->source_cache;
        std::lock_guard<std::mutex> g(sc.mu);
        e = (int64_t)sc.entries.size();
        b = (int64_t)sc.bytes;
        h = sc.hits;
        m = sc.misses;
    }
    if (entries) *entries = e;
    if (bytes) *bytes = b;
    if (hits) *hits = h;
    if (misses) *misses = m;
    return QEH_OK;
}

extern "C" int qeh_source_cache_budget(qeh_ctx *ctx, int64_t bytes) {
    if (!ctx || bytes < 0) return qeh::fail(QEH_E_INVALID, "qeh_source_cache_budget: bad argument");
    qeh::DeviceGuard dg(ctx->device);
    qeh::SourceCache &sc = source_cache(ctx);
    std::lock_guard<std::mutex> g(sc.mu);
    sc.budget = (size_t)bytes;
    sc.evict_oldest_until(sc.budget);
    return QEH_OK;
}
