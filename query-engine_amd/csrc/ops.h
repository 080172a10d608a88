// Host-side helpers shared between operator translation units.
#pragma once
#include <cstdlib>

#include <memory>
#include <vector>

#include "expr.h"
#include "grouptable.h"
#include "hashtable.h"
#include "qeh_internal.h"

namespace qeh {

// qeh_column -> kernel view.  Validation of dtype/length happens in callers.
ColRef make_colref(const qeh_column &c);
int check_column(const qeh_column &c, const char *what);
int make_colset(const qeh_column *cols, int n, ColSet *out);

// Device-wide exclusive scan of uint32 counts into uint64 offsets; returns
// the total through *total (synchronous read).  `out` may alias nothing.
int exclusive_scan_u32_dev(qeh_ctx *ctx, const uint32_t *in, uint64_t *out, int64_t n, uint64_t *total_dev);
int exclusive_scan_u32(qeh_ctx *ctx, const uint32_t *in, uint64_t *out, int64_t n, uint64_t *total);

// Join hash table built over `key` with payload either row ids
// (row_payload == nullptr) or row_payload[row].
struct BuiltTable {
    HashTable t{};
    DevBuf slots, payload, payload16;
    int64_t n_inserted = 0;
};
// Payload of build row i: ids[i] if ids, else dense[slot[i]] if slot (group
// ids straight from a group table), else i.
struct RowPayload {
    const uint32_t *ids = nullptr;
    const uint32_t *slot = nullptr;
    const uint64_t *dense = nullptr;
    const int64_t *values = nullptr;  // payload = values[i] - bias (frame of reference)
    int64_t bias = 0;
};
// DIRECT (perfect-hash) join tables, one entry per key offset: for dense key ranges (<= 4 entries
// per build row) always; for sparser ranges (<= 32 per row) when the entries are u16 and the table
// stays <= 512 MB -- e.g. the key shard one rank receives in a hash exchange, 1/N of a dense range,
// which then takes the LDS-slice pipeline instead of a linear-probing table whose every probe
// misses L2 (QEH_DIRECT_SPARSE=0 turns the sparse case off).
__host__ __device__ inline bool direct_table_ok_with(uint64_t range, uint64_t nv, uint64_t payload_max, bool sparse) {
    if (range == 0 || range >= (1ull << 32) || payload_max >= 0xFFFFFFFEull) return false;
    if (range <= 4 * nv + 1024) return true;
    return sparse && payload_max < 0xFFFFull && range <= 32 * nv && range * 2 <= (512ull << 20);
}
inline bool direct_sparse_allowed() {
    static const bool sparse = [] {
        const char *e = std::getenv("QEH_DIRECT_SPARSE");
        return !(e && e[0] == '0') && !std::getenv("QEH_NO_U16");
    }();
    return sparse;
}
inline bool direct_table_ok(uint64_t range, uint64_t nv, uint64_t payload_max) {
    return direct_table_ok_with(range, nv, payload_max, direct_sparse_allowed());
}
// Per-column [min, max, valid count] as the min/max kernels leave it in device memory.
struct MinMax {
    int64_t mn, mx;
    uint64_t cnt;
    uint32_t bad;  // unsupported key type seen
};
// The min/max kernels of `n` integer columns into dev_out[0..n) (no host sync), and the read-back of
// such a result (one synchronous read; also memoised like columns_minmax).
int columns_minmax_launch(qeh_ctx *ctx, const qeh_column *cols, int n, MinMax *dev_out);
// only the per-workgroup partials (part[column * *nb + workgroup], at most minmax_partials_max_blocks per column)
int columns_minmax_partials(qeh_ctx *ctx, const qeh_column *cols, int n, MinMax *part, int *nb);
int minmax_partials_max_blocks(qeh_ctx *ctx);
int columns_minmax_collect(qeh_ctx *ctx, const qeh_column *cols, int n, const MinMax *dev_out, int64_t *mn, int64_t *mx,
                           int64_t *valid);
// Stable sort of (one Int64 / Int32 key, one non-null 8-byte payload) carrying the payload through
// the radix passes (no gather): the sorted key and payload columns.  kPayloadSortNotEligible when
// the shapes do not fit (nothing allocated).
constexpr int kPayloadSortNotEligible = -3;
int sort_pairs_payload_parts(qeh_ctx *ctx, const qeh_column *keys, const qeh_column *vals, int nparts, bool asc,
                             bool nulls_first, qeh_column *out_key, qeh_column *out_val);
int sort_pairs_payload(qeh_ctx *ctx, const qeh_column &key, const qeh_column &val, bool asc, bool nulls_first,
                       qeh_column *out_key, qeh_column *out_val);
// min / max / valid count of an integer column (one synchronous read).
int column_minmax(qeh_ctx *ctx, const qeh_column &col, int64_t *mn, int64_t *mx, int64_t *valid);
// min / max / valid count of several integer columns, one synchronous read.
int columns_minmax(qeh_ctx *ctx, const qeh_column *cols, int n, int64_t *mn, int64_t *mx, int64_t *valid);
// LDS-slice materialising INNER join of one probe payload and one Int64 build
// payload (k_aggregate.hip); kSliceJoinNotEligible when the shapes do not fit.
constexpr int kSliceJoinNotEligible = -1;
int slice_join_materialise(qeh_ctx *ctx, const qeh_column &probe_key, const qeh_column &probe_val,
                           const qeh_column &build_key, const qeh_column &build_val, qeh_column *out_probe,
                           qeh_column *out_build, int64_t *out_rows);
int build_join_table(qeh_ctx *ctx, const qeh_column &key, const RowPayload &payload, uint64_t payload_max,
                     BuiltTable *out, int force_kind = -1);
inline int build_join_table(qeh_ctx *ctx, const qeh_column &key, const uint32_t *row_payload, uint64_t payload_max,
                            BuiltTable *out, int force_kind = -1) {
    RowPayload rp;
    rp.ids = row_payload;
    return build_join_table(ctx, key, rp, payload_max, out, force_kind);
}

// Group table over key tuples: slots hold a representative row id; dense ids
// 0..G-1 follow slot order.  rep_row[g] = a row carrying group g's key.
struct GroupTable {
    KeyCols keys{};
    DevBuf slots;    // uint32[cap], EMPTY = 0xFFFFFFFF
    DevBuf dense;    // uint64[cap] dense id per occupied slot
    DevBuf rep_row;  // uint32[G]
    uint64_t cap = 0;
    int64_t groups = 0;
    bool direct = false;  // slot = key - kmin (one integer key); not probe-able with group_find
    int64_t kmin = 0;
};
int build_group_table(qeh_ctx *ctx, const qeh_column *keys, int n_keys, int64_t n_rows, GroupTable *out,
                      uint32_t *slot_of_row /* optional, device uint32[n_rows] */, bool allow_direct = false);
// build_group_table + per-row slots (uint32[n_rows]; dense id = table->dense[slot]).
int group_slots_of_rows(qeh_ctx *ctx, const qeh_column *keys, int n_keys, int64_t n_rows, GroupTable *table,
                        DevBuf *slot_of_row);
// build_group_table + per-row dense ids (uint32[n_rows]).
int assign_group_ids(qeh_ctx *ctx, const qeh_column *keys, int n_keys, int64_t n_rows, GroupTable *table,
                     DevBuf *gid_of_row);

// Gather rows `idx[0..m)` of a column into a new owned column.  With `nullable_idx`, an index of
// kNullRow yields NULL (outer-join filler rows) and the output always carries a validity bitmap.
constexpr uint32_t kNullRow = 0xFFFFFFFFu;
int gather_column(qeh_ctx *ctx, const qeh_column &src, const uint32_t *idx, int64_t m, qeh_column *out,
                  bool nullable_idx = false);

// Concatenate parts (same dtype) into one owned column with offset 0 (k_merge.hip); one part =
// a normalising copy.
int concat_columns(qeh_ctx *ctx, const qeh_column *const *parts, int n_parts, qeh_column *out);

// Utf8 comparisons (k_utf8.hip): every comparison of two leaves with a Utf8 side is evaluated into
// a temporary BOOL column appended to `cols`, and the expression rewritten to read it.  Owns the
// temporaries; `changed` false means expr/cols are the inputs unchanged.
struct Utf8Rewrite {
    qeh_ctx *ctx = nullptr;
    std::vector<qeh_column> cols;
    std::vector<qeh_expr_node> nodes;
    qeh_expr expr{};
    std::vector<qeh_column> temps;
    std::vector<std::unique_ptr<DevBuf>> bufs;
    bool changed = false;
    Utf8Rewrite() = default;
    Utf8Rewrite(const Utf8Rewrite &) = delete;
    Utf8Rewrite &operator=(const Utf8Rewrite &) = delete;
    ~Utf8Rewrite();
};
int rewrite_utf8_compares(qeh_ctx *ctx, const qeh_column *cols, int n_cols, const qeh_expr *e, Utf8Rewrite *out);
bool expr_has_utf8(const qeh_expr *e, const int32_t *dtypes, int n_cols);

// Window functions over one bounded integer PARTITION BY key and one ORDER BY key by partitioning
// (k_window.hip): ROW_NUMBER / RANK / DENSE_RANK / NTILE into a fresh Int64 column.
// kWindowMsdNotEligible (nothing allocated) when the shapes do not fit.
constexpr int kWindowMsdNotEligible = -1;
// LAG / LEAD / FIRST_VALUE / LAST_VALUE when `arg` is the ORDER BY column itself.
int window_msd(qeh_ctx *ctx, int func, const qeh_column &part, const qeh_column &order, bool asc, int64_t param,
               const qeh_column *arg, const int64_t *dflt, qeh_column *out);
// Several integer PARTITION BY keys (2..4): their mixed-radix composite (one Int64 column, the keys'
// ranges multiplied) takes window_msd when the product of the ranges is within its key bound.
int window_msd_keys(qeh_ctx *ctx, int func, const qeh_column *parts, int n_part, const qeh_column &order, bool asc,
                    int64_t param, const qeh_column *arg, const int64_t *dflt, qeh_column *out);
// ROW_NUMBER / RANK / NTILE over a key range of <= 2^20 by three 512-way levels with whole-chunk
// writes (k_window3.hip); window_msd tries it first.
int window_w3(qeh_ctx *ctx, int func, const qeh_column &part, const qeh_column &order, bool asc, int64_t param,
              qeh_column *out);

// Order-preserving LDS-slice probe of an outer join over compact embedded records (k_outer_slice.hip):
// writes the build column (vmin + record - 1, validity) of every probe row in probe order and, for
// FULL, copies np probe columns and sets the records' matched flags.  kOuterSliceNotEligible (nothing
// launched) when the shape does not fit.
constexpr int kOuterSliceNotEligible = -1;
int outer_slice_probe(qeh_ctx *ctx, const qeh_column &pk, void *rec, int rw, int64_t kmin, uint64_t range, int64_t vmin,
                      bool full, int np, const int64_t *const *pcol, int64_t *const *pout, uint64_t *const *pvalid,
                      int64_t *bout, uint64_t *bvalid);

// The chunks of a pool grouped by their tag (k_outer_slice.hip): list ranges sbase[0..F], entries
// chunk id | (item count - 1) << 24 (chunk ids < 2^24; unused chunks carry a tag >= F).  `work`: the
// caller's device scratch of chunk_lists_work_words(F) words, alive until the two kernels have run.
size_t chunk_lists_work_words(int F);
int chunk_lists(qeh_ctx *ctx, const uint16_t *tag, const uint16_t *ccnt, uint64_t nchunks, int F, uint32_t *sbase,
                uint32_t *list, uint32_t *work);

// Non-zero entries of a device table of n 2-B or 4-B entries (k_build.hip; one synchronous read).
int count_nonzero_entries(qeh_ctx *ctx, const void *table, uint64_t n, int bytes, uint64_t *out);

// Error word -> status.
int kernel_error_status(uint32_t err, const char *op);

// Environment knob for forcing a table layout in tests ("direct"/"packed"/"wide").
int forced_table_kind();
// the device ranks a tile's rows stably by returning LDS atomics (checked once per process)
bool lds_atomic_rank_ok(qeh_ctx *ctx);

}  // namespace qeh
