// Arrow IPC stream encoding of a device batch: what
// SerializedBatch::from_batch does with arrow-rs's StreamWriter
// (crates/query-distributed/src/network.rs:56-72): a Schema message, one
// RecordBatch message, the end-of-stream marker.  Each message is the 0xFFFFFFFF
// continuation, the little-endian metadata length (padded to 8), the Message
// flatbuffer, then the body (buffers at 64-byte aligned offsets, as arrow-rs's
// default IpcWriteOptions align them).
//
// The flatbuffers are laid out front to back: a table is written before the
// objects it points to (uoffsets must point forward) and its offset fields are
// patched once those objects are placed; every table's vtable sits right
// before it.  The body comes straight from HBM: each column is first
// normalised to offset 0 on the device (validity / boolean bits re-aligned,
// Utf8 offsets re-based) and then copied into the host stream.
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "ops.h"

namespace qeh {
namespace {

// Pinned host buffers handed out by the IPC entry points (freed by qeh_host_free).  Pinning a few
// hundred MB costs more than the copy into them (hipHostMalloc locks and maps every page), so a freed
// buffer is kept (up to kPinKeep bytes in all) and handed out again to a request it fits within 2x.
struct PinCache {
    std::mutex mu;
    std::unordered_map<void *, size_t> live;      // handed out: size
    std::vector<std::pair<void *, size_t>> idle;  // freed and kept, oldest first
    size_t idle_bytes = 0;
};
PinCache &pins() {
    static PinCache *c = new PinCache;  // never destroyed: a buffer may be freed during interpreter exit
    return *c;
}
constexpr size_t kPinKeep = (size_t)1 << 30;

void *pinned_get(size_t n) {
    PinCache &c = pins();
    {
        std::lock_guard<std::mutex> g(c.mu);
        for (size_t i = 0; i < c.idle.size(); ++i) {
            const auto e = c.idle[i];
            if (e.second >= n && e.second <= 2 * n + ((size_t)1 << 20)) {
                c.idle.erase(c.idle.begin() + (std::ptrdiff_t)i);
                c.idle_bytes -= e.second;
                c.live[e.first] = e.second;
                return e.first;
            }
        }
    }
    void *p = nullptr;
    if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess || !p) return nullptr;
    std::lock_guard<std::mutex> g(c.mu);
    c.live[p] = n;
    return p;
}

void pinned_put(void *p) {
    PinCache &c = pins();
    std::vector<void *> drop;
    {
        std::lock_guard<std::mutex> g(c.mu);
        auto it = c.live.find(p);
        if (it == c.live.end() || it->second > kPinKeep) {
            drop.push_back(p);
            if (it != c.live.end()) c.live.erase(it);
        } else {
            c.idle.push_back({p, it->second});
            c.idle_bytes += it->second;
            c.live.erase(it);
            while (c.idle_bytes > kPinKeep) {
                drop.push_back(c.idle.front().first);
                c.idle_bytes -= c.idle.front().second;
                c.idle.erase(c.idle.begin());
            }
        }
    }
    for (void *q : drop) (void)hipHostFree(q);
}

class FbWriter {
  public:
    std::vector<uint8_t> b;

    size_t pos() const { return b.size(); }
    void align(size_t a) {
        while (b.size() % a) b.push_back(0);
    }
    template <typename T>
    size_t put(T v) {
        align(sizeof(T));
        const size_t at = b.size();
        b.resize(at + sizeof(T));
        std::memcpy(&b[at], &v, sizeof(T));
        return at;
    }
    template <typename T>
    void patch(size_t at, T v) {
        std::memcpy(&b[at], &v, sizeof(T));
    }
    // uoffset at `field` -> object at `target` (target > field)
    void link(size_t field, size_t target) { patch<uint32_t>(field, (uint32_t)(target - field)); }

    // A table with `nf` vtable slots; fields are added in declaration order of the
    // caller, each scalar aligned to its size inside the table.
    struct Table {
        size_t vt = 0, start = 0;
        int nf = 0;
    };
    Table begin_table(int nf) {
        align(4);
        Table t;
        t.nf = nf;
        t.vt = b.size();
        put<uint16_t>((uint16_t)(4 + 2 * nf));
        put<uint16_t>(0);  // table size, patched at end_table
        for (int i = 0; i < nf; ++i) put<uint16_t>(0);
        align(4);
        t.start = put<int32_t>(0);
        patch<int32_t>(t.start, (int32_t)(t.start - t.vt));  // vtable = table - soffset
        return t;
    }
    template <typename T>
    size_t field(Table &t, int slot, T v) {
        const size_t at = put<T>(v);
        patch<uint16_t>(t.vt + 4 + 2 * slot, (uint16_t)(at - t.start));
        return at;
    }
    size_t field_offset(Table &t, int slot) { return field<uint32_t>(t, slot, 0); }
    void end_table(Table &t) {
        align(4);
        patch<uint16_t>(t.vt + 2, (uint16_t)(b.size() - t.start));
    }
    size_t string(const std::string &s) {
        align(4);
        const size_t at = put<uint32_t>((uint32_t)s.size());
        b.insert(b.end(), s.begin(), s.end());
        b.push_back(0);
        return at;
    }
};

struct IpcType {
    uint8_t type;       // flatbuffers Type union: Int = 2, FloatingPoint = 3, Utf8 = 5, Bool = 6
    int32_t bit_width;  // Int
    bool is_signed;
    int16_t precision;  // FloatingPoint: SINGLE = 1, DOUBLE = 2
};

IpcType ipc_type(int dt) {
    switch (dt) {
        case QEH_DT_BOOL: return {6, 0, false, 0};
        case QEH_DT_INT32: return {2, 32, true, 0};
        case QEH_DT_INT64: return {2, 64, true, 0};
        case QEH_DT_UINT32: return {2, 32, false, 0};
        case QEH_DT_FLOAT32: return {3, 0, false, 1};
        case QEH_DT_FLOAT64: return {3, 0, false, 2};
        case QEH_DT_UTF8: return {5, 0, false, 0};
        default: return {0, 0, false, 0};
    }
}

// Message { version: short = V5 (4), header_type: ubyte, header: table, bodyLength: long }
// slots: 0 version, 1 header_type, 2 header, 3 bodyLength, 4 custom_metadata
size_t begin_message(FbWriter &w, uint8_t header_type, int64_t body_len, size_t *header_field) {
    const size_t root = w.put<uint32_t>(0);
    auto m = w.begin_table(5);
    w.link(root, m.start);
    w.field<int64_t>(m, 3, body_len);
    *header_field = w.field_offset(m, 2);
    w.field<int16_t>(m, 0, 4);
    w.field<uint8_t>(m, 1, header_type);
    w.end_table(m);
    return root;
}

void schema_message(FbWriter &w, const qeh_column *cols, const char *const *names, int n) {
    size_t hdr;
    begin_message(w, 1, 0, &hdr);
    // Schema { endianness: short (Little = 0), fields: [Field] }: slots 0 endianness, 1 fields
    auto s = w.begin_table(4);
    w.link(hdr, s.start);
    const size_t fields_field = w.field_offset(s, 1);
    w.end_table(s);
    w.align(4);
    const size_t vec = w.put<uint32_t>((uint32_t)n);
    w.link(fields_field, vec);
    std::vector<size_t> elem(n);
    for (int i = 0; i < n; ++i) elem[i] = w.put<uint32_t>(0);
    for (int i = 0; i < n; ++i) {
        // Field { name: string, nullable: bool, type_type: ubyte, type: table, dictionary, children: [Field] }
        // slots: 0 name, 1 nullable, 2 type_type, 3 type, 4 dictionary, 5 children, 6 custom_metadata
        const IpcType t = ipc_type(cols[i].dtype);
        auto f = w.begin_table(7);
        w.link(elem[i], f.start);
        const size_t name_field = w.field_offset(f, 0);
        const size_t type_field = w.field_offset(f, 3);
        const size_t children_field = w.field_offset(f, 5);
        w.field<uint8_t>(f, 1, 1);  // nullable (the reference's planner fields are nullable)
        w.field<uint8_t>(f, 2, t.type);
        w.end_table(f);
        w.link(name_field, w.string(names && names[i] ? names[i] : ("col_" + std::to_string(i))));
        auto ty = w.begin_table(2);
        w.link(type_field, ty.start);
        if (t.type == 2) {  // Int { bitWidth: int, is_signed: bool }
            w.field<int32_t>(ty, 0, t.bit_width);
            w.field<uint8_t>(ty, 1, t.is_signed ? 1 : 0);
        } else if (t.type == 3) {  // FloatingPoint { precision: short }
            w.field<int16_t>(ty, 0, t.precision);
        }
        w.end_table(ty);
        w.align(4);
        w.link(children_field, w.put<uint32_t>(0));  // no children
    }
}

struct BodyBuf {
    const void *dev;  // nullptr: zero-length buffer
    int64_t len;
    int64_t offset;  // inside the body
};

// RecordBatch { length: long, nodes: [FieldNode], buffers: [Buffer] }: slots 0 length, 1 nodes, 2 buffers
void batch_message(FbWriter &w, int64_t rows, const std::vector<std::pair<int64_t, int64_t>> &nodes,
                   const std::vector<BodyBuf> &bufs, int64_t body_len) {
    size_t hdr;
    begin_message(w, 3, body_len, &hdr);
    auto rb = w.begin_table(5);
    w.link(hdr, rb.start);
    w.field<int64_t>(rb, 0, rows);
    const size_t nodes_field = w.field_offset(rb, 1);
    const size_t bufs_field = w.field_offset(rb, 2);
    w.end_table(rb);
    // vectors of structs: count, then 8-byte aligned 16-byte elements
    auto struct_vec = [&](size_t field, size_t count) {
        while ((w.pos() + 4) % 8) w.b.push_back(0);
        const size_t at = w.put<uint32_t>((uint32_t)count);
        w.link(field, at);
    };
    struct_vec(nodes_field, nodes.size());
    for (auto &nd : nodes) {
        w.put<int64_t>(nd.first);
        w.put<int64_t>(nd.second);
    }
    struct_vec(bufs_field, bufs.size());
    for (auto &bb : bufs) {
        w.put<int64_t>(bb.offset);
        w.put<int64_t>(bb.len);
    }
}

void frame(std::vector<uint8_t> &out, const FbWriter &w) {
    std::vector<uint8_t> meta = w.b;
    while (meta.size() % 8) meta.push_back(0);
    const uint32_t cont = 0xFFFFFFFFu, len = (uint32_t)meta.size();
    out.insert(out.end(), (const uint8_t *)&cont, (const uint8_t *)&cont + 4);
    out.insert(out.end(), (const uint8_t *)&len, (const uint8_t *)&len + 4);
    out.insert(out.end(), meta.begin(), meta.end());
}

// ---- reading (SerializedBatch::to_batch, network.rs:75-90) ----------------------------
// A bounds-checked view of one flatbuffer: every position is validated against the
// buffer before it is read (the bytes come from the network).
struct FbReader {
    const uint8_t *b;
    size_t n;
    bool ok = true;

    template <typename T>
    T rd(size_t at) {
        if (at > n || n - at < sizeof(T)) {
            ok = false;
            return T{};
        }
        T v;
        std::memcpy(&v, b + at, sizeof(T));
        return v;
    }
    size_t deref(size_t at) {  // uoffset
        const uint32_t o = rd<uint32_t>(at);
        if (!ok || at + o >= n) {
            ok = false;
            return 0;
        }
        return at + o;
    }
    // position of field `slot` of the table at t, or 0 when absent
    size_t field(size_t t, int slot) {
        const int32_t so = rd<int32_t>(t);
        if (!ok) return 0;
        const int64_t vt = (int64_t)t - so;
        if (vt < 0 || (size_t)vt >= n) {
            ok = false;
            return 0;
        }
        const uint16_t vsize = rd<uint16_t>((size_t)vt);
        if ((size_t)(4 + 2 * slot) + 2 > vsize) return 0;
        const uint16_t off = rd<uint16_t>((size_t)vt + 4 + 2 * slot);
        return off ? t + off : 0;
    }
    template <typename T>
    T scalar(size_t t, int slot, T dflt) {
        const size_t f = field(t, slot);
        return f ? rd<T>(f) : dflt;
    }
    size_t table(size_t t, int slot) {
        const size_t f = field(t, slot);
        return f ? deref(f) : 0;
    }
    uint32_t vec_len(size_t v) { return rd<uint32_t>(v); }
    std::string str(size_t s) {
        const uint32_t len = rd<uint32_t>(s);
        if (!ok || s + 4 + len > n) {
            ok = false;
            return {};
        }
        return std::string((const char *)b + s + 4, len);
    }
};

struct IpcMsg {
    const uint8_t *meta = nullptr;
    size_t meta_len = 0;
    const uint8_t *body = nullptr;
    int64_t body_len = 0;
    uint8_t header_type = 0;
    size_t header = 0;  // position of the header table inside meta
};

int read_message(const uint8_t *p, size_t n, size_t *pos, IpcMsg *m, bool *eos) {
    *eos = false;
    if (*pos + 4 > n) {
        *eos = true;  // a stream may end without the marker
        return QEH_OK;
    }
    uint32_t len;
    std::memcpy(&len, p + *pos, 4);
    size_t at = *pos + 4;
    if (len == 0xFFFFFFFFu) {
        if (at + 4 > n) return fail(QEH_E_INVALID, "ipc: truncated message length");
        std::memcpy(&len, p + at, 4);
        at += 4;
    }
    if (len == 0) {
        *eos = true;
        return QEH_OK;
    }
    if (at + len > n) return fail(QEH_E_INVALID, "ipc: truncated message metadata");
    FbReader r{p + at, len};
    const size_t root = r.deref(0);
    const int16_t version = r.scalar<int16_t>(root, 0, 0);
    const uint8_t ht = r.scalar<uint8_t>(root, 1, 0);
    const size_t hdr = r.table(root, 2);
    const int64_t body_len = r.scalar<int64_t>(root, 3, 0);
    if (!r.ok || !hdr) return fail(QEH_E_INVALID, "ipc: malformed message");
    if (version < 3) return fail(QEH_E_UNSUPPORTED, "ipc: metadata version before V4");
    if (body_len < 0 || at + len + (size_t)body_len > n) return fail(QEH_E_INVALID, "ipc: truncated message body");
    m->meta = p + at;
    m->meta_len = len;
    m->body = p + at + len;
    m->body_len = body_len;
    m->header_type = ht;
    m->header = hdr;
    *pos = at + len + (size_t)body_len;
    return QEH_OK;
}

int dtype_of_ipc(FbReader &r, size_t field, int *dt) {
    const uint8_t tt = r.scalar<uint8_t>(field, 2, 0);
    const size_t ty = r.table(field, 3);
    const size_t ch = r.table(field, 5);
    if (ch && r.vec_len(ch) != 0) return fail(QEH_E_UNSUPPORTED, "ipc: nested types are not supported");
    if (r.field(field, 4)) return fail(QEH_E_UNSUPPORTED, "ipc: dictionary-encoded fields are not supported");
    switch (tt) {
        case 2: {
            const int32_t bw = ty ? r.scalar<int32_t>(ty, 0, 0) : 0;
            const bool sg = ty ? r.scalar<uint8_t>(ty, 1, 0) != 0 : false;
            if (bw == 64 && sg) *dt = QEH_DT_INT64;
            else if (bw == 32 && sg) *dt = QEH_DT_INT32;
            else if (bw == 32) *dt = QEH_DT_UINT32;
            else return fail(QEH_E_UNSUPPORTED, "ipc: integer width/signedness not supported");
            return QEH_OK;
        }
        case 3: {
            const int16_t pr = ty ? r.scalar<int16_t>(ty, 0, 0) : 0;
            if (pr == 1) *dt = QEH_DT_FLOAT32;
            else if (pr == 2) *dt = QEH_DT_FLOAT64;
            else return fail(QEH_E_UNSUPPORTED, "ipc: half floats are not supported");
            return QEH_OK;
        }
        case 5: *dt = QEH_DT_UTF8; return QEH_OK;
        case 6: *dt = QEH_DT_BOOL; return QEH_OK;
        default: return fail(QEH_E_UNSUPPORTED, "ipc: column type not supported");
    }
}

}  // namespace
}  // namespace qeh

using namespace qeh;

extern "C" int qeh_encode_arrow_ipc(qeh_ctx *ctx, const qeh_column *cols, const char *const *names, int n_cols,
                                    uint8_t **out_bytes, int64_t *out_size) {
    if (!ctx || !out_bytes || !out_size || n_cols < 0 || (n_cols > 0 && !cols))
        return fail(QEH_E_INVALID, "qeh_encode_arrow_ipc: bad argument");
    *out_bytes = nullptr;
    *out_size = 0;
    DeviceGuard dg(ctx->device);
    const int64_t rows = n_cols > 0 ? cols[0].length : 0;
    for (int i = 0; i < n_cols; ++i) {
        QEH_TRY(check_column(cols[i], "ipc"));
        if (cols[i].length != rows) return fail(QEH_E_INVALID, "ipc: columns have different lengths");
        if (ipc_type(cols[i].dtype).type == 0) return fail(QEH_E_UNSUPPORTED, "ipc: unsupported column type");
    }
    // normalise every column to offset 0 on the device (one copy; bits re-aligned)
    std::vector<qeh_column> norm(n_cols);
    int made = 0, s = QEH_OK;
    for (int i = 0; i < n_cols && s == QEH_OK; ++i) {
        const qeh_column *one = &cols[i];
        s = concat_columns(ctx, &one, 1, &norm[i]);
        if (s == QEH_OK) ++made;
    }
    auto release = [&]() {
        for (int i = 0; i < made; ++i) qeh_column_release(ctx, &norm[i]);
    };
    if (s != QEH_OK) {
        release();
        return s;
    }
    hipError_t he = hipStreamSynchronize(ctx->stream);
    if (he != hipSuccess) {
        release();
        return fail(QEH_E_HIP, std::string("ipc: ") + hipGetErrorString(he));
    }
    // body layout: per column validity, then values (or offsets + data), 64-byte aligned
    std::vector<std::pair<int64_t, int64_t>> nodes;
    std::vector<BodyBuf> bufs;
    int64_t body = 0;
    auto add = [&](const void *p, int64_t len) {
        bufs.push_back({len ? p : nullptr, len, body});
        body += (len + 63) / 64 * 64;
    };
    for (int i = 0; i < n_cols; ++i) {
        const qeh_column &c = norm[i];
        int64_t nulls = 0;
        if (c.validity) {
            nulls = c.null_count;
            if (nulls < 0) {  // count on the host from the normalised bitmap
                std::vector<uint8_t> vb((size_t)(rows + 7) / 8);
                if (!vb.empty() && (s = read_small(ctx, vb.data(), c.validity, vb.size())) != QEH_OK) break;
                nulls = 0;
                for (int64_t r = 0; r < rows; ++r) nulls += !((vb[(size_t)(r >> 3)] >> (r & 7)) & 1);
            }
        }
        nodes.push_back({rows, nulls});
        add(nulls ? c.validity : nullptr, nulls ? (rows + 7) / 8 : 0);
        if (c.dtype == QEH_DT_UTF8) {
            add(c.offsets, (rows + 1) * 4);
            add(c.values, c.values_bytes);
        } else if (c.dtype == QEH_DT_BOOL) {
            add(c.values, (rows + 7) / 8);
        } else {
            add(c.values, rows * (int64_t)dtype_size(c.dtype));
        }
    }
    if (s != QEH_OK) {
        release();
        return s;
    }
    std::vector<uint8_t> head;  // schema message + record batch metadata (small)
    {
        FbWriter w;
        schema_message(w, cols, names, n_cols);
        frame(head, w);
    }
    {
        FbWriter w;
        batch_message(w, rows, nodes, bufs, body);
        frame(head, w);
    }
    // one host allocation: metadata, the body copied straight from HBM, end-of-stream marker
    const size_t total = head.size() + (size_t)body + 8;
    // pinned: the body leaves HBM at the DMA rate instead of through pageable staging
    uint8_t *p = (uint8_t *)pinned_get(total);
    if (!p) {
        release();
        return fail(QEH_E_OOM, "ipc: host allocation");
    }
    std::memcpy(p, head.data(), head.size());
    uint8_t *bp = p + head.size();
    int64_t filled = 0;
    for (auto &bb : bufs) {
        if (bb.offset > filled) std::memset(bp + filled, 0, (size_t)(bb.offset - filled));
        if (bb.dev && bb.len) {
            he = hipMemcpyAsync(bp + bb.offset, bb.dev, (size_t)bb.len, hipMemcpyDeviceToHost, ctx->stream);
            if (he != hipSuccess) break;
        }
        filled = bb.offset + bb.len;
    }
    if (body > filled) std::memset(bp + filled, 0, (size_t)(body - filled));
    if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
    release();
    if (he != hipSuccess) {
        pinned_put(p);
        return fail(QEH_E_HIP, std::string("ipc: ") + hipGetErrorString(he));
    }
    const uint32_t eos[2] = {0xFFFFFFFFu, 0u};
    std::memcpy(p + total - 8, eos, 8);
    *out_bytes = p;
    *out_size = (int64_t)total;
    return QEH_OK;
}

// buffers returned by the IPC entry points are pinned host memory (kept for reuse, pinned_put)
extern "C" void qeh_host_free(void *p) {
    if (p) pinned_put(p);
}

extern "C" int qeh_decode_arrow_ipc(qeh_ctx *ctx, const uint8_t *bytes, int64_t size, qeh_column *out_cols, int max_cols,
                                    int *out_n_cols, char **out_names, int64_t *out_rows) {
    if (!ctx || (!bytes && size > 0) || size < 0 || !out_n_cols || !out_rows || (max_cols > 0 && !out_cols))
        return fail(QEH_E_INVALID, "qeh_decode_arrow_ipc: bad argument");
    *out_n_cols = 0;
    *out_rows = 0;
    if (out_names) *out_names = nullptr;
    DeviceGuard dg(ctx->device);
    size_t pos = 0;
    bool eos = false;
    IpcMsg schema_msg;
    QEH_TRY(read_message(bytes, (size_t)size, &pos, &schema_msg, &eos));
    if (eos || schema_msg.header_type != 1) return fail(QEH_E_INVALID, "ipc: stream does not start with a schema");
    FbReader sr{schema_msg.meta, schema_msg.meta_len};
    const size_t fields = sr.table(schema_msg.header, 1);
    const uint32_t nf = fields ? sr.vec_len(fields) : 0;
    if (!sr.ok) return fail(QEH_E_INVALID, "ipc: malformed schema");
    if (max_cols < 0 || nf > (uint32_t)max_cols) return fail(QEH_E_INVALID, "ipc: more columns than out_cols holds");
    std::vector<int> dts(nf);
    std::string names;
    for (uint32_t i = 0; i < nf; ++i) {
        const size_t f = sr.deref(fields + 4 + 4 * (size_t)i);
        if (!sr.ok) return fail(QEH_E_INVALID, "ipc: malformed field");
        QEH_TRY(dtype_of_ipc(sr, f, &dts[i]));
        const size_t nm = sr.table(f, 0);
        names += nm ? sr.str(nm) : std::string();
        names.push_back('\0');
        if (!sr.ok) return fail(QEH_E_INVALID, "ipc: malformed field name");
    }
    // the first record batch (to_batch returns the first one; network.rs:81-84)
    IpcMsg bm;
    for (;;) {
        QEH_TRY(read_message(bytes, (size_t)size, &pos, &bm, &eos));
        if (eos) return fail(QEH_E_INVALID, "No batch found in serialized data");
        if (bm.header_type == 3) break;
        if (bm.header_type == 2) return fail(QEH_E_UNSUPPORTED, "ipc: dictionary batches are not supported");
    }
    FbReader br{bm.meta, bm.meta_len};
    const int64_t rows = br.scalar<int64_t>(bm.header, 0, 0);
    const size_t nodes = br.table(bm.header, 1), bufs = br.table(bm.header, 2);
    if (br.field(bm.header, 3)) return fail(QEH_E_UNSUPPORTED, "ipc: compressed bodies are not supported");
    if (!br.ok || rows < 0 || rows > ((int64_t)1 << 40) || !nodes || !bufs || br.vec_len(nodes) != nf)
        return fail(QEH_E_INVALID, "ipc: malformed record batch");
    const uint32_t nb = br.vec_len(bufs);
    uint32_t bi = 0;
    auto buffer = [&](const uint8_t **p, int64_t *len) -> int {
        if (bi >= nb) return fail(QEH_E_INVALID, "ipc: too few buffers");
        const size_t at = bufs + 4 + 16 * (size_t)bi++;
        const int64_t off = br.rd<int64_t>(at), l = br.rd<int64_t>(at + 8);
        if (!br.ok || off < 0 || l < 0 || off > (int64_t)bm.body_len || l > (int64_t)bm.body_len - off) return fail(QEH_E_INVALID, "ipc: buffer outside the body");
        *p = bm.body + off;
        *len = l;
        return QEH_OK;
    };
    int made = 0, s = QEH_OK;
    for (uint32_t i = 0; i < nf && s == QEH_OK; ++i) {
        const size_t nd = nodes + 4 + 16 * (size_t)i;
        const int64_t len = br.rd<int64_t>(nd), nulls = br.rd<int64_t>(nd + 8);
        if (!br.ok || len != rows || nulls < 0 || nulls > rows) {
            s = fail(QEH_E_INVALID, "ipc: field node does not match the batch");
            break;
        }
        const uint8_t *vp, *dp, *op;
        int64_t vl, dl, ol;
        if ((s = buffer(&vp, &vl)) != QEH_OK) break;
        const bool has_valid = nulls > 0;
        if (has_valid && vl < (rows + 7) / 8) {
            s = fail(QEH_E_INVALID, "ipc: validity buffer too short");
            break;
        }
        qeh_column &c = out_cols[i];
        if (dts[i] == QEH_DT_UTF8) {
            if ((s = buffer(&op, &ol)) != QEH_OK || (s = buffer(&dp, &dl)) != QEH_OK) break;
            if (ol < (rows + 1) * 4) {
                s = fail(QEH_E_INVALID, "ipc: offsets buffer too short");
                break;
            }
            std::memset(&c, 0, sizeof(c));
            c.dtype = QEH_DT_UTF8;
            c.owned = 1;
            c.length = rows;
            void *o = nullptr, *d = nullptr;
            if ((s = ctx->pool->alloc((size_t)(rows + 1) * 4, &o)) != QEH_OK) break;
            if ((s = ctx->pool->alloc(std::max<size_t>((size_t)dl, 8), &d)) != QEH_OK) {
                ctx->pool->free(o);
                break;
            }
            c.offsets = (int32_t *)o;
            c.values = d;
            c.values_bytes = dl;
            // untrusted offsets: non-decreasing, inside the data buffer (device kernels index with them)
            int32_t prev, last;
            std::memcpy(&prev, op, 4);
            bool mono = prev >= 0;
            for (int64_t r = 1; mono && r <= rows; ++r) {
                int32_t cur;
                std::memcpy(&cur, op + r * 4, 4);
                mono = cur >= prev;
                prev = cur;
            }
            std::memcpy(&last, op + rows * 4, 4);
            if (!mono || last < 0 || last > dl) {
                ctx->pool->free(o);
                ctx->pool->free(d);
                s = fail(QEH_E_INVALID, "ipc: Utf8 offsets decreasing or outside the data buffer");
                break;
            }
            QEH_HIP(hipMemcpyAsync(o, op, (size_t)(rows + 1) * 4, hipMemcpyHostToDevice, ctx->stream));
            if (dl) QEH_HIP(hipMemcpyAsync(d, dp, (size_t)dl, hipMemcpyHostToDevice, ctx->stream));
            if (has_valid) {
                void *v = nullptr;
                if ((s = ctx->pool->alloc(std::max<size_t>((size_t)(rows + 63) / 64 * 8, 8), &v)) != QEH_OK) {
                    ctx->pool->free(o);
                    ctx->pool->free(d);
                    break;
                }
                c.validity = (uint8_t *)v;
            }
        } else {
            if ((s = buffer(&dp, &dl)) != QEH_OK) break;
            const int64_t need = dts[i] == QEH_DT_BOOL ? (rows + 7) / 8 : rows * (int64_t)dtype_size(dts[i]);
            if (dl < need) {
                s = fail(QEH_E_INVALID, "ipc: values buffer too short");
                break;
            }
            if ((s = alloc_column(ctx, dts[i], rows, has_valid, &c)) != QEH_OK) break;
            if (need) QEH_HIP(hipMemcpyAsync(c.values, dp, (size_t)need, hipMemcpyHostToDevice, ctx->stream));
        }
        if (has_valid) QEH_HIP(hipMemcpyAsync(c.validity, vp, (size_t)(rows + 7) / 8, hipMemcpyHostToDevice, ctx->stream));
        c.null_count = nulls;
        ++made;
    }
    if (s == QEH_OK) {
        hipError_t e = hipStreamSynchronize(ctx->stream);  // the host bytes are the caller's
        if (e != hipSuccess) s = fail(QEH_E_HIP, std::string("ipc: ") + hipGetErrorString(e));
    }
    if (s != QEH_OK) {
        for (int i = 0; i < made; ++i) qeh_column_release(ctx, &out_cols[i]);
        return s;
    }
    if (out_names) {
        char *p = (char *)pinned_get(std::max<size_t>(names.size(), 1));
        if (!p) {
            for (int i = 0; i < made; ++i) qeh_column_release(ctx, &out_cols[i]);
            return fail(QEH_E_OOM, "ipc: host allocation");
        }
        std::memcpy(p, names.data(), names.size());
        *out_names = p;
    }
    *out_n_cols = (int)nf;
    *out_rows = rows;
    return QEH_OK;
}
