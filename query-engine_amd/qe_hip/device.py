"""Device context and column handles over the qeh C ABI.

Host data enters as numpy arrays (values + optional boolean validity) laid out
exactly like Arrow primitive arrays once on the device (bit-packed booleans and
LSB-first validity bitmaps).  Every operator wrapper calls one C entry point of
include/qeh.h; nothing here computes results on the CPU.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .expr import AggregateExpr, PhysicalExpr

NP_OF = {abi.DT_INT32: np.int32, abi.DT_INT64: np.int64, abi.DT_FLOAT32: np.float32,
         abi.DT_FLOAT64: np.float64, abi.DT_UINT32: np.uint32}
DT_OF = {np.dtype(np.int32): abi.DT_INT32, np.dtype(np.int64): abi.DT_INT64,
         np.dtype(np.float32): abi.DT_FLOAT32, np.dtype(np.float64): abi.DT_FLOAT64,
         np.dtype(np.uint32): abi.DT_UINT32, np.dtype(np.bool_): abi.DT_BOOL}


def pack_bits(b: np.ndarray) -> np.ndarray:
    """bool[n] -> Arrow LSB-first bitmap bytes, padded to 8 bytes."""
    bits = np.packbits(np.asarray(b, dtype=bool), bitorder="little")
    pad = (-len(bits)) % 8
    return np.concatenate([bits, np.zeros(pad + (8 if len(bits) == 0 else 0), np.uint8)])


def unpack_bits(buf: np.ndarray, n: int, offset: int = 0) -> np.ndarray:
    return np.unpackbits(buf, bitorder="little")[offset:offset + n].astype(bool)


class DeviceColumn:
    """An Arrow-layout column in HBM.  `owned` columns came from the library
    pool (released with qeh_column_release); uploaded columns are owned by
    this handle's context allocations."""

    def __init__(self, ctx: "Context", c: abi.QehColumn, bufs: Sequence[int] = ()):
        self.ctx = ctx
        self.c = c
        self._bufs = list(bufs)  # pool buffers this handle allocated itself

    @property
    def dtype(self) -> int:
        return self.c.dtype

    def __len__(self) -> int:
        return self.c.length

    def release(self) -> None:
        if self.ctx is None:
            return
        if self.c.owned:
            abi.check(self.ctx.lib.qeh_column_release(self.ctx.h, C.byref(self.c)))
        for b in self._bufs:
            self.ctx.free(b)
        self._bufs = []
        self.ctx = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass

    def to_bytes(self) -> List[bytes]:
        """Utf8 column -> its strings as raw bytes (no decoding; e.g. encoded DataRow messages)."""
        assert self.c.dtype == abi.DT_UTF8
        n, off = self.c.length, self.c.offset
        offs = np.empty(n + 1, np.int32)
        self.ctx.d2h(offs, self.c.offsets + 4 * off, 4 * (n + 1))
        nb = int(offs[-1]) if n else 0
        data = np.empty(max(nb, 1), np.uint8)
        if nb:
            self.ctx.d2h(data, self.c.values, nb)
        raw = data.tobytes()
        return [raw[offs[i]:offs[i + 1]] for i in range(n)]

    def to_numpy(self) -> Tuple[np.ndarray, Optional[np.ndarray]]:
        """(values, validity-or-None) copied to the host."""
        n, off = self.c.length, self.c.offset
        ctx = self.ctx
        valid = None
        if self.c.validity and n > 0:
            nbytes = (off + n + 7) // 8
            vb = np.empty(nbytes, np.uint8)
            ctx.d2h(vb, self.c.validity, nbytes)
            valid = unpack_bits(vb, n, off)
        elif self.c.validity:
            valid = np.zeros(0, bool)
        if self.c.dtype == abi.DT_UTF8:
            offs = np.empty(n + 1, np.int32)
            ctx.d2h(offs, self.c.offsets + 4 * off, 4 * (n + 1))
            nb = int(offs[-1]) if n else 0
            data = np.empty(max(nb, 1), np.uint8)
            if nb:
                ctx.d2h(data, self.c.values, nb)
            raw = data.tobytes()
            out = np.array([raw[offs[i]:offs[i + 1]].decode() for i in range(n)], dtype=object)
            return out, valid
        if self.c.dtype == abi.DT_BOOL:
            nbytes = (off + n + 7) // 8
            vb = np.empty(max(nbytes, 1), np.uint8)
            if n > 0:
                ctx.d2h(vb, self.c.values, nbytes)
            return unpack_bits(vb, n, off), valid
        npdt = NP_OF[self.c.dtype]
        out = np.empty(n, npdt)
        if n > 0:
            ctx.d2h(out, self.c.values + off * out.itemsize, n * out.itemsize)
        return out, valid


class Context:
    def __init__(self, device: int = 0):
        self.lib = abi.load()
        h = C.c_void_p()
        abi.check(self.lib.qeh_init(device, C.byref(h)))
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            abi.check(self.lib.qeh_shutdown(self.h))
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- memory ----------------------------------------------------------
    def alloc(self, nbytes: int) -> int:
        p = C.c_void_p()
        abi.check(self.lib.qeh_device_alloc(self.h, max(int(nbytes), 8), C.byref(p)))
        return p.value

    def free(self, p: int) -> None:
        abi.check(self.lib.qeh_device_free(self.h, p))

    def h2d(self, dst: int, src: np.ndarray) -> None:
        src = np.ascontiguousarray(src)
        abi.check(self.lib.qeh_memcpy_h2d(self.h, dst, src.ctypes.data, src.nbytes))

    def d2h(self, dst: np.ndarray, src: int, nbytes: int) -> None:
        abi.check(self.lib.qeh_memcpy_d2h(self.h, dst.ctypes.data, src, nbytes))

    def lds_atomic_rank_ok(self) -> bool:
        """Whether the device ranks a tile's rows stably by LDS atomics (else the sort, exchange
        and window passes rank by ballot matching); a once-per-process self-check kernel."""
        s = self.lib.qeh_lds_atomic_rank_ok(self.h)
        if s < 0:
            abi.check(s)
        return s == 1

    def sync(self) -> None:
        abi.check(self.lib.qeh_synchronize(self.h))

    def set_stream(self, stream_handle: int) -> None:
        abi.check(self.lib.qeh_set_stream(self.h, stream_handle))
        self.stream_handle = stream_handle

    # ---- timing ----------------------------------------------------------
    def timing(self, on: bool) -> None:
        abi.check(self.lib.qeh_timing_enable(self.h, 1 if on else 0))

    def timing_reset(self) -> None:
        abi.check(self.lib.qeh_timing_reset(self.h))

    def kernel_time(self, name: str) -> Tuple[float, int]:
        ms, n = C.c_double(), C.c_int64()
        abi.check(self.lib.qeh_kernel_time(self.h, name.encode(), C.byref(ms), C.byref(n)))
        return ms.value, n.value

    # ---- columns ---------------------------------------------------------
    def upload(self, values: np.ndarray, valid: Optional[np.ndarray] = None, offset: int = 0) -> DeviceColumn:
        """numpy -> Arrow-layout device column.  `offset` prepends that many
        padding rows and records them as the Arrow array offset (exercises
        non-zero offsets)."""
        if isinstance(values, (list, tuple)) or (isinstance(values, np.ndarray) and values.dtype == object):
            return self._upload_utf8(list(values), valid)
        values = np.asarray(values)
        dt = DT_OF.get(values.dtype)
        if dt is None:
            raise TypeError(f"unsupported dtype {values.dtype}")
        n = len(values)
        c = abi.QehColumn(dtype=dt, owned=0, length=n, offset=offset, null_count=0)
        bufs = []
        if dt == abi.DT_BOOL:
            host = pack_bits(np.concatenate([np.zeros(offset, bool), values]))
        else:
            host = np.concatenate([np.zeros(offset, values.dtype), values])
        p = self.alloc(max(host.nbytes, 8))
        bufs.append(p)
        if host.nbytes:
            self.h2d(p, host)
        c.values = p
        if valid is not None:
            valid = np.asarray(valid, bool)
            vb = pack_bits(np.concatenate([np.zeros(offset, bool), valid]))
            q = self.alloc(max(vb.nbytes, 8))
            bufs.append(q)
            self.h2d(q, vb)
            c.validity = q
            c.null_count = int(n - valid.sum())
        return DeviceColumn(self, c, bufs)

    def _upload_utf8(self, strs, valid=None) -> DeviceColumn:
        n = len(strs)
        if valid is None:
            valid = np.array([x is not None for x in strs], bool)
        enc = [(x if isinstance(x, bytes) else (x or "").encode()) if v else b"" for x, v in zip(strs, valid)]
        offs = np.zeros(n + 1, np.int32)
        offs[1:] = np.cumsum([len(b) for b in enc]) if n else []
        data = np.frombuffer(b"".join(enc), np.uint8) if offs[-1] else np.zeros(8, np.uint8)
        po, pd = self.alloc(offs.nbytes), self.alloc(max(data.nbytes, 8))
        self.h2d(po, offs)
        self.h2d(pd, data)
        c = abi.QehColumn(dtype=abi.DT_UTF8, owned=0, length=n, offset=0, null_count=int(n - valid.sum()),
                          values=pd, offsets=po, values_bytes=int(offs[-1]))
        bufs = [po, pd]
        if not valid.all():
            vb = pack_bits(valid)
            q = self.alloc(vb.nbytes)
            self.h2d(q, vb)
            c.validity = q
            bufs.append(q)
        return DeviceColumn(self, c, bufs)

    def empty(self, dtype: int, n: int) -> DeviceColumn:
        """Uninitialised device column (no validity) from the pool."""
        item = np.dtype(NP_OF[dtype]).itemsize
        p = self.alloc(max(n * item, 8))
        c = abi.QehColumn(dtype=dtype, owned=0, length=n, offset=0, null_count=0, values=p)
        return DeviceColumn(self, c, [p])

    def generate(self, kind: int, seed: int, col_id: int, n: int, modulus: int = 0, lo: int = 0,
                 row0: int = 0) -> DeviceColumn:
        dt = abi.DT_FLOAT64 if kind == abi.GEN_UNIT_F64 else abi.DT_INT64
        col = self.empty(dt, n)
        abi.check(self.lib.qeh_generate(self.h, kind, seed, col_id, row0, n, modulus, lo, col.c.values))
        return col

    def _wrap(self, c: abi.QehColumn) -> DeviceColumn:
        return DeviceColumn(self, c)

    @staticmethod
    def _cols(cols: Sequence[DeviceColumn]):
        arr = (abi.QehColumn * max(len(cols), 1))(*[x.c for x in cols])
        return arr

    # ---- operators -------------------------------------------------------
    def filter(self, cols: Sequence[DeviceColumn], predicate: PhysicalExpr,
               out_idx: Optional[Sequence[int]] = None, max_rows: Optional[int] = None
               ) -> Tuple[List[DeviceColumn], int]:
        """qeh_filter; with `max_rows`, qeh_filter_limit (the first max_rows qualifying rows)."""
        out_idx = list(range(len(cols))) if out_idx is None else list(out_idx)
        e, keep = predicate.to_c()
        cin = self._cols(cols)
        oi = (C.c_int32 * max(len(out_idx), 1))(*out_idx)
        cout = (abi.QehColumn * max(len(out_idx), 1))()
        rows = C.c_int64()
        if max_rows is None:
            abi.check(self.lib.qeh_filter(self.h, cin, len(cols), C.byref(e), oi, len(out_idx), cout, C.byref(rows)))
        else:
            abi.check(self.lib.qeh_filter_limit(self.h, cin, len(cols), C.byref(e), oi, len(out_idx), int(max_rows),
                                                cout, C.byref(rows)))
        return [self._wrap(cout[i]) for i in range(len(out_idx))], rows.value

    def eval(self, cols: Sequence[DeviceColumn], expr: PhysicalExpr, n_rows: Optional[int] = None) -> DeviceColumn:
        e, keep = expr.to_c()
        cin = self._cols(cols)
        out = abi.QehColumn()
        n = n_rows if n_rows is not None else (len(cols[0]) if cols else 0)
        abi.check(self.lib.qeh_eval(self.h, cin, len(cols), C.byref(e), n, C.byref(out)))
        if not out.owned:  # zero-copy column reference: keep the source alive
            src = cols[expr.index]
            return DeviceColumn(self, out, []), src
        return self._wrap(out)

    def hash_aggregate(self, keys: Sequence[DeviceColumn], inputs: Sequence[DeviceColumn],
                       aggs: Sequence[Tuple[int, int]], input_batches: int = 1):
        ck, ci = self._cols(keys), self._cols(inputs)
        ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
        ok = (abi.QehColumn * max(len(keys), 1))()
        oa = (abi.QehColumn * max(len(aggs), 1))()
        g = C.c_int64()
        abi.check(self.lib.qeh_hash_aggregate(self.h, ck, len(keys), ci, len(inputs), ca, len(aggs),
                                              input_batches, ok, oa, C.byref(g)))
        if g.value == 0 and not ok[0].values and not oa[0].values:
            return [], [], 0
        return [self._wrap(ok[i]) for i in range(len(keys))], [self._wrap(oa[i]) for i in range(len(aggs))], g.value

    def filter_aggregate(self, cols: Sequence[DeviceColumn], predicate: Optional[PhysicalExpr],
                         key_idx: Sequence[int], aggs: Sequence[Tuple[int, int]], input_batches: int = 1):
        cc = self._cols(cols)
        ki = (C.c_int32 * max(len(key_idx), 1))(*key_idx)
        ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
        ok = (abi.QehColumn * max(len(key_idx), 1))()
        oa = (abi.QehColumn * max(len(aggs), 1))()
        g = C.c_int64()
        if predicate is not None:
            e, keep = predicate.to_c()
            ep = C.byref(e)
        else:
            ep = None
        abi.check(self.lib.qeh_filter_aggregate(self.h, cc, len(cols), ep, ki, len(key_idx), ca, len(aggs),
                                                input_batches, ok, oa, C.byref(g)))
        if g.value == 0 and not oa[0].values:
            return [], [], 0
        return [self._wrap(ok[i]) for i in range(len(key_idx))], [self._wrap(oa[i]) for i in range(len(aggs))], g.value

    def copy_d2d(self, dst: int, src: int, nbytes: int) -> None:
        abi.check(self.lib.qeh_memcpy_d2d(self.h, dst, src, nbytes))

    def wrap_device(self, dtype: int, ptr: int, n: int, validity: int = 0, offsets: int = 0,
                    values_bytes: int = 0) -> DeviceColumn:
        """View caller-owned device memory (e.g. a torch tensor) as a column (Utf8: `offsets` is
        the int32[n + 1] offsets buffer and `ptr` the bytes)."""
        c = abi.QehColumn(dtype=dtype, owned=0, length=n, offset=0, null_count=0 if not validity else -1,
                          values=ptr, validity=validity or None, offsets=offsets or None, values_bytes=values_bytes)
        return DeviceColumn(self, c, [])

    def hash_join_inner(self, probe_key: DeviceColumn, probe_cols: Sequence[DeviceColumn],
                        build_key: DeviceColumn, build_cols: Sequence[DeviceColumn]):
        cp, cb = self._cols(probe_cols), self._cols(build_cols)
        op = (abi.QehColumn * max(len(probe_cols), 1))()
        ob = (abi.QehColumn * max(len(build_cols), 1))()
        rows = C.c_int64()
        abi.check(self.lib.qeh_hash_join_inner(self.h, C.byref(probe_key.c), cp, len(probe_cols),
                                               C.byref(build_key.c), cb, len(build_cols), op, ob, C.byref(rows)))
        return ([self._wrap(op[i]) for i in range(len(probe_cols))],
                [self._wrap(ob[i]) for i in range(len(build_cols))], rows.value)

    def hash_join_outer(self, join_type: int, left_key: DeviceColumn, left_cols: Sequence[DeviceColumn],
                        right_key: DeviceColumn, right_cols: Sequence[DeviceColumn]):
        """qeh_hash_join_outer: join_type 1 LEFT, 2 RIGHT, 3 FULL (0 INNER)."""
        cl, cr = self._cols(left_cols), self._cols(right_cols)
        ol = (abi.QehColumn * max(len(left_cols), 1))()
        orr = (abi.QehColumn * max(len(right_cols), 1))()
        rows = C.c_int64()
        abi.check(self.lib.qeh_hash_join_outer(self.h, int(join_type), C.byref(left_key.c), cl, len(left_cols),
                                               C.byref(right_key.c), cr, len(right_cols), ol, orr, C.byref(rows)))

        def wrap(c, src):
            d = self._wrap(c)
            if not c.owned:
                d.parent = src  # a view of the input column: keep it alive
            return d
        return ([wrap(ol[i], left_cols[i]) for i in range(len(left_cols))],
                [wrap(orr[i], right_cols[i]) for i in range(len(right_cols))], rows.value)

    def join_filter_aggregate(self, probe_cols: Sequence[DeviceColumn], probe_key_idx: int,
                              predicate: Optional[PhysicalExpr], build_key: DeviceColumn,
                              build_group_keys: Sequence[DeviceColumn], aggs: Sequence[Tuple[int, int]]):
        cp = self._cols(probe_cols)
        cg = self._cols(build_group_keys)
        ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
        ok = (abi.QehColumn * max(len(build_group_keys), 1))()
        oa = (abi.QehColumn * max(len(aggs), 1))()
        g = C.c_int64()
        if predicate is not None:
            e, keep = predicate.to_c()
            ep = C.byref(e)
        else:
            ep = None
        abi.check(self.lib.qeh_join_filter_aggregate(self.h, cp, len(probe_cols), probe_key_idx, ep,
                                                     C.byref(build_key.c), cg, len(build_group_keys), ca,
                                                     len(aggs), ok, oa, C.byref(g)))
        return ([self._wrap(ok[i]) for i in range(len(build_group_keys))],
                [self._wrap(oa[i]) for i in range(len(aggs))], g.value)

    def direct_group_table_insert(self, build_key: DeviceColumn, group_key: DeviceColumn, key_min: int,
                                  key_range: int, group_min: int, table_ptr: int, check: bool = True) -> None:
        """qeh_direct_group_table_insert: this shard's rows into the caller's zeroed u16 table
        (check=False: qeh_direct_group_table_insert_async, no host wait; out-of-range rows skipped)."""
        fn = self.lib.qeh_direct_group_table_insert if check else self.lib.qeh_direct_group_table_insert_async
        abi.check(fn(self.h, C.byref(build_key.c), C.byref(group_key.c), key_min, key_range, group_min, table_ptr))

    def columns_minmax(self, cols: Sequence[DeviceColumn]) -> List[Tuple[int, int, int]]:
        """qeh_columns_minmax: [(min, max, non-null count)] of Int32 / Int64 columns, one read."""
        out = (C.c_int64 * (3 * len(cols)))()
        abi.check(self.lib.qeh_columns_minmax(self.h, self._cols(cols), len(cols), out))
        return [(out[3 * i], out[3 * i + 1], out[3 * i + 2]) for i in range(len(cols))]

    def dense_states_f64(self, keys: DeviceColumn, vals: Sequence[DeviceColumn], key_min: int, key_range: int,
                         out_ptr: int) -> None:
        """qeh_dense_states_f64: partial states into f64 lanes [1 + len(vals)][key_range] (caller-zeroed)."""
        abi.check(self.lib.qeh_dense_states_f64(self.h, C.byref(keys.c), self._cols(vals) if vals else None, len(vals),
                                                key_min, key_range, out_ptr))

    def dense_states_take(self, in_ptr: int, n_vals: int, key_min: int, key_range: int, world: int, rank: int,
                          key_dtype: int, out_dtypes: Sequence[int]):
        """qeh_dense_states_take: (keys, value columns, groups) this rank owns after the lane sum."""
        ok = abi.QehColumn()
        ov = (abi.QehColumn * max(n_vals, 1))()
        dts = (C.c_int32 * max(n_vals, 1))(*out_dtypes)
        g = C.c_int64()
        abi.check(self.lib.qeh_dense_states_take(self.h, in_ptr, n_vals, key_min, key_range, world, rank, key_dtype,
                                                 dts, C.byref(ok), ov, C.byref(g)))
        return self._wrap(ok), [self._wrap(ov[i]) for i in range(n_vals)], g.value

    def dense_states_take_status(self, in_ptr: int, n_vals: int, key_min: int, key_range: int, world: int, rank: int,
                                 key_dtype: int, out_dtypes: Sequence[int]):
        """qeh_dense_states_take_status: dense_states_take + the status lane, one host read."""
        ok = abi.QehColumn()
        ov = (abi.QehColumn * max(n_vals, 1))()
        dts = (C.c_int32 * max(n_vals, 1))(*out_dtypes)
        g = C.c_int64()
        st = C.c_double()
        abi.check(self.lib.qeh_dense_states_take_status(self.h, in_ptr, n_vals, key_min, key_range, world, rank,
                                                        key_dtype, dts, C.byref(ok), ov, C.byref(g), C.byref(st)))
        return self._wrap(ok), [self._wrap(ov[i]) for i in range(n_vals)], g.value, st.value

    def u16_count_nonzero(self, table_ptr: int, n: int) -> int:
        out = C.c_int64()
        abi.check(self.lib.qeh_u16_count_nonzero(self.h, table_ptr, n, C.byref(out)))
        return out.value

    def join_filter_aggregate_table(self, probe_cols: Sequence[DeviceColumn], probe_key_idx: int,
                                    predicate: Optional[PhysicalExpr], table_ptr: int, key_min: int, key_range: int,
                                    group_min: int, n_groups: int, group_dtype: int, aggs: Sequence[Tuple[int, int]]):
        """qeh_join_filter_aggregate_table: the fused operator against a DIRECT u16 table of
        (group slot + 1) entries (the table-form broadcast join)."""
        cp = self._cols(probe_cols)
        ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
        ok = (abi.QehColumn * 1)()
        oa = (abi.QehColumn * max(len(aggs), 1))()
        g = C.c_int64()
        e = keep = None
        if predicate is not None:
            e, keep = predicate.to_c()
        abi.check(self.lib.qeh_join_filter_aggregate_table(self.h, cp, len(probe_cols), probe_key_idx,
                                                           C.byref(e) if e is not None else None, table_ptr, key_min,
                                                           key_range, group_min, n_groups, group_dtype, ca, len(aggs),
                                                           ok, oa, C.byref(g)))
        return [self._wrap(ok[0])], [self._wrap(oa[i]) for i in range(len(aggs))], g.value

    def join_filter_aggregate_table_lanes(self, probe_cols: Sequence[DeviceColumn], probe_key_idx: int,
                                          predicate: Optional[PhysicalExpr], table_ptr: int, key_min: int,
                                          key_range: int, n_groups: int, aggs: Sequence[Tuple[int, int]],
                                          lanes_ptr: int) -> None:
        """qeh_join_filter_aggregate_table_lanes: the table-form fused operator writing the dense
        final stage's f64 lanes [1 + len(aggs)][n_groups] (row counts, then COUNT / float SUM partials)."""
        cp = self._cols(probe_cols)
        ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
        e = keep = None
        if predicate is not None:
            e, keep = predicate.to_c()
        abi.check(self.lib.qeh_join_filter_aggregate_table_lanes(self.h, cp, len(probe_cols), probe_key_idx,
                                                                 C.byref(e) if e is not None else None, table_ptr,
                                                                 key_min, key_range, n_groups, ca, len(aggs),
                                                                 lanes_ptr))

    def join_filter_aggregate_table_lanes_async(self, probe_cols: Sequence[DeviceColumn], probe_key_idx: int,
                                                predicate: Optional[PhysicalExpr], table_ptr: int, key_min: int,
                                                key_range: int, n_groups: int, aggs: Sequence[Tuple[int, int]],
                                                lanes_ptr: int, status_ptr: int) -> None:
        """qeh_join_filter_aggregate_table_lanes_async: as ..._lanes, but its status words (error bits,
        region overflow) go to device memory at status_ptr, one more lane after the (1 + aggs) * n_groups
        ones is 1.0 when either is set (lanes_ptr holds (1 + aggs) * n_groups + 1 doubles), and nothing
        waits on the host."""
        cp = self._cols(probe_cols)
        ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
        e = keep = None
        if predicate is not None:
            e, keep = predicate.to_c()
        abi.check(self.lib.qeh_join_filter_aggregate_table_lanes_async(self.h, cp, len(probe_cols), probe_key_idx,
                                                                       C.byref(e) if e is not None else None, table_ptr,
                                                                       key_min, key_range, n_groups, ca, len(aggs),
                                                                       lanes_ptr, status_ptr))

    def u16_count_nonzero_dev(self, table_ptr: int, n: int, out_ptr: int) -> None:
        """qeh_u16_count_nonzero_dev: the non-empty entries of a u16 table into device memory (8 B)."""
        abi.check(self.lib.qeh_u16_count_nonzero_dev(self.h, table_ptr, n, out_ptr))

    def u16_table_check_dev(self, table_ptr: int, n: int, max_entry: int, out_ptr: int) -> None:
        """qeh_u16_table_check_dev: entries in [1, max_entry] counted into device memory (8 B); entries
        above max_entry cleared in place (a later probe reads them as misses)."""
        abi.check(self.lib.qeh_u16_table_check_dev(self.h, table_ptr, n, max_entry, out_ptr))

    def broadcast_stats(self, build_key: DeviceColumn, group_key: DeviceColumn, extra: Sequence[int],
                        out_ptr: int) -> None:
        """qeh_broadcast_stats: [rows, key min, max, group min, max, *extra] of this dimension shard
        into device memory (no host wait)."""
        ex = (C.c_int64 * max(len(extra), 1))(*[int(q) for q in extra])
        abi.check(self.lib.qeh_broadcast_stats(self.h, C.byref(build_key.c), C.byref(group_key.c), ex, len(extra),
                                               out_ptr))

    # the items form of the distributed broadcast join (include/qeh.h qeh_fused_items_*)
    FUSED_ITEMS_SLICES = 160  # slices the item buffers hold (kSliceMaxF)

    def fused_items_begin(self, probe_cols: Sequence[DeviceColumn], probe_key_idx: int,
                          predicate: Optional[PhysicalExpr], aggs: Sequence[Tuple[int, int]], stats_ptr: int,
                          world: int, row_len: int) -> int:
        """qeh_fused_items_begin: plan from the gathered stats rows + phase A queued; returns the handle.
        Raises QehError(QEH_E_UNSUPPORTED) for shapes outside the items form."""
        cp = self._cols(probe_cols)
        ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
        e = keep = None
        if predicate is not None:
            e, keep = predicate.to_c()
        h = C.c_void_p()
        abi.check(self.lib.qeh_fused_items_begin(self.h, cp, len(probe_cols), probe_key_idx,
                                                 C.byref(e) if e is not None else None, ca, len(aggs), stats_ptr, world,
                                                 row_len, C.byref(h)))
        return h.value

    @staticmethod
    def fused_items_shape(max_rows: int, world: int) -> Tuple[int, int]:
        """(n_blocks, span) of the items form's build for the largest rank's row count: one workgroup per
        ~8 K rows, at most 512 spans over all ranks (phase B's bound), spans of ceil(rows / blocks) + 640
        u32 (multiples of 4)."""
        nb = max(1, min(512 // max(world, 1), -(-max_rows // 8192)))
        span = (-(-max_rows // nb) + 4 * 160 + 3) // 4 * 4
        return nb, span

    def fused_items_build(self, handle: int, build_key: DeviceColumn, group_key: DeviceColumn, n_blocks: int,
                          span: int, items_ptr: int, offs_ptr: int) -> None:
        """qeh_fused_items_build: this rank's build rows grouped by slice in n_blocks spans
        (items[n_blocks * span]; offs[n_blocks * 322]: run starts, then run rows, per span)."""
        abi.check(self.lib.qeh_fused_items_build(self.h, handle, C.byref(build_key.c), C.byref(group_key.c), n_blocks,
                                                 span, items_ptr, offs_ptr))

    def fused_items_finish(self, handle: int, items_ptr: int, span: int, offs_ptr: int, n_regions: int,
                           n_groups: int, lanes_ptr: int) -> None:
        """qeh_fused_items_finish: phase B over the gathered spans (n_regions) + the lanes (status last)."""
        abi.check(self.lib.qeh_fused_items_finish(self.h, handle, items_ptr, span, offs_ptr, n_regions, n_groups,
                                                  lanes_ptr))

    def fused_items_check(self, probe_cols: Sequence[DeviceColumn], probe_key_idx: int,
                          predicate: Optional[PhysicalExpr], aggs: Sequence[Tuple[int, int]]) -> bool:
        """qeh_fused_items_check: whether this rank's probe shard fits the items form (nothing queued)."""
        cp = self._cols(probe_cols)
        ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
        e = keep = None
        if predicate is not None:
            e, keep = predicate.to_c()
        s = self.lib.qeh_fused_items_check(self.h, cp, len(probe_cols), probe_key_idx,
                                           C.byref(e) if e is not None else None, ca, len(aggs))
        if s == abi.QEH_E_UNSUPPORTED:
            return False
        abi.check(s)
        return True

    def fused_items_abort(self, handle: int) -> None:
        abi.check(self.lib.qeh_fused_items_abort(self.h, handle))

    def shuffle_items_begin(self, probe_cols: Sequence[DeviceColumn], probe_key_idx: int,
                            predicate: Optional[PhysicalExpr], aggs: Sequence[Tuple[int, int]], stats_ptr: int,
                            world: int, rank: int, row_len: int) -> int:
        """qeh_shuffle_items_begin: the shuffle join's items form -- plan from the gathered stats rows and
        phase A over this rank's fact shard in the per-destination layout, queued; returns the handle."""
        cp = self._cols(probe_cols)
        ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
        e = keep = None
        if predicate is not None:
            e, keep = predicate.to_c()
        h = C.c_void_p()
        abi.check(self.lib.qeh_shuffle_items_begin(self.h, cp, len(probe_cols), probe_key_idx,
                                                   C.byref(e) if e is not None else None, ca, len(aggs), stats_ptr,
                                                   world, rank, row_len, C.byref(h)))
        return h.value

    def shuffle_items_pack(self, handle: int, world: int):
        """qeh_shuffle_items_pack: (ok, keys_ptr, vals_ptr, counts_ptr, blockcap, block_regions, totals[world])
        -- each destination's packed block (library-owned until shuffle_items_finish)."""
        kp, vp, cp = C.c_void_p(), C.c_void_p(), C.c_void_p()
        bc, br, ok = C.c_uint64(), C.c_int64(), C.c_int()
        tot = (C.c_int64 * world)()
        abi.check(self.lib.qeh_shuffle_items_pack(self.h, handle, C.byref(kp), C.byref(vp), C.byref(cp), C.byref(bc),
                                                  C.byref(br), tot, C.byref(ok)))
        return (bool(ok.value), kp.value or 0, vp.value or 0, cp.value or 0, bc.value, br.value,
                np.array(tot[:], np.int64))

    def shuffle_items_finish(self, handle: int, keys_ptr: int, vals_ptr: int, counts_ptr: int, src_offsets,
                             items_ptr: int, span: int, offs_ptr: int, n_regions: int, n_groups: int,
                             lanes_ptr: int) -> None:
        """qeh_shuffle_items_finish: phase B over the received blocks (source q's items from
        src_offsets[q]) with the gathered dimension spans, then the lanes (status last)."""
        so = (C.c_int64 * len(src_offsets))(*[int(x) for x in src_offsets])
        abi.check(self.lib.qeh_shuffle_items_finish(self.h, handle, keys_ptr, vals_ptr or None, counts_ptr, so,
                                                    items_ptr, span, offs_ptr, n_regions, n_groups, lanes_ptr))

    def join_filter_aggregate_prelaunch_stats(self, probe_cols: Sequence[DeviceColumn], probe_key_idx: int,
                                              predicate: Optional[PhysicalExpr], aggs: Sequence[Tuple[int, int]],
                                              stats_ptr: int, world: int, row_len: int) -> None:
        """qeh_join_filter_aggregate_prelaunch_stats: phase A planned on the device from the gathered
        qeh_broadcast_stats rows (no host wait); the adopting call reads the plan back."""
        cp = self._cols(probe_cols)
        ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
        e = keep = None
        if predicate is not None:
            e, keep = predicate.to_c()
        abi.check(self.lib.qeh_join_filter_aggregate_prelaunch_stats(self.h, cp, len(probe_cols), probe_key_idx,
                                                                     C.byref(e) if e is not None else None, ca,
                                                                     len(aggs), stats_ptr, world, row_len))

    def join_filter_aggregate_prelaunch(self, probe_cols: Sequence[DeviceColumn], probe_key_idx: int,
                                        predicate: Optional[PhysicalExpr], aggs: Sequence[Tuple[int, int]],
                                        build_key_range: Sequence[int], group_key_range: Sequence[int]) -> None:
        """qeh_join_filter_aggregate_prelaunch: start phase A from the build side's [min, max, count]
        ranges; the next join_filter_aggregate on the same probe columns adopts or discards it."""
        cp = self._cols(probe_cols)
        ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
        e = keep = None
        if predicate is not None:
            e, keep = predicate.to_c()
        br = (C.c_int64 * 3)(*[int(q) for q in build_key_range])
        gr = (C.c_int64 * 3)(*[int(q) for q in group_key_range])
        abi.check(self.lib.qeh_join_filter_aggregate_prelaunch(self.h, cp, len(probe_cols), probe_key_idx,
                                                               C.byref(e) if e is not None else None, ca, len(aggs),
                                                               br, gr))

    def sort_indices(self, keys: Sequence[DeviceColumn], ascending: Sequence[bool]) -> DeviceColumn:
        ck = self._cols(keys)
        asc = (C.c_int8 * max(len(keys), 1))(*[1 if a else 0 for a in ascending])
        out = abi.QehColumn()
        abi.check(self.lib.qeh_sort_indices(self.h, ck, len(keys), asc, C.byref(out)))
        return self._wrap(out)

    def sort_indices_nulls(self, keys: Sequence[DeviceColumn], ascending: Sequence[bool],
                           nulls_first: Sequence[bool]) -> DeviceColumn:
        ck = self._cols(keys)
        asc = (C.c_int8 * max(len(keys), 1))(*[1 if a else 0 for a in ascending])
        nf = (C.c_int8 * max(len(keys), 1))(*[1 if a else 0 for a in nulls_first])
        out = abi.QehColumn()
        abi.check(self.lib.qeh_sort_indices_nulls(self.h, ck, len(keys), asc, nf, C.byref(out)))
        return self._wrap(out)

    def concat(self, parts: Sequence[DeviceColumn]) -> DeviceColumn:
        out = abi.QehColumn()
        abi.check(self.lib.qeh_concat(self.h, self._cols(parts), len(parts), C.byref(out)))
        return self._wrap(out)

    def merge_sorted(self, parts: Sequence[Sequence[DeviceColumn]], key_idx: Sequence[int],
                     ascending: Sequence[bool], nulls_first: Sequence[bool]) -> Tuple[List[DeviceColumn], int]:
        """qeh_merge_sorted: parts = one column list per partition (same schema)."""
        ncols = len(parts[0]) if parts else 0
        flat = [c for p in parts for c in p]
        cp = self._cols(flat)
        ki = (C.c_int32 * max(len(key_idx), 1))(*key_idx)
        asc = (C.c_int8 * max(len(key_idx), 1))(*[1 if a else 0 for a in ascending])
        nf = (C.c_int8 * max(len(key_idx), 1))(*[1 if a else 0 for a in nulls_first])
        out = (abi.QehColumn * max(ncols, 1))()
        rows = C.c_int64()
        abi.check(self.lib.qeh_merge_sorted(self.h, cp, len(parts), ncols, ki, asc, nf, len(key_idx), out,
                                            C.byref(rows)))
        return [self._wrap(out[i]) for i in range(ncols)], rows.value

    def encode_pg_datarows(self, cols: Sequence[DeviceColumn]) -> DeviceColumn:
        """qeh_encode_pg_datarows: Utf8 column, string i = row i's DataRow message."""
        out = abi.QehColumn()
        abi.check(self.lib.qeh_encode_pg_datarows(self.h, self._cols(cols), len(cols), C.byref(out)))
        return self._wrap(out)

    def encode_arrow_ipc(self, cols: Sequence[DeviceColumn], names: Sequence[str]) -> np.ndarray:
        """qeh_encode_arrow_ipc: the batch as an Arrow IPC stream.  Returns a uint8 numpy view of
        the library's pinned host buffer (no copy; freed when the array is collected).
        `bytes(result)` or `pyarrow.py_buffer(result)` for consumers that need those."""
        import weakref
        nm = (C.c_char_p * max(len(names), 1))(*[n.encode() for n in names])
        p, size = C.c_void_p(), C.c_int64()
        abi.check(self.lib.qeh_encode_arrow_ipc(self.h, self._cols(cols), nm, len(cols), C.byref(p), C.byref(size)))
        holder = (C.c_uint8 * max(size.value, 1)).from_address(p.value)
        weakref.finalize(holder, self.lib.qeh_host_free, C.c_void_p(p.value))
        return np.frombuffer(holder, np.uint8, count=size.value)

    def decode_arrow_ipc(self, data: bytes, max_cols: int = 256) -> Tuple[List[str], List[DeviceColumn], int]:
        """qeh_decode_arrow_ipc: (names, device columns, rows) of the stream's first batch."""
        out = (abi.QehColumn * max_cols)()
        nc, rows, names = C.c_int(), C.c_int64(), C.c_void_p()
        buf = np.frombuffer(data, np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data, np.uint8)
        ptr = C.c_void_p(buf.ctypes.data if len(buf) else None)
        abi.check(self.lib.qeh_decode_arrow_ipc(self.h, ptr, len(buf), out, max_cols, C.byref(nc), C.byref(names),
                                                C.byref(rows)))
        parts: List[str] = []
        try:
            p = names.value
            for _ in range(nc.value):  # NUL-separated, one per column
                s = C.string_at(p)
                parts.append(s.decode())
                p += len(s) + 1
        finally:
            self.lib.qeh_host_free(names)
        return parts, [self._wrap(out[i]) for i in range(nc.value)], rows.value

    def partition_hash_move(self, keys: Sequence[DeviceColumn], n_parts: int, cols: Sequence[DeviceColumn]):
        """qeh_partition_hash_move: (counts, cols in partition-major order)."""
        counts = (C.c_int64 * n_parts)()
        out = (abi.QehColumn * max(len(cols), 1))()
        abi.check(self.lib.qeh_partition_hash_move(self.h, self._cols(keys), len(keys), n_parts, self._cols(cols),
                                                   len(cols), counts, out))
        return np.array(counts[:], np.int64), [self._wrap(out[i]) for i in range(len(cols))]

    def partition_hash_unmove(self, key: DeviceColumn, n_parts: int, moved: Sequence[DeviceColumn]) -> List[DeviceColumn]:
        """qeh_partition_hash_unmove: columns in partition-major order (as partition_hash_move over `key`
        left them) back into the key's input order."""
        out = (abi.QehColumn * max(len(moved), 1))()
        abi.check(self.lib.qeh_partition_hash_unmove(self.h, C.byref(key.c), n_parts, self._cols(moved), len(moved), out))
        return [self._wrap(out[i]) for i in range(len(moved))]

    def filter_partition_hash_move(self, cols: Sequence[DeviceColumn], predicate: PhysicalExpr, key_idx: int,
                                   n_parts: int, move_idx: Sequence[int]):
        """qeh_filter_partition_hash_move: (counts, cols[move_idx] of the qualifying rows in
        partition-major order).  Raises QehError(QEH_E_UNSUPPORTED) for shapes it does not take."""
        e, keep = predicate.to_c()
        counts = (C.c_int64 * n_parts)()
        mi = (C.c_int32 * len(move_idx))(*move_idx)
        out = (abi.QehColumn * len(move_idx))()
        abi.check(self.lib.qeh_filter_partition_hash_move(self.h, self._cols(cols), len(cols), C.byref(e), key_idx,
                                                          n_parts, mi, len(move_idx), counts, out))
        return np.array(counts[:], np.int64), [self._wrap(out[i]) for i in range(len(move_idx))]

    def slice(self, col: DeviceColumn, offset: int, length: int) -> DeviceColumn:
        """Zero-copy view of rows [offset, offset + length) (RecordBatch::slice); keeps `col` alive."""
        if offset < 0 or length < 0 or offset + length > len(col):
            raise IndexError("slice outside the column")
        c = abi.QehColumn()
        C.pointer(c)[0] = col.c
        c.owned = 0
        c.offset = col.c.offset + offset
        c.length = length
        c.null_count = -1 if col.c.validity else 0
        d = DeviceColumn(self, c)
        d.parent = col
        return d

    def take(self, col: DeviceColumn, indices: DeviceColumn) -> DeviceColumn:
        out = abi.QehColumn()
        abi.check(self.lib.qeh_take(self.h, C.byref(col.c), C.byref(indices.c), C.byref(out)))
        return self._wrap(out)

    def row_number(self, part: Sequence[DeviceColumn], order: Sequence[DeviceColumn],
                   ascending: Sequence[bool]) -> DeviceColumn:
        cp, co = self._cols(part), self._cols(order)
        asc = (C.c_int8 * max(len(order), 1))(*[1 if a else 0 for a in ascending])
        out = abi.QehColumn()
        abi.check(self.lib.qeh_row_number(self.h, cp, len(part), co, len(order), asc, C.byref(out)))
        return self._wrap(out)

    def window(self, func: int, part: Sequence[DeviceColumn], order: Sequence[DeviceColumn],
               ascending: Sequence[bool], arg: Optional[DeviceColumn] = None, param: int = 0,
               default=None) -> DeviceColumn:
        """``WindowFunctionType`` ``func`` (qe_hip.plan.WindowFunctionType) OVER (PARTITION BY
        part ORDER BY order): RANK / DENSE_RANK / NTILE(param) -> Int64; LAG / LEAD(arg, param)
        / FIRST_VALUE / LAST_VALUE(arg) -> arg's type, NULL outside the partition unless
        ``default`` is given (qeh_window)."""
        cp, co = self._cols(part), self._cols(order)
        asc = (C.c_int8 * max(len(order), 1))(*[1 if a else 0 for a in ascending])
        d = None
        if default is not None:
            dt = {abi.DT_INT32: np.int32, abi.DT_INT64: np.int64, abi.DT_FLOAT32: np.float32,
                  abi.DT_FLOAT64: np.float64}[arg.c.dtype]
            bits = np.zeros(1, np.int64)
            if np.dtype(dt).itemsize == 8:
                bits.view(dt)[0] = default
            else:
                bits[0] = int(np.array([default], dt).view(np.uint32)[0])
            d = C.byref(C.c_int64(int(bits[0])))
        out = abi.QehColumn()
        abi.check(self.lib.qeh_window(self.h, int(func), cp, len(part), co, len(order), asc,
                                      C.byref(arg.c) if arg is not None else None, int(param), d,
                                      C.byref(out)))
        return self._wrap(out)

    def hash_partition(self, key: DeviceColumn, n_parts: int):
        counts = (C.c_int64 * n_parts)()
        out = abi.QehColumn()
        abi.check(self.lib.qeh_hash_partition(self.h, C.byref(key.c), n_parts, counts, C.byref(out)))
        return np.array(counts[:], dtype=np.int64), self._wrap(out)

    def range_partition(self, key: DeviceColumn, splitters, ascending: bool = True):
        """Partition ids by order-key ranges (qeh_range_partition); splitters
        are ascending order keys (see ``order_keys``)."""
        sp = np.ascontiguousarray(np.asarray(splitters, dtype=np.int64))
        n_parts = len(sp) + 1
        counts = (C.c_int64 * n_parts)()
        out = abi.QehColumn()
        abi.check(self.lib.qeh_range_partition(self.h, C.byref(key.c), 1 if ascending else 0,
                                               sp.ctypes.data_as(C.POINTER(C.c_int64)), len(sp), counts,
                                               C.byref(out)))
        return np.array(counts[:], dtype=np.int64), self._wrap(out)

    def scatter(self, col: DeviceColumn, perm: DeviceColumn) -> DeviceColumn:
        """out[perm[i]] = col[i] (qeh_scatter)."""
        out = abi.QehColumn()
        abi.check(self.lib.qeh_scatter(self.h, C.byref(col.c), C.byref(perm.c), C.byref(out)))
        return self._wrap(out)


def order_keys(values: np.ndarray) -> np.ndarray:
    """Host twin of the device order key used by qeh_range_partition: ints as
    Int64, floats widened to Float64 and mapped to IEEE totalOrder."""
    v = np.asarray(values)
    if v.dtype.kind == "f":
        b = v.astype(np.float64).view(np.int64)
        return b ^ ((b >> 63).astype(np.uint64) >> np.uint64(1)).astype(np.int64)
    return v.astype(np.int64)


def agg(func: int, column: int) -> Tuple[int, int]:
    return (func, column)
