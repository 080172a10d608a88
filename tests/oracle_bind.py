"""ctypes binding of the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from typing import List, Optional, Sequence, Tuple

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
from qe_hip import abi  # noqa: E402  (enum values + expression node struct)

ORACLE_PATH = os.path.join(ROOT, "oracle", "liboracle.so")
NATIVE_PATH = os.path.join(ROOT, "oracle", "_native", "liboracle.so")  # -march=native build (bench.py)

NP_OF = {abi.DT_INT32: np.int32, abi.DT_INT64: np.int64, abi.DT_FLOAT32: np.float32,
         abi.DT_FLOAT64: np.float64, abi.DT_UINT32: np.uint32, abi.DT_BOOL: np.uint8}
DT_OF = {np.dtype(np.int32): abi.DT_INT32, np.dtype(np.int64): abi.DT_INT64,
         np.dtype(np.float32): abi.DT_FLOAT32, np.dtype(np.float64): abi.DT_FLOAT64,
         np.dtype(np.uint32): abi.DT_UINT32, np.dtype(np.bool_): abi.DT_BOOL}


class QoCol(C.Structure):
    _fields_ = [("dtype", C.c_int32), ("_pad", C.c_int32), ("length", C.c_int64),
                ("values", C.c_void_p), ("valid", C.c_void_p)]


class OracleError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"[{abi.STATUS_NAMES.get(status, status)}] {msg}")
        self.status = status
        self.message = msg


_lib = None


def use_native() -> bool:
    """Load the -march=native build (bench.py's CPU baseline) instead of the portable one.
    Must be called before the first oracle call; returns False when it is not built."""
    global ORACLE_PATH
    if _lib is None and os.path.exists(NATIVE_PATH):
        ORACLE_PATH = NATIVE_PATH
        return True
    return ORACLE_PATH == NATIVE_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_PATH):
            raise RuntimeError(f"{ORACLE_PATH} missing: run `make -C oracle`")
        L = C.CDLL(ORACLE_PATH)
        L.qo_last_error.restype = C.c_char_p
        L.qo_generate.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_int64, C.c_int64, C.c_int64,
                                  C.c_int64, C.c_void_p]
        L.qo_generate.restype = None
        _lib = L
    return _lib


def _check(s):
    if s != 0:
        raise OracleError(s, lib().qo_last_error().decode(errors="replace"))


class HostCol:
    """numpy values + optional bool validity, kept alive for the C call."""

    def __init__(self, values: np.ndarray, valid: Optional[np.ndarray] = None):
        v = np.ascontiguousarray(values)
        if v.dtype == np.bool_:
            v = v.astype(np.uint8)
            self.dtype = abi.DT_BOOL
        else:
            self.dtype = DT_OF[v.dtype]
        self.values = v
        self.valid = None if valid is None else np.ascontiguousarray(np.asarray(valid, bool).astype(np.uint8))
        self.c = QoCol(self.dtype, 0, len(v), v.ctypes.data if len(v) else None,
                       self.valid.ctypes.data if self.valid is not None and len(v) else None)
        if self.valid is not None and len(v) == 0:
            self.c.valid = None


def _arr(cols: Sequence[HostCol]):
    return (QoCol * max(len(cols), 1))(*[c.c for c in cols])


def _take(c: QoCol) -> Tuple[np.ndarray, np.ndarray]:
    n = c.length
    npdt = NP_OF[c.dtype]
    if n:
        vals = np.ctypeslib.as_array(C.cast(c.values, C.POINTER(np.ctypeslib.as_ctypes_type(npdt))), (n,)).copy()
        valid = np.ctypeslib.as_array(C.cast(c.valid, C.POINTER(C.c_uint8)), (n,)).astype(bool).copy()
    else:
        vals, valid = np.zeros(0, npdt), np.zeros(0, bool)
    if c.dtype == abi.DT_BOOL:
        vals = vals.astype(bool)
    lib().qo_col_free(C.byref(c))
    return vals, valid


def generate(kind, seed, col_id, n, modulus=0, lo=0, row0=0) -> np.ndarray:
    out = np.empty(n, np.float64 if kind == abi.GEN_UNIT_F64 else np.int64)
    lib().qo_generate(kind, seed, col_id, row0, n, modulus, lo, out.ctypes.data)
    return out


def eval_expr(cols: Sequence[HostCol], expr, n_rows: int):
    nodes = expr.postfix()
    na = (abi.QehExprNode * len(nodes))(*nodes)
    out = QoCol()
    _check(lib().qo_eval(_arr(cols), len(cols), C.c_int64(n_rows), na, len(nodes), C.byref(out)))
    dt = out.dtype
    return _take(out), dt


def filter(cols: Sequence[HostCol], pred, out_idx: Optional[Sequence[int]] = None):
    out_idx = list(range(len(cols))) if out_idx is None else list(out_idx)
    nodes = pred.postfix()
    na = (abi.QehExprNode * len(nodes))(*nodes)
    oi = (C.c_int32 * max(len(out_idx), 1))(*out_idx)
    out = (QoCol * max(len(out_idx), 1))()
    rows = C.c_int64()
    _check(lib().qo_filter(_arr(cols), len(cols), na, len(nodes), oi, len(out_idx), out, C.byref(rows)))
    dts = [out[i].dtype for i in range(len(out_idx))]
    return [_take(out[i]) for i in range(len(out_idx))], rows.value, dts


def hash_aggregate(keys: Sequence[HostCol], inputs: Sequence[HostCol], aggs, input_batches=1):
    ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
    ok = (QoCol * max(len(keys), 1))()
    oa = (QoCol * max(len(aggs), 1))()
    g = C.c_int64()
    _check(lib().qo_hash_aggregate(_arr(keys), len(keys), _arr(inputs), len(inputs), ca, len(aggs),
                                   C.c_int64(input_batches), ok, oa, C.byref(g)))
    if g.value == 0 and not oa[0].values:
        return [], [], 0, []
    dts = [oa[i].dtype for i in range(len(aggs))]
    return ([_take(ok[i]) for i in range(len(keys))], [_take(oa[i]) for i in range(len(aggs))], g.value, dts)


def hash_join_inner(probe_key: HostCol, probe_cols, build_key: HostCol, build_cols):
    op = (QoCol * max(len(probe_cols), 1))()
    ob = (QoCol * max(len(build_cols), 1))()
    rows = C.c_int64()
    _check(lib().qo_hash_join_inner(C.byref(probe_key.c), _arr(probe_cols), len(probe_cols), C.byref(build_key.c),
                                    _arr(build_cols), len(build_cols), op, ob, C.byref(rows)))
    return ([_take(op[i]) for i in range(len(probe_cols))], [_take(ob[i]) for i in range(len(build_cols))], rows.value)


def hash_join_outer(join_type: int, left_key: HostCol, left_cols, right_key: HostCol, right_cols):
    ol = (QoCol * max(len(left_cols), 1))()
    orr = (QoCol * max(len(right_cols), 1))()
    rows = C.c_int64()
    _check(lib().qo_hash_join_outer(int(join_type), C.byref(left_key.c), _arr(left_cols), len(left_cols),
                                    C.byref(right_key.c), _arr(right_cols), len(right_cols), ol, orr, C.byref(rows)))
    return ([_take(ol[i]) for i in range(len(left_cols))], [_take(orr[i]) for i in range(len(right_cols))], rows.value)


def join_filter_aggregate(probe_cols, probe_key_idx, pred, build_key: HostCol, build_group_keys, aggs):
    ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
    ok = (QoCol * max(len(build_group_keys), 1))()
    oa = (QoCol * max(len(aggs), 1))()
    g = C.c_int64()
    if pred is not None:
        nodes = pred.postfix()
        na = (abi.QehExprNode * len(nodes))(*nodes)
        nn = len(nodes)
    else:
        na, nn = None, 0
    _check(lib().qo_join_filter_aggregate(_arr(probe_cols), len(probe_cols), probe_key_idx, na, nn,
                                          C.byref(build_key.c), _arr(build_group_keys), len(build_group_keys),
                                          ca, len(aggs), ok, oa, C.byref(g)))
    return ([_take(ok[i]) for i in range(len(build_group_keys))], [_take(oa[i]) for i in range(len(aggs))],
            g.value)


def join_filter_aggregate_mt(probe_cols, probe_key_idx, pred, build_key: HostCol, build_group_keys, aggs,
                             threads: int):
    """qo_join_filter_aggregate_mt: the all-cores (OpenMP) CPU baseline of the metric query."""
    ca = (abi.QehAgg * max(len(aggs), 1))(*[abi.QehAgg(f, c) for f, c in aggs])
    ok = (QoCol * max(len(build_group_keys), 1))()
    oa = (QoCol * max(len(aggs), 1))()
    g = C.c_int64()
    if pred is not None:
        nodes = pred.postfix()
        na = (abi.QehExprNode * len(nodes))(*nodes)
        nn = len(nodes)
    else:
        na, nn = None, 0
    _check(lib().qo_join_filter_aggregate_mt(_arr(probe_cols), len(probe_cols), probe_key_idx, na, nn,
                                             C.byref(build_key.c), _arr(build_group_keys), len(build_group_keys),
                                             ca, len(aggs), int(threads), ok, oa, C.byref(g)))
    return ([_take(ok[i]) for i in range(len(build_group_keys))], [_take(oa[i]) for i in range(len(aggs))],
            g.value)


def _cartesian(fn, left, right):
    out = (QoCol * max(len(left) + len(right), 1))()
    rows = C.c_int64()
    _check(fn(_arr(left), len(left), _arr(right), len(right), out, C.byref(rows)))
    if rows.value < 0:
        return None, -1  # an empty side: no batch (executor.rs:350-352)
    return [_take(out[i]) for i in range(len(left) + len(right))], rows.value


def join_batches(left: Sequence[HostCol], right: Sequence[HostCol]):
    """qo_join_batches — literal join_batches (executor.rs:500-540): (columns, rows), left row-major."""
    return _cartesian(lib().qo_join_batches, left, right)


def cross_join(left: Sequence[HostCol], right: Sequence[HostCol]):
    """qo_cross_join — literal execute_cross_join (executor.rs:437-498): right row-major."""
    return _cartesian(lib().qo_cross_join, left, right)


def join_on(join_type: int, left: Sequence[HostCol], right: Sequence[HostCol], on):
    """qo_join_on: join on an arbitrary boolean expression over left ++ right columns."""
    nodes = on.postfix()
    na = (abi.QehExprNode * len(nodes))(*nodes)
    ol = (QoCol * max(len(left), 1))()
    orr = (QoCol * max(len(right), 1))()
    rows = C.c_int64()
    _check(lib().qo_join_on(int(join_type), _arr(left), len(left), _arr(right), len(right), na, len(nodes), ol, orr,
                            C.byref(rows)))
    return [_take(ol[i]) for i in range(len(left))], [_take(orr[i]) for i in range(len(right))], rows.value


def partition_hash(keys: Sequence[HostCol], n_parts: int):
    """(counts, partition-major row order) of Partitioner::partition_by_hash (qo_partition_hash)."""
    n = len(keys[0].values)
    counts = np.zeros(n_parts, np.int64)
    perm = np.empty(max(n, 1), np.uint32)
    _check(lib().qo_partition_hash(_arr(keys), len(keys), n_parts, counts.ctypes.data_as(C.c_void_p),
                                   perm.ctypes.data_as(C.c_void_p)))
    return counts, perm[:n]


def sort_indices_nulls(keys: Sequence[HostCol], ascending: Sequence[bool], nulls_first: Sequence[bool]) -> np.ndarray:
    n = len(keys[0].values) if keys else 0
    out = np.empty(max(n, 1), np.uint32)
    asc = (C.c_int8 * max(len(keys), 1))(*[1 if a else 0 for a in ascending])
    nf = (C.c_int8 * max(len(keys), 1))(*[1 if a else 0 for a in nulls_first])
    _check(lib().qo_sort_indices_nulls(_arr(keys), len(keys), asc, nf, C.c_int64(n), out.ctypes.data_as(C.c_void_p)))
    return out[:n]


def sort_indices(keys: Sequence[HostCol], ascending: Sequence[bool]) -> np.ndarray:
    n = len(keys[0].values) if keys else 0
    out = np.empty(max(n, 1), np.uint32)
    asc = (C.c_int8 * max(len(keys), 1))(*[1 if a else 0 for a in ascending])
    _check(lib().qo_sort_indices(_arr(keys), len(keys), asc, C.c_int64(n), out.ctypes.data_as(C.c_void_p)))
    return out[:n]


def window(func: int, part: Sequence[HostCol], order: Sequence[HostCol], ascending: Sequence[bool],
           arg: Optional[HostCol] = None, param: int = 0, default=None, n: Optional[int] = None):
    """qo_window: (values, valid).  Ranking functions -> int64 values, all valid; value functions
    -> values in the argument's dtype, valid = bool array."""
    if n is None:
        n = len((list(part) + list(order) + ([arg] if arg is not None else []))[0].values)
    bits = np.zeros(max(n, 1), np.int64)
    valid = np.zeros(max(n, 1), np.uint8)
    asc = (C.c_int8 * max(len(order), 1))(*[1 if a else 0 for a in ascending])
    d = None
    if default is not None:
        dv = np.zeros(1, np.int64)
        if arg.values.dtype.itemsize == 8:
            dv.view(arg.values.dtype)[0] = default
        else:
            dv.view(np.uint32)[0] = np.array([default], arg.values.dtype).view(np.uint32)[0]
        d = dv.ctypes.data_as(C.c_void_p)
    argp = C.byref(arg.c) if arg is not None else None
    _check(lib().qo_window(func, _arr(part), len(part), _arr(order), len(order), asc, argp, C.c_int64(param), d,
                           C.c_int64(n), bits.ctypes.data_as(C.c_void_p), valid.ctypes.data_as(C.c_void_p)))
    bits, valid = bits[:n], valid[:n].astype(bool)
    if func < 4 or arg is None:
        return bits, valid
    dt = arg.values.dtype
    vals = bits.view(dt) if dt.itemsize == 8 else bits.astype(np.uint32).view(dt)
    return vals, valid


def row_number(part: Sequence[HostCol], order: Sequence[HostCol], ascending: Sequence[bool]) -> np.ndarray:
    n = len((part or order)[0].values)
    out = np.empty(max(n, 1), np.int64)
    asc = (C.c_int8 * max(len(order), 1))(*[1 if a else 0 for a in ascending])
    _check(lib().qo_row_number(_arr(part), len(part), _arr(order), len(order), asc, C.c_int64(n),
                               out.ctypes.data_as(C.c_void_p)))
    return out[:n]
