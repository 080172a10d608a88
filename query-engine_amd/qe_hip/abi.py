"""ctypes declarations of the qeh C ABI (include/qeh.h).

This is the Python-side binding a caller uses (tests, bench, the distributed
layer).  It loads the in-tree ``libqeh.so`` and fails loudly when it is missing:
there is no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(HERE), "libqeh.so")

# ---- enums (include/qeh.h) -------------------------------------------------
QEH_OK, QEH_E_INVALID, QEH_E_OVERFLOW, QEH_E_DIV0, QEH_E_OOM = 0, 1, 2, 3, 4
QEH_E_UNSUPPORTED, QEH_E_HIP, QEH_E_TYPE, QEH_E_INTERNAL = 5, 6, 7, 8
STATUS_NAMES = {0: "OK", 1: "INVALID", 2: "OVERFLOW", 3: "DIV0", 4: "OOM", 5: "UNSUPPORTED",
                6: "HIP", 7: "TYPE", 8: "INTERNAL"}

DT_NULL, DT_BOOL, DT_INT32, DT_INT64, DT_FLOAT32, DT_FLOAT64, DT_UTF8, DT_UINT32 = range(8)

EX_COLUMN, EX_LITERAL, EX_BINARY, EX_UNARY = 1, 2, 3, 4
(OP_ADD, OP_SUB, OP_MUL, OP_DIV, OP_MOD, OP_EQ, OP_NEQ, OP_LT, OP_LTE, OP_GT, OP_GTE,
 OP_AND, OP_OR) = range(13)
UOP_NOT, UOP_MINUS = 0, 1
AGG_COUNT, AGG_SUM, AGG_AVG, AGG_MIN, AGG_MAX = range(5)
GEN_UNIFORM_MOD, GEN_UNIT_F64, GEN_PERMUTATION, GEN_SPARSE_KEY = 0, 1, 2, 3


class QehColumn(C.Structure):
    _fields_ = [("dtype", C.c_int32), ("owned", C.c_int32), ("length", C.c_int64),
                ("offset", C.c_int64), ("null_count", C.c_int64), ("values", C.c_void_p),
                ("validity", C.c_void_p), ("offsets", C.c_void_p), ("values_bytes", C.c_int64)]


class QehExprNode(C.Structure):
    _fields_ = [("kind", C.c_int32), ("op", C.c_int32), ("index", C.c_int32),
                ("lit_dtype", C.c_int32), ("lit_is_null", C.c_int32), ("_pad", C.c_int32),
                ("lit_i64", C.c_int64), ("lit_f64", C.c_double)]


class QehExpr(C.Structure):
    _fields_ = [("nodes", C.POINTER(QehExprNode)), ("n_nodes", C.c_int32)]


class QehAgg(C.Structure):
    _fields_ = [("func", C.c_int32), ("column", C.c_int32)]


# every exported symbol and its signature (also checked by the CPU tests)
P, I, I64, U64, SZ = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_size_t
COLP, EXPRP, AGGP = C.POINTER(QehColumn), C.POINTER(QehExpr), C.POINTER(QehAgg)
SIGNATURES = {
    "qeh_abi_version": (I, []),
    "qeh_last_error": (C.c_char_p, []),
    "qeh_init": (I, [I, C.POINTER(P)]),
    "qeh_shutdown": (I, [P]),
    "qeh_lds_atomic_rank_ok": (I, [P]),
    "qeh_set_stream": (I, [P, P]),
    "qeh_get_stream": (P, [P]),
    "qeh_synchronize": (I, [P]),
    "qeh_device_alloc": (I, [P, SZ, C.POINTER(P)]),
    "qeh_device_free": (I, [P, P]),
    "qeh_pool_trim": (I, [P]),
    "qeh_memcpy_h2d": (I, [P, P, P, SZ]),
    "qeh_memcpy_d2h": (I, [P, P, P, SZ]),
    "qeh_memcpy_d2d": (I, [P, P, P, SZ]),
    "qeh_memset": (I, [P, P, I, SZ]),
    "qeh_column_release": (I, [P, COLP]),
    "qeh_timing_enable": (I, [P, I]),
    "qeh_timing_reset": (I, [P]),
    "qeh_kernel_time": (I, [P, C.c_char_p, C.POINTER(C.c_double), C.POINTER(I64)]),
    "qeh_generate": (I, [P, I, U64, U64, I64, I64, I64, I64, P]),
    "qeh_filter": (I, [P, COLP, I, EXPRP, C.POINTER(C.c_int32), I, COLP, C.POINTER(I64)]),
    "qeh_filter_limit": (I, [P, COLP, I, EXPRP, C.POINTER(C.c_int32), I, I64, COLP, C.POINTER(I64)]),
    "qeh_eval": (I, [P, COLP, I, EXPRP, I64, COLP]),
    "qeh_expr_type": (I, [C.POINTER(C.c_int32), I, EXPRP, C.POINTER(C.c_int32)]),
    "qeh_hash_aggregate": (I, [P, COLP, I, COLP, I, AGGP, I, I64, COLP, COLP, C.POINTER(I64)]),
    "qeh_filter_aggregate": (I, [P, COLP, I, EXPRP, C.POINTER(C.c_int32), I, AGGP, I, I64, COLP, COLP,
                                 C.POINTER(I64)]),
    "qeh_hash_join_inner": (I, [P, COLP, COLP, I, COLP, COLP, I, COLP, COLP, C.POINTER(I64)]),
    "qeh_hash_join_outer": (I, [P, I, COLP, COLP, I, COLP, COLP, I, COLP, COLP, C.POINTER(I64)]),
    "qeh_join_filter_aggregate": (I, [P, COLP, I, I, EXPRP, COLP, COLP, I, AGGP, I, COLP, COLP,
                                      C.POINTER(I64)]),
    "qeh_join_filter_aggregate_prelaunch": (I, [P, COLP, I, I, EXPRP, AGGP, I, C.POINTER(I64), C.POINTER(I64)]),
    "qeh_direct_group_table_insert": (I, [P, COLP, COLP, I64, U64, I64, P]),
    "qeh_direct_group_table_insert_async": (I, [P, COLP, COLP, I64, U64, I64, P]),
    "qeh_u16_count_nonzero": (I, [P, P, U64, C.POINTER(I64)]),
    "qeh_u16_count_nonzero_dev": (I, [P, P, U64, P]),
    "qeh_u16_table_check_dev": (I, [P, P, U64, C.c_uint32, P]),
    "qeh_columns_minmax": (I, [P, COLP, I, C.POINTER(I64)]),
    "qeh_dense_states_f64": (I, [P, COLP, COLP, I, I64, I64, P]),
    "qeh_dense_states_take": (I, [P, P, I, I64, I64, I, I, C.c_int32, C.POINTER(C.c_int32), COLP, COLP, C.POINTER(I64)]),
    "qeh_dense_states_take_status": (I, [P, P, I, I64, I64, I, I, C.c_int32, C.POINTER(C.c_int32), COLP, COLP,
                                         C.POINTER(I64), C.POINTER(C.c_double)]),
    "qeh_join_filter_aggregate_table": (I, [P, COLP, I, I, EXPRP, P, I64, U64, I64, I64, C.c_int32, AGGP, I, COLP, COLP,
                                            C.POINTER(I64)]),
    "qeh_join_filter_aggregate_table_lanes": (I, [P, COLP, I, I, EXPRP, P, I64, U64, I64, AGGP, I, P]),
    "qeh_join_filter_aggregate_table_lanes_async": (I, [P, COLP, I, I, EXPRP, P, I64, U64, I64, AGGP, I, P, P]),
    "qeh_broadcast_stats": (I, [P, COLP, COLP, C.POINTER(I64), I, P]),
    "qeh_fused_items_begin": (I, [P, COLP, I, I, EXPRP, AGGP, I, P, I, I, C.POINTER(P)]),
    "qeh_fused_items_build": (I, [P, P, COLP, COLP, I, U64, P, P]),
    "qeh_fused_items_finish": (I, [P, P, P, U64, P, I, I64, P]),
    "qeh_fused_items_abort": (I, [P, P]),
    "qeh_shuffle_items_begin": (I, [P, COLP, I, I, EXPRP, AGGP, I, P, I, I, I, C.POINTER(P)]),
    "qeh_shuffle_items_pack": (I, [P, P, C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(U64), C.POINTER(I64),
                                   C.POINTER(I64), C.POINTER(I)]),
    "qeh_shuffle_items_finish": (I, [P, P, P, P, P, C.POINTER(I64), P, U64, P, I, I64, P]),
    "qeh_fused_items_check": (I, [P, COLP, I, I, EXPRP, AGGP, I]),
    "qeh_join_filter_aggregate_prelaunch_stats": (I, [P, COLP, I, I, EXPRP, AGGP, I, P, I, I]),
    "qeh_sort_indices": (I, [P, COLP, I, C.POINTER(C.c_int8), COLP]),
    "qeh_sort_indices_nulls": (I, [P, COLP, I, C.POINTER(C.c_int8), C.POINTER(C.c_int8), COLP]),
    "qeh_concat": (I, [P, COLP, I, COLP]),
    "qeh_merge_sorted": (I, [P, COLP, I, I, C.POINTER(C.c_int32), C.POINTER(C.c_int8), C.POINTER(C.c_int8), I, COLP,
                             C.POINTER(I64)]),
    "qeh_encode_pg_datarows": (I, [P, COLP, I, COLP]),
    "qeh_encode_arrow_ipc": (I, [P, COLP, C.POINTER(C.c_char_p), I, C.POINTER(C.c_void_p), C.POINTER(I64)]),
    "qeh_host_free": (None, [C.c_void_p]),
    "qeh_decode_arrow_ipc": (I, [P, C.c_void_p, I64, COLP, I, C.POINTER(I), C.POINTER(C.c_void_p), C.POINTER(I64)]),
    "qeh_partition_hash": (I, [P, COLP, I, I, C.POINTER(I64), COLP]),
    "qeh_partition_range": (I, [P, COLP, C.POINTER(I64), I, C.POINTER(I64), COLP]),
    "qeh_partition_hash_move": (I, [P, COLP, I, I, COLP, I, C.POINTER(I64), COLP]),
    "qeh_partition_hash_unmove": (I, [P, COLP, I, COLP, I, COLP]),
    "qeh_filter_partition_hash_move": (I, [P, COLP, I, EXPRP, I, I, C.POINTER(C.c_int32), I, C.POINTER(I64), COLP]),
    "qeh_take": (I, [P, COLP, COLP, COLP]),
    "qeh_row_number": (I, [P, COLP, I, COLP, I, C.POINTER(C.c_int8), COLP]),
    "qeh_window": (I, [P, I, COLP, I, COLP, I, C.POINTER(C.c_int8), COLP, I64, C.POINTER(I64), COLP]),
    "qeh_hash_partition": (I, [P, COLP, I, C.POINTER(I64), COLP]),
    "qeh_range_partition": (I, [P, COLP, I, C.POINTER(I64), I, C.POINTER(I64), COLP]),
    "qeh_scatter": (I, [P, COLP, COLP, COLP]),
    "qeh_validity_to_bytes": (I, [P, COLP, P]),
    "qeh_bytes_to_validity": (I, [P, P, I64, P]),
    "qeh_execute_plan": (I, [P, P, P, I, P, P, C.POINTER(I64)]),  # include/qeh_plan.h; typed in plan.py
    "qeh_source_cache_evict": (I, [P, C.c_uint64]),
    "qeh_source_cache_stats": (I, [P, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64), C.POINTER(I64)]),
    "qeh_source_cache_budget": (I, [P, I64]),
}

_lib = None


class QehError(RuntimeError):
    """A non-OK qeh status; ``status`` is the enum value, the message the
    library's thread-local error text (which mirrors the reference's)."""

    def __init__(self, status: int, message: str):
        super().__init__(f"[{STATUS_NAMES.get(status, status)}] {message}")
        self.status = status
        self.message = message


def load(path: str | None = None) -> C.CDLL:
    """Load libqeh.so (built in-tree by ``make -C query-engine_amd``)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # QEH_LIB_PATH: an experiment build of the library in place of the in-tree one (A/B runs)
    p = path or os.environ.get("QEH_LIB_PATH") or LIB_PATH
    # One HIP runtime per process: torch's wheel bundles its own libamdhip64
    # (same soname, libamdhip64.so.7).  If libqeh.so loaded /opt/rocm's copy
    # first, a later `import torch` would load a second runtime that finds no
    # device.  Importing torch first makes libqeh bind to the copy already
    # mapped, so torch streams/collectives and qeh kernels share one runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(p):
        raise RuntimeError(f"libqeh.so not found at {p}: build it with `make -C query-engine_amd` "
                           "(there is no CPU fallback)")
    lib = C.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        if (path or os.environ.get("QEH_LIB_PATH")) and not hasattr(lib, name):
            continue  # an older experiment build: calls into what it lacks fail where they are made
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(status: int) -> None:
    if status != QEH_OK:
        raise QehError(status, load().qeh_last_error().decode(errors="replace"))
