"""The drop-in boundary: libqeh.so loads on a CPU-only host and exports every
entry point include/qeh.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

import qe_hip
from qe_hip import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "qeh.h")).read() + open(os.path.join(ROOT, "include", "qeh_plan.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char \*|void \*)\s*(qeh_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_operator_surface():
    names = declared_functions()
    for required in ["qeh_init", "qeh_filter", "qeh_eval", "qeh_hash_aggregate", "qeh_filter_aggregate",
                     "qeh_hash_join_inner", "qeh_join_filter_aggregate", "qeh_sort_indices", "qeh_take",
                     "qeh_row_number", "qeh_window", "qeh_hash_partition", "qeh_last_error", "qeh_execute_plan"]:
        assert required in names


def test_library_exports_every_declared_symbol():
    lib = qe_hip.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
        assert name in abi.SIGNATURES, f"{name} missing from qe_hip/abi.py SIGNATURES"
    out = subprocess.run(["nm", "-D", "--defined-only", abi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\b(qeh_\w+)\b", out))
    assert set(declared_functions()) <= exported


def test_library_is_gfx950_code():
    data = open(abi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # offload bundle target id


def test_abi_version_and_struct_layout():
    lib = qe_hip.load()
    assert lib.qeh_abi_version() == 1
    assert ctypes.sizeof(abi.QehColumn) == 64
    assert ctypes.sizeof(abi.QehExprNode) == 40
    assert ctypes.sizeof(abi.QehAgg) == 8


def test_init_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(qe_hip.QehError) as e:
        qe_hip.Context(0)
    assert e.value.status == abi.QEH_E_HIP


def test_expression_typing_mirrors_reference_errors():
    """qeh_expr_type is host-only: it applies operators.rs typing rules."""
    from qe_hip import BinaryOp, UnaryExpr, UnaryOp, binop, col, lit
    lib = qe_hip.load()

    def ty(expr, dtypes):
        e, keep = expr.to_c()
        d = (ctypes.c_int32 * len(dtypes))(*dtypes)
        out = ctypes.c_int32()
        s = lib.qeh_expr_type(d, len(dtypes), ctypes.byref(e), ctypes.byref(out))
        return s, out.value, lib.qeh_last_error().decode()

    I64, F64, I32, F32, B = abi.DT_INT64, abi.DT_FLOAT64, abi.DT_INT32, abi.DT_FLOAT32, abi.DT_BOOL
    assert ty(binop(col(0), BinaryOp.Greater, lit(25)), [I64])[:2] == (0, B)
    assert ty(binop(col(0), BinaryOp.Greater, lit(25)), [F64])[:2] == (0, B)      # int literal coerced to f64
    assert ty(binop(col(0), BinaryOp.Less, lit(2.5)), [I32])[:2] == (0, B)
    assert ty(binop(col(0), BinaryOp.Add, lit(1)), [I64])[:2] == (0, I64)
    s, _, msg = ty(binop(col(0), BinaryOp.Multiply, lit(1.1)), [I64])            # no arithmetic coercion
    assert s == abi.QEH_E_TYPE and msg == "Unsupported types for multiplication"
    s, _, msg = ty(binop(col(0), BinaryOp.Modulo, lit(2.0)), [F64])
    assert s == abi.QEH_E_TYPE and msg == "Modulo operation requires integer arrays"
    s, _, msg = ty(UnaryExpr(UnaryOp.Not, col(0)), [I64])
    assert s == abi.QEH_E_TYPE and msg == "NOT operator requires boolean array"
    s, _, msg = ty(binop(col(0), BinaryOp.And, col(1)), [B, I64])
    assert s == abi.QEH_E_TYPE and msg == "AND requires boolean arrays"
    s, _, msg = ty(col(3), [I64])
    assert s == abi.QEH_E_INVALID and msg == "Column index 3 out of bounds"
    s, _, msg = ty(binop(col(0), BinaryOp.Equal, col(1)), [I64, B])
    assert s == abi.QEH_E_TYPE and "Invalid comparison operation: Int64 == Boolean" in msg
    assert ty(binop(col(0), BinaryOp.Equal, col(1)), [F32, I64])[:2] == (0, B)    # both cast to f64
