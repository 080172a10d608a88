"""Python mirror of the reference's physical expression types.

Mirrors ``PhysicalExpr`` / ``BinaryOp`` / ``UnaryOp`` / ``AggregateExpr``
(crates/query-executor/src/physical_plan.rs:74-157) and ``ScalarValue``
(crates/query-planner/src/logical_plan.rs:147-161) so tests construct plans the
way the reference's converters do (crates/query-pgwire/src/backend.rs:727-756),
then serialises them to the postfix ``qeh_expr`` of include/qeh.h.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional, Union

from . import abi


# ---- ScalarValue ----------------------------------------------------------
@dataclass(frozen=True)
class ScalarValue:
    dtype: int
    value: Optional[Union[int, float, bool, str]]

    @staticmethod
    def Int64(v): return ScalarValue(abi.DT_INT64, v)

    @staticmethod
    def Int32(v): return ScalarValue(abi.DT_INT32, v)

    @staticmethod
    def Float64(v): return ScalarValue(abi.DT_FLOAT64, v)

    @staticmethod
    def Float32(v): return ScalarValue(abi.DT_FLOAT32, v)

    @staticmethod
    def Boolean(v): return ScalarValue(abi.DT_BOOL, v)

    @staticmethod
    def Utf8(v): return ScalarValue(abi.DT_UTF8, v)


ScalarValue.Null = ScalarValue(abi.DT_NULL, None)


# ---- PhysicalExpr ---------------------------------------------------------
class BinaryOp:
    Add, Subtract, Multiply, Divide, Modulo = abi.OP_ADD, abi.OP_SUB, abi.OP_MUL, abi.OP_DIV, abi.OP_MOD
    Equal, NotEqual, Less, LessEqual = abi.OP_EQ, abi.OP_NEQ, abi.OP_LT, abi.OP_LTE
    Greater, GreaterEqual, And, Or = abi.OP_GT, abi.OP_GTE, abi.OP_AND, abi.OP_OR


class UnaryOp:
    Not, Minus = abi.UOP_NOT, abi.UOP_MINUS


class AggregateFunction:
    Count, Sum, Avg, Min, Max = abi.AGG_COUNT, abi.AGG_SUM, abi.AGG_AVG, abi.AGG_MIN, abi.AGG_MAX


class PhysicalExpr:
    def postfix(self) -> List[abi.QehExprNode]:
        out: List[abi.QehExprNode] = []
        self._emit(out)
        return out

    def columns(self) -> List[int]:
        return sorted({n.index for n in self.postfix() if n.kind == abi.EX_COLUMN})

    def to_c(self):
        """(QehExpr, keepalive) for a C call."""
        nodes = self.postfix()
        arr = (abi.QehExprNode * len(nodes))(*nodes)
        e = abi.QehExpr(C.cast(arr, C.POINTER(abi.QehExprNode)), len(nodes))
        # Utf8 literal bytes are referenced by address (index = length, lit_i64 = pointer)
        return e, (arr, [n._utf8 for n in nodes if hasattr(n, "_utf8")])

    # operator sugar so tests read naturally
    def __and__(self, o): return BinaryExpr(self, BinaryOp.And, o)
    def __or__(self, o): return BinaryExpr(self, BinaryOp.Or, o)


@dataclass
class Column(PhysicalExpr):
    name: str
    index: int

    def _emit(self, out):
        out.append(abi.QehExprNode(kind=abi.EX_COLUMN, index=self.index))


@dataclass
class Literal(PhysicalExpr):
    value: ScalarValue

    def _emit(self, out):
        v = self.value
        n = abi.QehExprNode(kind=abi.EX_LITERAL, lit_dtype=v.dtype)
        if v.dtype == abi.DT_NULL or v.value is None:
            n.lit_is_null = 1
        elif v.dtype in (abi.DT_FLOAT32, abi.DT_FLOAT64):
            n.lit_f64 = float(v.value)
        elif v.dtype == abi.DT_UTF8:
            b = v.value.encode() if isinstance(v.value, str) else bytes(v.value)
            buf = C.create_string_buffer(b, max(len(b), 1))
            n.index = len(b)
            n.lit_i64 = C.addressof(buf)
            n._utf8 = buf
        else:
            n.lit_i64 = int(v.value)
        out.append(n)


@dataclass
class BinaryExpr(PhysicalExpr):
    left: PhysicalExpr
    op: int
    right: PhysicalExpr

    def _emit(self, out):
        self.left._emit(out)
        self.right._emit(out)
        out.append(abi.QehExprNode(kind=abi.EX_BINARY, op=self.op))


@dataclass
class UnaryExpr(PhysicalExpr):
    op: int
    expr: PhysicalExpr

    def _emit(self, out):
        self.expr._emit(out)
        out.append(abi.QehExprNode(kind=abi.EX_UNARY, op=self.op))


@dataclass
class AggregateExpr:
    func: int
    expr: PhysicalExpr


def col(index: int, name: str = "") -> Column:
    return Column(name or f"c{index}", index)


def lit(v) -> Literal:
    """Literal typed like the reference planner types SQL literals
    (planner.rs:669-686): ints -> Int64, decimals -> Float64."""
    if v is None:
        return Literal(ScalarValue.Null)
    if isinstance(v, bool):
        return Literal(ScalarValue.Boolean(v))
    if isinstance(v, int):
        return Literal(ScalarValue.Int64(v))
    if isinstance(v, float):
        return Literal(ScalarValue.Float64(v))
    if isinstance(v, (str, bytes)):  # string literals -> Utf8
        return Literal(ScalarValue.Utf8(v))
    if isinstance(v, ScalarValue):
        return Literal(v)
    raise TypeError(v)


def binop(l, op, r) -> BinaryExpr:
    return BinaryExpr(l, op, r)
