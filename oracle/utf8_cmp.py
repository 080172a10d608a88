"""CPU restatement of the reference's Utf8 comparisons.

TEST INFRASTRUCTURE ONLY (the checker for tests/test_utf8.py); the product path is k_utf8_cmp on
the device, reached through qeh_filter / qeh_filter_limit / qeh_eval.

Follows crates/query-executor/src/operators.rs:509-538: each comparison arm runs
coerce_numeric_types (:616-675), which leaves Utf8 operands untouched (it only widens numeric
types, :672 falls back to the arrays as they are), then arrow-rs 53.4.1's cmp::{eq, neq, lt,
lt_eq, gt, gt_eq} (Cargo.lock:156-377; not vendored, restated here).  On two StringArrays those
compare the UTF-8 bytes lexicographically (memcmp order, a proper prefix is smaller), and a NULL
on either side gives NULL.  A Utf8 literal is broadcast to the batch length by
create_literal_array (:322-347); Utf8(None) becomes a NullArray, and any Utf8 side against a
different type is arrow's "Invalid comparison operation: <l> <op> <r>" error.

Pinned by tests/golden/utf8_cmp.npz (tools/gen_golden_utf8.py, Arrow C++ via pyarrow 25, whose
string comparison kernels use the same byte order and null propagation).
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple, Union

import numpy as np

OPS = ("eq", "neq", "lt", "lt_eq", "gt", "gt_eq")


def _cmp(a: bytes, b: bytes, op: str) -> bool:
    # Python bytes ordering is memcmp order with the shorter prefix first: arrow's order.
    return {"eq": a == b, "neq": a != b, "lt": a < b, "lt_eq": a <= b, "gt": a > b, "gt_eq": a >= b}[op]


def _as_bytes(s) -> Optional[bytes]:
    if s is None:
        return None
    return s.encode() if isinstance(s, str) else bytes(s)


Side = Union[str, bytes, Sequence[Optional[Union[str, bytes]]]]


def compare(left: Side, op: str, right: Side, n: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
    """(values, validity) of `left op right`; a str/bytes side is a literal broadcast to n rows,
    a sequence side is a column whose None entries are NULL."""
    def column(side):
        if isinstance(side, (str, bytes)):
            return None
        return [_as_bytes(s) for s in side]
    lc, rc = column(left), column(right)
    if n is None:
        n = len(lc) if lc is not None else len(rc)
    vals = np.zeros(n, bool)
    valid = np.zeros(n, bool)
    lb, rb = _as_bytes(left) if lc is None else None, _as_bytes(right) if rc is None else None
    for i in range(n):
        a = lb if lc is None else lc[i]
        b = rb if rc is None else rc[i]
        if a is None or b is None:
            continue
        valid[i] = True
        vals[i] = _cmp(a, b, op)
    return vals, valid


def filter_rows(mask: np.ndarray, valid: np.ndarray) -> np.ndarray:
    """Row indices arrow's filter keeps (NULL predicate -> dropped; executor.rs:139-147)."""
    return np.flatnonzero(mask & valid)
