"""Comparison helpers for parity tests (bit-exact ints, tolerance for float aggregates)."""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np

FLOAT_RTOL = 1e-6   # north_star: SUM/AVG floats within 1e-6 relative


def rows_of(cols: Sequence[Tuple[np.ndarray, Optional[np.ndarray]]]) -> List[tuple]:
    """Columns -> list of row tuples with None for NULL."""
    if not cols:
        return []
    n = len(cols[0][0])
    out = []
    for i in range(n):
        row = []
        for vals, valid in cols:
            if valid is not None and not valid[i]:
                row.append(None)
            else:
                v = vals[i]
                row.append(v.item() if hasattr(v, "item") else v)
        out.append(tuple(row))
    return out


def _key(row):
    return tuple((0, 0) if v is None else (1, v) for v in row)


def sorted_rows(cols) -> List[tuple]:
    return sorted(rows_of(cols), key=_key)


def assert_rows_equal(got: List[tuple], want: List[tuple], float_cols: Sequence[int] = (), rtol=FLOAT_RTOL):
    assert len(got) == len(want), f"row count {len(got)} != {len(want)}"
    for i, (g, w) in enumerate(zip(got, want)):
        assert len(g) == len(w)
        for j, (a, b) in enumerate(zip(g, w)):
            if j in float_cols and a is not None and b is not None:
                if math.isnan(a) and math.isnan(b):
                    continue
                assert abs(a - b) <= rtol * max(abs(a), abs(b), 1e-300) or a == b, \
                    f"row {i} col {j}: {a} vs {b} (rtol {rtol})"
            else:
                assert a == b, f"row {i} col {j}: {a!r} vs {b!r}\n got={g}\nwant={w}"


def assert_grouped_equal(gk, ga, wk, wa, float_aggs: Sequence[int] = (), rtol=FLOAT_RTOL):
    """Compare (keys, aggs) multisets sorted by key columns."""
    nk = len(gk)
    got = sorted_rows(list(gk) + list(ga))
    want = sorted_rows(list(wk) + list(wa))
    assert_rows_equal(got, want, float_cols=[nk + j for j in float_aggs], rtol=rtol)
