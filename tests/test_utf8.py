"""Utf8 comparisons in predicates and projections (k_utf8.hip through qeh_filter /
qeh_filter_limit / qeh_eval) vs the CPU restatement oracle/utf8_cmp.py, which follows
operators.rs:509-538 (arrow cmp kernels on StringArray: byte order, NULL in -> NULL out).
The oracle itself is pinned by tests/golden/utf8_cmp.npz (Arrow C++ string compares,
tools/gen_golden_utf8.py).  Bit-exact: row sets, row order, bytes, validity."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import utf8_cmp as uo  # noqa: E402
from qe_hip import BinaryOp, QehError, abi, binop, col, lit  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "utf8_cmp.npz")
OPS = {"eq": BinaryOp.Equal, "neq": BinaryOp.NotEqual, "lt": BinaryOp.Less, "lt_eq": BinaryOp.LessEqual,
       "gt": BinaryOp.Greater, "gt_eq": BinaryOp.GreaterEqual}


def golden():
    z = np.load(GOLD, allow_pickle=False)

    def strs(name):
        offs, data, valid = z[name + "_offsets"], z[name + "_bytes"].tobytes(), z[name + "_valid"]
        return [data[offs[i]:offs[i + 1]] if valid[i] else None for i in range(len(offs) - 1)]
    return z, strs("a"), strs("b"), strs("lit")


# ---- CPU: oracle pinned by Arrow's string kernels ---------------------------------------------
@pytest.mark.parametrize("op", uo.OPS)
def test_oracle_utf8_compare_matches_arrow(op):
    z, a, b, lits = golden()
    v, m = uo.compare(a, op, b)
    assert np.array_equal(m, z[f"col_{op}_valid"]) and np.array_equal(v & m, z[f"col_{op}_values"] & m)
    for j, s in enumerate(lits):
        v, m = uo.compare(a, op, s)
        assert np.array_equal(m, z[f"lit{j}_{op}_valid"]), (op, s)
        assert np.array_equal(v & m, z[f"lit{j}_{op}_values"] & m), (op, s)


def test_utf8_literal_node_encoding():
    import ctypes as C
    e, keep = binop(col(0), BinaryOp.Equal, lit("ab\x00c")).to_c()
    node = e.nodes[1]
    assert node.kind == abi.EX_LITERAL and node.lit_dtype == abi.DT_UTF8 and node.index == 4
    assert C.string_at(node.lit_i64, node.index) == b"ab\x00c"


# ---- GPU parity -------------------------------------------------------------------------------
def check_filter(ctx, strs, ids, pred, want_rows, max_rows=None, other=None):
    cols = [ctx.upload(strs), ctx.upload(ids)] + ([ctx.upload(*other)] if other else [])
    out, rows = ctx.filter(cols, pred, out_idx=[0, 1], max_rows=max_rows)
    want_rows = want_rows if max_rows is None else want_rows[:max_rows]
    assert rows == len(want_rows)
    got_ids = out[1].to_numpy()[0]
    assert np.array_equal(got_ids, ids[want_rows])
    got_s = out[0].to_bytes()
    assert got_s == [strs[i] for i in want_rows]


@pytest.mark.gpu
@pytest.mark.parametrize("op", uo.OPS)
def test_filter_utf8_column_vs_literal(ctx, op):
    _, a, _, lits = golden()
    ids = np.arange(len(a), dtype=np.int64)
    for s in lits:
        v, m = uo.compare(a, op, s)
        check_filter(ctx, a, ids, binop(col(0), OPS[op], lit(s)), uo.filter_rows(v, m))
        v, m = uo.compare(s, op, a, n=len(a))  # literal on the left
        check_filter(ctx, a, ids, binop(lit(s), OPS[op], col(0)), uo.filter_rows(v, m))


@pytest.mark.gpu
@pytest.mark.parametrize("op", uo.OPS)
def test_filter_utf8_column_vs_column(ctx, op):
    _, a, b, _ = golden()
    ids = np.arange(len(a), dtype=np.int64)
    v, m = uo.compare(a, op, b)
    cols = [ctx.upload(a), ctx.upload(ids), ctx.upload(b)]
    out, rows = ctx.filter(cols, binop(col(0), OPS[op], col(2)), out_idx=[1, 2])
    want = uo.filter_rows(v, m)
    assert rows == len(want)
    assert np.array_equal(out[0].to_numpy()[0], ids[want])
    assert out[1].to_bytes() == [b[i] for i in want]


@pytest.mark.gpu
def test_filter_utf8_and_numeric_with_limit(ctx):
    _, a, _, _ = golden()
    n = len(a)
    r = np.random.default_rng(5)
    x = r.integers(0, 100, n).astype(np.int64)
    xv = r.random(n) > 0.1
    ids = np.arange(n, dtype=np.int64)
    sv, sm = uo.compare(a, "gt", "B")
    # arrow `and` (non-Kleene): NULL if either side NULL; filter drops NULL
    want = np.flatnonzero(sv & sm & (x > 49) & xv)
    pred = binop(col(0), BinaryOp.Greater, lit("B")) & binop(col(2), BinaryOp.Greater, lit(49))
    check_filter(ctx, a, ids, pred, want, other=(x, xv))
    check_filter(ctx, a, ids, pred, want, max_rows=17, other=(x, xv))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 65, 100_003])
def test_eval_utf8_compare_projection(ctx, n):
    r = np.random.default_rng(n)
    words = ["", "a", "ab", "abc", "b", "ba", "é", None]
    a = [words[i] for i in r.integers(0, len(words), n)]
    b = [words[i] for i in r.integers(0, len(words), n)]
    for op in uo.OPS:
        out = ctx.eval([ctx.upload(a), ctx.upload(b)], binop(col(0), OPS[op], col(1)), n_rows=n)
        v, m = uo.compare(a, op, b, n=n)
        gv, gm = out.to_numpy()
        gm = np.ones(n, bool) if gm is None else gm
        assert np.array_equal(gm, m) and np.array_equal(gv.astype(bool) & m, v & m), op


@pytest.mark.gpu
def test_filter_utf8_sliced_input(ctx):
    _, a, _, _ = golden()
    ids = np.arange(len(a), dtype=np.int64)
    ca, ci = ctx.upload(a), ctx.upload(ids)
    off, ln = 333, 1200
    out, rows = ctx.filter([ctx.slice(ca, off, ln), ctx.slice(ci, off, ln)],
                           binop(col(0), BinaryOp.LessEqual, lit("ab")))
    v, m = uo.compare(a[off:off + ln], "lt_eq", "ab")
    want = uo.filter_rows(v, m) + off
    assert rows == len(want)
    assert np.array_equal(out[1].to_numpy()[0], ids[want])
    assert out[0].to_bytes() == [a[i] for i in want]


@pytest.mark.gpu
def test_utf8_compare_type_errors(ctx):
    cols = [ctx.upload(["a", "b"]), ctx.upload(np.array([1, 2], np.int64))]
    with pytest.raises(QehError) as ei:
        ctx.filter(cols, binop(col(0), BinaryOp.Equal, col(1)))
    assert "Invalid comparison operation: Utf8 == Int64" in ei.value.message
    with pytest.raises(QehError) as ei:
        ctx.filter(cols, binop(col(0), BinaryOp.Less, lit(None)))
    assert "Invalid comparison operation: Utf8 < Null" in ei.value.message


@pytest.mark.gpu
def test_config1_filter_on_name(ctx):
    """employees.csv (reference data/employees.csv:1-7): WHERE name >= 'Charlie' AND age > 28."""
    names = ["Alice", "Bob", "Charlie", "Diana", "Eve", "Frank"]
    ages = np.array([25, 30, 35, 28, 32, 29], np.int64)
    cols = [ctx.upload(names), ctx.upload(ages)]
    out, rows = ctx.filter(cols, binop(col(0), BinaryOp.GreaterEqual, lit("Charlie"))
                           & binop(col(1), BinaryOp.Greater, lit(28)))
    assert rows == 3
    assert out[0].to_bytes() == [b"Charlie", b"Eve", b"Frank"]
    assert list(out[1].to_numpy()[0]) == [35, 32, 29]
