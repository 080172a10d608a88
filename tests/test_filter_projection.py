"""FilterExec / ProjectionExec parity: device (qeh_filter / qeh_eval through the
C ABI) vs the CPU oracle restating executor.rs:93-155 and operators.rs:13-743.
Filter output must be bit-exact AND order-identical (arrow filter preserves
order); projections bit-exact including validity."""
import numpy as np
import pytest

import oracle_bind as ob
from qe_hip import BinaryOp, QehError, ScalarValue, UnaryExpr, UnaryOp, abi, binop, col, lit
from qe_hip.expr import Literal

RNG = np.random.default_rng(1234)


def table(n, nulls=True, seed=0):
    r = np.random.default_rng(seed)
    cols = [
        (r.integers(0, 100, n).astype(np.int64), r.random(n) > 0.1 if nulls else None),           # 0 x int64
        (r.integers(-1000, 1000, n).astype(np.int32), r.random(n) > 0.2 if nulls else None),      # 1 i int32
        (r.random(n), r.random(n) > 0.15 if nulls else None),                                     # 2 v f64
        (r.random(n).astype(np.float32), None),                                                   # 3 f f32
        (r.random(n) > 0.5, r.random(n) > 0.1 if nulls else None),                                # 4 b bool
        (r.integers(-(2 ** 40), 2 ** 40, n).astype(np.int64), None),                              # 5 big int64
    ]
    return cols


def same_col(got, want, what=""):
    gv, gvalid = got
    wv, wvalid = want
    assert len(gv) == len(wv), f"{what}: length {len(gv)} != {len(wv)}"
    gm = np.ones(len(gv), bool) if gvalid is None else gvalid
    wm = wvalid
    assert np.array_equal(gm, wm), f"{what}: validity differs"
    a, b = np.asarray(gv)[wm], np.asarray(wv).astype(np.asarray(gv).dtype)[wm]
    assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), f"{what}: values differ"


def run_filter(ctx, cols, pred, offset=0):
    dev = [ctx.upload(v, m, offset=offset) for v, m in cols]
    out, rows = ctx.filter(dev, pred)
    got = [c.to_numpy() for c in out]
    want, wrows, _ = ob.filter([ob.HostCol(v, m) for v, m in cols], pred)
    assert rows == wrows
    for j, (g, w) in enumerate(zip(got, want)):
        same_col(g, w, f"col {j}")
    return rows


PREDS = {
    "gt_int": binop(col(0), BinaryOp.Greater, lit(49)),
    "le_float_vs_int_literal": binop(col(2), BinaryOp.LessEqual, lit(0)),
    "int32_vs_float_literal": binop(col(1), BinaryOp.Less, lit(12.5)),
    "f32_vs_f64": binop(col(3), BinaryOp.GreaterEqual, col(2)),
    "and_or": (binop(col(0), BinaryOp.Greater, lit(20)) & binop(col(2), BinaryOp.Less, lit(0.5)))
              | binop(col(1), BinaryOp.Equal, lit(7)),
    "not_bool": UnaryExpr(UnaryOp.Not, col(4)),
    "bare_bool": col(4),
    "arith": binop(binop(binop(col(0), BinaryOp.Multiply, lit(3)), BinaryOp.Add, col(5)), BinaryOp.Greater, lit(0)),
    "modulo": binop(binop(col(0), BinaryOp.Modulo, lit(7)), BinaryOp.Equal, lit(3)),
    "int32_arith": binop(binop(col(1), BinaryOp.Subtract, col(1)), BinaryOp.Equal,
                         Literal(ScalarValue.Int32(0))),
    "neg_float": binop(UnaryExpr(UnaryOp.Minus, col(2)), BinaryOp.Greater, lit(-0.25)),
    "div_float": binop(binop(col(2), BinaryOp.Divide, col(2)), BinaryOp.Equal, lit(1.0)),
    "ne_int64_int32": binop(col(5), BinaryOp.NotEqual, col(1)),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(PREDS))
def test_filter_predicates(ctx, name):
    run_filter(ctx, table(50_000, seed=sum(map(ord, name))), PREDS[name])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 63, 2047, 2048, 2049, 100_001, 3_000_000])
def test_filter_sizes_and_order(ctx, n):
    rows = run_filter(ctx, table(n, nulls=n % 2 == 1, seed=n), PREDS["gt_int"])
    if n > 10_000:
        assert 0 < rows < n


@pytest.mark.gpu
@pytest.mark.parametrize("offset", [1, 5, 64, 77])
def test_filter_nonzero_arrow_offsets(ctx, offset):
    run_filter(ctx, table(10_000, seed=offset), PREDS["and_or"], offset=offset)


@pytest.mark.gpu
def test_filter_all_and_none(ctx):
    t = table(5000, nulls=False)
    assert run_filter(ctx, t, binop(col(0), BinaryOp.GreaterEqual, lit(0))) == 5000
    assert run_filter(ctx, t, binop(col(0), BinaryOp.Greater, lit(1000))) == 0


@pytest.mark.gpu
def test_filter_errors_match_reference(ctx):
    t = table(1000, nulls=False)
    dev = [ctx.upload(v, m) for v, m in t]
    hc = [ob.HostCol(v, m) for v, m in t]
    cases = [
        (binop(col(0), BinaryOp.Add, lit(1)), abi.QEH_E_TYPE),                                         # not boolean
        (binop(binop(col(5), BinaryOp.Multiply, lit(2 ** 40)), BinaryOp.Greater, lit(0)), abi.QEH_E_OVERFLOW),
        (binop(binop(col(0), BinaryOp.Divide, binop(col(0), BinaryOp.Subtract, col(0))), BinaryOp.Greater, lit(0)),
         abi.QEH_E_DIV0),
        (binop(binop(col(0), BinaryOp.Multiply, lit(1.5)), BinaryOp.Greater, lit(0)), abi.QEH_E_TYPE),  # no coercion
        (binop(col(0), BinaryOp.Greater, lit(None)), abi.QEH_E_TYPE),                                  # NullArray
    ]
    for pred, status in cases:
        with pytest.raises(QehError) as e:
            ctx.filter(dev, pred)
        with pytest.raises(ob.OracleError) as w:
            ob.filter(hc, pred)
        assert e.value.status == status == w.value.status, (e.value, w.value)
        assert e.value.message == w.value.message


PROJ = {
    "add_i64": binop(col(0), BinaryOp.Add, lit(5)),
    "mul_f64": binop(col(2), BinaryOp.Multiply, col(2)),
    "f32_div": binop(col(3), BinaryOp.Divide, col(3)),
    "i32_mod": binop(col(1), BinaryOp.Modulo, Literal(ScalarValue.Int32(7))),
    "mod_by_zero_is_null": binop(col(0), BinaryOp.Modulo, binop(col(0), BinaryOp.Subtract, col(0))),
    "neg_i32": UnaryExpr(UnaryOp.Minus, col(1)),
    "cmp": binop(col(0), BinaryOp.Less, col(5)),
    "not": UnaryExpr(UnaryOp.Not, col(4)),
    "nested": binop(binop(col(5), BinaryOp.Subtract, col(0)), BinaryOp.Divide, lit(3)),
    "literal": lit(42),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(PROJ))
def test_projection_expressions(ctx, name):
    t = table(20_011, seed=len(name))
    dev = [ctx.upload(v, m) for v, m in t]
    r = ctx.eval(dev, PROJ[name])
    got_col = r[0] if isinstance(r, tuple) else r
    got = got_col.to_numpy()
    (wv, wm), wdt = ob.eval_expr([ob.HostCol(v, m) for v, m in t], PROJ[name], 20_011)
    assert got_col.dtype == wdt
    same_col(got, (wv, wm), name)


@pytest.mark.gpu
def test_projection_column_reference_is_zero_copy(ctx):
    t = table(1000)
    dev = [ctx.upload(v, m) for v, m in t]
    view, src = ctx.eval(dev, col(2))
    assert view.c.values == dev[2].c.values and view.c.owned == 0


FAST_PREDS = {
    "gt_int": binop(col(0), BinaryOp.Greater, lit(49)),
    "float_col_int_lit": binop(col(1), BinaryOp.LessEqual, lit(0)),
    "int_col_float_lit": binop(col(0), BinaryOp.Less, lit(12.5)),
    "and": binop(col(0), BinaryOp.Greater, lit(20)) & binop(col(1), BinaryOp.Less, lit(0.5)),
    "or": binop(col(2), BinaryOp.Greater, lit(0)) | binop(col(1), BinaryOp.Less, lit(0.25)),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(FAST_PREDS))
@pytest.mark.parametrize("n", [0, 1, 2047, 2049, 1_000_003])
def test_fast_filter_non_null_8byte_columns(ctx, monkeypatch, name, n):
    """All-8-byte, non-null inputs take k_filter_fast (register tiles + LDS-staged
    runs); same rows, same order as the generic kernel and the oracle."""
    r = np.random.default_rng(n + len(name))
    cols = [(r.integers(0, 100, n).astype(np.int64), None), (r.random(n) - 0.25, None),
            (r.integers(-(2 ** 40), 2 ** 40, n).astype(np.int64), None)]
    rows = run_filter(ctx, cols, FAST_PREDS[name])
    monkeypatch.setenv("QEH_NO_FAST_FILTER", "1")
    assert run_filter(ctx, cols, FAST_PREDS[name]) == rows


@pytest.mark.gpu
def test_fast_filter_output_subset_and_aligned_offset(ctx):
    r = np.random.default_rng(5)
    n = 300_000
    x = r.integers(0, 100, n).astype(np.int64)
    v = r.random(n)
    dev = [ctx.upload(x, offset=2), ctx.upload(v, offset=4)]
    pred = binop(col(0), BinaryOp.Greater, lit(49))
    out, rows = ctx.filter(dev, pred, [1])
    keep = x > 49
    assert rows == int(keep.sum())
    assert np.array_equal(out[0].to_numpy()[0], v[keep])


def run_filter_limit(ctx, cols, pred, cap, offset=0):
    """qeh_filter_limit == the oracle's full filter, then the first `cap` rows (LimitExec)."""
    dev = [ctx.upload(v, m, offset=offset) for v, m in cols]
    out, rows = ctx.filter(dev, pred, max_rows=cap)
    want, wrows, _ = ob.filter([ob.HostCol(v, m) for v, m in cols], pred)
    assert rows == min(wrows, cap)
    for j, (g, w) in enumerate(zip([c.to_numpy() for c in out], want)):
        wv, wm = w
        same_col(g, (np.asarray(wv)[:cap], np.asarray(wm)[:cap]), f"col {j} cap {cap}")
    return rows


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["gt_int", "and_or", "bare_bool", "arith", "modulo"])
@pytest.mark.parametrize("cap", [0, 1, 31, 33, 2048, 5000, 10 ** 9])
def test_filter_limit_generic(ctx, name, cap):
    """Generic kernel (nullable int/float/bool columns): rows past the cap are dropped inside the
    filter; validity and bit-packed booleans stay exact at the cut."""
    run_filter_limit(ctx, table(20_011, seed=cap % 97), PREDS[name], cap)


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [0, 1, 7, 4096, 100_000, 10 ** 9])
@pytest.mark.parametrize("n", [1, 2049, 3_000_001])
def test_filter_limit_fast_early_exit(ctx, monkeypatch, cap, n):
    """k_filter_fast with a cap: tiles claimed after `cap` rows are placed publish a >= cap prefix
    and stop (no hang, no missing rows); the same rows with the generic kernel."""
    r = np.random.default_rng(n + cap)
    cols = [(r.integers(0, 100, n).astype(np.int64), None), (r.random(n), None)]
    pred = binop(col(0), BinaryOp.Greater, lit(49))
    rows = run_filter_limit(ctx, cols, pred, cap)
    monkeypatch.setenv("QEH_NO_FAST_FILTER", "1")
    assert run_filter_limit(ctx, cols, pred, cap) == rows


@pytest.mark.gpu
def test_filter_limit_still_raises_past_the_cap(ctx):
    """A predicate that can raise is evaluated on every row even under a cap (the reference
    evaluates the whole batch before LimitExec slices it)."""
    n = 100_000
    big = np.zeros(n, np.int64)
    big[-1] = 2 ** 62  # overflows only on the last row
    dev = [ctx.upload(np.arange(n, dtype=np.int64)), ctx.upload(big)]
    pred = binop(binop(col(1), BinaryOp.Multiply, lit(4)), BinaryOp.GreaterEqual, lit(0))
    with pytest.raises(QehError) as e:
        ctx.filter(dev, pred, max_rows=10)
    assert e.value.status == abi.QEH_E_OVERFLOW

