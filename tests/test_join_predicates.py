"""Joins whose `on` is not a single integer equi-key, through the plan executor (§8 row a9).

The reference's `on` is any boolean expression over the concatenated schema
(query-planner/src/planner.rs:148-157); the contract is "exactly the pairs of
join_batches' Cartesian product on which `on` evaluates TRUE", extended for LEFT / RIGHT / FULL
by the rows without such a pair.  The oracle restates that literally (qo_join_on: Cartesian
product, `on` evaluated column-at-a-time); the device runs AND-ed equi conjuncts as a hash join
(packed composite keys), checks the rest of `on` over the candidate pairs, and runs a pure
non-equi `on` over the Cartesian product.  Row order is not part of the join contract:
multisets are compared, except for the literal Cartesian joins whose order the reference fixes.
"""
import numpy as np
import pyarrow as pa
import pytest

import oracle_bind as ob
from helpers import assert_grouped_equal, rows_of, sorted_rows
from qe_hip import AggregateExpr, AggregateFunction as AF, BinaryOp, abi, binop, col, lit
from qe_hip import Filter, HashAggregate, HashJoin, JoinType, MemoryDataSource, QueryExecutor, Scan
from qe_hip.expr import Column
from test_executor import as_cols, source

JT = {"inner": (JoinType.Inner, 0), "left": (JoinType.Left, 1), "right": (JoinType.Right, 2),
      "full": (JoinType.Full, 3)}


@pytest.fixture(scope="module")
def qx(ctx):
    return QueryExecutor(ctx)


def tables(seed, nl=700, nr=500, wide=False):
    r = np.random.default_rng(seed)
    lo, hi = (-(2 ** 62), 2 ** 62) if wide else (0, 12)
    lk1 = r.integers(0, 12, nl)
    lk2 = r.integers(lo, hi, nl) if not wide else r.choice(r.integers(lo, hi, 20), nl)
    rk1 = r.integers(0, 12, nr)
    rk2 = r.integers(lo, hi, nr) if not wide else r.choice(np.concatenate([lk2[:10], r.integers(lo, hi, 10)]), nr)
    left = pa.table({
        "a.k1": pa.array(lk1, pa.int64(), mask=r.random(nl) < 0.05),
        "a.k2": pa.array(lk2.astype(np.int64), pa.int64()),
        "a.x": pa.array(r.integers(-50, 50, nl), pa.int64(), mask=r.random(nl) < 0.05),
        "a.f": pa.array(np.round(r.random(nl), 1)),
    })
    right = pa.table({
        "b.k1": pa.array(rk1.astype(np.int32), pa.int32(), mask=r.random(nr) < 0.05),  # Int32 = Int64 keys
        "b.k2": pa.array(rk2.astype(np.int64), pa.int64()),
        "b.y": pa.array(r.integers(-50, 50, nr), pa.int64()),
        "b.f": pa.array(np.round(r.random(nr), 1)),
    })
    return left, right


def host(t):
    return [ob.HostCol(v, m) for v, m in as_cols(t.to_batches())]


# column indices over the concatenated schema: a.k1 a.k2 a.x a.f | b.k1 b.k2 b.y b.f
K1 = binop(Column("a.k1", 0), BinaryOp.Equal, Column("b.k1", 4))
K2 = binop(Column("a.k2", 1), BinaryOp.Equal, Column("b.k2", 5))
RES = binop(Column("a.x", 2), BinaryOp.Greater, Column("b.y", 6))
ONS = {
    "composite": K1 & K2,
    "equi_residual": K1 & RES,
    "composite_residual": (K2 & RES) & K1,
    "non_equi": binop(Column("a.x", 2), BinaryOp.Less, binop(Column("b.y", 6), BinaryOp.Subtract, lit(40))),
    "or": K1 | binop(Column("a.x", 2), BinaryOp.Equal, Column("b.y", 6)),
    "float_equi": binop(Column("a.f", 3), BinaryOp.Equal, Column("b.f", 7)) & K1,
    "reversed_sides": binop(Column("b.k1", 4), BinaryOp.Equal, Column("a.k1", 0)) & RES,
}


def check(qx, left, right, on, jt):
    jtype, code = JT[jt]
    out = qx.execute(HashJoin(Scan(source(left)), Scan(source(right)), jtype, on))
    lo, ro, rows = ob.join_on(code, host(left), host(right), on)
    got = as_cols(out)
    if rows == 0:
        assert out == [] or out[0].num_rows == 0
        return
    assert out[0].num_rows == rows
    assert out[0].schema.names == left.schema.names + right.schema.names
    assert sorted_rows(got) == sorted_rows(lo + ro)


@pytest.mark.gpu
@pytest.mark.parametrize("jt", ["inner", "left", "right", "full"])
@pytest.mark.parametrize("name", sorted(ONS))
def test_join_on_general_predicate(qx, name, jt):
    left, right = tables(sorted(ONS).index(name) + 11)
    check(qx, left, right, ONS[name], jt)


@pytest.mark.gpu
@pytest.mark.parametrize("jt", ["inner", "left", "full"])
def test_join_composite_key_beyond_63_bits_is_hashed(qx, jt):
    """Two equi keys spanning 2^63 each: the packed key would not fit, so the tuple is hashed and
    the whole `on` re-checked on every candidate pair."""
    left, right = tables(77, wide=True)
    check(qx, left, right, K1 & K2, jt)


@pytest.mark.gpu
def test_join_composite_larger_inner(qx):
    """A composite-key INNER join at a size where the hash join's table paths matter."""
    r = np.random.default_rng(5)
    n, m = 400_000, 60_000
    left = pa.table({"a.k1": r.integers(0, 300, n), "a.k2": r.integers(0, 200, n), "a.v": r.random(n)})
    rk = np.stack(np.unravel_index(r.permutation(300 * 200)[:m], (300, 200)))
    right = pa.table({"b.k1": rk[0].astype(np.int64), "b.k2": rk[1].astype(np.int64),
                      "b.a": np.arange(m, dtype=np.int64)})
    on = binop(Column("a.k1", 0), BinaryOp.Equal, Column("b.k1", 3)) & \
        binop(Column("a.k2", 1), BinaryOp.Equal, Column("b.k2", 4))
    out = qx.execute(HashJoin(Scan(source(left)), Scan(source(right)), JoinType.Inner, on))
    hl, hr = host(left), host(right)
    # the oracle's equi join on a combined key (k1 * 200 + k2) gives the same pairs
    ck = lambda t: ob.HostCol(t.column(0).to_numpy() * 200 + t.column(1).to_numpy())  # noqa: E731
    wp, wb, rows = ob.hash_join_inner(ck(left), hl, ck(right), hr)
    assert out[0].num_rows == rows
    assert sorted_rows(as_cols(out)) == sorted_rows(wp + wb)


@pytest.mark.gpu
def test_cartesian_joins_keep_the_reference_row_order(qx):
    """INNER without `on` = join_batches (left row-major, executor.rs:500-540); CROSS =
    execute_cross_join (right row-major, executor.rs:437-498): row order bit-exact."""
    a = pa.table({"a.x": np.arange(5, dtype=np.int64), "a.f": np.linspace(0, 1, 5)})
    b = pa.table({"b.y": pa.array([7, 8, 9], pa.int64(), mask=[False, True, False])})
    out = qx.execute(HashJoin(Scan(source(a)), Scan(source(b)), JoinType.Inner, None))
    want, _ = ob.join_batches(host(a), host(b))
    assert rows_of(as_cols(out)) == rows_of(want)
    out = qx.execute(HashJoin(Scan(source(a)), Scan(source(b)), JoinType.Cross, None))
    want, _ = ob.cross_join(host(a), host(b))
    assert rows_of(as_cols(out)) == rows_of(want)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_literal_metric_query_through_the_plan(qx, seed):
    """The one form of the metric query the reference answers correctly: a global aggregate over
    Filter(f.k = d.k AND f.x > 49) of the un-keyed join (executor.rs:131-188, join_batches).
    Device plan == the oracle's literal Cartesian path == the intended hash join + aggregate."""
    r = np.random.default_rng(seed)
    n, nd = 1500, 600
    fact = pa.table({"f.x": r.integers(0, 100, n), "f.k": pa.array(r.integers(0, nd + 50, n), pa.int64(),
                                                                   mask=r.random(n) < 0.03),
                     "f.v": r.random(n)})
    dk = r.permutation(nd).astype(np.int64)
    dk[3] = dk[4]
    dim = pa.table({"d.k": dk, "d.g": r.integers(0, 9, nd)})
    pred = binop(Column("f.k", 1), BinaryOp.Equal, Column("d.k", 3)) & \
        binop(Column("f.x", 0), BinaryOp.Greater, lit(49))
    plan = HashAggregate(Filter(HashJoin(Scan(source(fact, 2)), Scan(source(dim)), JoinType.Inner, None), pred), [],
                         [AggregateExpr(AF.Sum, Column("f.v", 2)), AggregateExpr(AF.Count, Column("f.v", 2))])
    got = qx.execute(plan)[0].to_pylist()[0]
    # literal: Cartesian (join_batches), filter, global aggregate
    cart, rows = ob.join_batches(host(fact), host(dim))
    filt, _, _ = ob.filter([ob.HostCol(v, m) for v, m in cart], pred)
    _, la, g, _ = ob.hash_aggregate([], [ob.HostCol(*c) for c in filt], [(AF.Sum, 2), (AF.Count, 2)])
    assert got["col_1"] == la[1][0][0]
    assert got["col_0"] == pytest.approx(la[0][0][0], rel=1e-9)
    # intended semantics: hash join + filter + aggregate (no group key)
    _, ia, _ = ob.join_filter_aggregate(host(fact), 1, binop(col(0), BinaryOp.Greater, lit(49)), host(dim)[0], [],
                                        [(AF.Sum, 2), (AF.Count, 2)])
    assert ia[1][0][0] == got["col_1"]
    assert ia[0][0][0] == pytest.approx(got["col_0"], rel=1e-9)
    # and the same query with the equi key in `on` (the planner's shape) agrees
    plan2 = HashAggregate(Filter(HashJoin(Scan(source(fact, 2)), Scan(source(dim)), JoinType.Inner,
                                          binop(Column("f.k", 1), BinaryOp.Equal, Column("d.k", 3))),
                                 binop(Column("f.x", 0), BinaryOp.Greater, lit(49))), [],
                          [AggregateExpr(AF.Sum, Column("f.v", 2)), AggregateExpr(AF.Count, Column("f.v", 2))])
    got2 = qx.execute(plan2)[0].to_pylist()[0]
    assert got2["col_1"] == got["col_1"] and got2["col_0"] == pytest.approx(got["col_0"], rel=1e-9)
