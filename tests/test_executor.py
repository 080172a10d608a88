"""Plan-level parity: qe_hip.QueryExecutor.execute(PhysicalPlan) — the drop-in
for `QueryExecutor::execute` (executor.rs:19-21) — on the device, vs the CPU
oracle and the reference's known answers.  Plans are built the way the
reference's converters build them (crates/query-pgwire/src/backend.rs:614-756):
column indices over the concatenation of table-prefixed schemas."""
import json
import os

import numpy as np
import pyarrow as pa
import pytest

import oracle_bind as ob
from helpers import assert_grouped_equal, assert_rows_equal, rows_of, sorted_rows
from qe_hip import AggregateExpr, AggregateFunction as AF, BinaryOp, UnaryExpr, UnaryOp, abi, binop, col, lit
from qe_hip import (Filter, HashAggregate, HashJoin, JoinType, Limit, MemoryDataSource, Projection, QueryExecutor,
                    Scan, Sort, SubqueryScan, Window, WindowExpr, WindowFunctionType)
from qe_hip.expr import Column

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def qx(ctx):
    return QueryExecutor(ctx)


def source(table: pa.Table, chunks=1):
    batches = table.to_batches()
    if chunks > 1 and table.num_rows:
        step = max(1, table.num_rows // chunks)
        batches = [table.slice(i, step).to_batches()[0] for i in range(0, table.num_rows, step)]
    return MemoryDataSource(table.schema, batches)


def as_cols(batches, names=None):
    if not batches:
        return []
    t = pa.Table.from_batches(batches)
    out = []
    for c in t.columns:
        a = c.combine_chunks()
        valid = ~np.asarray(a.is_null().to_numpy(zero_copy_only=False), bool)
        if pa.types.is_string(a.type):
            vals = np.array([x if x is not None else "" for x in a.to_pylist()], dtype=object)
        elif pa.types.is_boolean(a.type):
            vals = np.asarray(a.fill_null(False).to_numpy(zero_copy_only=False), bool)
        else:
            vals = np.asarray(a.fill_null(0).to_numpy(zero_copy_only=False))
        out.append((vals, valid))
    return out


@pytest.mark.gpu
def test_config1_employees_known_answer(qx):
    """BASELINE config 1: SELECT name,age FROM employees WHERE age>25."""
    import pyarrow.csv as pacsv
    emp = pacsv.read_csv(os.path.join(GOLD, "employees.csv"))
    emp = emp.rename_columns([f"employees.{c}" for c in emp.column_names])
    plan = Projection(
        Filter(Scan(source(emp)), binop(Column("employees.age", 2), BinaryOp.Greater, lit(25))),
        [Column("employees.name", 1), Column("employees.age", 2)],
        ["employees.name", "employees.age"])
    out = qx.execute(plan)
    assert len(out) == 1
    b = out[0]
    assert b.schema.names == ["employees.name", "employees.age"]
    assert [f.type for f in b.schema] == [pa.string(), pa.int64()]
    want = [tuple(r) for r in json.load(open(os.path.join(GOLD, "manifest.json")))["fixtures"]["employees"]["rows"]]
    assert list(zip(b.column(0).to_pylist(), b.column(1).to_pylist())) == want


def metric_tables(n, nd, groups=1024, seed=0x5EED):
    x = ob.generate(abi.GEN_UNIFORM_MOD, seed, 1, n, 100)
    k = ob.generate(abi.GEN_UNIFORM_MOD, seed, 2, n, nd)
    v = ob.generate(abi.GEN_UNIT_F64, seed, 3, n)
    dk = ob.generate(abi.GEN_PERMUTATION, seed, 0, nd, nd)
    dg = ob.generate(abi.GEN_UNIFORM_MOD, seed, 5, nd, groups)
    fact = pa.table({"f.x": x, "f.k": k, "f.v": v})
    dim = pa.table({"d.k": dk, "d.g": dg})
    return fact, dim


def metric_plan(fact, dim, chunks=1):
    """SELECT d.g, SUM(f.v), COUNT(f.v) FROM fact f JOIN dim d ON f.k = d.k
    WHERE f.x > 49 GROUP BY d.g  ->  HashAggregate(Filter(HashJoin))."""
    join = HashJoin(Scan(source(fact, chunks)), Scan(source(dim)), JoinType.Inner,
                    binop(Column("f.k", 1), BinaryOp.Equal, Column("d.k", 3)))
    filt = Filter(join, binop(Column("f.x", 0), BinaryOp.Greater, lit(49)))
    return HashAggregate(filt, [Column("d.g", 4)],
                         [AggregateExpr(AF.Sum, Column("f.v", 2)), AggregateExpr(AF.Count, Column("f.v", 2))])


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False])
def test_metric_query_plan(qx, monkeypatch, fused):
    if not fused:
        monkeypatch.setenv("QEH_NO_FUSION", "1")  # materialise join -> filter -> aggregate
    fact, dim = metric_tables(300_000, 20_000, 256)
    out = qx.execute(metric_plan(fact, dim, chunks=3))
    got = as_cols(out)
    wk, wa, wg = ob.join_filter_aggregate(
        [ob.HostCol(fact.column(i).to_numpy()) for i in range(3)], 1, binop(col(0), BinaryOp.Greater, lit(49)),
        ob.HostCol(dim.column(0).to_numpy()), [ob.HostCol(dim.column(1).to_numpy())], [(AF.Sum, 2), (AF.Count, 2)])
    assert out[0].schema.names == ["d.g", "col_0", "col_1"]
    assert_grouped_equal(got[:1], got[1:], wk, wa, float_aggs=[0])


@pytest.mark.gpu
def test_config2_filter_group_by(qx):
    """BASELINE config 2 shape: SELECT k, SUM(v), COUNT(v), SUM(vi) FROM t WHERE x > 49 GROUP BY k."""
    r = np.random.default_rng(2)
    n = 500_000
    t = pa.table({"t.x": r.integers(0, 100, n), "t.k": r.integers(0, 1024, n), "t.v": r.random(n),
                  "t.vi": r.integers(-(2 ** 20), 2 ** 20, n)})
    plan = HashAggregate(Filter(Scan(source(t, 4)), binop(Column("t.x", 0), BinaryOp.Greater, lit(49))),
                         [Column("t.k", 1)],
                         [AggregateExpr(AF.Sum, Column("t.v", 2)), AggregateExpr(AF.Count, Column("t.v", 2)),
                          AggregateExpr(AF.Sum, Column("t.vi", 3))])
    got = as_cols(qx.execute(plan))
    hc = [ob.HostCol(t.column(i).to_numpy()) for i in range(4)]
    fc, rows, _ = ob.filter(hc, binop(col(0), BinaryOp.Greater, lit(49)))
    fh = [ob.HostCol(v, m) for v, m in fc]
    wk, wa, wg, _ = ob.hash_aggregate([fh[1]], fh, [(AF.Sum, 2), (AF.Count, 2), (AF.Sum, 3)])
    assert_grouped_equal(got[:1], got[1:], wk, wa, float_aggs=[0])


@pytest.mark.gpu
def test_global_aggregate_quirks(qx):
    t = pa.table({"t.x": np.arange(10, dtype=np.int64), "t.v": np.linspace(0, 1, 10)})
    aggs = [AggregateExpr(AF.Count, Column("t.x", 0)), AggregateExpr(AF.Sum, Column("t.v", 1)),
            AggregateExpr(AF.Avg, Column("t.x", 0)), AggregateExpr(AF.Min, Column("t.v", 1)),
            AggregateExpr(AF.Max, Column("t.x", 0))]
    out = qx.execute(HashAggregate(Scan(source(t)), [], aggs))
    assert out[0].schema.names == ["col_0", "col_1", "col_2", "col_3", "col_4"]
    assert out[0].to_pylist() == [{"col_0": 10, "col_1": pytest.approx(5.0), "col_2": 4.5, "col_3": 0.0, "col_4": 9}]
    # filter drops every row -> no batches -> the reference's aggregate returns vec![] (executor.rs:178-186)
    none = qx.execute(HashAggregate(Filter(Scan(source(t)), binop(Column("t.x", 0), BinaryOp.Greater, lit(100))), [],
                                    aggs))
    assert none == []
    # no aggregates -> no batches (executor.rs:163-165)
    assert qx.execute(HashAggregate(Scan(source(t)), [Column("t.x", 0)], [])) == []


@pytest.mark.gpu
def test_sort_limit_subquery_window(qx):
    r = np.random.default_rng(5)
    n = 50_000
    k = pa.array(r.integers(0, 40, n), pa.int64(), mask=r.random(n) < 0.05)
    v = pa.array(r.integers(-100, 100, n), pa.int64())
    w = pa.array(r.random(n))
    t = pa.table({"t.k": k, "t.v": v, "t.w": w})
    srt = Sort(Scan(source(t, 5)), [Column("t.k", 0), Column("t.w", 2)], [True, False])
    out = qx.execute(Limit(SubqueryScan(srt), 100, 1000))
    perm = ob.sort_indices([ob.HostCol(*c) for c in as_cols([t.to_batches()[0]])[0:1]] +
                           [ob.HostCol(*as_cols([t.to_batches()[0]])[2])], [True, False])
    want = t.take(pa.array(perm[100:1100]))
    assert rows_of(as_cols(out)) == rows_of(as_cols(want.to_batches()))
    win = Window(Scan(source(t, 2)), [WindowExpr(WindowFunctionType.RowNumber, [], [Column("t.k", 0)],
                                                 [Column("t.v", 1)])], ["t.k", "t.v", "t.w", "rn"])
    out = qx.execute(win)
    assert out[0].schema.names == ["t.k", "t.v", "t.w", "rn"]
    cols = as_cols([t.to_batches()[0]])
    want_rn = ob.row_number([ob.HostCol(*cols[0])], [ob.HostCol(*cols[1])], [True])
    assert np.array_equal(out[0].column(3).to_numpy(), want_rn)


@pytest.mark.gpu
@pytest.mark.parametrize("key_col,asc,key_dt,nulls", [(0, True, pa.int64(), True), (1, False, pa.int32(), False),
                                                      (0, False, pa.int64(), False)])
def test_sort_key_and_payload_columns(qx, monkeypatch, key_col, asc, key_dt, nulls):
    """Sort of a two-column table by one Int key column: the payload column rides through the radix
    passes (no permutation, no gathers); stable, NULL keys first -- equal to the oracle's stable sort
    and to the permutation path (QEH_NO_PAYLOAD_SORT=1)."""
    r = np.random.default_rng(11 + key_col)
    n = 90_001
    k = pa.array(r.integers(-3000, 3000, n), key_dt, mask=(r.random(n) < 0.07) if nulls else None)
    v = pa.array(r.random(n))
    t = pa.table({"t.k": k, "t.v": v} if key_col == 0 else {"t.v": v, "t.k": k})
    plan = Sort(Scan(source(t, 3)), [Column("t.k", key_col)], [asc])
    got = as_cols(qx.execute(plan))
    kc = as_cols([t.combine_chunks().to_batches()[0]])[key_col]
    perm = ob.sort_indices([ob.HostCol(kc[0].astype(np.int64), kc[1])], [asc])
    want = t.take(pa.array(perm))
    assert rows_of(got) == rows_of(as_cols(want.to_batches()))
    monkeypatch.setenv("QEH_NO_PAYLOAD_SORT", "1")
    assert rows_of(as_cols(qx.execute(plan))) == rows_of(got)


@pytest.mark.gpu
def test_projection_join_and_errors(qx):
    a = pa.table({"a.id": np.arange(100, dtype=np.int64), "a.x": np.arange(100, dtype=np.int64) * 2})
    b = pa.table({"b.id": np.arange(0, 200, 2, dtype=np.int64), "b.name": [f"n{i}" for i in range(100)]})
    join = HashJoin(Scan(source(a)), Scan(source(b)), JoinType.Inner,
                    binop(Column("a.id", 0), BinaryOp.Equal, Column("b.id", 2)))
    plan = Projection(join, [Column("a.id", 0), binop(Column("a.x", 1), BinaryOp.Add, lit(1)), Column("b.name", 3)],
                      ["a.id", "?column?", "b.name"])
    out = qx.execute(plan)
    assert out[0].num_rows == 50
    assert out[0].column(2).to_pylist()[:3] == ["n0", "n1", "n2"]
    assert out[0].column(1).to_pylist()[:3] == [1, 5, 9]
    # reference error text (operators.rs:384-507): no arithmetic coercion
    import qe_hip
    bad = Projection(Scan(source(a)), [binop(Column("a.x", 1), BinaryOp.Multiply, lit(1.5))], ["y"])
    with pytest.raises(qe_hip.QehError, match="Unsupported types for multiplication"):
        qx.execute(bad)
    # cross join: left row-major Cartesian product (executor.rs:437-498)
    small = pa.table({"s.x": np.arange(3, dtype=np.int64)})
    out = qx.execute(HashJoin(Scan(source(small)), Scan(source(small)), JoinType.Cross, None))
    assert out[0].num_rows == 9
    # any empty side -> no batches (executor.rs:350-352)
    empty = MemoryDataSource(small.schema, [])
    assert qx.execute(HashJoin(Scan(source(small)), Scan(empty), JoinType.Inner,
                               binop(Column("s.x", 0), BinaryOp.Equal, Column("s.x", 1)))) == []


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["x_gt_49", "and_or", "not_b", "x_times_3_ne_i", "f_ge_v"])
def test_device_filter_matches_arrow_goldens(qx, name):
    """Device filter on the Arrow C++ golden vectors (tests/golden/filter.npz)."""
    from test_oracle_golden import COLS, PREDS
    z = np.load(os.path.join(GOLD, "filter.npz"), allow_pickle=False)
    arrays = {f"t.{c}": pa.array(z[f"in_{c}"], mask=~z[f"in_{c}__valid"]) for c in COLS}
    t = pa.table(arrays)
    out = qx.execute(Filter(Scan(source(t, 3)), PREDS[name]))
    want = [(z[f"{name}__{c}"], z[f"{name}__{c}__valid"]) for c in COLS]
    assert rows_of(as_cols(out)) == rows_of(want)


@pytest.mark.gpu
def test_device_scan_cache(ctx):
    """§8 f1: a DataSource with a cache key keeps its device columns between queries; results stay
    identical to the uncached import, insert() retires the stale copy, evict/budget drop entries."""
    qx = QueryExecutor(ctx)
    qx.cache_evict()
    fact, dim = metric_tables(200_000, 10_000, 128)
    plain = qx.execute(metric_plan(fact, dim, chunks=2))
    fsrc = MemoryDataSource(fact.schema, fact.to_batches(max_chunksize=70_000), device_cache=True)
    dsrc = MemoryDataSource(dim.schema, dim.to_batches(), device_cache=True)

    def plan():
        join = HashJoin(Scan(fsrc), Scan(dsrc), JoinType.Inner,
                        binop(Column("f.k", 1), BinaryOp.Equal, Column("d.k", 3)))
        filt = Filter(join, binop(Column("f.x", 0), BinaryOp.Greater, lit(49)))
        return HashAggregate(filt, [Column("d.g", 4)],
                             [AggregateExpr(AF.Sum, Column("f.v", 2)), AggregateExpr(AF.Count, Column("f.v", 2))])

    s0 = qx.cache_stats()
    first = qx.execute(plan())
    s1 = qx.cache_stats()
    assert s1["misses"] - s0["misses"] == 2 and s1["entries"] == 2
    assert s1["bytes"] == 200_000 * 24 + 10_000 * 16
    second = qx.execute(plan())
    s2 = qx.cache_stats()
    assert s2["hits"] - s1["hits"] == 2 and s2["misses"] == s1["misses"]
    for a in (first, second):
        assert_rows_equal(sorted_rows(as_cols(a)), sorted_rows(as_cols(plain)), float_cols=[1])

    # insert(): new key, so the next query imports the grown table
    extra = pa.table({"f.x": np.full(5, 99, np.int64), "f.k": np.asarray(dim.column(0))[:5],
                      "f.v": np.ones(5)}).to_batches()[0]
    fsrc.insert(extra)
    grown = qx.execute(plan())
    s3 = qx.cache_stats()
    assert s3["misses"] - s2["misses"] == 1
    want = qx.execute(HashAggregate(Filter(
        HashJoin(Scan(source(pa.concat_tables([fact, pa.Table.from_batches([extra])]))), Scan(source(dim)),
                 JoinType.Inner, binop(Column("f.k", 1), BinaryOp.Equal, Column("d.k", 3))),
        binop(Column("f.x", 0), BinaryOp.Greater, lit(49))), [Column("d.g", 4)],
        [AggregateExpr(AF.Sum, Column("f.v", 2)), AggregateExpr(AF.Count, Column("f.v", 2))]))
    assert_rows_equal(sorted_rows(as_cols(grown)), sorted_rows(as_cols(want)), float_cols=[1])

    qx.cache_evict(dsrc)
    assert qx.cache_stats()["entries"] == 2  # old fact key + new fact key
    qx.cache_budget(200_005 * 24)  # room for the newest fact copy only
    assert qx.cache_stats()["entries"] == 1
    qx.cache_evict()
    assert qx.cache_stats()["entries"] == 0 and qx.cache_stats()["bytes"] == 0
    qx.cache_budget(64 << 30)

    # nullable + string + bool columns through a cached scan
    t = pa.table({"t.s": pa.array(["a", None, "ccc", "dd"] * 50), "t.b": pa.array([True, False, None, True] * 50),
                  "t.i": pa.array([1, None, 3, 4] * 50, pa.int64())})
    ts = MemoryDataSource(t.schema, t.to_batches(max_chunksize=64), device_cache=True)
    p = Filter(Scan(ts), binop(Column("t.i", 2), BinaryOp.Greater, lit(1)))
    a, b = qx.execute(p), qx.execute(p)
    ref = qx.execute(Filter(Scan(source(t)), binop(Column("t.i", 2), BinaryOp.Greater, lit(1))))
    assert [x.to_pylist() for x in pa.Table.from_batches(a).columns] == \
        [x.to_pylist() for x in pa.Table.from_batches(b).columns] == \
        [x.to_pylist() for x in pa.Table.from_batches(ref).columns]
    assert qx.cache_stats()["hits"] >= 1
    qx.cache_evict()


def _arrow_rows(batches):
    if not batches:
        return []
    t = pa.Table.from_batches(batches)
    return list(zip(*[c.to_pylist() for c in t.columns])), t.schema.names


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["limit_filter", "limit_proj_filter", "proj_filter_expr", "limit_proj_expr",
                                   "limit_skip_past_end", "limit_zero"])
def test_fused_filter_projection_limit(qx, monkeypatch, shape):
    """§8 f1: Limit(Projection(Filter(Scan))) and its sub-shapes run as one capped filter over the
    projected columns; results equal the unfused chain (QEH_NO_FUSION) and the oracle filter."""
    r = np.random.default_rng(len(shape))
    n = 400_003
    t = pa.table({"t.x": pa.array(r.integers(0, 100, n), pa.int64()),
                  "t.s": pa.array([f"s{i % 977}" if i % 13 else None for i in range(n)]),
                  "t.v": pa.array(r.random(n), mask=r.random(n) < 0.1),
                  "t.b": pa.array(r.random(n) < 0.5),
                  "t.i": pa.array(r.integers(-(2 ** 20), 2 ** 20, n), pa.int64())})
    pred = binop(Column("t.x", 0), BinaryOp.Greater, lit(90))
    filt = Filter(Scan(source(t, 3)), pred)
    cols_proj = Projection(filt, [Column("t.i", 4), Column("t.s", 1), Column("t.b", 3), Column("t.v", 2)],
                           ["t.i", "t.s", "t.b", "t.v"])
    expr_proj = Projection(filt, [binop(Column("t.i", 4), BinaryOp.Add, Column("t.x", 0)), Column("t.s", 1)],
                           ["y", "t.s"])
    plan = {"limit_filter": Limit(filt, 17, 5000),
            "limit_proj_filter": Limit(cols_proj, 0, 1234),
            "proj_filter_expr": expr_proj,
            "limit_proj_expr": Limit(expr_proj, 3, 10),
            "limit_skip_past_end": Limit(cols_proj, 10 ** 8, 5),
            "limit_zero": Limit(filt, 0, 0)}[shape]
    fused = _arrow_rows(qx.execute(plan))
    monkeypatch.setenv("QEH_NO_FUSION", "1")
    plain = _arrow_rows(qx.execute(plan))
    assert fused == plain
    if shape == "limit_proj_filter":
        keep = np.nonzero(np.asarray(t.column(0)) > 90)[0][:1234]
        rows, names = fused
        assert names == ["t.i", "t.s", "t.b", "t.v"]
        assert [x[0] for x in rows] == np.asarray(t.column(4))[keep].tolist()
        assert [x[1] for x in rows] == [t.column(1)[int(i)].as_py() for i in keep]


@pytest.mark.gpu
@pytest.mark.parametrize("jt", ["Left", "Right", "Full"])
def test_outer_join_plans(qx, jt):
    """HashJoin{join_type: Left/Right/Full} through QueryExecutor (Utf8 payload included): rows ==
    the oracle's outer join; the NULL-filled side keeps its types; an empty side -> no batches
    (executor.rs:350-352)."""
    r = np.random.default_rng(3)
    a = pa.table({"a.id": pa.array(r.integers(0, 400, 3000), pa.int64(), mask=r.random(3000) < 0.05),
                  "a.s": pa.array([f"a{i}" for i in range(3000)])})
    b = pa.table({"b.id": pa.array(r.permutation(600)[:500], pa.int64()),
                  "b.x": pa.array(r.random(500)),
                  "b.t": pa.array([f"b{i}" if i % 5 else None for i in range(500)])})
    code = getattr(JoinType, jt)
    plan = HashJoin(Scan(source(a, 2)), Scan(source(b)), code, binop(Column("a.id", 0), BinaryOp.Equal, Column("b.id", 2)))
    out = qx.execute(plan)
    assert out[0].schema.names == ["a.id", "a.s", "b.id", "b.x", "b.t"]
    got = pa.Table.from_batches(out)
    got_rows = sorted(zip(*[c.to_pylist() for c in got.columns]), key=lambda t: tuple((x is None, x) for x in t))
    aid = ob.HostCol(*as_cols(a.to_batches())[0])
    bc = as_cols(b.to_batches())
    li, ri, n = ob.hash_join_outer({"Left": 1, "Right": 2, "Full": 3}[jt], aid,
                                   [aid, ob.HostCol(np.arange(3000, dtype=np.int64))],
                                   ob.HostCol(*bc[0]), [ob.HostCol(*bc[0]), ob.HostCol(*bc[1]),
                                                        ob.HostCol(np.arange(500, dtype=np.int64))])
    assert got.num_rows == n
    s_of_a, t_of_b = a.column(1).to_pylist(), b.column(2).to_pylist()
    want = []
    for i in range(n):
        ai = li[1][0][i] if li[1][1][i] else None
        bi = ri[2][0][i] if ri[2][1][i] else None
        want.append((int(li[0][0][i]) if li[0][1][i] else None, None if ai is None else s_of_a[ai],
                     int(ri[0][0][i]) if ri[0][1][i] else None, float(ri[1][0][i]) if ri[1][1][i] else None,
                     None if bi is None else t_of_b[bi]))
    want.sort(key=lambda t: tuple((x is None, x) for x in t))
    assert got_rows == want
    empty = MemoryDataSource(b.schema, [])
    assert qx.execute(HashJoin(Scan(source(a)), Scan(empty), code,
                               binop(Column("a.id", 0), BinaryOp.Equal, Column("b.id", 2)))) == []
    # build side of non-null 8-byte columns only: LEFT / RIGHT return the preserved side as views
    # of the scanned columns; the result must survive the inputs' release
    b2 = b.select(["b.id", "b.x"])
    plan2 = HashJoin(Scan(source(a, 2)), Scan(source(b2)), code,
                     binop(Column("a.id", 0), BinaryOp.Equal, Column("b.id", 2)))
    out2 = pa.Table.from_batches(qx.execute(plan2))
    got2 = sorted(zip(*[c.to_pylist() for c in out2.columns]), key=lambda t: tuple((x is None, x) for x in t))
    want2 = sorted([w[:4] for w in want], key=lambda t: tuple((x is None, x) for x in t))
    assert got2 == want2


@pytest.mark.gpu
def test_window_functions_through_the_plan(qx):
    """Window node with RANK / DENSE_RANK / NTILE(4) / LAG(w, 2, 0.5) / LAST_VALUE(v)
    (WindowFunctionType, physical_plan.rs:160-179) vs the oracle."""
    from qe_hip.plan import WindowFunctionType as W
    r = np.random.default_rng(11)
    n = 40_000
    k = pa.array(r.integers(0, 30, n), pa.int64(), mask=r.random(n) < 0.05)
    v = pa.array(r.integers(-10, 10, n), pa.int64())
    w = pa.array(r.random(n), mask=r.random(n) < 0.1)
    t = pa.table({"t.k": k, "t.v": v, "t.w": w})
    part, order = [Column("t.k", 0)], [Column("t.v", 1)]
    exprs = [WindowExpr(W.Rank, [], part, order), WindowExpr(W.DenseRank, [], part, order),
             WindowExpr(W.Ntile, [lit(4)], part, order), WindowExpr(W.Lag, [Column("t.w", 2), lit(2), lit(0.5)], part, order),
             WindowExpr(W.LastValue, [Column("t.v", 1)], part, order)]
    names = ["t.k", "t.v", "t.w", "rk", "drk", "q", "lag", "lv"]
    out = qx.execute(Window(Scan(source(t, 3)), exprs, names))
    assert out[0].schema.names == names
    cols = as_cols([t.to_batches()[0]])
    hk, hv, hw = ob.HostCol(*cols[0]), ob.HostCol(*cols[1]), ob.HostCol(*cols[2])
    assert np.array_equal(out[0].column(3).to_numpy(), ob.window(W.Rank, [hk], [hv], [True])[0])
    assert np.array_equal(out[0].column(4).to_numpy(), ob.window(W.DenseRank, [hk], [hv], [True])[0])
    assert np.array_equal(out[0].column(5).to_numpy(), ob.window(W.Ntile, [hk], [hv], [True], param=4)[0])
    lag_v, lag_ok = ob.window(W.Lag, [hk], [hv], [True], arg=hw, param=2, default=0.5)
    got = out[0].column(6)
    assert np.array_equal(got.is_valid().to_numpy(zero_copy_only=False), lag_ok)
    assert np.array_equal(got.to_numpy(zero_copy_only=False)[lag_ok], lag_v[lag_ok])
    assert np.array_equal(out[0].column(7).to_numpy(zero_copy_only=False), ob.window(W.LastValue, [hk], [hv], [True], arg=hv)[0])
