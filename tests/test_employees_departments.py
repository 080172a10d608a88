"""Known answers on the reference's own data: data/employees.csv joined with data/departments.csv on
dept_id (copied as data fixtures, tests/golden/; answers derived by hand, manifest.json
"employees_departments", checked against pyarrow by tools/gen_golden.py).  The only reference-held
input that exercises the join and group-by operators (HashJoinExec / HashAggregateExec,
executor.rs:157-190, 363-435): Frank's dept_id is the literal NULL and must match nothing, department
104 has no employee.

CPU: the oracle's intended-semantics join / outer join / group-by / join + filter + group-by against
the fixture.  GPU: the same queries as PhysicalPlans through qeh_execute_plan (QueryExecutor), plans
built the way the reference's converters build them (column indices over the concatenation of the
table-prefixed schemas: employees 0-4, departments 5-8)."""
import json
import os

import numpy as np
import pyarrow as pa
import pyarrow.csv as pacsv
import pytest

import oracle_bind as ob
from qe_hip import AggregateExpr, AggregateFunction as AF, BinaryOp, binop, lit
from qe_hip import Filter, HashAggregate, HashJoin, JoinType, MemoryDataSource, Projection, QueryExecutor, Scan
from qe_hip.expr import Column

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIX = json.load(open(os.path.join(GOLD, "manifest.json")))["fixtures"]["employees_departments"]


def tables():
    emp = pacsv.read_csv(os.path.join(GOLD, "employees.csv"))  # "NULL" is read as a NULL
    dep = pacsv.read_csv(os.path.join(GOLD, "departments.csv"))
    return emp, dep


def norm(rows):
    return sorted([tuple(r) for r in rows], key=repr)


def arr(t, name):
    a = t[name].combine_chunks()
    valid = ~np.asarray(a.is_null().to_numpy(zero_copy_only=False), bool)
    return np.asarray(a.fill_null(0).to_numpy(zero_copy_only=False)).astype(np.int64), valid


# ---- the oracle (CPU) -------------------------------------------------------------------------

@pytest.mark.parametrize("kind", ["inner", "left", "right", "full"])
def test_oracle_join_known_answer(kind):
    emp, dep = tables()
    ek, em = arr(emp, "dept_id")
    dk, dm = arr(dep, "dept_id")
    eid = np.arange(emp.num_rows, dtype=np.int64)  # row ids as payloads, mapped to names below
    did = np.arange(dep.num_rows, dtype=np.int64)
    if kind == "inner":
        (le,), (ld,), rows = ob.hash_join_inner(ob.HostCol(ek, em), [ob.HostCol(eid)], ob.HostCol(dk, dm),
                                                [ob.HostCol(did)])
    else:
        jt = {"left": 1, "right": 2, "full": 3}[kind]
        (le,), (ld,), rows = ob.hash_join_outer(jt, ob.HostCol(ek, em), [ob.HostCol(eid)], ob.HostCol(dk, dm),
                                                [ob.HostCol(did)])
    names, dnames = emp["name"].to_pylist(), dep["dept_name"].to_pylist()
    got = [(names[a] if va else None, dnames[b] if vb else None) for a, va, b, vb in zip(le[0], le[1], ld[0], ld[1])]
    assert rows == len(FIX[kind]["rows"])
    assert norm(got) == norm(FIX[kind]["rows"])


def test_oracle_group_by_known_answer():
    emp, _ = tables()
    k, km = arr(emp, "dept_id")
    s, sm = arr(emp, "salary")
    keys, aggs, g, _ = ob.hash_aggregate([ob.HostCol(k, km)], [ob.HostCol(s, sm)],
                                         [(AF.Count, 0), (AF.Sum, 0), (AF.Avg, 0)])
    got = [(int(kv) if kvld else None, int(c), int(sv), float(av))
           for kv, kvld, c, sv, av in zip(keys[0][0], keys[0][1], aggs[0][0], aggs[1][0], aggs[2][0])]
    assert g == 4
    assert norm(got) == norm(FIX["group_by_dept"]["rows"])


def test_oracle_join_filter_group_by_known_answer():
    emp, dep = tables()
    cols = [ob.HostCol(*arr(emp, c)) for c in ("age", "dept_id", "salary")]
    pred = binop(Column("e.age", 0), BinaryOp.Greater, lit(25))
    keys, aggs, g = ob.join_filter_aggregate(cols, 1, pred, ob.HostCol(*arr(dep, "dept_id")),
                                             [ob.HostCol(*arr(dep, "dept_id"))], [(AF.Count, 2), (AF.Sum, 2)])
    got = [(int(a), int(b), int(c)) for a, b, c in zip(keys[0][0], aggs[0][0], aggs[1][0])]
    assert g == 3
    assert norm(got) == norm(FIX["join_filter_group_by"]["rows"])


# ---- the device, through the plan executor ------------------------------------------------------

def sources():
    emp, dep = tables()
    emp = emp.rename_columns([f"employees.{c}" for c in emp.column_names])
    dep = dep.rename_columns([f"departments.{c}" for c in dep.column_names])
    return (MemoryDataSource(emp.schema, emp.to_batches()), MemoryDataSource(dep.schema, dep.to_batches()))


ON = binop(Column("employees.dept_id", 4), BinaryOp.Equal, Column("departments.dept_id", 5))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["inner", "left", "right", "full"])
def test_device_join_known_answer(ctx, kind):
    es, ds = sources()
    jt = {"inner": JoinType.Inner, "left": JoinType.Left, "right": JoinType.Right, "full": JoinType.Full}[kind]
    plan = Projection(HashJoin(Scan(es), Scan(ds), jt, ON),
                      [Column("employees.name", 1), Column("departments.dept_name", 6)],
                      ["employees.name", "departments.dept_name"])
    out = QueryExecutor(ctx).execute(plan)
    t = pa.Table.from_batches(out)
    got = list(zip(t.column(0).to_pylist(), t.column(1).to_pylist()))
    assert norm(got) == norm(FIX[kind]["rows"])


@pytest.mark.gpu
def test_device_group_by_known_answer(ctx):
    es, _ = sources()
    s = Column("employees.salary", 3)
    plan = HashAggregate(Scan(es), [Column("employees.dept_id", 4)],
                         [AggregateExpr(AF.Count, s), AggregateExpr(AF.Sum, s), AggregateExpr(AF.Avg, s)])
    t = pa.Table.from_batches(QueryExecutor(ctx).execute(plan))
    got = list(zip(*[t.column(i).to_pylist() for i in range(4)]))
    assert norm(got) == norm(FIX["group_by_dept"]["rows"])


@pytest.mark.gpu
def test_device_join_filter_group_by_known_answer(ctx):
    """The metric query's shape (HashAggregate(Filter(HashJoin))) on the reference's data."""
    es, ds = sources()
    join = HashJoin(Scan(es), Scan(ds), JoinType.Inner, ON)
    filt = Filter(join, binop(Column("employees.age", 2), BinaryOp.Greater, lit(25)))
    s = Column("employees.salary", 3)
    plan = HashAggregate(filt, [Column("departments.dept_id", 5)], [AggregateExpr(AF.Count, s), AggregateExpr(AF.Sum, s)])
    t = pa.Table.from_batches(QueryExecutor(ctx).execute(plan))
    got = list(zip(*[t.column(i).to_pylist() for i in range(3)]))
    assert norm(got) == norm(FIX["join_filter_group_by"]["rows"])
