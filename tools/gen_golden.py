#!/usr/bin/env python3
"""Generate tests/golden/* fixtures (run in the build container only).

The reference (Rust + arrow-rs 53.4.1) cannot be built here, so golden outputs
for the arrow kernels the reference calls come from Arrow C++ (pyarrow 25),
which implements the same Arrow semantics for these kernels:
  cmp::{eq,neq,lt,lt_eq,gt,gt_eq}  -> pc.equal/.../greater_equal (null-propagating)
  compute::{and,or,not}            -> pc.and_/pc.or_/pc.invert   (non-Kleene)
  numeric::{add,sub,mul,div} ints  -> pc.add_checked/subtract_checked/multiply_checked/divide_checked
  filter_record_batch              -> pc.filter(null_selection_behavior="drop")
  compute::{sum,min,max}, count    -> pc.sum/min/max/count (non-overflowing data: pyarrow
                                      widens Int32 sums, arrow-rs wraps them)
Intended-semantics operators are pinned the same way:
  GROUP BY -> Table.group_by().aggregate();  INNER / LEFT / RIGHT / FULL JOIN -> Table.join(...);
  Sort     -> pc.sort_indices(null_placement="at_start") (stable);
  ROW_NUMBER -> numpy lexsort (no Arrow kernel; documented as numpy-pinned).
Config 1's known answer comes from the reference's own data/employees.csv
(SURVEY.md §8 row c), copied here as a data fixture.
Every fixture is an .npz written with allow_pickle=False.
"""
import json
import os
import shutil

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import pyarrow.csv as pacsv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden")
N = 4096


def col_arrays(arr: pa.Array):
    """values (nulls filled with 0) + validity."""
    valid = ~np.asarray(arr.is_null().to_numpy(zero_copy_only=False), bool)
    t = arr.type
    if pa.types.is_boolean(t):
        vals = np.asarray(arr.fill_null(False).to_numpy(zero_copy_only=False), bool)
    else:
        vals = np.asarray(arr.fill_null(0).to_numpy(zero_copy_only=False))
    return vals, valid


def base_table(seed=20251226):
    r = np.random.default_rng(seed)
    def nulls(p):
        return r.random(N) < p
    x = pa.array(r.integers(0, 100, N), pa.int64(), mask=nulls(0.1))
    i = pa.array(r.integers(-1000, 1000, N).astype(np.int32), pa.int32(), mask=nulls(0.15))
    v = pa.array(np.round(r.random(N), 6), pa.float64(), mask=nulls(0.12))
    f = pa.array(r.random(N).astype(np.float32), pa.float32(), mask=nulls(0.05))
    b = pa.array(r.random(N) > 0.5, pa.bool_(), mask=nulls(0.1))
    k = pa.array(r.integers(0, 37, N), pa.int64(), mask=nulls(0.05))
    return pa.table({"x": x, "i": i, "v": v, "f": f, "b": b, "k": k})


def save(name, **arrays):
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **arrays)


def put_table(prefix, t: pa.Table, d: dict):
    for name in t.column_names:
        vals, valid = col_arrays(t.column(name).combine_chunks())
        d[f"{prefix}{name}"] = vals
        d[f"{prefix}{name}__valid"] = valid


def main():
    os.makedirs(OUT, exist_ok=True)
    manifest = {"generator": "tools/gen_golden.py", "pyarrow": pa.__version__, "fixtures": {}}
    t = base_table()

    # ---- filter predicates (expression encodings are rebuilt by the tests from these names)
    preds = {
        "x_gt_49": pc.greater(t["x"], 49),
        "v_le_half": pc.less_equal(t["v"], 0.5),
        "i_lt_f64": pc.less(pc.cast(t["i"], pa.float64()), 12.5),
        "f_ge_v": pc.greater_equal(pc.cast(t["f"], pa.float64()), t["v"]),
        "and_or": pc.or_(pc.and_(pc.greater(t["x"], 20), pc.less(t["v"], 0.5)), pc.equal(t["i"], 7)),
        "not_b": pc.invert(t["b"]),
        "x_plus_x_gt_50": pc.greater(pc.add_checked(t["x"], t["x"]), 50),
        "x_times_3_ne_i": pc.not_equal(pc.multiply_checked(t["x"], 3), pc.cast(t["i"], pa.int64())),
    }
    d = {}
    put_table("in_", t, d)
    for name, mask in preds.items():
        ft = t.filter(mask, null_selection_behavior="drop")
        put_table(f"{name}__", ft, d)
        d[f"{name}__rows"] = np.array([ft.num_rows])
    save("filter", **d)
    manifest["fixtures"]["filter"] = {"rows": N, "predicates": list(preds)}

    # ---- global aggregates (evaluate_aggregate): non-overflowing data
    d = {}
    put_table("in_", t, d)
    for c in ["x", "v", "f", "i"]:
        a = t[c]
        d[f"{c}__count"] = np.array([pc.count(a).as_py()])
        d[f"{c}__sum"] = np.array([pc.sum(a).as_py()], dtype=np.float64 if c in ("v", "f") else np.int64)
        d[f"{c}__avg"] = np.array([pc.mean(a).as_py()])
        d[f"{c}__min"] = np.array([pc.min(a).as_py()])
        d[f"{c}__max"] = np.array([pc.max(a).as_py()])
    save("global_agg", **d)
    manifest["fixtures"]["global_agg"] = {"columns": ["x", "v", "f", "i"]}

    # ---- grouped aggregate (intended semantics)
    g = t.group_by(["k"], use_threads=False).aggregate(
        [("v", "sum"), ("v", "count"), ("v", "mean"), ("x", "min"), ("x", "max"), ("x", "sum")])
    d = {}
    put_table("in_", t, d)
    put_table("out_", g, d)
    save("group_agg", **d)
    manifest["fixtures"]["group_agg"] = {"groups": g.num_rows, "columns": g.column_names}

    # ---- inner join (intended semantics)
    r = np.random.default_rng(7)
    left = pa.table({"lk": pa.array(r.integers(0, 300, 3000), pa.int64(), mask=r.random(3000) < 0.05),
                     "lv": pa.array(r.random(3000))})
    right = pa.table({"rk": pa.array(r.integers(0, 250, 400), pa.int64(), mask=r.random(400) < 0.05),
                      "ra": pa.array(r.integers(-9, 9, 400), pa.int64())})
    j = left.join(right, keys="lk", right_keys="rk", join_type="inner", use_threads=False)
    j = j.select(["lk", "lv", "ra"])
    d = {}
    put_table("left_", left, d)
    put_table("right_", right, d)
    put_table("out_", j, d)
    save("join", **d)
    manifest["fixtures"]["join"] = {"rows": j.num_rows}

    # ---- LEFT / RIGHT / FULL outer joins on the same inputs (Arrow's hash join,
    # NULL keys never match, both key columns kept)
    for jt in ("left outer", "right outer", "full outer"):
        j = left.join(right, keys="lk", right_keys="rk", join_type=jt, use_threads=False, coalesce_keys=False)
        j = j.select(["lk", "lv", "rk", "ra"])
        d = {}
        put_table("out_", j, d)
        name = "join_" + jt.split()[0]
        save(name, **d)
        manifest["fixtures"][name] = {"rows": j.num_rows, "inputs": "join.npz left_/right_"}

    # ---- stable multi-key sort, nulls first
    keys = [("k", "ascending"), ("v", "descending"), ("x", "ascending")]
    idx = pc.sort_indices(t, sort_keys=keys, null_placement="at_start")
    d = {}
    put_table("in_", t, d)
    d["perm"] = np.asarray(idx.to_numpy(), np.uint32)
    save("sort", **d)
    manifest["fixtures"]["sort"] = {"keys": keys}

    # ---- Merge::sorted (distributed/operators.rs:143-193): three partitions concatenated, then
    # sorted with per-key descending / nulls_first (Arrow sort_indices is stable; the reference's
    # lexsort_to_indices may order ties either way)
    parts = [t.slice(0, 1000), t.slice(1000, 1500), t.slice(2500, N - 2500)]
    cat = pa.concat_tables(parts)
    mkeys = [("k", "descending", "at_end"), ("x", "ascending", "at_start"), ("v", "ascending", "at_end")]
    midx = pc.sort_indices(cat, sort_keys=mkeys)
    d = {"part_rows": np.array([p.num_rows for p in parts], np.int64)}
    put_table("in_", cat, d)
    d["perm"] = np.asarray(midx.to_numpy(), np.uint32)
    save("merge_sorted", **d)
    manifest["fixtures"]["merge_sorted"] = {"keys": mkeys, "parts": [p.num_rows for p in parts]}

    # ---- ROW_NUMBER() OVER (PARTITION BY k ORDER BY x) (numpy-pinned)
    kk, kv = col_arrays(t["k"].combine_chunks())
    xx, xv = col_arrays(t["x"].combine_chunks())
    # lexsort: last key primary. nulls first -> sort by valid flag before value
    order = np.lexsort((np.arange(N), xx, xv, kk, kv))
    rn = np.zeros(N, np.int64)
    prev = None
    cnt = 0
    for pos in order:
        key = (bool(kv[pos]), int(kk[pos]) if kv[pos] else 0)
        cnt = cnt + 1 if key == prev else 1
        prev = key
        rn[pos] = cnt
    d = {}
    put_table("in_", t, d)
    d["rn"] = rn
    save("row_number", **d)
    manifest["fixtures"]["row_number"] = {"partition_by": "k", "order_by": "x"}

    # ---- config 1: the reference's data/employees.csv and its known answer
    src = "/root/reference/data/employees.csv"
    dst = os.path.join(OUT, "employees.csv")
    if os.path.exists(src):
        shutil.copyfile(src, dst)
    emp = pacsv.read_csv(dst)
    ans = emp.filter(pc.greater(emp["age"], 25)).select(["name", "age"])
    manifest["fixtures"]["employees"] = {
        "query": "SELECT name,age FROM employees WHERE age>25",
        "schema": ["employees.name: Utf8", "employees.age: Int64"],
        "rows": [[n, a] for n, a in zip(ans["name"].to_pylist(), ans["age"].to_pylist())],
    }
    employees_departments(manifest)
    json.dump(manifest, open(os.path.join(OUT, "manifest.json"), "w"), indent=1)
    print(json.dumps(manifest["fixtures"]["employees"]))


# Known answers on the reference's own data/employees.csv and data/departments.csv, joined on dept_id:
# the only reference-held input that exercises the join and group-by operators.  The rows below were
# derived by hand from the two files (6 employees, Frank's dept_id is the literal text NULL -- read as a
# NULL, which never matches; read as the text "NULL" by a reader that keeps it, it equals no department
# id either, so the answer is the same; department 104 has no employee), then checked against
# pyarrow's hash join and group_by when this script runs.
EMP_DEPT = {
    "inner": {
        "query": "SELECT e.name, d.dept_name FROM employees e JOIN departments d ON e.dept_id = d.dept_id",
        "rows": [["Alice", "Engineering"], ["Bob", "Sales"], ["Charlie", "Engineering"], ["Diana", "HR"],
                 ["Eve", "Sales"]]},
    "left": {
        "query": "SELECT e.name, d.dept_name FROM employees e LEFT JOIN departments d ON e.dept_id = d.dept_id",
        "rows": [["Alice", "Engineering"], ["Bob", "Sales"], ["Charlie", "Engineering"], ["Diana", "HR"],
                 ["Eve", "Sales"], ["Frank", None]]},
    "right": {
        "query": "SELECT e.name, d.dept_name FROM employees e RIGHT JOIN departments d ON e.dept_id = d.dept_id",
        "rows": [["Alice", "Engineering"], ["Bob", "Sales"], ["Charlie", "Engineering"], ["Diana", "HR"],
                 ["Eve", "Sales"], [None, "Marketing"]]},
    "full": {
        "query": "SELECT e.name, d.dept_name FROM employees e FULL JOIN departments d ON e.dept_id = d.dept_id",
        "rows": [["Alice", "Engineering"], ["Bob", "Sales"], ["Charlie", "Engineering"], ["Diana", "HR"],
                 ["Eve", "Sales"], ["Frank", None], [None, "Marketing"]]},
    "group_by_dept": {
        "query": "SELECT dept_id, COUNT(salary), SUM(salary), AVG(salary) FROM employees GROUP BY dept_id",
        "rows": [[101, 2, 170000, 85000.0], [102, 2, 175000, 87500.0], [103, 1, 80000, 80000.0],
                 [None, 1, 78000, 78000.0]]},
    "join_filter_group_by": {
        "query": "SELECT d.dept_id, COUNT(e.salary), SUM(e.salary) FROM employees e JOIN departments d "
                 "ON e.dept_id = d.dept_id WHERE e.age > 25 GROUP BY d.dept_id",
        "rows": [[101, 1, 95000], [102, 2, 175000], [103, 1, 80000]]},
}


def employees_departments(manifest):
    src = "/root/reference/data/departments.csv"
    dst = os.path.join(OUT, "departments.csv")
    if os.path.exists(src):
        shutil.copyfile(src, dst)
    emp = pacsv.read_csv(os.path.join(OUT, "employees.csv"))
    dep = pacsv.read_csv(dst)
    def rows(t, cols):
        return sorted([list(r) for r in zip(*[t[c].to_pylist() for c in cols])], key=repr)
    for how, name in (("inner", "inner"), ("left outer", "left"), ("right outer", "right"), ("full outer", "full")):
        j = emp.join(dep, "dept_id", join_type=how)
        assert rows(j, ["name", "dept_name"]) == sorted(EMP_DEPT[name]["rows"], key=repr), name
    g = emp.group_by("dept_id").aggregate([("salary", "count"), ("salary", "sum"), ("salary", "mean")])
    assert rows(g, ["dept_id", "salary_count", "salary_sum", "salary_mean"]) == \
        sorted(EMP_DEPT["group_by_dept"]["rows"], key=repr)
    j = emp.filter(pc.greater(emp["age"], 25)).join(dep, "dept_id", join_type="inner")
    g = j.group_by("dept_id").aggregate([("salary", "count"), ("salary", "sum")])
    assert rows(g, ["dept_id", "salary_count", "salary_sum"]) == sorted(EMP_DEPT["join_filter_group_by"]["rows"], key=repr)
    manifest["fixtures"]["employees_departments"] = dict(EMP_DEPT, inputs=["employees.csv", "departments.csv"],
                                                         key="dept_id")


if __name__ == "__main__":
    main()
