"""Pin the CPU oracle before trusting it (CPU-only, no GPU):
  * against golden vectors produced by Arrow C++ (pyarrow) for the arrow-rs
    kernels the reference calls (tools/gen_golden.py, tests/golden/*.npz);
  * against the reference's own known answers: config 1 on data/employees.csv
    and distributed/operators.rs:343-374 (sorted merge [3,1],[4,2] -> [1,2,3,4]).
"""
import json
import os

import numpy as np
import pytest

import oracle_bind as ob
from helpers import assert_grouped_equal, rows_of, sorted_rows
from qe_hip import AggregateFunction as AF
from qe_hip import BinaryOp, UnaryExpr, UnaryOp, abi, binop, col, lit

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
COLS = ["x", "i", "v", "f", "b", "k"]

PREDS = {
    "x_gt_49": binop(col(0), BinaryOp.Greater, lit(49)),
    "v_le_half": binop(col(2), BinaryOp.LessEqual, lit(0.5)),
    "i_lt_f64": binop(col(1), BinaryOp.Less, lit(12.5)),
    "f_ge_v": binop(col(3), BinaryOp.GreaterEqual, col(2)),
    "and_or": (binop(col(0), BinaryOp.Greater, lit(20)) & binop(col(2), BinaryOp.Less, lit(0.5)))
              | binop(col(1), BinaryOp.Equal, lit(7)),
    "not_b": UnaryExpr(UnaryOp.Not, col(4)),
    "x_plus_x_gt_50": binop(binop(col(0), BinaryOp.Add, col(0)), BinaryOp.Greater, lit(50)),
    "x_times_3_ne_i": binop(binop(col(0), BinaryOp.Multiply, lit(3)), BinaryOp.NotEqual, col(1)),
}


def load(name):
    return np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)


def cols_of(z, prefix, names):
    return [(z[f"{prefix}{n}"], z[f"{prefix}{n}__valid"]) for n in names]


def golden_inputs(z):
    return [ob.HostCol(v, m) for v, m in cols_of(z, "in_", COLS)]


@pytest.mark.parametrize("name", sorted(PREDS))
def test_oracle_filter_matches_arrow(name):
    z = load("filter")
    got, rows, _ = ob.filter(golden_inputs(z), PREDS[name])
    assert rows == int(z[f"{name}__rows"][0])
    want = cols_of(z, f"{name}__", COLS)
    assert rows_of(got) == rows_of(want)  # same rows, same order


def test_oracle_global_aggregates_match_arrow():
    z = load("global_agg")
    inputs = golden_inputs(z)
    for c in ["x", "v", "f", "i"]:
        j = COLS.index(c)
        aggs = [(AF.Count, j), (AF.Sum, j), (AF.Avg, j), (AF.Min, j), (AF.Max, j)]
        _, out, g, _ = ob.hash_aggregate([], inputs, aggs)
        assert g == 1
        vals = [o[0][0] for o in out]
        assert vals[0] == z[f"{c}__count"][0]
        rtol = 1e-4 if c == "f" else 1e-12  # Float32 SUM accumulates in f32 (arrow-rs and the oracle)
        assert vals[1] == pytest.approx(z[f"{c}__sum"][0], rel=rtol)
        assert vals[2] == pytest.approx(z[f"{c}__avg"][0], rel=rtol)
        assert vals[3] == z[f"{c}__min"][0] and vals[4] == z[f"{c}__max"][0]


def test_oracle_global_aggregate_no_batches_quirk():
    """executor.rs:178-186: no input batches -> no output row at all."""
    z = load("global_agg")
    k, a, g, _ = ob.hash_aggregate([], golden_inputs(z), [(AF.Count, 0)], input_batches=0)
    assert g == 0


def test_oracle_group_by_matches_arrow():
    z = load("group_agg")
    inputs = golden_inputs(z)
    aggs = [(AF.Sum, 2), (AF.Count, 2), (AF.Avg, 2), (AF.Min, 0), (AF.Max, 0), (AF.Sum, 0)]
    keys, out, g, _ = ob.hash_aggregate([inputs[5]], inputs, aggs)
    want_k = cols_of(z, "out_", ["k"])
    want_a = cols_of(z, "out_", ["v_sum", "v_count", "v_mean", "x_min", "x_max", "x_sum"])
    assert g == len(want_k[0][0])
    assert_grouped_equal(keys, out, want_k, want_a, float_aggs=[0, 2], rtol=1e-12)


def test_oracle_inner_join_matches_arrow():
    z = load("join")
    (lk, lkv), (lv, lvv) = cols_of(z, "left_", ["lk", "lv"])
    (rk, rkv), (ra, rav) = cols_of(z, "right_", ["rk", "ra"])
    p, b, rows = ob.hash_join_inner(ob.HostCol(lk, lkv), [ob.HostCol(lk, lkv), ob.HostCol(lv, lvv)],
                                    ob.HostCol(rk, rkv), [ob.HostCol(ra, rav)])
    want = cols_of(z, "out_", ["lk", "lv", "ra"])
    assert rows == len(want[0][0])
    assert sorted_rows(p + b) == sorted_rows(want)


@pytest.mark.parametrize("jt", ["left", "right", "full"])
def test_oracle_outer_join_matches_arrow(jt):
    """LEFT / RIGHT / FULL joins: the oracle's rows == Arrow's hash join (tests/golden/join_*.npz),
    NULL-filled sides included, as multisets."""
    z = load("join")
    (lk, lkv), (lv, lvv) = cols_of(z, "left_", ["lk", "lv"])
    (rk, rkv), (ra, rav) = cols_of(z, "right_", ["rk", "ra"])
    code = {"left": 1, "right": 2, "full": 3}[jt]
    lo, ro, rows = ob.hash_join_outer(code, ob.HostCol(lk, lkv), [ob.HostCol(lk, lkv), ob.HostCol(lv, lvv)],
                                      ob.HostCol(rk, rkv), [ob.HostCol(rk, rkv), ob.HostCol(ra, rav)])
    want = cols_of(load("join_" + jt), "out_", ["lk", "lv", "rk", "ra"])
    assert rows == len(want[0][0])
    assert sorted_rows(lo + ro) == sorted_rows(want)


def test_oracle_outer_join_known_answer():
    """Hand-derived: left keys [1, 2, 2, NULL, 5], right keys [2, 3, NULL, 2, 1]."""
    lk = ob.HostCol(np.array([1, 2, 2, 0, 5], np.int64), np.array([1, 1, 1, 0, 1], bool))
    rk = ob.HostCol(np.array([2, 3, 0, 2, 1], np.int64), np.array([1, 1, 0, 1, 1], bool))
    li = ob.HostCol(np.arange(5, dtype=np.int64))
    ri = ob.HostCol(np.arange(10, 15, dtype=np.int64))
    pairs = {}
    for code in (1, 2, 3):
        lo, ro, n = ob.hash_join_outer(code, lk, [li], rk, [ri])
        pairs[code] = sorted_rows(lo + ro)
    inner = [(0, 14), (1, 10), (1, 13), (2, 10), (2, 13)]
    assert pairs[1] == sorted_rows_of(inner + [(3, None), (4, None)])
    assert pairs[2] == sorted_rows_of(inner + [(None, 11), (None, 12)])
    assert pairs[3] == sorted_rows_of(inner + [(3, None), (4, None), (None, 11), (None, 12)])


def sorted_rows_of(rows):
    from helpers import _key
    return sorted(rows, key=_key)


MERGE_KEYS = [("k", False, False), ("x", True, True), ("v", True, False)]  # (column, ascending, nulls_first)


def test_oracle_merge_sorted_matches_arrow():
    """Merge::sorted's ordering (distributed/operators.rs:143-193) with per-key nulls_first:
    the oracle's stable lexsort == Arrow's sort_indices on tests/golden/merge_sorted.npz."""
    z = load("merge_sorted")
    cols = dict(zip([c for c, _, _ in MERGE_KEYS], cols_of(z, "in_", [c for c, _, _ in MERGE_KEYS])))
    perm = ob.sort_indices_nulls([ob.HostCol(*cols[c]) for c, _, _ in MERGE_KEYS], [a for _, a, _ in MERGE_KEYS],
                                 [nf for _, _, nf in MERGE_KEYS])
    assert np.array_equal(perm, z["perm"])


def test_oracle_sort_matches_arrow():
    z = load("sort")
    inputs = golden_inputs(z)
    perm = ob.sort_indices([inputs[5], inputs[2], inputs[0]], [True, False, True])
    assert np.array_equal(perm, z["perm"])


def test_oracle_row_number_matches_numpy():
    z = load("row_number")
    inputs = golden_inputs(z)
    rn = ob.row_number([inputs[5]], [inputs[0]], [True])
    assert np.array_equal(rn, z["rn"])


def test_oracle_config1_employees_known_answer():
    """SELECT name,age FROM employees WHERE age>25 (BASELINE config 1): the
    filter runs on the age column; names ride along by row index."""
    man = json.load(open(os.path.join(GOLD, "manifest.json")))
    want = [tuple(r) for r in man["fixtures"]["employees"]["rows"]]
    lines = open(os.path.join(GOLD, "employees.csv")).read().strip().splitlines()[1:]
    names = [ln.split(",")[1] for ln in lines]
    age = np.array([int(ln.split(",")[2]) for ln in lines], np.int64)
    rowid = np.arange(len(lines), dtype=np.int64)
    got, rows, _ = ob.filter([ob.HostCol(rowid), ob.HostCol(age)], binop(col(1), BinaryOp.Greater, lit(25)))
    assert [(names[i], int(a)) for i, a in zip(got[0][0], got[1][0])] == want
    assert want == [("Bob", 30), ("Charlie", 35), ("Diana", 28), ("Eve", 32), ("Frank", 29)]


def test_oracle_sorted_merge_known_answer():
    """distributed/operators.rs:343-374: merge of [3,1] and [4,2] sorted -> [1,2,3,4]."""
    v = np.array([3, 1, 4, 2], np.int64)
    perm = ob.sort_indices([ob.HostCol(v)], [True])
    assert v[perm].tolist() == [1, 2, 3, 4]


def test_oracle_generator_is_deterministic_and_bijective():
    a = ob.generate(abi.GEN_PERMUTATION, 0x5EED, 0, 1_000_000, 1_000_000)
    assert np.array_equal(np.sort(a), np.arange(1_000_000))
    x1 = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 1, 1000, 100, row0=500)
    x2 = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 1, 1500, 100)
    assert np.array_equal(x1, x2[500:])
    v = ob.generate(abi.GEN_UNIT_F64, 0x5EED, 3, 100_000)
    assert v.min() >= 0.0 and v.max() < 1.0


def test_oracle_errors_mirror_reference_messages():
    x = ob.HostCol(np.array([1, 2, 3], np.int64))
    f = ob.HostCol(np.array([1.0, 2.0, 3.0]))
    with pytest.raises(ob.OracleError, match="Unsupported types for addition"):
        ob.eval_expr([x, f], binop(col(0), BinaryOp.Add, col(1)), 3)
    with pytest.raises(ob.OracleError, match="Filter predicate must return boolean"):
        ob.filter([x], binop(col(0), BinaryOp.Add, lit(1)))
    with pytest.raises(ob.OracleError, match="Arithmetic overflow"):
        ob.eval_expr([ob.HostCol(np.array([2 ** 62], np.int64))], binop(col(0), BinaryOp.Multiply, lit(4)), 1)
    with pytest.raises(ob.OracleError, match="Divide by zero"):
        ob.eval_expr([x], binop(col(0), BinaryOp.Divide, lit(0)), 3)
    (v, m), _ = ob.eval_expr([x], binop(col(0), BinaryOp.Modulo, lit(0)), 3)
    assert not m.any()  # operators.rs:711-743: % 0 -> NULL
