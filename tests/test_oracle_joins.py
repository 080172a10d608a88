"""CPU-only pinning of the oracle's join restatements (no GPU):
  * the literal Cartesian joins the reference actually runs — join_batches
    (executor.rs:500-540: INNER/LEFT/RIGHT/FULL, left row-major) and execute_cross_join
    (executor.rs:437-498: right row-major) — against hand-derived known answers;
  * the one form of the metric query the reference answers correctly: Filter(f.k = d.k AND
    f.x > 49) over the literal Cartesian join, then a GLOBAL aggregate (executor.rs:131-188),
    against the oracle's intended-semantics hash join + aggregate;
  * qo_join_on (arbitrary `on`) against the hash joins and the Arrow join goldens;
  * the all-cores CPU baseline (qo_join_filter_aggregate_mt) against the 1-thread oracle.
"""
import os

import numpy as np
import pytest

import oracle_bind as ob
from helpers import assert_grouped_equal, rows_of, sorted_rows
from qe_hip import AggregateFunction as AF
from qe_hip import BinaryOp, abi, binop, col, lit

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_join_batches_known_answer_left_row_major():
    l = [ob.HostCol(np.array([1, 2], np.int64)), ob.HostCol(np.array([0.5, 1.5]))]
    r = [ob.HostCol(np.array([10, 20, 30], np.int64), np.array([1, 0, 1], bool))]
    cols, rows = ob.join_batches(l, r)
    assert rows == 6
    assert rows_of(cols) == [(1, 0.5, 10), (1, 0.5, None), (1, 0.5, 30),
                             (2, 1.5, 10), (2, 1.5, None), (2, 1.5, 30)]


def test_cross_join_known_answer_right_row_major():
    l = [ob.HostCol(np.array([1, 2], np.int64))]
    r = [ob.HostCol(np.array([10, 20, 30], np.int64))]
    cols, rows = ob.cross_join(l, r)
    assert rows == 6
    assert rows_of(cols) == [(1, 10), (2, 10), (1, 20), (2, 20), (1, 30), (2, 30)]


def test_cartesian_join_empty_side_has_no_batch():
    """executor.rs:350-352: either side empty -> no batches at all (even for outer joins)."""
    l = [ob.HostCol(np.array([1, 2], np.int64))]
    e = [ob.HostCol(np.zeros(0, np.int64))]
    assert ob.join_batches(l, e) == (None, -1)
    assert ob.cross_join(e, l) == (None, -1)


def metric_tables(seed, n=400, nd=150):
    r = np.random.default_rng(seed)
    x = r.integers(0, 100, n).astype(np.int64)
    k = r.integers(0, nd + 20, n).astype(np.int64)  # some fact keys miss the dim
    km = r.random(n) > 0.05
    v = r.random(n)
    vm = r.random(n) > 0.05
    dk = r.permutation(nd).astype(np.int64)
    dk[5] = dk[6]  # one duplicated dim key: its fact rows join twice
    dkm = r.random(nd) > 0.03
    dg = r.integers(0, 7, nd).astype(np.int64)
    return (x, None), (k, km), (v, vm), (dk, dkm), (dg, None)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_literal_metric_query_global_aggregate_equals_intended_join(seed):
    """SELECT SUM(f.v), COUNT(f.v) FROM fact f, dim d WHERE f.k = d.k AND f.x > 49 as the
    reference executes it: join_batches (Cartesian), execute_filter, global execute_aggregate
    (executor.rs:131-188) — equals the oracle's hash join + filter + aggregate with no group
    key, and the sum over the GROUP BY d.g groups of the intended query."""
    (x, _), (k, km), (v, vm), (dk, dkm), (dg, _) = metric_tables(seed)
    fact = [ob.HostCol(x), ob.HostCol(k, km), ob.HostCol(v, vm)]
    dim = [ob.HostCol(dk, dkm), ob.HostCol(dg)]
    cart, rows = ob.join_batches(fact, dim)
    assert rows == len(x) * len(dk)
    pred = binop(col(1), BinaryOp.Equal, col(3)) & binop(col(0), BinaryOp.Greater, lit(49))
    hc = [ob.HostCol(vals, m) for vals, m in cart]
    filt, frows, _ = ob.filter(hc, pred)
    _, lit_aggs, g, _ = ob.hash_aggregate([], [ob.HostCol(*c) for c in filt], [(AF.Sum, 2), (AF.Count, 2)])
    assert g == 1
    lit_sum, lit_cnt = lit_aggs[0][0][0], lit_aggs[1][0][0]
    # intended semantics, no group key
    _, ia, ig = ob.join_filter_aggregate(fact, 1, binop(col(0), BinaryOp.Greater, lit(49)), dim[0], [],
                                         [(AF.Sum, 2), (AF.Count, 2)])
    assert ig == 1
    assert ia[1][0][0] == lit_cnt
    assert ia[0][0][0] == pytest.approx(lit_sum, rel=1e-12)
    # grouped form: the per-group totals add up to the global answer
    gk, ga, gg = ob.join_filter_aggregate(fact, 1, binop(col(0), BinaryOp.Greater, lit(49)), dim[0], [dim[1]],
                                          [(AF.Sum, 2), (AF.Count, 2)])
    assert int(ga[1][0].sum()) == lit_cnt
    assert float(ga[0][0][ga[0][1]].sum()) == pytest.approx(lit_sum, rel=1e-12)
    # and the filtered Cartesian rows are exactly the intended inner join's rows
    p, b, jrows = ob.hash_join_inner(fact[1], fact, dim[0], dim)
    jsel = [c for c in p + b]
    keep = jsel[0][0] > 49
    want = [(vals[keep], m[keep]) for vals, m in jsel]
    assert sorted_rows(filt) == sorted_rows(want)


def load(name):
    return np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)


@pytest.mark.parametrize("jt,code", [("inner", 0), ("left", 1), ("right", 2), ("full", 3)])
def test_join_on_equi_matches_arrow_goldens(jt, code):
    """qo_join_on with on = l.lk = r.rk reproduces Arrow's hash joins (tests/golden/join*.npz)."""
    z = load("join")
    lk, lkv, lv, lvv = z["left_lk"], z["left_lk__valid"], z["left_lv"], z["left_lv__valid"]
    rk, rkv, ra, rav = z["right_rk"], z["right_rk__valid"], z["right_ra"], z["right_ra__valid"]
    left = [ob.HostCol(lk, lkv), ob.HostCol(lv, lvv)]
    right = [ob.HostCol(rk, rkv), ob.HostCol(ra, rav)]
    lo, ro, rows = ob.join_on(code, left, right, binop(col(0), BinaryOp.Equal, col(2)))
    if jt == "inner":
        want = [(z[f"out_{c}"], z[f"out_{c}__valid"]) for c in ["lk", "lv", "ra"]]
        got = lo + ro[1:]
    else:
        g = load("join_" + jt)
        want = [(g[f"out_{c}"], g[f"out_{c}__valid"]) for c in ["lk", "lv", "rk", "ra"]]
        got = lo + ro
    assert rows == len(want[0][0])
    assert sorted_rows(got) == sorted_rows(want)


def test_join_on_residual_and_non_equi_known_answers():
    lk = ob.HostCol(np.array([1, 2, 2, 3], np.int64))
    lx = ob.HostCol(np.array([5, 1, 9, 4], np.int64))
    rk = ob.HostCol(np.array([2, 1, 2, 7], np.int64))
    ry = ob.HostCol(np.array([3, 0, 8, 1], np.int64))
    # equi + residual: l.k = r.k AND l.x > r.y
    on = binop(col(0), BinaryOp.Equal, col(2)) & binop(col(1), BinaryOp.Greater, col(3))
    lo, ro, n = ob.join_on(0, [lk, lx], [rk, ry], on)
    assert rows_of(lo + ro) == [(1, 5, 1, 0), (2, 9, 2, 3), (2, 9, 2, 8)]
    lo, ro, n = ob.join_on(1, [lk, lx], [rk, ry], on)  # LEFT: unmatched left rows in place
    assert rows_of(lo + ro) == [(1, 5, 1, 0), (2, 1, None, None), (2, 9, 2, 3), (2, 9, 2, 8),
                                (3, 4, None, None)]
    lo, ro, n = ob.join_on(2, [lk, lx], [rk, ry], on)  # RIGHT: right-row order
    assert rows_of(lo + ro) == [(2, 9, 2, 3), (1, 5, 1, 0), (2, 9, 2, 8), (None, None, 7, 1)]
    # pure non-equi: l.x < r.y
    lo, ro, n = ob.join_on(3, [lk, lx], [rk, ry], binop(col(1), BinaryOp.Less, col(3)))
    assert rows_of(lo + ro) == [(1, 5, 2, 8), (2, 1, 2, 3), (2, 1, 2, 8), (2, 9, None, None), (3, 4, 2, 8),
                                (None, None, 1, 0), (None, None, 7, 1)]


@pytest.mark.parametrize("threads", [1, 4])
def test_all_cores_baseline_matches_oracle(threads):
    n, nd = 300_000, 20_000
    x = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 1, n, 100)
    k = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 2, n, nd + 500)
    v = ob.generate(abi.GEN_UNIT_F64, 0x5EED, 3, n)
    dk = ob.generate(abi.GEN_PERMUTATION, 0x5EED, 0, nd, nd)
    dk[7] = dk[8]  # a duplicate build key
    dg = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 5, nd, 300)
    pred = binop(col(0), BinaryOp.Greater, lit(49))
    aggs = [(AF.Sum, 2), (AF.Count, 2), (AF.Min, 0), (AF.Max, 2)]
    fact = [ob.HostCol(x), ob.HostCol(k), ob.HostCol(v)]
    wk, wa, wg = ob.join_filter_aggregate(fact, 1, pred, ob.HostCol(dk), [ob.HostCol(dg)], aggs)
    gk, ga, g = ob.join_filter_aggregate_mt(fact, 1, pred, ob.HostCol(dk), [ob.HostCol(dg)], aggs, threads)
    assert g == wg
    assert_grouped_equal(gk, ga, wk, wa, float_aggs=[0])
