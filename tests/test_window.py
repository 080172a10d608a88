"""RANK / DENSE_RANK / NTILE / LAG / LEAD / FIRST_VALUE / LAST_VALUE (`WindowFunctionType`,
physical_plan.rs:160-170) on the device through qeh_window vs the CPU oracle (qo_window).

The reference executor passes Window through (executor.rs:76-80), so there is no reference
output to pin against: the oracle follows docs/WINDOW_FUNCTIONS.md and is pinned by the doc's
own worked examples (test_oracle_doc_examples, CPU).  Everything else is parity with the oracle,
bit-exact (integer results and copied value bits)."""
import numpy as np
import pytest

import oracle_bind as ob
from qe_hip.plan import WindowFunctionType as W

RANKING = [W.RowNumber, W.Rank, W.DenseRank, W.Ntile]
VALUE = [W.Lag, W.Lead, W.FirstValue, W.LastValue]


def test_oracle_doc_examples():
    """docs/WINDOW_FUNCTIONS.md:44-137: ORDER BY salary DESC over Alice 60000, Charlie 80000,
    Diana 90000, Eve 80000 (RANK/DENSE_RANK tie example), and NTILE(4) over four salaries."""
    sal = np.array([60000, 80000, 90000, 80000], np.int64)  # Alice, Charlie, Diana, Eve
    rank, _ = ob.window(W.Rank, [], [ob.HostCol(sal)], [False])
    dense, _ = ob.window(W.DenseRank, [], [ob.HostCol(sal)], [False])
    assert rank.tolist() == [4, 2, 1, 2]     # Diana 1, Charlie 2, Eve 2, Alice 4 (skips 3)
    assert dense.tolist() == [3, 2, 1, 2]    # no gap
    sal4 = np.array([60000, 70000, 80000, 90000], np.int64)  # Alice, Bob, Charlie, Diana
    nt, _ = ob.window(W.Ntile, [], [ob.HostCol(sal4)], [False], param=4)
    assert nt.tolist() == [4, 3, 2, 1]
    # LAG(sales, 1) OVER (ORDER BY date): first row has no predecessor -> NULL (:139-160)
    sales = np.array([100.0, 150.0, 120.0])
    date = np.array([1, 2, 3], np.int64)
    lag, ok = ob.window(W.Lag, [], [ob.HostCol(date)], [True], arg=ob.HostCol(sales), param=1)
    assert ok.tolist() == [False, True, True] and lag[1:].tolist() == [100.0, 150.0]
    lead, ok = ob.window(W.Lead, [], [ob.HostCol(date)], [True], arg=ob.HostCol(sales), param=1)
    assert ok.tolist() == [True, True, False] and lead[:2].tolist() == [150.0, 120.0]
    # FIRST_VALUE(salary) OVER (PARTITION BY department ORDER BY salary DESC) (:177-190)
    dept = np.array([1, 2, 1, 2, 1], np.int64)
    s = np.array([10, 40, 30, 20, 30], np.int64)
    fv, _ = ob.window(W.FirstValue, [ob.HostCol(dept)], [ob.HostCol(s)], [False], arg=ob.HostCol(s))
    assert fv.tolist() == [30, 40, 30, 40, 30]
    lv, _ = ob.window(W.LastValue, [ob.HostCol(dept)], [ob.HostCol(s)], [True], arg=ob.HostCol(s))
    assert lv.tolist() == [30, 40, 30, 40, 30]  # whole-partition frame: the max


def test_oracle_ntile_uneven_and_small():
    k = np.zeros(10, np.int64)
    v = np.arange(10, dtype=np.int64)
    nt, _ = ob.window(W.Ntile, [ob.HostCol(k)], [ob.HostCol(v)], [True], param=4)
    assert nt.tolist() == [1, 1, 1, 2, 2, 2, 3, 3, 4, 4]  # 10 = 3 + 3 + 2 + 2
    nt, _ = ob.window(W.Ntile, [ob.HostCol(k[:3])], [ob.HostCol(v[:3])], [True], param=5)
    assert nt.tolist() == [1, 2, 3]


def _data(n, parts, seed, nulls):
    r = np.random.default_rng(seed)
    k = r.integers(0, parts, n).astype(np.int64)
    v = r.integers(-20, 20, n).astype(np.int64)  # many ties
    a = r.normal(size=n)
    km = vm = am = None
    if nulls:
        km, vm, am = (r.random(n) > 0.05), (r.random(n) > 0.1), (r.random(n) > 0.2)
    return k, km, v, vm, a, am


def _check(ctx, func, k, km, v, vm, a, am, asc=True, param=0, default=None, arg_dtype=None):
    arg_h = ob.HostCol(a.astype(arg_dtype) if arg_dtype else a, am)
    arg_d = ctx.upload(arg_h.values, am)
    got = ctx.window(func, [ctx.upload(k, km)], [ctx.upload(v, vm)], [asc],
                     arg=arg_d if func in VALUE else None, param=param, default=default).to_numpy()
    want_v, want_ok = ob.window(func, [ob.HostCol(k, km)], [ob.HostCol(v, vm)], [asc],
                                arg=arg_h if func in VALUE else None, param=param, default=default)
    gv, gm = got
    if func in RANKING:
        assert gm is None or gm.all()
        assert np.array_equal(gv, want_v)
    else:
        gm = np.ones(len(gv), bool) if gm is None else gm
        assert np.array_equal(gm, want_ok)
        assert np.array_equal(gv[gm].view(np.uint8), want_v[want_ok].view(np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("func", [W.Rank, W.DenseRank])
@pytest.mark.parametrize("n,parts,nulls", [(0, 3, False), (1, 1, False), (5000, 7, True), (1_000_000, 1000, False)])
def test_rank_dense_rank(ctx, func, n, parts, nulls):
    _check(ctx, func, *_data(n, parts, n + parts, nulls))
    _check(ctx, func, *_data(n, parts, n + 1, nulls), asc=False)


@pytest.mark.gpu
@pytest.mark.parametrize("buckets", [1, 3, 4, 1000])
@pytest.mark.parametrize("n,parts", [(1, 1), (9999, 13), (300_000, 50)])
def test_ntile(ctx, buckets, n, parts):
    _check(ctx, W.Ntile, *_data(n, parts, n + buckets, True), param=buckets)


@pytest.mark.gpu
@pytest.mark.parametrize("func", [W.Lag, W.Lead])
@pytest.mark.parametrize("offset", [0, 1, 3, 100])
def test_lag_lead(ctx, func, offset):
    d = _data(20_000, 31, offset, True)
    _check(ctx, func, *d, param=offset)
    _check(ctx, func, *d, param=offset, default=-1.5)  # default where the offset leaves the partition
    _check(ctx, func, *d, param=offset, arg_dtype=np.int32, default=7)
    _check(ctx, func, *d, param=offset, arg_dtype=np.float32, asc=False)


@pytest.mark.gpu
@pytest.mark.parametrize("func", [W.FirstValue, W.LastValue])
@pytest.mark.parametrize("n,parts", [(1, 1), (50_000, 100), (1_000_000, 3)])
def test_first_last_value(ctx, func, n, parts):
    d = _data(n, parts, n, True)
    _check(ctx, func, *d)
    _check(ctx, func, *d, asc=False, arg_dtype=np.int64)


@pytest.mark.gpu
def test_window_over_empty_clause(ctx):
    """OVER (): one partition in input order; the argument column gives the row count."""
    a = np.arange(1000, dtype=np.int64) * 3
    arg = ctx.upload(a)
    rk = ctx.window(W.Rank, [], [], [], arg=arg).to_numpy()[0]
    assert (rk == 1).all()
    nt = ctx.window(W.Ntile, [], [], [], arg=arg, param=3).to_numpy()[0]
    want, _ = ob.window(W.Ntile, [], [], [], param=3, n=1000)
    assert np.array_equal(nt, want)
    lag, ok = ctx.window(W.Lag, [], [], [], arg=arg, param=2).to_numpy()
    assert not ok[:2].any() and np.array_equal(lag[2:], a[:-2])


@pytest.mark.gpu
def test_window_errors(ctx):
    import qe_hip
    k = ctx.upload(np.zeros(4, np.int64))
    with pytest.raises(qe_hip.QehError):
        ctx.window(W.Ntile, [k], [k], [True], param=0)
    with pytest.raises(qe_hip.QehError):
        ctx.window(W.Lag, [k], [k], [True])  # value function without an argument
