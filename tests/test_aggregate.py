"""HashAggregate parity (device vs oracle): global aggregates and GROUP BY on
every key type, NULL keys (one group), the INT64_MIN key (the HBM table's
empty marker), group-table regrowth at high cardinality, fused predicates,
and the multi-key group-table path.  Integers exact, float SUM/AVG 1e-6."""
import numpy as np
import pytest

import oracle_bind as ob
from helpers import assert_grouped_equal
from qe_hip import AggregateFunction as AF
from qe_hip import BinaryOp, binop, col, lit

AGGS = [(AF.Sum, 1), (AF.Count, 1), (AF.Avg, 1), (AF.Min, 1), (AF.Max, 1), (AF.Sum, 2), (AF.Min, 2), (AF.Count, 0)]


def data(n, key, seed=0, nulls=True):
    r = np.random.default_rng(seed)
    v = r.random(n)
    vm = r.random(n) > 0.1 if nulls else None
    w = r.integers(-10 ** 6, 10 ** 6, n).astype(np.int64)
    km = r.random(n) > 0.05 if nulls else None
    return [(key, km), (v, vm), (w, None)]


def run(ctx, cols, key_idx, aggs, pred=None, float_aggs=(0, 2)):
    dev = [ctx.upload(*c) for c in cols]
    if pred is None:
        gk, ga, g = ctx.hash_aggregate([dev[i] for i in key_idx], dev, aggs)
    else:
        gk, ga, g = ctx.filter_aggregate(dev, pred, key_idx, aggs)
    got_k = [c.to_numpy() for c in gk]
    got_a = [c.to_numpy() for c in ga]
    hc = [ob.HostCol(*c) for c in cols]
    if pred is not None:
        fc, _, _ = ob.filter(hc, pred)
        hc = [ob.HostCol(v, m) for v, m in fc]
    wk, wa, wg, _ = ob.hash_aggregate([hc[i] for i in key_idx], hc, aggs)
    assert g == wg
    assert_grouped_equal(got_k, got_a, wk, wa, float_aggs=float_aggs)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["int64", "int32", "float64", "float32", "bool"])
def test_group_by_key_types(ctx, kind):
    r = np.random.default_rng(1)
    n = 300_000
    key = {"int64": r.integers(-500, 500, n).astype(np.int64),
           "int32": r.integers(-500, 500, n).astype(np.int32),
           "float64": np.round(r.standard_normal(n), 1),
           "float32": np.round(r.standard_normal(n), 1).astype(np.float32),
           "bool": r.random(n) > 0.3}[kind]
    run(ctx, data(n, key), [0], AGGS)


@pytest.mark.gpu
def test_group_by_special_keys_and_regrowth(ctx):
    r = np.random.default_rng(2)
    n = 400_000
    key = r.integers(0, 200_000, n).astype(np.int64)  # > 65536 distinct: the HBM table regrows
    key[::1000] = np.iinfo(np.int64).min               # the table's empty marker as a real key
    key[1::1000] = np.iinfo(np.int64).max
    run(ctx, data(n, key, seed=3), [0], AGGS)


@pytest.mark.gpu
def test_group_by_with_fused_predicate(ctx):
    r = np.random.default_rng(4)
    n = 1_000_003
    cols = [(r.integers(0, 1024, n).astype(np.int64), None), (r.random(n), None),
            (r.integers(-(2 ** 20), 2 ** 20, n).astype(np.int64), None), (r.integers(0, 100, n).astype(np.int64), None)]
    pred = binop(col(3), BinaryOp.Greater, lit(49))
    run(ctx, cols, [0], [(AF.Sum, 1), (AF.Count, 1), (AF.Sum, 2)], pred=pred, float_aggs=(0,))


@pytest.mark.gpu
def test_group_by_multi_key_group_table_path(ctx):
    r = np.random.default_rng(5)
    n = 200_000
    cols = [(r.integers(0, 30, n).astype(np.int32), r.random(n) > 0.1), (r.random(n), None),
            (r.integers(-9, 9, n).astype(np.int64), None), (r.integers(0, 7, n).astype(np.int64), None)]
    run(ctx, cols, [0, 3], [(AF.Sum, 1), (AF.Max, 2), (AF.Count, 1)], float_aggs=(0,))


@pytest.mark.gpu
def test_group_by_lds_path_vs_group_table_path(ctx, monkeypatch):
    r = np.random.default_rng(6)
    n = 100_000
    cols = data(n, r.integers(0, 5000, n).astype(np.int64), seed=6)
    run(ctx, cols, [0], AGGS)
    monkeypatch.setenv("QEH_NO_LDS_GROUPBY", "1")
    run(ctx, cols, [0], AGGS)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 1000, 3_000_000])
def test_global_aggregates(ctx, n):
    r = np.random.default_rng(n)
    cols = [(r.integers(-100, 100, n).astype(np.int64), r.random(n) > 0.2), (r.random(n), r.random(n) > 0.5),
            (r.integers(-(2 ** 31), 2 ** 31 - 1, n).astype(np.int32), None), (r.random(n).astype(np.float32), None)]
    aggs = [(AF.Count, 0), (AF.Sum, 0), (AF.Avg, 0), (AF.Min, 0), (AF.Max, 0), (AF.Sum, 1), (AF.Avg, 1),
            (AF.Min, 1), (AF.Max, 1), (AF.Sum, 2), (AF.Min, 3), (AF.Max, 3)]
    dev = [ctx.upload(*c) for c in cols]
    _, ga, g = ctx.hash_aggregate([], dev, aggs)
    _, wa, wg, _ = ob.hash_aggregate([], [ob.HostCol(*c) for c in cols], aggs)
    assert g == wg == 1
    assert_grouped_equal([], [c.to_numpy() for c in ga], [], wa, float_aggs=(5, 6))


@pytest.mark.gpu
def test_int32_sum_wraps_like_arrow_rs(ctx):
    """compute::sum(Int32Array) wraps in i32 before the `as i64` (operators.rs:755-757)."""
    v = np.full(10, 2 ** 30, np.int32)
    _, ga, _ = ctx.hash_aggregate([], [ctx.upload(v)], [(AF.Sum, 0)])
    assert ga[0].to_numpy()[0][0] == np.int64(np.int32(np.int64(10 * 2 ** 30) & 0xFFFFFFFF).astype(np.int32))
    _, wa, _, _ = ob.hash_aggregate([], [ob.HostCol(v)], [(AF.Sum, 0)])
    assert wa[0][0][0] == ga[0].to_numpy()[0][0]


@pytest.mark.gpu
@pytest.mark.parametrize("keys", [[0], [0, 3]])
def test_more_aggregates_than_one_kernel_carries(ctx, keys):
    """>8 aggregates run as key-ordered chunks that line up row for row."""
    r = np.random.default_rng(7)
    n = 250_000
    cols = [(r.integers(0, 3000, n).astype(np.int64), r.random(n) > 0.05), (r.random(n), r.random(n) > 0.3),
            (r.integers(-99, 99, n).astype(np.int32), None), (r.integers(0, 3, n).astype(np.int64), None)]
    aggs = [(AF.Sum, 1), (AF.Count, 1), (AF.Avg, 1), (AF.Min, 1), (AF.Max, 1), (AF.Sum, 2), (AF.Min, 2),
            (AF.Max, 2), (AF.Count, 0), (AF.Avg, 2), (AF.Count, 3), (AF.Sum, 3)]
    run(ctx, cols, keys, aggs, float_aggs=(0, 2, 9))


@pytest.mark.gpu
@pytest.mark.parametrize("groups", [7, 1024, 5000, 300_000])
def test_group_by_fast_path_no_nulls(ctx, groups):
    """Non-null 8-byte columns take k_group_agg_fast (LDS key hash); >2048 keys
    per workgroup spill to the HBM table; ragged tail through the generic kernel."""
    r = np.random.default_rng(groups)
    n = 2_000_003
    key = r.integers(0, groups, n).astype(np.int64) * 7919 - 3
    key[::50_000] = np.iinfo(np.int64).min
    cols = [(key, None), (r.random(n), None), (r.integers(-(2 ** 40), 2 ** 40, n).astype(np.int64), None),
            (r.integers(0, 100, n).astype(np.int64), None)]
    aggs = [(AF.Sum, 1), (AF.Count, 1), (AF.Min, 2), (AF.Max, 2), (AF.Sum, 2)]
    run(ctx, cols, [0], aggs, pred=binop(col(3), BinaryOp.Greater, lit(49)), float_aggs=(0,))
    run(ctx, cols, [0], aggs[:3], float_aggs=(0,))


@pytest.mark.gpu
def test_group_by_fast_path_float_key(ctx):
    r = np.random.default_rng(31)
    n = 500_000
    key = np.round(r.standard_normal(n), 1)
    cols = [(key, None), (r.integers(-9, 9, n).astype(np.int64), None)]
    run(ctx, cols, [0], [(AF.Sum, 1), (AF.Count, 1), (AF.Avg, 1)], float_aggs=(2,))
