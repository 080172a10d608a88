"""The stable tile ranking by returning LDS atomics (k_rs_scatter, k_part_scatter(_small), the window
partition passes) relies on ds_add_rtn serving a wave's lanes in lane order.  The library checks that
once per process on the device (qeh_lds_atomic_rank_ok, a self-test kernel) and ranks by ballot
matching when it fails; these tests run every pass family both ways (QEH_RS_BALLOT / QEH_WM_BALLOT
force the ballot ranking) and compare both with the oracle, so a device whose atomics were not
lane-ordered could not hide behind either path."""
import numpy as np
import pytest

import oracle_bind as ob
from qe_hip import AggregateFunction as AF, BinaryOp, binop, col, lit  # noqa: F401
from qe_hip.plan import WindowFunctionType as W


@pytest.mark.gpu
def test_self_check_reports_lane_ordered_atomics(ctx):
    ok = ctx.lds_atomic_rank_ok()
    assert ok in (True, False)
    assert ctx.lds_atomic_rank_ok() == ok  # cached per process
    # gfx950 serves one instruction's lanes in lane order (tools/ubench/lds_order_ubench.hip)
    assert ok, "LDS atomics failed the lane-order self-check: the passes run the ballot ranking"


@pytest.mark.gpu
@pytest.mark.parametrize("ballot", [False, True])
def test_sort_both_rankings_vs_oracle(ctx, monkeypatch, ballot):
    if ballot:
        monkeypatch.setenv("QEH_RS_BALLOT", "1")
    r = np.random.default_rng(5)
    n = 300_001
    a = r.integers(-3, 3, n).astype(np.int64)           # many ties: stability decides the order
    b = r.integers(-(2 ** 40), 2 ** 40, n).astype(np.int64)
    got = ctx.sort_indices([ctx.upload(a), ctx.upload(b)], [True, False]).to_numpy()[0]
    want = ob.sort_indices_nulls([ob.HostCol(a), ob.HostCol(b)], [True, False], [True, True])
    assert np.array_equal(got, want)
    k = r.integers(-1000, 1000, n).astype(np.int64)
    v = r.random(n)
    cols, rows = ctx.merge_sorted([[ctx.upload(k[:n // 2]), ctx.upload(v[:n // 2])],
                                   [ctx.upload(k[n // 2:]), ctx.upload(v[n // 2:])]], [0], [False], [False])
    perm = ob.sort_indices_nulls([ob.HostCol(k)], [False], [False])
    assert np.array_equal(cols[0].to_numpy()[0], k[perm])
    assert np.array_equal(cols[1].to_numpy()[0], v[perm])  # payload order = stable order


@pytest.mark.gpu
@pytest.mark.parametrize("ballot", [False, True])
@pytest.mark.parametrize("parts", [3, 8, 40])
def test_partition_move_both_rankings_keep_input_order(ctx, monkeypatch, ballot, parts):
    if ballot:
        monkeypatch.setenv("QEH_RS_BALLOT", "1")
    r = np.random.default_rng(parts)
    n = 250_003
    k = r.integers(0, 1 << 30, n).astype(np.int64)
    rowid = np.arange(n, dtype=np.int64)
    counts, moved = ctx.partition_hash_move([ctx.upload(k)], parts, [ctx.upload(k), ctx.upload(rowid)])
    got_k, got_id = moved[0].to_numpy()[0], moved[1].to_numpy()[0]
    assert np.array_equal(got_k, k[got_id])
    start = 0
    for c in counts:
        seg = got_id[start:start + c]
        assert np.all(np.diff(seg) > 0)  # stable: each partition keeps the input order
        start += c
    assert start == n and np.array_equal(np.sort(got_id), rowid)


@pytest.mark.gpu
@pytest.mark.parametrize("ballot", [False, True])
@pytest.mark.parametrize("func", [W.RowNumber, W.Rank])
def test_window_partition_path_both_rankings_vs_oracle(ctx, monkeypatch, ballot, func):
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    if ballot:
        monkeypatch.setenv("QEH_WM_BALLOT", "1")
    r = np.random.default_rng(9)
    n = 400_000
    k = r.integers(0, 5000, n).astype(np.int64)
    v = r.integers(-20, 20, n).astype(np.int64)  # ties: the input-order tiebreak is the stability check
    if func == W.RowNumber:
        got = ctx.row_number([ctx.upload(k)], [ctx.upload(v)], [True]).to_numpy()[0]
        want = ob.row_number([ob.HostCol(k)], [ob.HostCol(v)], [True])
    else:
        got = ctx.window(func, [ctx.upload(k)], [ctx.upload(v)], [True]).to_numpy()[0]
        want, _ = ob.window(func, [ob.HostCol(k)], [ob.HostCol(v)], [True])
    assert np.array_equal(got, want)
