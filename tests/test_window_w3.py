"""The three-level window pipeline (k_window3.hip: ROW_NUMBER / RANK / NTILE over one PARTITION BY key
of at most 2^20 consecutive values) against the oracle (qo_row_number / qo_window, which follow
docs/WINDOW_FUNCTIONS.md:44-140).  QEH_WINDOW_MSD=1 forces the partitioning paths below their default
size threshold.  Shapes the pipeline declines -- a key range above 2^20, heavy keys overflowing a
region or sub-bucket, a bucket of many equal order keys, DENSE_RANK -- must reach the k_window.hip or
LSD path and stay correct."""
import numpy as np
import pytest


@pytest.fixture(autouse=True)
def _w3_on(monkeypatch):
    monkeypatch.setenv("QEH_WINDOW_W3", "1")  # the pipeline is opt-in (k_window3.hip window_w3)

import oracle_bind as ob
from qe_hip import abi
from qe_hip.plan import WindowFunctionType as W


def _run(ctx, func, k, v, asc, param=0):
    """(device result, oracle result, the three-level pipeline ran to the end)"""
    ctx.timing(True)
    ctx.timing_reset()
    if func == W.RowNumber:
        got = ctx.row_number([ctx.upload(k)], [ctx.upload(v)], [asc]).to_numpy()[0]
        want = ob.row_number([ob.HostCol(k)], [ob.HostCol(v)], [asc])
    else:
        got = ctx.window(func, [ctx.upload(k)], [ctx.upload(v)], [asc], param=param).to_numpy()[0]
        want, _ = ob.window(func, [ob.HostCol(k)], [ob.HostCol(v)], [asc], param=param)
    ran = ctx.kernel_time("w3_place")[1] > 0
    old = ctx.kernel_time("window_sort")[1] > 0 or ctx.kernel_time("radix_pass")[1] > 0
    ctx.timing(False)
    return got, want, ran and not old


FUNCS = [(W.RowNumber, 0), (W.Rank, 0), (W.Ntile, 3)]


@pytest.mark.gpu
@pytest.mark.parametrize("func,param", FUNCS + [(W.Ntile, 1), (W.Ntile, 1000)])
@pytest.mark.parametrize("n,parts,k0", [(1, 1, 0), (1000, 7, 5), (70_000, 1 << 20, 0), (300_001, 1000, -500),
                                        (2_000_000, 4096, 1 << 40), (3_000_000, 1 << 20, -(1 << 19))])
@pytest.mark.parametrize("asc", [True, False])
def test_w3_matches_oracle(ctx, monkeypatch, func, param, n, parts, k0, asc):
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(n + parts)
    k = r.integers(0, parts, n).astype(np.int64) + k0
    v = r.integers(-40, 40, n).astype(np.int64)  # many ties: RANK peers, input-order tiebreak
    got, want, ran = _run(ctx, func, k, v, asc, param)
    assert ran
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("kdt", [np.int32, np.int64])
@pytest.mark.parametrize("vdt", [np.int32, np.int64, np.float64, np.float32])
def test_w3_key_and_order_types(ctx, monkeypatch, kdt, vdt):
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(3)
    n = 400_000
    k = r.integers(-3000, 3000, n).astype(kdt)
    if vdt == np.int32:
        v = r.integers(-(2 ** 31), 2 ** 31, n, dtype=np.int64).astype(np.int32)
        v[:2] = [-(2 ** 31), 2 ** 31 - 1]
    elif vdt == np.int64:
        v = r.integers(-(2 ** 63), 2 ** 63 - 1, n, dtype=np.int64)
        v[:3] = [np.iinfo(np.int64).min, np.iinfo(np.int64).max, np.iinfo(np.int64).max]
    else:
        v = np.round(r.standard_normal(n), 2).astype(vdt)
        v[:4] = [-0.0, 0.0, np.inf, -np.inf]
    for func in (W.RowNumber, W.Rank):
        for asc in (True, False):
            got, want, ran = _run(ctx, func, k, v, asc)
            assert ran and np.array_equal(got, want), (func, asc)


@pytest.mark.gpu
def test_w3_config5_shape_default_threshold(ctx, monkeypatch):
    """Without forcing: 2^22 rows, k in [0, 2^20), v over 2^62 (config 5 scaled down) take the pipeline."""
    n = 1 << 22
    k = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 7, n, 2 ** 20)
    v = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 8, n, 2 ** 62, lo=-(2 ** 61))
    for func, param in FUNCS:
        got, want, ran = _run(ctx, func, k, v, True, param)
        assert ran and np.array_equal(got, want), func


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["heavy_key", "equal_order_keys", "range_above_2_20", "dense_rank"])
def test_w3_declines_and_the_answer_stays_right(ctx, monkeypatch, case):
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(11)
    n = 300_000
    k = r.integers(0, 5000, n).astype(np.int64)
    v = r.integers(-(2 ** 40), 2 ** 40, n).astype(np.int64)
    func = W.Rank
    if case == "heavy_key":        # one key's rows overflow its sub-bucket
        k[:6000] = 42
    elif case == "equal_order_keys":  # a bucket of > 64 equal order keys
        k[:500] = 7
        v[:500] = 123
    elif case == "range_above_2_20":
        k[0] = 1 << 21
    else:
        func = W.DenseRank
    got, want, ran = _run(ctx, func, k, v, True)
    assert not ran
    assert np.array_equal(got, want)
