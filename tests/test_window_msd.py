"""The partitioning window path (k_window.hip: ROW_NUMBER / RANK / DENSE_RANK / NTILE over one
bounded integer PARTITION BY key and one ORDER BY key) against the oracle (qo_row_number /
qo_window, which follow docs/WINDOW_FUNCTIONS.md:44-140).  QEH_WINDOW_MSD=1 forces the path below
its default size threshold so small cases exercise every kernel; a group larger than the
wave sort's 2048 rows must fall back to the LSD path and stay correct."""
import numpy as np
import pytest

import oracle_bind as ob
from qe_hip.plan import WindowFunctionType as W


def _msd_ran(ctx):
    """a partitioning path ran: k_window.hip's, or the three-level one (k_window3.hip) tried first"""
    return ctx.kernel_time("window_sort")[1] > 0 or ctx.kernel_time("w3_place")[1] > 0


def _run(ctx, func, k, v, asc, param=0):
    ctx.timing(True)
    ctx.timing_reset()
    if func == W.RowNumber:
        got = ctx.row_number([ctx.upload(k)], [ctx.upload(v)], [asc]).to_numpy()[0]
        want = ob.row_number([ob.HostCol(k)], [ob.HostCol(v)], [asc])
    else:
        got = ctx.window(func, [ctx.upload(k)], [ctx.upload(v)], [asc], param=param).to_numpy()[0]
        want, _ = ob.window(func, [ob.HostCol(k)], [ob.HostCol(v)], [asc], param=param)
    ran = _msd_ran(ctx)
    ctx.timing(False)
    return got, want, ran


@pytest.mark.gpu
@pytest.mark.parametrize("func,param", [(W.RowNumber, 0), (W.Rank, 0), (W.DenseRank, 0), (W.Ntile, 3)])
@pytest.mark.parametrize("n,parts", [(1, 1), (1000, 7), (70_000, 1 << 20), (300_001, 1000), (2_000_000, 4096)])
@pytest.mark.parametrize("asc", [True, False])
def test_msd_window_matches_oracle(ctx, monkeypatch, func, param, n, parts, asc):
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(n + parts)
    k = r.integers(0, parts, n).astype(np.int64) + 1000  # offset range (k - kmin)
    v = r.integers(-40, 40, n).astype(np.int64)  # many ties: RANK / DENSE_RANK peers, input-order tiebreak
    got, want, ran = _run(ctx, func, k, v, asc, param)
    assert ran
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("vdt", [np.int32, np.float64, np.float32])
def test_msd_window_order_key_types(ctx, monkeypatch, vdt):
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(3)
    n = 200_000
    k = r.integers(-500, 500, n).astype(np.int32)
    if vdt == np.int32:
        v = r.integers(-(2 ** 31), 2 ** 31, n, dtype=np.int64).astype(np.int32)
        v[:2] = [-(2 ** 31), 2 ** 31 - 1]
    else:
        v = np.round(r.standard_normal(n), 2).astype(vdt)
        v[:4] = [-0.0, 0.0, np.inf, -np.inf]
    for func in (W.RowNumber, W.Rank):
        got, want, ran = _run(ctx, func, k, v, False)
        assert ran and np.array_equal(got, want)


@pytest.mark.gpu
def test_msd_window_full_range_order_key(ctx, monkeypatch):
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(4)
    n = 100_000
    k = r.integers(0, 30, n).astype(np.int64)
    v = r.integers(-(2 ** 63), 2 ** 63 - 1, n, dtype=np.int64)
    v[:3] = [np.iinfo(np.int64).min, np.iinfo(np.int64).max, np.iinfo(np.int64).max]
    for asc in (True, False):
        got, want, ran = _run(ctx, W.RowNumber, k, v, asc)
        assert ran and np.array_equal(got, want)


@pytest.mark.gpu
def test_msd_window_big_group_falls_back(ctx, monkeypatch):
    """A PARTITION BY group above 2048 rows: the wave sort declines, the LSD path answers."""
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(5)
    n = 50_000
    k = r.integers(0, 100, n).astype(np.int64)
    k[:5000] = 42
    v = r.integers(-9, 9, n).astype(np.int64)
    got, want, _ = _run(ctx, W.Rank, k, v, True)
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_msd_window_default_threshold_full_shape(ctx):
    """Without forcing: 2^21 rows, k in [0, 2^20) (the config-5 shape scaled down) take the path."""
    n = 1 << 21
    from qe_hip import abi
    kk = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 7, n, 2 ** 20)
    vv = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 8, n, 2 ** 62, lo=-(2 ** 61))
    got, want, ran = _run(ctx, W.RowNumber, kk, vv, True)
    assert ran and np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("func,param,default", [(W.Lag, 1, None), (W.Lag, 3, 7), (W.Lead, 1, None), (W.Lead, 2, -5),
                                                (W.FirstValue, 0, None), (W.LastValue, 0, None)])
@pytest.mark.parametrize("vdt", [np.int64, np.int32, np.float64, np.float32])
@pytest.mark.parametrize("asc", [True, False])
def test_msd_value_functions_of_the_order_column(ctx, monkeypatch, func, param, default, vdt, asc):
    """LAG / LEAD / FIRST_VALUE / LAST_VALUE whose argument is the ORDER BY column (the config-5
    window bench's LAG(v, 1)): values decoded from the group's order keys, NULL (or the default)
    outside the partition."""
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(11)
    n = 300_000
    k = r.integers(0, 700, n).astype(np.int64)
    if vdt in (np.int64, np.int32):
        v = r.integers(-50, 50, n).astype(vdt)
    else:
        v = np.round(r.standard_normal(n), 2).astype(vdt)
    d = None if default is None else vdt(default)
    ctx.timing(True)
    ctx.timing_reset()
    dv = ctx.upload(v)
    got_v, got_m = ctx.window(func, [ctx.upload(k)], [dv], [asc], arg=dv, param=param, default=d).to_numpy()
    ran = _msd_ran(ctx)
    ctx.timing(False)
    want_v, want_m = ob.window(func, [ob.HostCol(k)], [ob.HostCol(v)], [asc], arg=ob.HostCol(v), param=param,
                               default=d)
    assert ran
    assert np.array_equal(got_m, want_m)
    assert np.array_equal(got_v[want_m].view(np.uint8), want_v[want_m].view(np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("func,param", [(W.RowNumber, 0), (W.Rank, 0), (W.DenseRank, 0), (W.Ntile, 4)])
@pytest.mark.parametrize("vdt", [np.int64, np.float64])
@pytest.mark.parametrize("parts", [300, 700])
def test_msd_window_counting_sort_groups(ctx, monkeypatch, func, param, vdt, parts):
    """Spread order keys (the group counting sort's case: buckets of the top key bits, exact rank
    inside a bucket) with some duplicated values inside groups, so buckets hold equal keys ranked
    by input position; group sizes up to ~1900 rows take both the 1024- and 2048-row kernels."""
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(21)
    n = 400_000
    k = r.integers(0, parts, n).astype(np.int64)
    if vdt == np.int64:
        v = r.integers(-(2 ** 62), 2 ** 62, n, dtype=np.int64)
    else:
        v = r.standard_normal(n) * 1e6
    dup = r.random(n) < 0.1
    src = r.integers(0, n, n)
    same = k[src] == k  # copy a value from another row of the same group where one was drawn
    v[dup & same] = v[src[dup & same]]
    # a few near-equal keys in one bucket
    v[:64] = v[0] + np.arange(64, dtype=v.dtype) * (1 if vdt == np.int64 else 1e-9)
    k[:64] = k[0]
    got, want, ran = _run(ctx, func, k, v.astype(vdt), True, param)
    assert ran and np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("func,param", [(W.RowNumber, 0), (W.Rank, 0), (W.DenseRank, 0), (W.Ntile, 5)])
def test_msd_window_clustered_big_groups(ctx, monkeypatch, func, param):
    """Groups of 1025..2048 rows with many ties: the counting sort queues them and the 2048-row
    network kernel sorts the queue; one small clustered group and spread groups alongside."""
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(23)
    n = 300_000
    k = r.integers(0, 200, n).astype(np.int64)
    v = r.integers(-(2 ** 40), 2 ** 40, n).astype(np.int64)
    clustered = k < 100
    v[clustered] = r.integers(-30, 30, int(clustered.sum()))
    k[:700] = 500  # a small group, clustered too
    v[:700] = r.integers(0, 3, 700)
    got, want, ran = _run(ctx, func, k, v, True, param)
    assert ran and np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("func,param,default", [(W.Lag, 1, None), (W.Lead, 2, 9), (W.FirstValue, 0, None),
                                                (W.LastValue, 0, None)])
@pytest.mark.parametrize("asc", [True, False])
def test_msd_value_functions_big_and_clustered_groups(ctx, monkeypatch, func, param, default, asc):
    """Value functions over groups of 1025..2048 rows (the 2048-row counting sort), clustered groups
    of both size classes (the network kernels' queue) and small spread groups, in one call."""
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(29)
    n = 400_000
    k = r.integers(0, 260, n).astype(np.int64)  # ~1540 rows per group
    v = r.integers(-(2 ** 50), 2 ** 50, n).astype(np.int64)
    v[k < 60] = r.integers(-20, 20, int((k < 60).sum()))  # clustered big groups
    small = r.random(n) < 0.02
    k[small] = 1000 + r.integers(0, 40, int(small.sum()))  # small groups, half of them clustered
    v[small & (k < 1020)] = r.integers(0, 5, int((small & (k < 1020)).sum()))
    d = None if default is None else np.int64(default)
    ctx.timing(True)
    ctx.timing_reset()
    dv = ctx.upload(v)
    got_v, got_m = ctx.window(func, [ctx.upload(k)], [dv], [asc], arg=dv, param=param, default=d).to_numpy()
    ran = _msd_ran(ctx)
    ctx.timing(False)
    want_v, want_m = ob.window(func, [ob.HostCol(k)], [ob.HostCol(v)], [asc], arg=ob.HostCol(v), param=param,
                               default=d)
    assert ran
    assert np.array_equal(got_m, want_m)
    assert np.array_equal(got_v[want_m], want_v[want_m])


@pytest.mark.gpu
@pytest.mark.parametrize("func,param", [(W.Lead, 2 ** 62), (W.Lag, 2 ** 62), (W.Lead, 0), (W.Lag, 5000)])
def test_msd_value_functions_extreme_offsets(ctx, monkeypatch, func, param):
    """Offsets far past every partition (all NULL / default) and offset 0 (the row itself)."""
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(31)
    n = 100_000
    k = r.integers(0, 300, n).astype(np.int64)
    v = r.integers(-(2 ** 40), 2 ** 40, n).astype(np.int64)
    for d in (None, np.int64(-7)):
        dv = ctx.upload(v)
        got_v, got_m = ctx.window(func, [ctx.upload(k)], [dv], [True], arg=dv, param=param, default=d).to_numpy()
        want_v, want_m = ob.window(func, [ob.HostCol(k)], [ob.HostCol(v)], [True], arg=ob.HostCol(v), param=param,
                                   default=d)
        assert np.array_equal(got_m, want_m)
        assert np.array_equal(got_v[want_m], want_v[want_m])


@pytest.mark.gpu
def test_row_number_full_size_properties(ctx):
    """BASELINE config 5 at its full size (ROW_NUMBER() OVER (PARTITION BY k ORDER BY v), 1e9 rows,
    k in [0, 2^20), generated in HBM), checked against independent torch computations on the
    device: every group's numbers sum to m(m+1)/2 and lie in [1, m] (m = the group's row count from
    bincount), and for 64 sampled groups the numbers equal those of a stable sort by (k, v, row)."""
    import torch
    from qe_hip import abi
    from qe_hip.distributed import TYPESTR, _DeviceView
    n, parts = 1_000_000_000, 1 << 20
    k = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 7, n, parts)
    v = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 8, n, 2 ** 62, lo=-(2 ** 61))
    rn = ctx.row_number([k], [v], [True])

    def view(col):
        return torch.as_tensor(_DeviceView(col.c.values, len(col), TYPESTR[col.dtype], col), device="cuda")

    tk, tv, tr = view(k), view(v), view(rn)
    m = torch.bincount(tk, minlength=parts)
    assert int(m.sum()) == n
    assert int(tr.min()) >= 1 and bool((tr <= m[tk]).all())
    assert int(tr.sum()) == int((m * (m + 1) // 2).sum())
    sample = torch.randperm(parts, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5))[:64]
    idx = torch.nonzero(torch.isin(tk, sample)).squeeze(1)  # ascending row order
    sk, sv = tk[idx], tv[idx]
    o1 = torch.argsort(sv, stable=True)          # by v, ties by row
    o2 = torch.argsort(sk[o1], stable=True)      # then by k
    order = o1[o2]
    ks = sk[order]
    starts = torch.ones_like(ks, dtype=torch.bool)
    starts[1:] = ks[1:] != ks[:-1]
    pos = torch.arange(len(ks), device="cuda")
    first = torch.cummax(torch.where(starts, pos, torch.zeros_like(pos)), 0).values
    want = torch.empty_like(pos)
    want[order] = pos - first + 1
    assert torch.equal(tr[idx], want)


@pytest.mark.gpu
def test_row_number_full_size_vs_oracle_sample(ctx):
    """BASELINE config 5 at its full size (1e9 rows, k in [0, 2^20)) against the oracle itself on 1024
    sampled PARTITION BY groups (~1e6 rows): a group's row numbers depend only on its own rows in input
    order, so the oracle's ROW_NUMBER over the sampled groups' rows (regenerated on the host by chunks,
    input order kept) must equal the device's numbers at those rows exactly."""
    import torch
    from qe_hip import abi
    from qe_hip.distributed import TYPESTR, _DeviceView
    n, parts = 1_000_000_000, 1 << 20
    k = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 7, n, parts)
    v = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 8, n, 2 ** 62, lo=-(2 ** 61))
    rn = ctx.row_number([k], [v], [True])
    tr = torch.as_tensor(_DeviceView(rn.c.values, len(rn), TYPESTR[rn.dtype], rn), device="cuda")
    sample = np.sort(np.random.default_rng(9).choice(parts, 1024, replace=False))
    rows, ks, vs = [], [], []
    step = 100_000_000
    for r0 in range(0, n, step):
        m = min(step, n - r0)
        hk = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 7, m, parts, row0=r0)
        sel = np.nonzero(np.isin(hk, sample, assume_unique=False))[0]
        hv = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 8, m, 2 ** 62, lo=-(2 ** 61), row0=r0)
        rows.append(sel + r0)
        ks.append(hk[sel])
        vs.append(hv[sel])
        del hk, hv
    rows, ks, vs = np.concatenate(rows), np.concatenate(ks), np.concatenate(vs)
    want = ob.row_number([ob.HostCol(ks)], [ob.HostCol(vs)], [True])
    got = tr[torch.as_tensor(rows, device="cuda")].cpu().numpy()
    assert len(rows) > 500_000
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("func,param", [(W.RowNumber, 0), (W.Rank, 0), (W.Ntile, 3)])
@pytest.mark.parametrize("n,parts,k0", [(300_001, (1 << 20) + 5, -7), (2_000_000, 1 << 22, 1 << 40), (1_500_000, 1 << 24, -(1 << 30))])
@pytest.mark.parametrize("asc", [True, False])
def test_msd_window_sub_keys_vs_oracle(ctx, monkeypatch, func, param, n, parts, k0, asc):
    """Key ranges above 2^20 (up to 2^24) for ROW_NUMBER / RANK / NTILE: a group holds 2^sb consecutive
    keys and the group sort buckets by (sub-key, order key), numbering each sub-key's rows from 1."""
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(n + parts)
    k = r.integers(0, parts, n).astype(np.int64) + k0
    k[:2] = [k0, k0 + parts - 1]  # the whole range present
    v = r.integers(-40, 40, n).astype(np.int64)  # ties: RANK peers, input-order tiebreak
    got, want, ran = _run(ctx, func, k, v, asc, param)
    assert ran
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("asc", [True, False])
def test_msd_window_sub_keys_dense_rank(ctx, monkeypatch, asc):
    """DENSE_RANK over key ranges above 2^20: peer-group starts counted from each sub-key's first row."""
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(12)
    n = 1_200_000
    k = r.integers(0, 1 << 22, n).astype(np.int64) - 5
    v = r.integers(-5, 5, n).astype(np.int64)
    got, want, ran = _run(ctx, W.DenseRank, k, v, asc)
    assert ran and np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("func,param,default", [(W.Lag, 1, None), (W.Lead, 2, -5), (W.FirstValue, 0, None),
                                                (W.LastValue, 0, None)])
@pytest.mark.parametrize("asc", [True, False])
def test_msd_value_functions_sub_keys(ctx, monkeypatch, func, param, default, asc):
    """LAG / LEAD / FIRST_VALUE / LAST_VALUE of the ORDER BY column over key ranges above 2^20: the
    source row is found inside the row's own sub-key run."""
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(13)
    n = 900_000
    k = r.integers(0, (1 << 21) + 3, n).astype(np.int64)
    v = r.integers(-50, 50, n).astype(np.int64)
    d = None if default is None else np.int64(default)
    ctx.timing(True)
    ctx.timing_reset()
    dv = ctx.upload(v)
    got_v, got_m = ctx.window(func, [ctx.upload(k)], [dv], [asc], arg=dv, param=param, default=d).to_numpy()
    ran = _msd_ran(ctx)
    ctx.timing(False)
    want_v, want_m = ob.window(func, [ob.HostCol(k)], [ob.HostCol(v)], [asc], arg=ob.HostCol(v), param=param, default=d)
    assert ran
    assert np.array_equal(got_m, want_m)
    assert np.array_equal(got_v[want_m], want_v[want_m])


@pytest.mark.gpu
def test_msd_window_sub_keys_fallbacks(ctx, monkeypatch):
    """Above 2^20 keys, a group above 2048 rows falls back to the LSD path and stays equal to the oracle."""
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(12)
    n = 400_000
    k = r.integers(0, 1 << 22, n).astype(np.int64)
    v = r.integers(-5, 5, n).astype(np.int64)
    k[:5000] = 777  # one group of > 2048 rows
    for func in (W.RowNumber, W.DenseRank):
        got, want, _ = _run(ctx, func, k, v, True)
        assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("func,param", [(W.RowNumber, 0), (W.Rank, 0), (W.DenseRank, 0), (W.Ntile, 4)])
@pytest.mark.parametrize("ranges", [(64, 4096), (100, 50, 30), (3000, 2000)])
def test_msd_window_several_partition_keys(ctx, monkeypatch, func, param, ranges):
    """PARTITION BY two or three integer keys: their mixed-radix composite takes the partitioning path
    when the product of the ranges fits it (2^20 keys, 2^24 for ROW_NUMBER / RANK / NTILE), else the
    LSD path; equal to the oracle either way."""
    monkeypatch.setenv("QEH_WINDOW_MSD", "1")
    r = np.random.default_rng(sum(ranges))
    n = 500_000
    ks = [(r.integers(0, q, n) - q // 3).astype(np.int64 if i % 2 == 0 else np.int32) for i, q in enumerate(ranges)]
    v = r.integers(-30, 30, n).astype(np.int64)
    ctx.timing(True)
    ctx.timing_reset()
    dk = [ctx.upload(k) for k in ks]
    hk = [ob.HostCol(k.astype(np.int64)) for k in ks]
    if func == W.RowNumber:
        got = ctx.row_number(dk, [ctx.upload(v)], [True]).to_numpy()[0]
        want = ob.row_number(hk, [ob.HostCol(v)], [True])
    else:
        got = ctx.window(func, dk, [ctx.upload(v)], [True], param=param).to_numpy()[0]
        want, _ = ob.window(func, hk, [ob.HostCol(v)], [True], param=param)
    ran = _msd_ran(ctx)
    ctx.timing(False)
    assert ran == (int(np.prod(ranges)) <= (1 << 24))
    assert np.array_equal(got, want)
