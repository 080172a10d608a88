"""HashJoin (INNER, materialising), Sort, ROW_NUMBER and hash partitioning:
device through the C ABI vs the CPU oracle (intended semantics).
Integer/index results bit-exact.  Join output is compared as a multiset, and
additionally in order when the build keys are unique (left-row order = the
order of the reference's filtered Cartesian product, executor.rs:500-540)."""
import numpy as np
import pytest

import oracle_bind as ob
from helpers import rows_of, sorted_rows


def col_pair(c):
    return c.to_numpy()


def join_both(ctx, pk, pcols, bk, bcols):
    dp = [ctx.upload(*c) for c in pcols]
    db = [ctx.upload(*c) for c in bcols]
    op, obd, rows = ctx.hash_join_inner(ctx.upload(*pk), dp, ctx.upload(*bk), db)
    got = [c.to_numpy() for c in op] + [c.to_numpy() for c in obd]
    wp, wb, wrows = ob.hash_join_inner(ob.HostCol(*pk), [ob.HostCol(*c) for c in pcols], ob.HostCol(*bk),
                                       [ob.HostCol(*c) for c in bcols])
    assert rows == wrows
    return got, wp + wb


@pytest.mark.gpu
@pytest.mark.parametrize("n_probe,n_build", [(0, 10), (10, 0), (1, 1), (5000, 100), (1_000_000, 100_000)])
def test_join_unique_build_in_order(ctx, n_probe, n_build):
    r = np.random.default_rng(n_probe + n_build)
    bk = r.permutation(max(n_build, 1))[:n_build].astype(np.int64) * 3
    ba = r.integers(-5, 5, n_build).astype(np.int64)
    pk = r.integers(0, 3 * max(n_build, 1), n_probe).astype(np.int64)
    pv = r.random(n_probe)
    got, want = join_both(ctx, (pk, None), [(pv, None), (pk, None)], (bk, None), [(ba, None), (bk, None)])
    assert rows_of(got) == rows_of(want)  # same order


@pytest.mark.gpu
def test_join_duplicates_nulls_int32_keys(ctx):
    r = np.random.default_rng(9)
    bk = r.integers(0, 500, 3000).astype(np.int32)
    bkv = r.random(3000) > 0.1
    ba = r.random(3000)
    pk = r.integers(0, 600, 40_000).astype(np.int64)
    pkv = r.random(40_000) > 0.05
    pb = r.random(40_000) > 0.5
    got, want = join_both(ctx, (pk, pkv), [(pk, pkv), (pb, None)], (bk, bkv), [(ba, bkv), (bk, bkv)])
    assert sorted_rows(got) == sorted_rows(want)


@pytest.mark.gpu
@pytest.mark.parametrize("nbuild", [1, 7, 5_000, 300_000])
@pytest.mark.parametrize("payload", ["rows", "rows_null_keys", "dup_keys"])
def test_bucket_table_sparse_keys(ctx, monkeypatch, nbuild, payload):
    """The BUCKET layout (64-B buckets of 5-6 keys, chained by insert counts) for sparse 64-bit keys: the
    INNER / LEFT join's build-row payloads are 32-bit for large builds, 16-bit below 65535 rows; a repeated
    build key falls back to WIDE; NULL keys never match; keys absent from the build miss."""
    monkeypatch.setenv("QEH_FORCE_TABLE", "bucket")
    r = np.random.default_rng(nbuild + len(payload))
    bk = r.integers(-(2 ** 62), 2 ** 62, nbuild, dtype=np.int64)
    bkv = None
    if payload == "dup_keys" and nbuild > 1:
        bk[-1] = bk[0]
    if payload == "rows_null_keys":
        bkv = r.random(nbuild) > 0.1
    pk = np.concatenate([bk[r.integers(0, nbuild, 200_000)], r.integers(-(2 ** 62), 2 ** 62, 50_000, dtype=np.int64)])
    pv = r.random(len(pk))
    got, want = join_both(ctx, (pk, None), [(pk, None), (pv, None)], (bk, bkv), [(bk, bkv)])
    assert sorted_rows(got) == sorted_rows(want)
    got, want = outer_both(ctx, "left", (pk, None), [(pk, None), (pv, None)], (bk, bkv), [(bk, bkv)])
    assert sorted_rows(got) == sorted_rows(want)


@pytest.mark.gpu
@pytest.mark.parametrize("table", ["direct", "packed", "wide", "bucket"])
def test_join_table_layouts(ctx, monkeypatch, table):
    monkeypatch.setenv("QEH_FORCE_TABLE", table)
    r = np.random.default_rng(2)
    bk = r.integers(-(2 ** 20), 2 ** 20, 20_000).astype(np.int64)
    pk = bk[r.integers(0, len(bk), 100_000)]
    got, want = join_both(ctx, (pk, None), [(pk, None)], (bk, None), [(bk, None)])
    assert sorted_rows(got) == sorted_rows(want)


@pytest.mark.gpu
@pytest.mark.parametrize("n_probe,n_build,key0,arange", [(1_000_003, 300_000, 0, 1000), (500_000, 200_001, -77_777, 60_000),
                                                         (300_000, 100_000, 5, 70_000),
                                                         (700_001, 250_000, 1 << 40, 1 << 50)])  # wide: fused join
def test_join_slice_path(ctx, monkeypatch, n_probe, n_build, key0, arange):
    """The LDS-slice materialising join (config 3 shape: one probe payload, one
    Int64 build payload), forced on small tables; misses below and above the key
    range; ragged tail.  Payloads within 16 bits ride in the u16 table as a frame
    of reference; wider ones fall back to the ordered fused join.  Multiset compare."""
    monkeypatch.setenv("QEH_SLICE_MIN_BYTES", "0")
    r = np.random.default_rng(n_build)
    bk = r.permutation(n_build).astype(np.int64) + key0
    ba = r.integers(-(arange // 2), arange - arange // 2, n_build).astype(np.int64)
    pk = r.integers(key0 - 1000, key0 + n_build + 1000, n_probe).astype(np.int64)
    pv = r.random(n_probe)
    got, want = join_both(ctx, (pk, None), [(pv, None)], (bk, None), [(ba, None)])
    assert sorted_rows(got) == sorted_rows(want)


@pytest.mark.gpu
@pytest.mark.parametrize("n_probe,n_build,n_miss", [(1_000_003, 300_000, 0), (819_200, 131_072, 0), (600_011, 200_000, 1),
                                                    (400_000, 150_000, 777)])
def test_join_slice_path_exact_regions(ctx, monkeypatch, n_probe, n_build, n_miss):
    """Slice join with exact region sizes: when every probe row matches, the probe payload
    stays where phase A wrote it (the output column) and phase B only adds the build payload;
    any miss (one, or many) sends it through the compacting emit.  Ragged tails included."""
    monkeypatch.setenv("QEH_SLICE_MIN_BYTES", "0")
    r = np.random.default_rng(n_probe)
    bk = r.permutation(n_build).astype(np.int64) + 12_345
    ba = r.integers(-30_000, 30_000, n_build).astype(np.int64)
    pk = bk[r.integers(0, n_build, n_probe)]
    if n_miss:
        pk[r.choice(n_probe, n_miss, replace=False)] = -5  # below the key range
    pv = r.random(n_probe)
    got, want = join_both(ctx, (pk, None), [(pv, None)], (bk, None), [(ba, None)])
    assert len(got[0][0]) == n_probe - n_miss
    assert sorted_rows(got) == sorted_rows(want)


def sort_both(ctx, keys, asc):
    perm = ctx.sort_indices([ctx.upload(*k) for k in keys], asc).to_numpy()[0]
    want = ob.sort_indices([ob.HostCol(*k) for k in keys], asc)
    return perm, want


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 255, 256, 257, 100_000, 2_000_000])
def test_sort_single_int64_stable(ctx, n):
    r = np.random.default_rng(n)
    k = r.integers(-1000, 1000, n).astype(np.int64)  # many ties -> stability matters
    perm, want = sort_both(ctx, [(k, None)], [True])
    assert np.array_equal(perm, want)


@pytest.mark.gpu
def test_sort_multi_key_mixed_types_nulls_desc(ctx):
    r = np.random.default_rng(4)
    n = 300_000
    a = r.integers(0, 20, n).astype(np.int32)
    av = r.random(n) > 0.05
    b = np.round(r.standard_normal(n), 2)
    bv = r.random(n) > 0.1
    c = r.integers(-(2 ** 62), 2 ** 62, n).astype(np.int64)
    d = r.random(n) > 0.5
    for asc in ([True, False, True, True], [False, True, False, False]):
        perm, want = sort_both(ctx, [(a, av), (b, bv), (c, None), (d, None)], asc)
        assert np.array_equal(perm, want)


@pytest.mark.gpu
def test_sort_full_range_int64_and_negative_zero(ctx):
    k = np.array([2 ** 63 - 1, -(2 ** 63), 0, -1, 1, 2 ** 63 - 1, -(2 ** 63)], np.int64)
    perm, want = sort_both(ctx, [(k, None)], [True])
    assert np.array_equal(perm, want)
    f = np.array([0.0, -0.0, 1.5, -1.5, np.inf, -np.inf, 0.0], np.float64)  # totalOrder: -0.0 < +0.0
    perm, want = sort_both(ctx, [(f, None)], [True])
    assert np.array_equal(perm, want)


@pytest.mark.gpu
def test_take_gather(ctx):
    r = np.random.default_rng(8)
    v = r.random(10_000)
    m = r.random(10_000) > 0.3
    idx = r.integers(0, 10_000, 5000).astype(np.uint32)
    out = ctx.take(ctx.upload(v, m), ctx.upload(idx))
    gv, gm = out.to_numpy()
    assert np.array_equal(gm, m[idx])
    assert np.array_equal(gv[gm], v[idx][m[idx]])


@pytest.mark.gpu
@pytest.mark.parametrize("n,parts", [(0, 4), (1, 1), (10_000, 7), (1_000_000, 1024)])
def test_row_number(ctx, n, parts):
    r = np.random.default_rng(n)
    k = r.integers(0, parts, n).astype(np.int64)
    v = r.integers(-50, 50, n).astype(np.int64)  # ties inside partitions: broken by input position
    rn = ctx.row_number([ctx.upload(k)], [ctx.upload(v)], [True]).to_numpy()[0]
    want = ob.row_number([ob.HostCol(k)], [ob.HostCol(v)], [True])
    assert np.array_equal(rn, want)


@pytest.mark.gpu
@pytest.mark.parametrize("hi_vals,asc", [(4, True), (4, False), (1, True)])
def test_row_number_pair_key_truncated(ctx, hi_vals, asc):
    """PARTITION BY k ORDER BY v with a 62-bit v range: the pair sort keeps only
    the top bits of v and fixes up runs of rows that share them (hi_vals=4:
    runs of ~a dozen rows, sorted in place; hi_vals=1: one run per partition
    longer than the fix-up cap, so the operator falls back to the per-column
    sort).  Ties in v broken by input position."""
    r = np.random.default_rng(hi_vals)
    n = 400_000
    k = r.integers(0, 2 ** 12, n).astype(np.int64)
    hi = r.integers(0, hi_vals, n).astype(np.int64)
    lo = r.integers(0, 2 ** 33, n).astype(np.int64)
    v = (hi << 58) + lo - 2 ** 61
    v[::1000] = v[::1000] // (2 ** 20) * (2 ** 20)  # a few exact duplicates of the low bits too
    v[7] = 2 ** 61  # 62-bit span
    v[11] = v[12]
    k[11] = k[12]
    rn = ctx.row_number([ctx.upload(k)], [ctx.upload(v)], [asc]).to_numpy()[0]
    want = ob.row_number([ob.HostCol(k)], [ob.HostCol(v)], [asc])
    assert np.array_equal(rn, want)


@pytest.mark.gpu
def test_sort_two_keys_pair_path(ctx):
    r = np.random.default_rng(21)
    n = 200_000
    a = r.integers(-5, 5, n).astype(np.int32)
    b = r.integers(-(2 ** 62), 2 ** 62, n).astype(np.int64)
    b[::3] = b[1::3][: len(b[::3])]  # ties in b
    for asc in ([True, True], [False, True], [True, False]):
        perm, want = sort_both(ctx, [(a, None), (b, None)], asc)
        assert np.array_equal(perm, want)
    f = np.round(r.standard_normal(n), 1)
    perm, want = sort_both(ctx, [(f, None), (a, None)], [False, True])
    assert np.array_equal(perm, want)


@pytest.mark.gpu
@pytest.mark.parametrize("dt,lo,hi", [(np.int32, -(2 ** 31), 2 ** 31 - 1), (np.int64, -(2 ** 63), 2 ** 63 - 1),
                                      (np.int64, 0, 2 ** 32 - 1)])
def test_row_number_single_partition_full_width_order_key(ctx, dt, lo, hi):
    """One distinct PARTITION BY value and an ORDER BY key whose span needs exactly 32 or 64
    bits: the pair encoding gives the partition key zero bits (part_shift = key width), and
    every row must still count as one partition (ROW_NUMBER 1..n, RANK by order value)."""
    from qe_hip.plan import WindowFunctionType as WF
    r = np.random.default_rng(31)
    n = 20_000
    k = np.full(n, 7, np.int64)
    v = r.integers(lo, hi, n, dtype=np.int64, endpoint=True).astype(dt)
    v[0], v[1] = lo, hi
    v[5] = v[6]  # a tie
    rn = ctx.row_number([ctx.upload(k)], [ctx.upload(v)], [True]).to_numpy()[0]
    want = ob.row_number([ob.HostCol(k)], [ob.HostCol(v)], [True])
    assert np.array_equal(rn, want)
    assert sorted(rn.tolist()) == list(range(1, n + 1))
    rk = ctx.window(WF.Rank, [ctx.upload(k)], [ctx.upload(v)], [False]).to_numpy()[0]
    want_rk, _ = ob.window(WF.Rank, [ob.HostCol(k)], [ob.HostCol(v)], [False])
    assert np.array_equal(rk, want_rk)


@pytest.mark.gpu
def test_row_number_nulls_desc_two_order_keys(ctx):
    r = np.random.default_rng(12)
    n = 50_000
    k = r.integers(0, 30, n).astype(np.int32)
    kv = r.random(n) > 0.1
    v = r.random(n)
    vv = r.random(n) > 0.2
    w = r.integers(0, 3, n).astype(np.int64)
    rn = ctx.row_number([ctx.upload(k, kv)], [ctx.upload(v, vv), ctx.upload(w)], [False, True]).to_numpy()[0]
    want = ob.row_number([ob.HostCol(k, kv)], [ob.HostCol(v, vv), ob.HostCol(w)], [False, True])
    assert np.array_equal(rn, want)


@pytest.mark.gpu
@pytest.mark.parametrize("parts", [1, 2, 8, 256])
def test_hash_partition_conserves_rows(ctx, parts):
    """partition.rs:400-415 pins row conservation; we also pin determinism,
    stability within a partition and key -> single partition."""
    r = np.random.default_rng(parts)
    k = r.integers(0, 5000, 200_000).astype(np.int64)
    kv = r.random(200_000) > 0.01
    counts, perm = ctx.hash_partition(ctx.upload(k, kv), parts)
    p = perm.to_numpy()[0]
    assert counts.sum() == len(k)
    assert np.array_equal(np.sort(p), np.arange(len(k), dtype=np.uint32))  # a permutation
    offs = np.concatenate([[0], np.cumsum(counts)])
    seen = {}
    for q in range(parts):
        rows = p[offs[q]:offs[q + 1]]
        assert np.all(np.diff(rows.astype(np.int64)) > 0)  # stable within a partition
        for key in np.unique(np.where(kv[rows], k[rows], -1)):
            assert seen.setdefault(int(key), q) == q  # one partition per key
    counts2, perm2 = ctx.hash_partition(ctx.upload(k, kv), parts)
    assert np.array_equal(counts, counts2) and np.array_equal(perm2.to_numpy()[0], p)


@pytest.mark.gpu
def test_sort_many_tiles_per_block_wide_keys(ctx):
    """> 1024 blocks x 2048-row tiles: several tiles per block, 8 passes of 8 bits, low-entropy top digit."""
    r = np.random.default_rng(21)
    n = 6_000_001
    k = r.integers(-(2 ** 62), 2 ** 62, n).astype(np.int64)
    k[::7] = 5  # heavy duplicate run
    perm, want = sort_both(ctx, [(k, None)], [False])
    assert np.array_equal(perm, want)


@pytest.mark.gpu
def test_row_number_full_range_nullable_partition_key(ctx):
    """Null-flag pass case (2^64 values + NULL): partition flags fall back to comparing the key column."""
    r = np.random.default_rng(22)
    n = 40_000
    k = r.integers(0, 50, n).astype(np.int64)
    k[0], k[1] = np.iinfo(np.int64).min, np.iinfo(np.int64).max
    kv = r.random(n) > 0.1
    v = r.integers(-9, 9, n).astype(np.int64)
    rn = ctx.row_number([ctx.upload(k, kv)], [ctx.upload(v)], [True]).to_numpy()[0]
    want = ob.row_number([ob.HostCol(k, kv)], [ob.HostCol(v)], [True])
    assert np.array_equal(rn, want)


@pytest.mark.gpu
@pytest.mark.parametrize("asc", [True, False])
def test_range_partition_orders_partitions(ctx, asc):
    from qe_hip.device import order_keys
    r = np.random.default_rng(23)
    n = 100_000
    v = np.round(r.standard_normal(n), 2)
    m = r.random(n) > 0.05
    split = np.sort(order_keys(np.array([-1.0, -0.0, 0.5, 1.25])))
    counts, perm = ctx.range_partition(ctx.upload(v, m), split, asc)
    p = perm.to_numpy()[0]
    assert counts.sum() == n and np.array_equal(np.sort(p), np.arange(n, dtype=np.uint32))
    offs = np.concatenate([[0], np.cumsum(counts)])
    ok = order_keys(v)
    want_part = np.where(m, (split[None, :] < ok[:, None]).sum(1) if asc else (split[None, :] > ok[:, None]).sum(1), 0)
    for q in range(len(counts)):
        rows = p[offs[q]:offs[q + 1]]
        assert np.all(np.diff(rows.astype(np.int64)) > 0)
        assert np.all(want_part[rows] == q)


@pytest.mark.gpu
def test_scatter_inverts_take(ctx):
    r = np.random.default_rng(24)
    n = 300_001
    v = r.integers(-(2 ** 62), 2 ** 62, n).astype(np.int64)
    perm = r.permutation(n).astype(np.uint32)
    dp = ctx.upload(perm)
    back = ctx.scatter(ctx.take(ctx.upload(v), dp), dp).to_numpy()[0]
    assert np.array_equal(back, v)
    f = r.random(n).astype(np.float32)
    assert np.array_equal(ctx.scatter(ctx.take(ctx.upload(f), dp), dp).to_numpy()[0], f)


@pytest.mark.gpu
@pytest.mark.parametrize("np_,nb", [(0, 1), (1, 1), (3, 3), (2, 2)])
@pytest.mark.parametrize("n_probe", [2047, 2049, 300_001])
def test_join_fused_materialise_matches_unfused(ctx, monkeypatch, np_, nb, n_probe):
    """The fused probe (records embedded by key offset, LDS-staged output) against
    the index-pair + gather path and the oracle, in probe-row order."""
    r = np.random.default_rng(np_ * 10 + nb + n_probe)
    n_build = 50_000
    bk = (r.permutation(2 * n_build)[:n_build] - 7000).astype(np.int64)  # DIRECT, half the offsets absent
    bcols = [(bk, None)] + [(r.integers(-(2 ** 62), 2 ** 62, n_build).astype(np.int64), None),
                            (r.random(n_build), None)][: nb - 1]
    pk = r.integers(-9000, 2 * n_build - 5000, n_probe).astype(np.int64)
    pcols = [(r.random(n_probe), None), (pk, None), (r.integers(0, 9, n_probe).astype(np.int64), None)][:np_]
    got, want = join_both(ctx, (pk, None), pcols, (bk, None), bcols)
    assert rows_of(got) == rows_of(want)
    monkeypatch.setenv("QEH_NO_FUSED_JOIN", "1")
    got2, _ = join_both(ctx, (pk, None), pcols, (bk, None), bcols)
    assert rows_of(got2) == rows_of(got)


@pytest.mark.gpu
def test_join_fused_with_array_offsets(ctx):
    r = np.random.default_rng(77)
    bk = r.permutation(10_000).astype(np.int64)
    ba = r.integers(0, 100, 10_000).astype(np.int64)
    pk = r.integers(0, 12_000, 100_000).astype(np.int64)
    pv = r.random(100_000)
    dp = [ctx.upload(pv, offset=2)]
    op, obd, rows = ctx.hash_join_inner(ctx.upload(pk, offset=4), dp, ctx.upload(bk, offset=2), [ctx.upload(ba, offset=6)])
    wp, wb, wrows = ob.hash_join_inner(ob.HostCol(pk), [ob.HostCol(pv)], ob.HostCol(bk), [ob.HostCol(ba)])
    assert rows == wrows
    assert rows_of([c.to_numpy() for c in op + obd]) == rows_of(wp + wb)


# ---- LEFT / RIGHT / FULL ---------------------------------------------
JT = {"left": 1, "right": 2, "full": 3}


def outer_both(ctx, jt, lk, lcols, rk, rcols):
    dl = [ctx.upload(*c) for c in lcols]
    dr = [ctx.upload(*c) for c in rcols]
    ol, orr, rows = ctx.hash_join_outer(JT[jt], ctx.upload(*lk), dl, ctx.upload(*rk), dr)
    got = [c.to_numpy() for c in ol] + [c.to_numpy() for c in orr]
    wl, wr, wrows = ob.hash_join_outer(JT[jt], ob.HostCol(*lk), [ob.HostCol(*c) for c in lcols], ob.HostCol(*rk),
                                       [ob.HostCol(*c) for c in rcols])
    assert rows == wrows
    return got, wl + wr


@pytest.mark.gpu
@pytest.mark.parametrize("jt", ["left", "right", "full"])
def test_outer_join_arrow_goldens(ctx, jt):
    """Device == Arrow's hash join on the committed fixtures (tests/golden/join_*.npz)."""
    import os
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    z = np.load(os.path.join(gold, "join.npz"), allow_pickle=False)
    w = np.load(os.path.join(gold, f"join_{jt}.npz"), allow_pickle=False)

    def c(zz, name):
        return zz[name], zz[name + "__valid"]
    lk, lv, rk, ra = c(z, "left_lk"), c(z, "left_lv"), c(z, "right_rk"), c(z, "right_ra")
    dl = [ctx.upload(*lk), ctx.upload(*lv)]
    dr = [ctx.upload(*rk), ctx.upload(*ra)]
    ol, orr, rows = ctx.hash_join_outer(JT[jt], ctx.upload(*lk), dl, ctx.upload(*rk), dr)
    got = [x.to_numpy() for x in ol + orr]
    want = [c(w, "out_" + n) for n in ("lk", "lv", "rk", "ra")]
    assert rows == len(want[0][0])
    assert sorted_rows(got) == sorted_rows(want)


@pytest.mark.gpu
@pytest.mark.parametrize("jt", ["left", "right", "full"])
@pytest.mark.parametrize("shape", ["unique", "dups_nulls_int32", "empty_left", "empty_right", "disjoint", "large"])
def test_outer_join_vs_oracle(ctx, jt, shape):
    r = np.random.default_rng(len(shape) * 7 + JT[jt])
    if shape == "unique":
        rk = (r.permutation(5000) * 2).astype(np.int64)
        lk = r.integers(0, 10_000, 20_000).astype(np.int64)
        lkv = rkv = None
    elif shape == "dups_nulls_int32":
        rk = r.integers(0, 300, 2000).astype(np.int32)
        lk = r.integers(0, 400, 30_000).astype(np.int64)
        lkv, rkv = r.random(len(lk)) > 0.05, r.random(len(rk)) > 0.1
    elif shape == "empty_left":
        lk, rk = np.zeros(0, np.int64), r.integers(0, 50, 100).astype(np.int64)
        lkv = rkv = None
    elif shape == "empty_right":
        lk, rk = r.integers(0, 50, 100).astype(np.int64), np.zeros(0, np.int64)
        lkv = rkv = None
    elif shape == "disjoint":
        lk, rk = np.arange(0, 1000, dtype=np.int64), np.arange(5000, 5500, dtype=np.int64)
        lkv = rkv = None
    else:
        rk = r.permutation(400_000).astype(np.int64)[:300_000]
        lk = r.integers(0, 500_000, 2_000_000).astype(np.int64)
        lkv = rkv = None
    if lkv is None:
        lkv = np.ones(len(lk), bool) if shape == "dups_nulls_int32" else None
    lcols = [(lk, lkv), (r.random(len(lk)), r.random(len(lk)) > 0.2), (r.random(len(lk)) > 0.5, None)]
    rcols = [(rk, rkv), (r.integers(-9, 9, len(rk)).astype(np.int32), None)]
    got, want = outer_both(ctx, jt, (lk, lkv), lcols, (rk, rkv), rcols)
    assert sorted_rows(got) == sorted_rows(want)


@pytest.mark.gpu
@pytest.mark.parametrize("jt", ["left", "right", "full"])
def test_outer_join_unique_in_place_matches_compacting_path(ctx, monkeypatch, jt):
    """Unique build keys take the in-place path (one row per probe row, probe order); the
    compacting path (QEH_OUTER_COMPACT) and the oracle give the same rows, and LEFT keeps
    probe order exactly."""
    r = np.random.default_rng(11)
    rk = (r.permutation(30_000) * 3).astype(np.int64)[:20_000]
    lk = r.integers(0, 90_000, 70_001).astype(np.int64)
    lkv = r.random(len(lk)) > 0.03
    lcols = [(lk, lkv), (r.random(len(lk)), r.random(len(lk)) > 0.2)]
    rcols = [(r.integers(-5, 5, len(rk)).astype(np.int64), r.random(len(rk)) > 0.1), (rk, None)]
    got, want = outer_both(ctx, jt, (lk, lkv), lcols, (rk, None), rcols)
    assert sorted_rows(got) == sorted_rows(want)
    if jt == "left":
        assert rows_of(got) == rows_of(want)
    monkeypatch.setenv("QEH_OUTER_COMPACT", "1")
    got2, _ = outer_both(ctx, jt, (lk, lkv), lcols, (rk, None), rcols)
    assert sorted_rows(got2) == sorted_rows(want)


@pytest.mark.gpu
@pytest.mark.parametrize("jt", ["left", "right"])
@pytest.mark.parametrize("nb", [1, 2, 3])
def test_outer_join_embedded_build_path(ctx, jt, nb):
    """LEFT/RIGHT over a unique DIRECT build with non-null 8-byte payloads: the fused embedded
    probe (k_outer_embed) writes the build columns in probe order and returns the preserved
    side as views; rows == oracle, in order."""
    r = np.random.default_rng(nb * 5 + len(jt))
    nbuild, nprobe = 50_000, 300_007
    bk = (r.permutation(80_000)[:nbuild] - 1000).astype(np.int64)
    pk = r.integers(-3000, 82_000, nprobe).astype(np.int64)
    pkv = r.random(nprobe) > 0.02
    bcols = [(bk, None), (r.random(nbuild), None), (r.integers(-9, 9, nbuild).astype(np.int64), None)][:nb]
    pcols = [(pk, pkv), (r.random(nprobe) > 0.5, r.random(nprobe) > 0.1)]
    if jt == "left":
        got, want = outer_both(ctx, jt, (pk, pkv), pcols, (bk, None), bcols)
    else:
        got, want = outer_both(ctx, jt, (bk, None), bcols, (pk, pkv), pcols)
    assert rows_of(got) == rows_of(want)


@pytest.mark.gpu
@pytest.mark.parametrize("bkind", ["int_narrow", "int_mid", "float", "two_cols", "int_wide"])
@pytest.mark.parametrize("npc,nprobe", [(0, 1), (1, 64), (2, 300_007), (3, 131_072)])
def test_full_join_fused_paths(ctx, bkind, npc, nprobe):
    """FULL over a unique DIRECT build (k_full_embed / k_outer_embed32 + the appended unmatched build rows):
    NULL probe keys, build keys never probed, probe columns copied (0-3, non-null 8-byte), the build columns
    as 2-B / 4-B records (one narrow Int64 column) or 8-B records with the flag word; every row vs the oracle."""
    r = np.random.default_rng(npc * 7 + nprobe + len(bkind))
    nbuild = 40_000
    bk = (r.permutation(90_000)[:nbuild] + 500).astype(np.int64)
    pk = r.integers(0, 91_000, nprobe).astype(np.int64)
    pkv = r.random(nprobe) > 0.03
    if bkind == "int_narrow":
        bcols = [(r.integers(-700, 700, nbuild).astype(np.int64), None)]
    elif bkind == "int_mid":  # 4-B records
        bcols = [(r.integers(-(1 << 20), 1 << 20, nbuild).astype(np.int64), None)]
    elif bkind == "int_wide":
        bcols = [(r.integers(-(2 ** 62), 2 ** 62, nbuild).astype(np.int64), None)]
    elif bkind == "float":
        bcols = [(r.random(nbuild), None)]
    else:
        bcols = [(r.random(nbuild), None), (bk * 3, None)]
    pcols = [(pk, None), (r.random(nprobe), None), (r.integers(-5, 5, nprobe).astype(np.int64), None)][:npc]
    got, want = outer_both(ctx, "full", (pk, pkv), pcols, (bk, None), bcols)
    assert sorted_rows(got) == sorted_rows(want)


@pytest.mark.gpu
@pytest.mark.parametrize("jt", ["left", "right", "full"])
@pytest.mark.parametrize("rec", ["u16", "u32"])
@pytest.mark.parametrize("shape", ["uniform", "one_slice", "ragged_int32", "big"])
def test_outer_slice_probe(ctx, monkeypatch, jt, rec, shape):
    """The order-preserving slice probe (k_outer_slice.hip, forced below its size threshold): phase A
    partitions the probe rows' key offsets by table slice with a replayable ranking, phase B looks them up
    in LDS (FULL: matched flags), phase C restores probe order.  Every output row equals the oracle's in
    order (the preserved side's rows come first, in probe order; FULL's unmatched build rows after them,
    compared as a multiset): NULL probe keys, keys below / above the build range, 2-B and 4-B records,
    one slice taking every row (many chunks per tile), Int32 keys and a ragged last tile."""
    monkeypatch.setenv("QEH_OUTER_SLICE", "1")
    r = np.random.default_rng(len(jt) * 31 + len(rec) * 7 + len(shape))
    nbuild, span, nprobe, kdt = 60_000, 300_000, 700_001, np.int64
    if shape == "big":
        nbuild, span, nprobe = 1_500_000, 6_000_000, 6_000_000
    elif shape == "ragged_int32":
        nprobe, kdt = 123_457, np.int32
    bk = (r.permutation(span)[:nbuild] + 1000).astype(kdt)
    if shape == "one_slice":
        pk = r.integers(1000, 1000 + 30_000, nprobe).astype(kdt)
    else:
        pk = r.integers(0, span + 3000, nprobe).astype(kdt)
    pkv = r.random(nprobe) > 0.05
    lo, hi = (-700, 700) if rec == "u16" else (-(1 << 24), 1 << 24)
    bcol = (r.integers(lo, hi, nbuild).astype(np.int64), None)
    pcols = [(r.random(nprobe), None), (pk.astype(np.int64), None)] if jt == "full" else [(r.random(nprobe), None)]
    ctx.timing(True)
    ctx.timing_reset()
    try:
        if jt == "right":
            got, want = outer_both(ctx, jt, (bk, None), [bcol], (pk, pkv), pcols)
        else:
            got, want = outer_both(ctx, jt, (pk, pkv), pcols, (bk, None), [bcol])
        ran = ctx.kernel_time("outer_slice")[1]
    finally:
        ctx.timing(False)
    assert ran == 1
    # probe-order rows: exact, position by position (values compared where valid)
    for (gv, gm), (wv, wm) in zip(got, want):
        gm = np.ones(len(gv), bool) if gm is None else gm
        wm = np.ones(len(wv), bool) if wm is None else wm
        assert len(gv) == len(wv)
        m = min(len(gv), nprobe)
        assert np.array_equal(gm[:m], wm[:m])
        assert np.array_equal(gv[:m][gm[:m]], wv[:m][wm[:m]])
    if jt == "full":
        tail = lambda cols: sorted_rows([(v[nprobe:], None if m is None else m[nprobe:]) for v, m in cols])
        assert tail(got) == tail(want)


@pytest.mark.gpu
@pytest.mark.parametrize("jt", ["left", "full"])
def test_outer_join_full_size_vs_oracle(ctx, jt):
    """The outer-join bench shape at its full size (2e8 probe rows with keys over twice the build's
    range, 1e7 build rows, 2-B records: the order-preserving slice probe) against the oracle's
    qo_hash_join_outer: the probe rows' part of the output in probe order, chunk by chunk (a LEFT /
    FULL join is row-wise in the probe side), values and validity exact; FULL's unmatched build rows
    after them as a multiset."""
    from qe_hip import abi
    seed, n, nd = 0x5EED, 200_000_000, 10_000_000
    fk = ctx.generate(abi.GEN_UNIFORM_MOD, seed, 2, n, 2 * nd)
    fv = ctx.generate(abi.GEN_UNIFORM_MOD, seed, 3, n, 1 << 40)
    dk = ctx.generate(abi.GEN_PERMUTATION, seed, 0, nd, nd)
    da = ctx.generate(abi.GEN_UNIFORM_MOD, seed, 6, nd, 1000)
    ctx.timing(True)
    ctx.timing_reset()
    try:
        lo, ro, rows = ctx.hash_join_outer(JT[jt], fk, [fv], dk, [da])
        ran = ctx.kernel_time("outer_slice")[1]
    finally:
        ctx.timing(False)
    assert ran == 1
    gv, gm = lo[0].to_numpy()
    ga, gam = ro[0].to_numpy()
    del lo, ro, fk, fv, dk, da
    hdk = ob.HostCol(ob.generate(abi.GEN_PERMUTATION, seed, 0, nd, nd))
    hda = ob.HostCol(ob.generate(abi.GEN_UNIFORM_MOD, seed, 6, nd, 1000))
    step = 25_000_000
    for r0 in range(0, n, step):
        m = min(step, n - r0)
        hk = ob.HostCol(ob.generate(abi.GEN_UNIFORM_MOD, seed, 2, m, 2 * nd, row0=r0))
        hv = ob.HostCol(ob.generate(abi.GEN_UNIFORM_MOD, seed, 3, m, 1 << 40, row0=r0))
        wl, wr, wrows = ob.hash_join_outer(JT["left"], hk, [hv], hdk, [hda])
        assert wrows == m  # unique build keys: one row per probe row
        (wv, _), (wa, wam) = wl[0], wr[0]
        assert np.array_equal(gv[r0:r0 + m], wv)
        want_m = np.ones(m, bool) if wam is None else wam
        got_m = np.ones(m, bool) if gam is None else gam[r0:r0 + m]
        assert np.array_equal(got_m, want_m)
        assert np.array_equal(ga[r0:r0 + m][got_m], wa[want_m])
    if jt == "full":
        # the build rows no probe key matched, after the probe rows, with the probe side NULL
        tail = ga[n:]
        assert gm is not None and not gm[n:].any()
        hit = np.zeros(nd, bool)
        for r0 in range(0, n, step):
            m = min(step, n - r0)
            hk = ob.generate(abi.GEN_UNIFORM_MOD, seed, 2, m, 2 * nd, row0=r0)
            hit[hk[hk < nd]] = True
        dkh = ob.generate(abi.GEN_PERMUTATION, seed, 0, nd, nd)
        dah = ob.generate(abi.GEN_UNIFORM_MOD, seed, 6, nd, 1000)
        want_tail = np.sort(dah[~hit[dkh]])
        assert rows == n + len(want_tail)
        assert np.array_equal(np.sort(tail), want_tail)
    else:
        assert rows == n


@pytest.mark.gpu
def test_row_number_windowed_scatter_path(ctx, monkeypatch):
    """n > 2^22: the direct scatter and the experimental windowed scatter (QEH_RN_WINDOWED:
    (destination, rn) pairs grouped by output window by one radix pass) both match the oracle."""
    r = np.random.default_rng(21)
    n = 5_000_001
    k = r.integers(0, 1 << 16, n).astype(np.int64)
    v = r.integers(-(2 ** 40), 2 ** 40, n).astype(np.int64)
    got = ctx.row_number([ctx.upload(k)], [ctx.upload(v)], [True]).to_numpy()[0]
    want = ob.row_number([ob.HostCol(k)], [ob.HostCol(v)], [True])
    assert np.array_equal(got, want)
    monkeypatch.setenv("QEH_RN_WINDOWED", "1")
    assert np.array_equal(ctx.row_number([ctx.upload(k)], [ctx.upload(v)], [True]).to_numpy()[0], want)
