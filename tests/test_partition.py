"""Partitioner / Exchange on the device: crates/query-distributed/src/
partition.rs and operators.rs:15-73.  Known answers are the reference's own tests
(partition.rs:381-455); range ownership is checked against a restatement of
find_range_partition (partition.rs:320-341)."""
import numpy as np
import pytest

from qe_hip import DeviceBatch, Exchange, Partitioner, PartitionStrategy
from qe_hip.partition import PartitionError


def batch(ctx, ids, names):
    return DeviceBatch(["id", "name"], [ctx.upload(np.array(ids, np.int64)), ctx.upload(np.array(names, dtype=object))])


def rows(b):
    cols = [c.to_numpy() for c in b.columns]
    return [tuple(None if (m is not None and not m[i]) else (v[i].item() if hasattr(v[i], "item") else v[i])
                  for v, m in cols) for i in range(b.num_rows())]


@pytest.mark.gpu
def test_reference_partitioner_known_answers(ctx):
    bs = [batch(ctx, [1, 2], ["a", "b"]), batch(ctx, [3, 4], ["c", "d"]), batch(ctx, [5, 6], ["e", "f"]),
          batch(ctx, [7, 8], ["g", "h"])]
    parts = Partitioner.round_robin(ctx, 2).partition(bs)  # test_round_robin_partition
    assert len(parts) == 2 and [len(p.batches) for p in parts] == [2, 2]
    assert [rows(b) for b in parts[0].batches] == [rows(bs[0]), rows(bs[2])]
    parts = Partitioner.hash(ctx, ["id"], 3).partition([batch(ctx, [1, 2, 3, 4, 5], list("abcde"))])
    assert len(parts) == 3 and sum(p.row_count() for p in parts) == 5  # test_hash_partition
    parts = Partitioner(ctx, PartitionStrategy.Single()).partition(bs[:2])  # test_single_partition
    assert len(parts) == 1 and len(parts[0].batches) == 2 and parts[0].row_count() == 4
    assert Partitioner.round_robin(ctx, 4).num_partitions() == 4  # test_num_partitions
    assert Partitioner.hash(ctx, [], 8).num_partitions() == 8
    assert Partitioner(ctx, PartitionStrategy.Single()).num_partitions() == 1
    assert Exchange.gather(ctx).num_partitions() == 1 and Exchange.hash(ctx, ["id"], 5).num_partitions() == 5


@pytest.mark.gpu
@pytest.mark.parametrize("keys", [["k"], ["s"], ["k", "s"], ["k", "missing"]])
def test_hash_partition_multi_key_conserves_and_colocates(ctx, keys):
    r = np.random.default_rng(len(keys))
    n = 50_000
    k = r.integers(-30, 30, n).astype(np.int64)
    km = r.random(n) > 0.05
    s = np.array([f"v{int(x)}" for x in r.integers(0, 40, n)], dtype=object)
    sm = r.random(n) > 0.1
    b = DeviceBatch(["k", "s", "v"], [ctx.upload(k, km), ctx.upload(s, sm), ctx.upload(r.random(n))])
    parts = Exchange.hash(ctx, keys, 7).execute([b, b])
    got = [t for p in parts for bb in p.batches for t in rows(bb)]
    assert sorted(got, key=str) == sorted(rows(b) * 2, key=str)
    ki = [["k", "s", "v"].index(x) for x in keys if x in ("k", "s", "v")]
    owner = {}
    for p in parts:
        for bb in p.batches:
            assert bb.num_rows() > 0  # empty partition batches are not added
            for t in rows(bb):
                kt = tuple(t[i] for i in ki)
                assert owner.setdefault(kt, p.index) == p.index


@pytest.mark.gpu
def test_range_partition_first_boundary_below_and_errors(ctx):
    r = np.random.default_rng(2)
    n = 20_000
    k = r.integers(-100, 100, n).astype(np.int64)
    km = r.random(n) > 0.1
    bounds = [-50, 0, 0, 60]  # as given, not sorted-deduplicated: the first boundary above wins
    b = DeviceBatch(["k"], [ctx.upload(k, km)])
    parts = Partitioner(ctx, PartitionStrategy.Range("k", bounds)).partition([b])
    assert len(parts) == 5
    for p in parts:
        for bb in p.batches:
            for (x,) in rows(bb):
                want = 0 if x is None else next((i for i, v in enumerate(bounds) if x < v), len(bounds))
                assert p.index == want
    # a non-Int64 key column lands in partition 0 (find_range_partition handles Int64 only)
    f = DeviceBatch(["k"], [ctx.upload(r.random(100))])
    parts = Partitioner(ctx, PartitionStrategy.Range("k", [0])).partition([f])
    assert parts[0].row_count() == 100 and parts[1].row_count() == 0
    with pytest.raises(PartitionError, match="Key column 'zz' not found"):
        Partitioner(ctx, PartitionStrategy.Range("zz", [0])).partition([b])
    with pytest.raises(PartitionError, match="No key columns found in batch"):
        Partitioner.hash(ctx, ["zz"], 2).partition([b])


@pytest.mark.gpu
@pytest.mark.parametrize("n,parts", [(0, 3), (1, 1), (4095, 2), (4097, 8), (300_001, 256), (2_000_003, 8)])
def test_partition_hash_move_matches_permutation(ctx, n, parts):
    """qeh_partition_hash_move == qeh_partition_hash's permutation + gathers (same counts, same
    stable partition-major order), with 1-5 movable columns and a nullable / Utf8 column that
    take the gather path."""
    r = np.random.default_rng(n + parts)
    k = r.integers(-1000, 1000, n).astype(np.int64)
    cols = [ctx.upload(k), ctx.upload(r.random(n)), ctx.upload(r.integers(0, 9, n).astype(np.int64)),
            ctx.upload(r.random(n)), ctx.upload(r.random(n)),
            ctx.upload(r.integers(0, 5, n).astype(np.int64), r.random(n) > 0.3),
            ctx.upload(np.array([f"t{i % 11}" for i in range(n)], dtype=object))]
    counts, moved = ctx.partition_hash_move([cols[0]], parts, cols)
    import ctypes as C
    from qe_hip import abi
    c2 = (C.c_int64 * parts)()
    perm = abi.QehColumn()
    abi.check(ctx.lib.qeh_partition_hash(ctx.h, ctx._cols([cols[0]]), 1, parts, c2, C.byref(perm)))
    perm = ctx._wrap(perm)
    assert list(counts) == list(c2[:]) and counts.sum() == n
    for c, m in zip(cols, moved):
        want = ctx.take(c, perm).to_numpy()
        got = m.to_numpy()
        assert np.array_equal(got[0], want[0]) if got[1] is None else \
            (np.array_equal(got[1], want[1]) and np.array_equal(got[0][got[1]], want[0][want[1]]))


@pytest.mark.gpu
@pytest.mark.parametrize("n,parts", [(0, 2), (1, 1), (4097, 2), (300_001, 7), (2_000_003, 8)])
@pytest.mark.parametrize("int32_key", [False, True])
def test_filter_partition_hash_move_matches_filter_then_partition(ctx, n, parts, int32_key):
    """qeh_filter_partition_hash_move == qeh_filter followed by qeh_partition_hash_move (same
    per-partition counts, same stable partition-major rows): the shuffle's filter fused into the
    exchange's id pass (config 4's probe side)."""
    from qe_hip import BinaryOp, binop, col, lit
    r = np.random.default_rng(n * 3 + parts)
    x = r.integers(0, 100, n).astype(np.int64)
    k = r.integers(-5000, 5000, n).astype(np.int32 if int32_key else np.int64)
    v = r.random(n)
    w = r.integers(-9, 9, n).astype(np.int64)
    cols = [ctx.upload(x), ctx.upload(k), ctx.upload(v), ctx.upload(w)]
    pred = binop(binop(col(0, "x"), BinaryOp.Greater, lit(49)), BinaryOp.And,
                 binop(col(3, "w"), BinaryOp.NotEqual, lit(0)))
    move = [1, 2, 3] if not int32_key else [2, 3]
    counts, moved = ctx.filter_partition_hash_move(cols, pred, 1, parts, move)
    kept, _ = ctx.filter(cols, pred, out_idx=[1] + move)
    want_counts, want = ctx.partition_hash_move([kept[0]], parts, kept[1:])
    assert list(counts) == list(want_counts)
    assert counts.sum() == int(((x > 49) & (w != 0)).sum())
    for got, exp in zip(moved, want):
        assert np.array_equal(got.to_numpy()[0], exp.to_numpy()[0])


@pytest.mark.gpu
def test_filter_partition_hash_move_declines_general_predicates(ctx):
    """A predicate that is not a list of column-literal comparisons: QEH_E_UNSUPPORTED (the
    distributed plan then filters and partitions separately)."""
    from qe_hip import BinaryOp, abi, binop, col, lit
    n = 1000
    cols = [ctx.upload(np.arange(n, dtype=np.int64)), ctx.upload(np.ones(n))]
    pred = binop(binop(col(0, "a"), BinaryOp.Add, lit(1)), BinaryOp.Greater, lit(5))
    with pytest.raises(abi.QehError) as ei:
        ctx.filter_partition_hash_move(cols, pred, 0, 2, [1])
    assert ei.value.status == abi.QEH_E_UNSUPPORTED


def test_oracle_partition_hash_restates_partition_by_hash():
    """qo_partition_hash (the oracle's partition.rs:151-212) against a numpy restatement of the
    same row hash: per-partition counts, partition-major stable order, NULL keys hashed as an
    empty key; rows are conserved (partition.rs:400-415)."""
    import oracle_bind as ob
    M = (1 << 64) - 1

    def mix(k):
        k ^= k >> 33
        k = (k * 0xff51afd7ed558ccd) & M
        k ^= k >> 33
        k = (k * 0xc4ceb9fe1a85ec53) & M
        return k ^ (k >> 33)

    r = np.random.default_rng(8)
    n = 3000
    a = r.integers(-2**62, 2**62, n).astype(np.int64)
    am = r.random(n) > 0.1
    b = r.integers(-9, 9, n).astype(np.int32)
    for keys, parts in (([ob.HostCol(a)], 8), ([ob.HostCol(a, am), ob.HostCol(b)], 5), ([ob.HostCol(b)], 1)):
        counts, perm = ob.partition_hash(keys, parts)
        ids = []
        for i in range(n):
            h = 0x9E3779B97F4A7C15
            for c in keys:
                if c.valid is not None and not c.valid[i]:
                    continue
                v = int(c.values[i]) & M
                h = mix(h ^ ((mix(v) + 0x9E3779B97F4A7C15 + ((h << 6) & M) + (h >> 2)) & M))
            ids.append(h % parts)
        ids = np.array(ids)
        assert np.array_equal(counts, np.bincount(ids, minlength=parts))
        assert np.array_equal(perm, np.argsort(ids, kind="stable").astype(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("nullable_key", [False, True])
def test_partition_hash_move_8_ways_vs_oracle(ctx, nullable_key):
    """Config 4's exchange pass against the oracle at 1e7 rows: qeh_partition_hash_move into 8
    partitions == the oracle's partition_by_hash (partition.rs:151-212) order, counts and rows,
    bit for bit (Int64 key with or without NULLs, Float64 and Int64 payloads)."""
    import oracle_bind as ob
    n, parts = 10_000_000, 8
    r = np.random.default_rng(44)
    k = r.integers(-10**12, 10**12, n).astype(np.int64)
    km = (r.random(n) > 0.01) if nullable_key else None
    v = r.random(n)
    w = r.integers(-10**9, 10**9, n).astype(np.int64)
    key = ctx.upload(k, km)
    counts, moved = ctx.partition_hash_move([key], parts, [key, ctx.upload(v), ctx.upload(w)])
    wc, perm = ob.partition_hash([ob.HostCol(k, km)], parts)
    assert list(counts) == list(wc)
    gk, gm = moved[0].to_numpy()
    assert np.array_equal(gk[gm] if gm is not None else gk, k[perm][km[perm]] if km is not None else k[perm])
    if km is not None:
        assert np.array_equal(gm, km[perm])
    assert np.array_equal(moved[1].to_numpy()[0], v[perm])
    assert np.array_equal(moved[2].to_numpy()[0], w[perm])


@pytest.mark.gpu
@pytest.mark.parametrize("int32_key", [False, True])
def test_filter_partition_hash_move_8_ways_vs_oracle(ctx, int32_key):
    """Config 4's per-rank probe leg (qeh_filter_partition_hash_move: filter fused into the
    8-way hash exchange pass) against the oracle at 1e7 rows: the oracle filter (executor.rs:
    131-155) then the oracle partition_by_hash (partition.rs:151-212) give the same per-partition
    counts and the same partition-major (k, v) rows, bit for bit."""
    import oracle_bind as ob
    from qe_hip import BinaryOp, binop, col, lit
    n, parts = 10_000_000, 8
    r = np.random.default_rng(45)
    x = r.integers(0, 100, n).astype(np.int64)
    k = r.integers(0, 10_000_000, n).astype(np.int32 if int32_key else np.int64)
    v = r.random(n)
    pred = binop(binop(col(0, "x"), BinaryOp.Greater, lit(49)), BinaryOp.And,
                 binop(col(0, "x"), BinaryOp.LessEqual, lit(97)))
    move = [2] if int32_key else [1, 2]  # moved columns are 8-byte (an Int32 key is hashed, not moved)
    counts, moved = ctx.filter_partition_hash_move([ctx.upload(x), ctx.upload(k), ctx.upload(v)], pred, 1, parts,
                                                   move)
    (fk, _), (fv, _) = ob.filter([ob.HostCol(x), ob.HostCol(k), ob.HostCol(v)], pred, out_idx=[1, 2])[0]
    wc, perm = ob.partition_hash([ob.HostCol(fk)], parts)
    assert list(counts) == list(wc) and counts.sum() == int(((x > 49) & (x <= 97)).sum())
    if not int32_key:
        assert np.array_equal(moved[0].to_numpy()[0], fk[perm])
    assert np.array_equal(moved[-1].to_numpy()[0], fv[perm])


@pytest.mark.gpu
@pytest.mark.parametrize("n,parts", [(1, 2), (8191, 3), (8192 * 5 + 17, 8), (2_000_003, 16)])
def test_partition_hash_unmove_inverts_move(ctx, n, parts):
    """qeh_partition_hash_unmove(move(x)) == x: the reverse of the stable hash move, for any row count
    (ragged segments and tiles) and up to 16 partitions; and it places a column computed on the moved
    rows (here the moved row ids) back at each row's input position."""
    r = np.random.default_rng(n + parts)
    k = r.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    v = r.random(n)
    rowid = np.arange(n, dtype=np.int64)
    counts, moved = ctx.partition_hash_move([ctx.upload(k)], parts, [ctx.upload(k), ctx.upload(v), ctx.upload(rowid)])
    assert int(counts.sum()) == n
    back = ctx.partition_hash_unmove(ctx.upload(k), parts, [moved[1], moved[2]])
    assert np.array_equal(back[0].to_numpy()[0], v)
    assert np.array_equal(back[1].to_numpy()[0], rowid)
