"""One rank of a multi-process rehearsal of qe_hip.distributed (launched by
tests/test_distributed.py as separate processes; RANK/WORLD_SIZE/MASTER_* in
the environment).  mode "exchange": CPU-only gloo all-to-all of partition-major
rows.  mode "gpu": every rank computes on cuda:0, collectives over gloo (host
tensors) — the one-GPU rehearsal of the RCCL path."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def rows_for(rank, n=5000):
    r = np.random.default_rng(100 + rank)
    k = r.integers(0, 997, n).astype(np.int64)
    v = r.random(n)
    return k, v


def mode_exchange(rank, world):
    from qe_hip.distributed import exchange
    k, v = rows_for(rank)
    part = k % world  # stand-in partition function (the device hash is tested on the GPU)
    order = np.argsort(part, kind="stable")
    counts = np.bincount(part, minlength=world)
    recv_counts, (rk, rv) = exchange(torch.tensor(counts), [torch.from_numpy(k[order]), torch.from_numpy(v[order])])
    all_k = np.concatenate([rows_for(r)[0] for r in range(world)])
    all_v = np.concatenate([rows_for(r)[1] for r in range(world)])
    mine = all_k % world == rank
    assert int(recv_counts.sum()) == int(mine.sum())
    got = sorted(zip(rk.numpy().tolist(), rv.numpy().tolist()))
    want = sorted(zip(all_k[mine].tolist(), all_v[mine].tolist()))
    assert got == want


def mode_exchange_bytes(rank, world):
    """Variable-size payloads (the bytes of Utf8 columns) ride the same all-to-all with their own
    per-rank byte counts (exchange(..., byte_splits))."""
    from qe_hip.distributed import exchange
    r = np.random.default_rng(7 + rank)
    n = 3000
    dest = r.integers(0, world, n)
    strs = [f"r{rank}-{i}-" + "x" * int(r.integers(0, 9)) for i in range(n)]
    order = np.argsort(dest, kind="stable")
    counts = np.bincount(dest, minlength=world)
    enc = [strs[i].encode() for i in order]
    lens = np.array([len(b) for b in enc], np.int32)
    data = np.frombuffer(b"".join(enc), np.uint8).copy()
    bounds = np.concatenate([[0], np.cumsum(counts)])
    cum = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    splits = [int(cum[bounds[q + 1]] - cum[bounds[q]]) for q in range(world)]
    rc, (rl, rd) = exchange(torch.tensor(counts), [torch.from_numpy(lens), torch.from_numpy(data)], byte_splits={1: splits})
    raw = rd.numpy().tobytes()
    c2 = np.concatenate([[0], np.cumsum(rl.numpy().astype(np.int64))])
    got = sorted(raw[c2[i]:c2[i + 1]].decode() for i in range(len(rl)))
    want = []
    for q in range(world):
        rq = np.random.default_rng(7 + q)
        dq = rq.integers(0, world, n)
        sq = [f"r{q}-{i}-" + "x" * int(rq.integers(0, 9)) for i in range(n)]
        want += [sq[i] for i in range(n) if dq[i] == rank]
    assert got == sorted(want)


def mode_exchange_chunked(rank, world):
    """The chunked all-to-all (distributed._all_to_all / _a2a_rounds, the logic the RCCL branch
    shares) with A2A_CHUNK_BYTES tiny, so one payload moves in many rounds: uneven partitions,
    zero partitions (rank 1 sends nothing to rank 0; the last rank has no rows at all), a 2-D
    payload and a byte-split payload.  Received rows must equal what every source sent, in
    source-rank-major, stable order."""
    from qe_hip import distributed as D
    D.A2A_CHUNK_BYTES = 40  # 5 int64 rows / 2 (3 x f32) rows / 40 bytes per peer per round

    def shard(q):
        r = np.random.default_rng(900 + q)
        n = 0 if q == world - 1 else 37 + 53 * q
        dest = r.integers(0, world, n)
        if q == 1:
            dest[dest == 0] = world - 1  # rank 1 -> rank 0: zero rows
        k = (q * 100_000 + np.arange(n)).astype(np.int64)  # globally unique, source-ordered ids
        w = r.random((n, 3)).astype(np.float32)
        strs = [f"{q}:{i}" + "z" * int(r.integers(0, 30)) for i in range(n)]
        return dest, k, w, strs

    dest, k, w, strs = shard(rank)
    order = np.argsort(dest, kind="stable")
    counts = np.bincount(dest, minlength=world).astype(np.int64)
    enc = [strs[i].encode() for i in order]
    lens = np.array([len(b) for b in enc], np.int32)
    data = np.frombuffer(b"".join(enc), np.uint8).copy() if enc else np.zeros(0, np.uint8)
    bounds = np.concatenate([[0], np.cumsum(counts)])
    cum = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    splits = [int(cum[bounds[q + 1]] - cum[bounds[q]]) for q in range(world)]
    rc, (rk, rw, rl, rd) = exchange_host(torch.tensor(counts), [torch.from_numpy(k[order]), torch.from_numpy(w[order]),
                                                                torch.from_numpy(lens), torch.from_numpy(data)],
                                         byte_splits={3: splits})
    want_k, want_w, want_s = [], [], []
    for q in range(world):
        dq, kq, wq, sq = shard(q)
        sel = np.nonzero(dq == rank)[0]  # stable: source order inside each source
        want_k.append(kq[sel])
        want_w.append(wq[sel])
        want_s += [sq[i] for i in sel]
    assert np.array_equal(rk.numpy(), np.concatenate(want_k))
    assert np.array_equal(rw.numpy(), np.concatenate(want_w).reshape(-1, 3))
    raw = rd.numpy().tobytes()
    c2 = np.concatenate([[0], np.cumsum(rl.numpy().astype(np.int64))])
    assert [raw[c2[i]:c2[i + 1]].decode() for i in range(len(rl))] == want_s
    assert int(rc.sum()) == len(want_s)


def exchange_host(counts, payloads, byte_splits=None):
    from qe_hip.distributed import exchange
    return exchange(counts, payloads, byte_splits=byte_splits)


def mode_gpu_exchange(rank, world):
    """DistributedExecutor.exchange: device Partitioner (Hash over Int64 + Utf8 keys, Range over
    Int64, Single) + all-to-all of Int64 / Float64 / Utf8 / Boolean columns with NULLs."""
    import qe_hip
    from qe_hip.distributed import DistributedExecutor
    from qe_hip.partition import DeviceBatch, Hash, Range, Single
    ctx = qe_hip.Context(0)
    dx = DistributedExecutor(ctx)

    def rows(q):
        r = np.random.default_rng(50 + q)
        n = 4000 + 123 * q
        k = r.integers(-50, 50, n).astype(np.int64)
        km = r.random(n) > 0.05
        s = np.array([f"s{int(x) % 7}" for x in r.integers(0, 100, n)], dtype=object)
        sm = r.random(n) > 0.1
        b = r.random(n) > 0.5
        bm = r.random(n) > 0.2
        v = r.random(n)
        return k, km, s, sm, b, bm, v

    def as_rows(cols):
        out = []
        vs = [c.to_numpy() for c in cols]
        for i in range(len(cols[0])):
            out.append(tuple(None if (m is not None and not m[i]) else (x[i].item() if hasattr(x[i], "item") else x[i])
                             for x, m in vs))
        return out

    k, km, s, sm, b, bm, v = rows(rank)
    batch = DeviceBatch(["k", "s", "b", "v"], [ctx.upload(k, km), ctx.upload(s, sm), ctx.upload(b, bm), ctx.upload(v)])
    everything = []
    for q in range(world):
        kq, kmq, sq, smq, bq, bmq, vq = rows(q)
        everything += [(None if not kmq[i] else int(kq[i]), None if not smq[i] else sq[i],
                        None if not bmq[i] else bool(bq[i]), float(vq[i])) for i in range(len(kq))]
    key = lambda t: tuple((x is None, x) for x in t)  # noqa: E731
    for strat in (Hash(["k", "s"], world), Range("k", [int(x) for x in np.linspace(-40, 40, world - 1)]) if world > 1
                  else Range("k", []), Single()):
        got = dx.exchange(strat, batch)
        mine = as_rows(got.columns)
        allrecv = [None] * world
        dist.all_gather_object(allrecv, mine)
        union = sorted([t for part in allrecv for t in part], key=key)
        assert union == sorted(everything, key=key), type(strat).__name__
        if isinstance(strat, Hash):
            owner = {}
            for q, part in enumerate(allrecv):
                for t in part:
                    assert owner.setdefault((t[0], t[1]), q) == q  # equal keys share a rank
        elif isinstance(strat, Range):
            bnd = strat.boundaries
            for t in mine:
                if t[0] is None:
                    assert rank == 0
                else:
                    assert rank == next((i for i, x in enumerate(bnd) if t[0] < x), len(bnd))
        else:
            assert (len(mine) == len(everything)) if rank == 0 else not mine
    ctx.close()


def mode_gpu(rank, world):
    import qe_hip
    import oracle_bind as ob
    from helpers import assert_grouped_equal, sorted_rows
    from qe_hip import AggregateFunction as AF, BinaryOp, abi, binop, col, lit
    from qe_hip.distributed import DistributedExecutor
    ctx = qe_hip.Context(0)
    dx = DistributedExecutor(ctx)
    # --- shuffle join: fact shard per rank x dim shard per rank
    def fact(r):
        g = np.random.default_rng(10 + r)
        return g.integers(0, 3000, 40_000).astype(np.int64), g.random(40_000)
    def dim(r):
        keys = np.arange(r, 3000, world, dtype=np.int64)  # disjoint shards of a unique key set
        return keys, keys * 7
    fk, fv = fact(rank)
    dk, da = dim(rank)
    op, obd, rows = dx.hash_join_inner(0, [ctx.upload(fk), ctx.upload(fv)], 0, [ctx.upload(dk), ctx.upload(da)])
    res = dx.gather_to_root(op + obd)
    if rank == 0:
        FK = np.concatenate([fact(r)[0] for r in range(world)])
        FV = np.concatenate([fact(r)[1] for r in range(world)])
        DK = np.concatenate([dim(r)[0] for r in range(world)])
        DA = np.concatenate([dim(r)[1] for r in range(world)])
        wp, wb, wrows = ob.hash_join_inner(ob.HostCol(FK), [ob.HostCol(FK), ob.HostCol(FV)], ob.HostCol(DK),
                                           [ob.HostCol(DK), ob.HostCol(DA)])
        assert sorted_rows(res) == sorted_rows(wp + wb)
    # --- distributed group by (partial/final)
    g = np.random.default_rng(50 + rank)
    k = g.integers(0, 300, 30_000).astype(np.int64)
    v = g.integers(-1000, 1000, 30_000).astype(np.int64)
    keys, aggs_out, ng = dx.group_by([ctx.upload(k)], [ctx.upload(v)], [(AF.Sum, 0), (AF.Count, 0), (AF.Min, 0),
                                                                        (AF.Max, 0)])
    res = dx.gather_to_root(keys + aggs_out)
    if rank == 0:
        K = np.concatenate([np.random.default_rng(50 + r).integers(0, 300, 30_000) for r in range(world)])
        V = np.concatenate([np.random.default_rng(50 + r).integers(-1000, 1000, 30_000) for r in range(world)])
        # regenerate exactly as the ranks did (same two draws per rank)
        K, V = [], []
        for r in range(world):
            gg = np.random.default_rng(50 + r)
            K.append(gg.integers(0, 300, 30_000))
            V.append(gg.integers(-1000, 1000, 30_000))
        K, V = np.concatenate(K).astype(np.int64), np.concatenate(V).astype(np.int64)
        wk, wa, wg, _ = ob.hash_aggregate([ob.HostCol(K)], [ob.HostCol(V)], [(AF.Sum, 0), (AF.Count, 0), (AF.Min, 0),
                                                                               (AF.Max, 0)])
        assert_grouped_equal(res[:1], res[1:], wk, wa)
    # --- the BASELINE metric path: broadcast dim, sharded fact
    n, nd = 200_000, 20_000
    x = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 1, n, 100, row0=rank * n)
    kk = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 2, n, nd, row0=rank * n)
    vv = ob.generate(abi.GEN_UNIT_F64, 0x5EED, 3, n, row0=rank * n)
    dkk = ob.generate(abi.GEN_PERMUTATION, 0x5EED, 0, nd, nd)
    dg = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 5, nd, 256)
    pred = binop(col(0), BinaryOp.Greater, lit(49))
    keys, aggs_out, ng = dx.join_filter_aggregate_broadcast([ctx.upload(x), ctx.upload(kk), ctx.upload(vv)], 1, pred,
                                                            ctx.upload(dkk), [ctx.upload(dg)], [(AF.Sum, 2), (AF.Count, 2)])
    res = dx.gather_to_root(keys + aggs_out)
    if rank == 0:
        X = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 1, n * world, 100)
        KK = ob.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 2, n * world, nd)
        VV = ob.generate(abi.GEN_UNIT_F64, 0x5EED, 3, n * world)
        wk, wa, wg = ob.join_filter_aggregate([ob.HostCol(X), ob.HostCol(KK), ob.HostCol(VV)], 1, pred, ob.HostCol(dkk),
                                              [ob.HostCol(dg)], [(AF.Sum, 2), (AF.Count, 2)])
        assert_grouped_equal(res[:1], res[1:], wk, wa, float_aggs=[0])
    # --- distributed ROW_NUMBER (hash shuffle by partition key, reverse exchange, scatter)
    def win(r):
        g = np.random.default_rng(70 + r)
        kk = g.integers(0, 200, 25_000).astype(np.int64)
        km = g.random(25_000) > 0.05
        vv = g.integers(-30, 30, 25_000).astype(np.int64)
        return kk, km, vv
    wk_, wm_, wv_ = win(rank)
    rn = dx.row_number([ctx.upload(wk_, wm_)], [ctx.upload(wv_)], [False])
    res = dx.gather_to_root([rn])
    if rank == 0:
        K = np.concatenate([win(r)[0] for r in range(world)])
        M = np.concatenate([win(r)[1] for r in range(world)])
        V = np.concatenate([win(r)[2] for r in range(world)])
        want = ob.row_number([ob.HostCol(K, M)], [ob.HostCol(V)], [False])
        assert np.array_equal(res[0][0], want)
    # --- distributed RANK and LAG(w, 2, default) (same placement as ROW_NUMBER)
    from qe_hip.plan import WindowFunctionType as WF
    ww_ = np.random.default_rng(170 + rank).normal(size=len(wk_))
    wwm_ = np.random.default_rng(171 + rank).random(len(wk_)) > 0.1
    rk = dx.window(WF.Rank, [ctx.upload(wk_, wm_)], [ctx.upload(wv_)], [False])
    lg = dx.window(WF.Lag, [ctx.upload(wk_, wm_)], [ctx.upload(wv_)], [True], arg=ctx.upload(ww_, wwm_), param=2,
                   default=0.25)
    res = dx.gather_to_root([rk, lg])
    if rank == 0:
        WW = np.concatenate([np.random.default_rng(170 + r).normal(size=len(win(r)[0])) for r in range(world)])
        WM = np.concatenate([np.random.default_rng(171 + r).random(len(win(r)[0])) > 0.1 for r in range(world)])
        want_rk, _ = ob.window(WF.Rank, [ob.HostCol(K, M)], [ob.HostCol(V)], [False])
        assert np.array_equal(res[0][0], want_rk)
        want_lv, want_ok = ob.window(WF.Lag, [ob.HostCol(K, M)], [ob.HostCol(V)], [True], arg=ob.HostCol(WW, WM),
                                     param=2, default=0.25)
        assert np.array_equal(res[1][1], want_ok)
        assert np.array_equal(res[1][0][want_ok], want_lv[want_ok])
    # --- the moved route (non-null Int64 PARTITION BY and ORDER BY keys): partition_hash_move carries the
    # rows, partition_hash_unmove returns the numbers into input order -- ROW_NUMBER, DENSE_RANK, NTILE
    rn2 = dx.row_number([ctx.upload(wk_)], [ctx.upload(wv_)], [True])
    dr2 = dx.window(WF.DenseRank, [ctx.upload(wk_)], [ctx.upload(wv_)], [False])
    nt2 = dx.window(WF.Ntile, [ctx.upload(wk_)], [ctx.upload(wv_)], [True], param=3)
    res = dx.gather_to_root([rn2, dr2, nt2])
    if rank == 0:
        assert np.array_equal(res[0][0], ob.row_number([ob.HostCol(K)], [ob.HostCol(V)], [True]))
        assert np.array_equal(res[1][0], ob.window(WF.DenseRank, [ob.HostCol(K)], [ob.HostCol(V)], [False])[0])
        assert np.array_equal(res[2][0], ob.window(WF.Ntile, [ob.HostCol(K)], [ob.HostCol(V)], [True], param=3)[0])
    # --- distributed ORDER BY (sampled range partition, stable local sort)
    def srt(r):
        g = np.random.default_rng(90 + r)
        a = np.round(g.standard_normal(30_000), 1)
        am = g.random(30_000) > 0.1
        b = g.integers(0, 5, 30_000).astype(np.int64)
        return a, am, b
    for asc in ([True, False], [False, True]):
        a_, am_, b_ = srt(rank)
        rid = (np.arange(30_000) + rank * 30_000).astype(np.int64)  # global input position
        out = dx.sort([ctx.upload(a_, am_), ctx.upload(b_), ctx.upload(rid)], [0, 1], asc)
        res = dx.gather_to_root(out)
        if rank == 0:
            A = np.concatenate([srt(r)[0] for r in range(world)])
            AM = np.concatenate([srt(r)[1] for r in range(world)])
            B = np.concatenate([srt(r)[2] for r in range(world)])
            perm = ob.sort_indices([ob.HostCol(A, AM), ob.HostCol(B)], asc)
            assert np.array_equal(res[2][0], perm.astype(np.int64))
    ctx.close()


def metric_shards(rank, world, n=120_000, nd=30_000, groups=97):
    """This rank's fact shard (x, k with NULLs and misses, v) and dim shard (k with one
    duplicate, g) of one table split by rows; plus the whole tables for the oracle."""
    def fact(q):
        g = np.random.default_rng(300 + q)
        x = g.integers(0, 100, n).astype(np.int64)
        k = g.integers(0, nd + 1000, n).astype(np.int64)
        km = g.random(n) > 0.02
        v = g.random(n)
        return x, k, km, v
    dk_all = np.random.default_rng(5).permutation(nd).astype(np.int64)
    dk_all[11] = dk_all[12]
    dg_all = np.random.default_rng(6).integers(0, groups, nd).astype(np.int64)
    b = np.linspace(0, nd, world + 1).astype(int)
    whole = [np.concatenate(c) for c in zip(*[fact(q) for q in range(world)])]
    return fact(rank), (dk_all[b[rank]:b[rank + 1]], dg_all[b[rank]:b[rank + 1]]), whole, (dk_all, dg_all)


def check_metric_plans(rank, world, dx, ctx):
    """Config 4's hash-partitioned join + aggregate and the sharded broadcast join, both vs the
    oracle's intended-semantics join + filter + aggregate over the whole tables."""
    import oracle_bind as ob
    from helpers import assert_grouped_equal
    from qe_hip import AggregateFunction as AF, BinaryOp, binop, col, lit
    (x, k, km, v), (dk, dg), (X, K, KM, V), (DK, DG) = metric_shards(rank, world)
    pred = binop(col(0), BinaryOp.Greater, lit(49))
    fact = [ctx.upload(x), ctx.upload(k, km), ctx.upload(v)]
    # float MAX: the broadcast join merges partial states by shuffle; SUM / COUNT and integer
    # MIN / MAX / SUM: by dense all-reduce (DistributedExecutor._final_dense)
    for aggs, floats, final in (([(AF.Sum, 2), (AF.Count, 2), (AF.Max, 2)], [0, 2], "shuffle"),
                                ([(AF.Sum, 2), (AF.Count, 2), (AF.Min, 0), (AF.Max, 0), (AF.Sum, 0)], [0], "dense")):
        want = ob.join_filter_aggregate([ob.HostCol(X), ob.HostCol(K, KM), ob.HostCol(V)], 1, pred, ob.HostCol(DK),
                                        [ob.HostCol(DG)], aggs)
        for name, fn in (("shuffle", dx.join_filter_aggregate_shuffle),
                         ("broadcast", lambda *a: dx.join_filter_aggregate_broadcast(*a, build_sharded=True))):
            keys, aggs_out, ng = fn(fact, 1, pred, ctx.upload(dk), [ctx.upload(dg)], aggs)
            if name == "broadcast":
                assert dx.last_final == final, (dx.last_final, final)
                # the dimension repeats a key: the table form (device payloads) detects it and falls back
                if dx.device == "cuda":
                    assert dx.last_build == "allgather", dx.last_build
            res = dx.gather_to_root(keys + aggs_out)
            if rank == 0:
                assert_grouped_equal(res[:1], res[1:], want[0], want[1], float_aggs=floats), name
    # a non-null key: the shuffle's probe side takes the fused id + histogram pass (k_ids_hist_pred)
    aggs = [(AF.Sum, 2), (AF.Count, 2)]
    want = ob.join_filter_aggregate([ob.HostCol(X), ob.HostCol(K), ob.HostCol(V)], 1, pred, ob.HostCol(DK),
                                    [ob.HostCol(DG)], aggs)
    keys, aggs_out, ng = dx.join_filter_aggregate_shuffle([ctx.upload(x), ctx.upload(k), ctx.upload(v)], 1, pred,
                                                          ctx.upload(dk), [ctx.upload(dg)], aggs)
    if world > 1 and dx.device == "cuda":
        # the dimension repeats a key (dk_all[11] == dk_all[12]): the items form sees it and falls back
        assert dx.last_shuffle == "two_pass", dx.last_shuffle
    res = dx.gather_to_root(keys + aggs_out)
    if rank == 0:
        assert_grouped_equal(res[:1], res[1:], want[0], want[1], float_aggs=[0])


def mode_gpu_cfg4(rank, world):
    """BASELINE config 4 as named (hash-partitioned join + aggregate) and the sharded broadcast
    join, two ranks on one GPU over gloo; plus an exchange where only one rank's shard has a
    validity bitmap (nullability must be agreed, or the collectives pair up wrongly)."""
    import qe_hip
    from qe_hip.distributed import DistributedExecutor
    ctx = qe_hip.Context(0)
    dx = DistributedExecutor(ctx)
    check_metric_plans(rank, world, dx, ctx)
    r = np.random.default_rng(40 + rank)
    n = 5000 + 17 * rank
    a = r.integers(0, 50, n).astype(np.int64)
    am = (r.random(n) > 0.2) if rank == 0 else None  # rank 0's shard has NULLs, the others none
    b = r.random(n)
    keys = dx.shuffle(ctx.upload(a, am), [ctx.upload(a, am), ctx.upload(b)])
    got = dx.gather_to_root(keys)
    full = dx.allgather_columns([ctx.upload(a, am), ctx.upload(b)])
    if rank == 0:
        rows = []
        for q in range(world):
            rq = np.random.default_rng(40 + q)
            nq = 5000 + 17 * q
            aq = rq.integers(0, 50, nq).astype(np.int64)
            mq = (rq.random(nq) > 0.2) if q == 0 else np.ones(nq, bool)
            bq = rq.random(nq)
            rows += [(int(aq[i]) if mq[i] else None, float(bq[i])) for i in range(nq)]
        from helpers import rows_of, _key
        assert sorted(rows_of(got), key=_key) == sorted(rows, key=_key)
        fv = [c.to_numpy() for c in full]
        assert rows_of([(fv[0][0], fv[0][1]), (fv[1][0], fv[1][1])]) == rows  # rank order, NULLs kept
    ctx.close()


def mode_gpu_devtensors(rank, world):
    """The RCCL path's device-tensor code with several ranks (two on one GPU): collectives over gloo
    on CUDA tensors (DistributedExecutor(device="cuda")), the library on a torch stream as in the
    bench.  Exercises what a host-tensor rehearsal skips: zero-copy column views as payloads, the
    dimension all-gather overlapped with a prelaunched phase A (and its adoption), the dense
    all-reduce final aggregate, validity flags agreed across ranks (only one rank's fact / dim shard
    carries a bitmap), and the chunked all-to-all with a tiny chunk."""
    import torch
    import qe_hip
    import oracle_bind as ob
    from helpers import assert_grouped_equal
    from qe_hip import AggregateFunction as AF, BinaryOp, binop, col, lit
    from qe_hip import distributed as D
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx = qe_hip.Context(0)
    ctx.set_stream(s.cuda_stream)
    dx = D.DistributedExecutor(ctx, device="cuda")
    check_metric_plans(rank, world, dx, ctx)
    # the metric shape at a size where the slice pipeline (phase A prelaunched beside the
    # all-gather) runs, sharded fact and dim, dense final
    n, nd = 3_000_000, 4_000_000
    x = ob.generate(abi_gen("UNIFORM_MOD"), 0x5EED, 1, n, 100, row0=rank * n)
    kk = ob.generate(abi_gen("UNIFORM_MOD"), 0x5EED, 2, n, nd, row0=rank * n)
    vv = ob.generate(abi_gen("UNIT_F64"), 0x5EED, 3, n, row0=rank * n)
    dk_all = ob.generate(abi_gen("PERMUTATION"), 0x5EED, 0, nd, nd)
    dg_all = ob.generate(abi_gen("UNIFORM_MOD"), 0x5EED, 5, nd, 1024)
    b = np.linspace(0, nd, world + 1).astype(int)
    pred = binop(col(0), BinaryOp.Greater, lit(49))
    aggs = [(AF.Sum, 2), (AF.Count, 2)]
    if rank == 0:
        X = ob.generate(abi_gen("UNIFORM_MOD"), 0x5EED, 1, n * world, 100)
        KK = ob.generate(abi_gen("UNIFORM_MOD"), 0x5EED, 2, n * world, nd)
        VV = ob.generate(abi_gen("UNIT_F64"), 0x5EED, 3, n * world)
        wk, wa, wg = ob.join_filter_aggregate([ob.HostCol(X), ob.HostCol(KK), ob.HostCol(VV)], 1, pred,
                                              ob.HostCol(dk_all), [ob.HostCol(dg_all)], aggs)
    # the items form (default): every rank groups its dim shard by slice, the items are all-gathered,
    # phase A runs once; then the table form (QEH_NO_ITEMS_BCAST): shard tables summed, the
    # prelaunched phase A adopted
    for form in ("items", "table"):
        if form == "table":
            os.environ["QEH_NO_ITEMS_BCAST"] = "1"
        ctx.timing(True)
        ctx.timing_reset()
        keys, aggs_out, ng = dx.join_filter_aggregate_broadcast(
            [ctx.upload(x), ctx.upload(kk), ctx.upload(vv)], 1, pred, ctx.upload(dk_all[b[rank]:b[rank + 1]]),
            [ctx.upload(dg_all[b[rank]:b[rank + 1]])], aggs, build_sharded=True)
        launches = ctx.kernel_time("slice_partition")[1]
        ctx.timing(False)
        os.environ.pop("QEH_NO_ITEMS_BCAST", None)
        assert dx.last_final == "dense"
        assert dx.last_build == form, (dx.last_build, form)
        assert launches == 1, launches  # one phase A (the table form: the prelaunch adopted, not re-run)
        res = dx.gather_to_root(keys + aggs_out)
        if rank == 0:
            assert_grouped_equal(res[:1], res[1:], wk, wa, float_aggs=[0])
    fact = [ctx.upload(x), ctx.upload(kk), ctx.upload(vv)]
    # config 4's shape: the shuffle join's items form -- phase A per destination on every rank, the packed
    # blocks exchanged (all-to-all of keys, values and region counts), phase B on the receiving rank --
    # then the two-pass exchange (QEH_NO_ITEMS_SHUFFLE), both vs the oracle
    for form in ("items", "two_pass"):
        if form == "two_pass":
            os.environ["QEH_NO_ITEMS_SHUFFLE"] = "1"
        keys, aggs_out, ng = dx.join_filter_aggregate_shuffle(fact, 1, pred, ctx.upload(dk_all[b[rank]:b[rank + 1]]),
                                                              [ctx.upload(dg_all[b[rank]:b[rank + 1]])], aggs)
        os.environ.pop("QEH_NO_ITEMS_SHUFFLE", None)
        assert dx.last_shuffle == form, (dx.last_shuffle, form)
        res = dx.gather_to_root(keys + aggs_out)
        if rank == 0:
            assert_grouped_equal(res[:1], res[1:], wk, wa, float_aggs=[0])
    # the items shuffle with COUNT only (no value column) and rank 1's fact shard empty; then probe keys
    # crowded into one slice (a region fills up on every rank: the pack's flag sends every rank to the
    # two-pass form) -- both vs the oracle
    cnt_only = [(AF.Count, 2)]
    empty = rank == 1
    fx = [ctx.upload(x[:0] if empty else x), ctx.upload(kk[:0] if empty else kk), ctx.upload(vv[:0] if empty else vv)]
    keys, aggs_out, ng = dx.join_filter_aggregate_shuffle(fx, 1, pred, ctx.upload(dk_all[b[rank]:b[rank + 1]]),
                                                          [ctx.upload(dg_all[b[rank]:b[rank + 1]])], cnt_only)
    assert dx.last_shuffle == "items", dx.last_shuffle
    res = dx.gather_to_root(keys + aggs_out)
    if rank == 0:
        keep = np.ones(n * world, bool)
        keep[n:2 * n] = False  # rank 1's rows
        ck, ca, _ = ob.join_filter_aggregate([ob.HostCol(X[keep]), ob.HostCol(KK[keep]), ob.HostCol(VV[keep])], 1, pred,
                                             ob.HostCol(dk_all), [ob.HostCol(dg_all)], cnt_only)
        assert_grouped_equal(res[:1], res[1:], ck, ca)
    ksk = (kk % 60_000).astype(np.int64)
    keys, aggs_out, ng = dx.join_filter_aggregate_shuffle([ctx.upload(x), ctx.upload(ksk), ctx.upload(vv)], 1, pred,
                                                          ctx.upload(dk_all[b[rank]:b[rank + 1]]),
                                                          [ctx.upload(dg_all[b[rank]:b[rank + 1]])], aggs)
    assert dx.last_shuffle == "two_pass", dx.last_shuffle
    res = dx.gather_to_root(keys + aggs_out)
    if rank == 0:
        KSK = (KK % 60_000).astype(np.int64)
        sk_, sa_, _ = ob.join_filter_aggregate([ob.HostCol(X), ob.HostCol(KSK), ob.HostCol(VV)], 1, pred,
                                               ob.HostCol(dk_all), [ob.HostCol(dg_all)], aggs)
        assert_grouped_equal(res[:1], res[1:], sk_, sa_, float_aggs=[0])
    # a build key held by two ranks (rank 0 and the last rank) with SUM + COUNT: the no-wait table
    # form sums the two entries to one above G (both group slots >= G / 2), which the table check
    # clears before the probe reads it; the non-empty count then falls short on every rank and every
    # rank falls back to the all-gather form (multi-match join) -- vs the oracle's join
    lo0, hi0 = b[0], b[1]
    lo1, hi1 = b[world - 1], b[world]
    i0 = lo0 + int(np.nonzero(dg_all[lo0:hi0] >= 700)[0][0])
    i1 = lo1 + int(np.nonzero(dg_all[lo1:hi1] >= 700)[0][0])
    dk_dup = dk_all.copy()
    dk_dup[i1] = dk_dup[i0]
    keys, aggs_out, ng = dx.join_filter_aggregate_broadcast(
        fact, 1, pred, ctx.upload(dk_dup[b[rank]:b[rank + 1]]), [ctx.upload(dg_all[b[rank]:b[rank + 1]])], aggs,
        build_sharded=True)
    assert dx.last_build == "allgather", dx.last_build
    res = dx.gather_to_root(keys + aggs_out)
    if rank == 0:
        dk_, da_, _ = ob.join_filter_aggregate([ob.HostCol(X), ob.HostCol(KK), ob.HostCol(VV)], 1, pred,
                                               ob.HostCol(dk_dup), [ob.HostCol(dg_all)], aggs)
        assert_grouped_equal(res[:1], res[1:], dk_, da_, float_aggs=[0])
    # probe keys crowded into one 2^16-key slice: the prelaunched phase A overflows its regions on
    # every rank, the status lane of the lanes' all-reduce tells every rank, and every rank redoes the
    # probe with the checks inline (the synchronous lanes call) -- vs the oracle
    ksk = (kk % 60_000).astype(np.int64)
    keys, aggs_out, ng = dx.join_filter_aggregate_broadcast(
        [ctx.upload(x), ctx.upload(ksk), ctx.upload(vv)], 1, pred, ctx.upload(dk_all[b[rank]:b[rank + 1]]),
        [ctx.upload(dg_all[b[rank]:b[rank + 1]])], aggs, build_sharded=True)
    assert dx.last_build == "table", dx.last_build
    assert dx.last_table_redo, "the region overflow did not reach the redo branch"
    res = dx.gather_to_root(keys + aggs_out)
    if rank == 0:
        KSK = (KK % 60_000).astype(np.int64)
        sk_, sa_, _ = ob.join_filter_aggregate([ob.HostCol(X), ob.HostCol(KSK), ob.HostCol(VV)], 1, pred,
                                               ob.HostCol(dk_all), [ob.HostCol(dg_all)], aggs)
        assert_grouped_equal(res[:1], res[1:], sk_, sa_, float_aggs=[0])
    # rank-local bitmaps: only rank 0's fact shard has NULLs in the aggregate input (every rank
    # must then skip the dense final, which cannot carry all-NULL groups), only rank 1's dim key
    # shard has a (NULL-free) bitmap (every rank must then skip the overlapped all-gather)
    vmask = (np.random.default_rng(7).random(n) > 0.3) if rank == 0 else None
    dkm = np.ones(b[rank + 1] - b[rank], bool) if rank == 1 else None
    keys, aggs_out, ng = dx.join_filter_aggregate_broadcast(
        [ctx.upload(x), ctx.upload(kk), ctx.upload(vv, vmask)], 1, pred, ctx.upload(dk_all[b[rank]:b[rank + 1]], dkm),
        [ctx.upload(dg_all[b[rank]:b[rank + 1]])], aggs, build_sharded=True)
    assert dx.last_final == "shuffle"
    assert dx.last_build == "allgather"  # a bitmap on one rank's dimension shard: no table form
    res = dx.gather_to_root(keys + aggs_out)
    if rank == 0:
        VM = np.concatenate([np.random.default_rng(7).random(n) > 0.3] + [np.ones(n, bool)] * (world - 1))
        wk, wa, wg = ob.join_filter_aggregate([ob.HostCol(X), ob.HostCol(KK), ob.HostCol(VV, VM)], 1, pred,
                                              ob.HostCol(dk_all), [ob.HostCol(dg_all)], aggs)
        assert_grouped_equal(res[:1], res[1:], wk, wa, float_aggs=[0])
    # chunked exchange on device tensors, one shard with a bitmap, a tiny chunk (many rounds)
    D.A2A_CHUNK_BYTES = 4096
    r = np.random.default_rng(40 + rank)
    m = 20_000 + 17 * rank
    a = r.integers(0, 50, m).astype(np.int64)
    am = (r.random(m) > 0.2) if rank == 0 else None
    v = r.random(m)
    got = dx.gather_to_root(dx.shuffle(ctx.upload(a, am), [ctx.upload(a, am), ctx.upload(v)]))
    if rank == 0:
        from helpers import rows_of, _key
        rows = []
        for q in range(world):
            rq = np.random.default_rng(40 + q)
            mq = 20_000 + 17 * q
            aq = rq.integers(0, 50, mq).astype(np.int64)
            vm = (rq.random(mq) > 0.2) if q == 0 else np.ones(mq, bool)
            vq = rq.random(mq)
            rows += [(int(aq[i]) if vm[i] else None, float(vq[i])) for i in range(mq)]
        assert sorted(rows_of(got), key=_key) == sorted(rows, key=_key)
    torch.cuda.synchronize()
    ctx.set_stream(0)
    ctx.close()


def abi_gen(name):
    from qe_hip import abi
    return getattr(abi, "GEN_" + name)


def mode_nccl1(rank, world):
    """The RCCL path itself: world_size 1 over the "nccl" backend (device tensors through
    all_gather / all_to_all on the GPU): exchange, shuffle join, partial/final GROUP BY, the
    sharded broadcast join and config 4's shuffle join, each vs the oracle."""
    import torch
    import qe_hip
    import oracle_bind as ob
    from helpers import assert_grouped_equal, sorted_rows
    from qe_hip import AggregateFunction as AF
    from qe_hip.distributed import DistributedExecutor
    from qe_hip.partition import DeviceBatch, Hash
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx = qe_hip.Context(0)
    ctx.set_stream(s.cuda_stream)
    dx = DistributedExecutor(ctx)
    assert dx.device == "cuda"
    r = np.random.default_rng(3)
    n = 50_000
    k = r.integers(-100, 100, n).astype(np.int64)
    km = r.random(n) > 0.1
    st = np.array([f"s{i % 13}" for i in range(n)], dtype=object)
    b = r.random(n) > 0.5
    v = r.random(n)
    got = dx.exchange(Hash(["k"], 1), DeviceBatch(["k", "s", "b", "v"], [ctx.upload(k, km), ctx.upload(st),
                                                                         ctx.upload(b), ctx.upload(v)]))
    want = [(k, km), (st, None), (b, None), (v, None)]
    assert sorted_rows([c.to_numpy() for c in got.columns]) == sorted_rows(want)
    fk = r.integers(0, 3000, 40_000).astype(np.int64)
    fv = r.random(40_000)
    dk = np.arange(0, 3000, 2, dtype=np.int64)
    da = dk * 7
    op, obd, rows = dx.hash_join_inner(0, [ctx.upload(fk), ctx.upload(fv)], 0, [ctx.upload(dk), ctx.upload(da)])
    wp, wb, wrows = ob.hash_join_inner(ob.HostCol(fk), [ob.HostCol(fk), ob.HostCol(fv)], ob.HostCol(dk),
                                       [ob.HostCol(dk), ob.HostCol(da)])
    assert rows == wrows
    assert sorted_rows([c.to_numpy() for c in op + obd]) == sorted_rows(wp + wb)
    gkey = r.integers(0, 300, 30_000).astype(np.int64)
    gv = r.integers(-1000, 1000, 30_000).astype(np.int64)
    aggs = [(AF.Sum, 0), (AF.Count, 0), (AF.Min, 0), (AF.Max, 0)]
    keys, aggs_out, ng = dx.group_by([ctx.upload(gkey)], [ctx.upload(gv)], aggs)
    wk, wa, wg, _ = ob.hash_aggregate([ob.HostCol(gkey)], [ob.HostCol(gv)], aggs)
    assert ng == wg
    assert_grouped_equal([c.to_numpy() for c in keys], [c.to_numpy() for c in aggs_out], wk, wa)
    check_metric_plans(rank, world, dx, ctx)
    torch.cuda.synchronize()
    ctx.set_stream(0)
    ctx.close()


def main():
    mode = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if mode == "nccl1":
        import torch
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        {"exchange": mode_exchange, "exchange_bytes": mode_exchange_bytes, "exchange_chunked": mode_exchange_chunked,
         "gpu": mode_gpu,
         "gpu_exchange": mode_gpu_exchange, "gpu_cfg4": mode_gpu_cfg4, "nccl1": mode_nccl1,
         "gpu_devtensors": mode_gpu_devtensors}[mode](rank, world)
        dist.barrier()
    finally:
        dist.destroy_process_group()
    print(f"rank {rank} ok")


if __name__ == "__main__":
    main()
