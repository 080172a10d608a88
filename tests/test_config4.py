"""BASELINE config 4 (hash-partitioned join + aggregate, 8 ranks) at its full per-rank size, on one GPU.

One rank of DistributedExecutor.join_filter_aggregate_shuffle (the reference's distributed plan:
query-distributed/src/planner.rs:200-249, the hash exchange of partition.rs:151-212) runs, besides the
RCCL all-to-alls, three device legs:
  1. its 1e9 fact rows through the fused filter + 8-way hash exchange pass
     (qeh_filter_partition_hash_move: x > 49 evaluated in the partition pass, (k, v) of the selected
     rows written partition-major);
  2. the 8-way hash exchange of the dimension (qeh_partition_hash_move of (k, g));
  3. the local fused join + partial aggregate over the partition it keeps (qeh_join_filter_aggregate).
Here rank 5 of 8 runs all three over its own shard (rows [5e9, 6e9) of the 8e9-row fact table, the
counter-based generator's rows) and keeps partition 5 of it; the dimension is the whole 1e7-row table
(every rank's dim shard hash-moved gives the same partition 5).  The oracle restates each leg on the
host: the filter, qo_partition_hash (partition_by_hash) for the partition counts and row order, and
qo_join_filter_aggregate_mt for the join + aggregate of partition 5's rows against the whole dimension
(keys of other partitions cannot match).  Partition counts and moved rows bit-exact, COUNT bit-exact,
SUM(v) within 1e-6 relative."""
import os

import numpy as np
import pytest

import oracle_bind as ob
from helpers import assert_grouped_equal
from qe_hip import AggregateFunction as AF
from qe_hip import BinaryOp, abi, binop, col, lit

SEED = 0x5EED


def _host_threads():
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else n)


@pytest.mark.gpu
def test_config4_rank_leg_full_size_vs_oracle(ctx):
    n, nd, world, rank, groups = 1_000_000_000, 10_000_000, 8, 5, 1024
    pred = binop(col(0, "f.x"), BinaryOp.Greater, lit(49))
    aggs = [(AF.Sum, 1), (AF.Count, 1)]
    # leg 1 on the device: this rank's fact shard, filter fused into the 8-way exchange pass
    x = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100, row0=rank * n)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, nd, row0=rank * n)
    v = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n, row0=rank * n)
    pc, pm = ctx.filter_partition_hash_move([x, k, v], pred, 1, world, [1, 2])
    del x, k, v
    off = int(pc[:rank].sum())
    pk, pv = ctx.slice(pm[0], off, int(pc[rank])), ctx.slice(pm[1], off, int(pc[rank]))
    # leg 2: the dimension's 8-way exchange
    dk = ctx.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
    dg = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 5, nd, groups)
    bc, bm = ctx.partition_hash_move([dk], world, [dk, dg])
    boff = int(bc[:rank].sum())
    bk, bg = ctx.slice(bm[0], boff, int(bc[rank])), ctx.slice(bm[1], boff, int(bc[rank]))
    # leg 3: the local fused join + partial aggregate of the kept partition
    gk, ga, g = ctx.join_filter_aggregate([pk, pv], 0, None, bk, [bg], aggs)
    got_k = [c.to_numpy() for c in gk]
    got_a = [c.to_numpy() for c in ga]
    got_pk, got_pv = pk.to_numpy()[0], pv.to_numpy()[0]
    got_bk, got_bg = bk.to_numpy()[0], bg.to_numpy()[0]
    del gk, ga, pk, pv, pm, bk, bg, bm
    # the oracle, leg by leg, over the same rows generated on the host
    hx = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100, row0=rank * n)
    sel = hx > 49
    del hx
    hk = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, nd, row0=rank * n)
    fk = hk[sel]
    del hk
    hv = ob.generate(abi.GEN_UNIT_F64, SEED, 3, n, row0=rank * n)
    fv = hv[sel]
    del hv, sel
    wc, perm = ob.partition_hash([ob.HostCol(fk)], world)
    assert list(pc) == list(wc) and int(pc.sum()) == len(fk)
    rows = perm[off:off + int(wc[rank])]
    del perm
    want_pk, want_pv = fk[rows], fv[rows]
    del fk, fv, rows
    assert np.array_equal(got_pk, want_pk)  # stable partition-major order, bit for bit
    assert np.array_equal(got_pv.view(np.int64), want_pv.view(np.int64))
    hdk = ob.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
    hdg = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 5, nd, groups)
    dwc, dperm = ob.partition_hash([ob.HostCol(hdk)], world)
    assert list(bc) == list(dwc)
    drows = dperm[boff:boff + int(dwc[rank])]
    assert np.array_equal(got_bk, hdk[drows]) and np.array_equal(got_bg, hdg[drows])
    wk, wa, wg = ob.join_filter_aggregate_mt([ob.HostCol(want_pk), ob.HostCol(want_pv)], 0, None, ob.HostCol(hdk),
                                             [ob.HostCol(hdg)], aggs, _host_threads())
    assert g == wg == groups
    assert_grouped_equal(got_k, got_a, wk, wa, float_aggs=[0])
    assert int(got_a[1][0].sum()) == len(want_pk)  # every kept row's key is in the dimension


def _canon(keys, vals_i64):
    """(key, value bits) pairs in a canonical order -- lexicographic by (value bits, key) through two
    stable device sorts -- so two multisets compare with torch.equal."""
    import torch
    o = torch.sort(keys, stable=True).indices
    keys, vals_i64 = keys[o], vals_i64[o]
    o = torch.sort(vals_i64, stable=True).indices
    return keys[o], vals_i64[o]


@pytest.mark.gpu
def test_config4_items_form_full_size_vs_oracle(ctx):
    """Config 4's first-choice plan, the shuffle join's items form (DistributedExecutor._shuffle_items:
    qeh_shuffle_items_begin / _pack / _finish), at its full per-rank size: rank 5 of 8 with 1e9 fact rows.

    Send side, rank 5's shard (rows [5e9, 6e9)): phase A in the per-destination layout, then the pack.
    Every destination's region counts summed per slice equal the oracle's filter + slice partition
    (partition.rs:151-212 restated as the items form's partition function: rank ((k - kmin) >> 16) mod
    world) bit for bit, and each remote destination's packed block holds exactly the oracle's multiset of
    (key, value bits) for that destination (the 16-bit key offsets re-based by their region's slice).

    Receive side: rank 5's finish over what it would receive -- its own block in place (full size) and
    block 5 of the seven other sources, each run through the same begin / pack over the first 1.25e8 rows
    of its own shard -- with every rank's dimension shard as items; its lanes equal the oracle's join +
    aggregate (qo_join_filter_aggregate_mt) over the union of those rows: COUNT exact, SUM within 1e-6."""
    import torch
    from qe_hip.distributed import _DeviceView
    n, n_src, nd, W, me, groups = 1_000_000_000, 125_000_000, 10_000_000, 8, 5, 1024
    pred = binop(col(0, "f.x"), BinaryOp.Greater, lit(49))
    aggs = [(AF.Sum, 2), (AF.Count, 2)]
    # every rank's dimension shard and its stats row (the all-gather's stand-in: concatenation)
    db = np.linspace(0, nd, W + 1).astype(np.int64)
    dshards = [(ctx.generate(abi.GEN_PERMUTATION, SEED, 0, int(db[r + 1] - db[r]), nd, row0=int(db[r])),
                ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 5, int(db[r + 1] - db[r]), groups, row0=int(db[r])))
               for r in range(W)]
    row_len = 7
    rows = []
    for dk, dg in dshards:
        row = torch.empty(row_len, dtype=torch.int64, device="cuda")
        ctx.broadcast_stats(dk, dg, [0, 1], row.data_ptr())
        rows.append(row)
    ctx.sync()
    M = torch.cat(rows)
    Mh = M.cpu().numpy().reshape(W, row_len)
    kmin, kmax, gmin, gmax = int(Mh[:, 1].min()), int(Mh[:, 2].max()), int(Mh[:, 3].min()), int(Mh[:, 4].max())
    G, F = gmax - gmin + 1, ((kmax - kmin + 1) + 65535) >> 16
    S = -(-F // W)

    def fact(r, rows_):
        return [ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 1, rows_, 100, row0=r * n),
                ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, rows_, nd, row0=r * n),
                ctx.generate(abi.GEN_UNIT_F64, SEED, 3, rows_, row0=r * n)]

    # ---- send side of rank 5 at full size ----
    f5 = fact(me, n)
    h = ctx.shuffle_items_begin(f5, 1, pred, aggs, M.data_ptr(), W, me, row_len)
    ok, kp, vp, cp, bc, E, tot = ctx.shuffle_items_pack(h, W)  # (waits for phase A)
    assert ok and E % S == 0
    del f5
    grid = E // S
    kt = torch.as_tensor(_DeviceView(kp, W * bc, "<i2", None))
    vt = torch.as_tensor(_DeviceView(vp, W * bc, "<i8", None))
    ct = torch.as_tensor(_DeviceView(cp, W * E, "<i4", None)).to(torch.int64)
    # the oracle: filter + slice partition of the same rows, generated on the host
    hx = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100, row0=me * n)
    sel = hx > 49
    del hx
    fk = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, nd, row0=me * n)[sel]
    fv = ob.generate(abi.GEN_UNIT_F64, SEED, 3, n, row0=me * n)[sel]
    del sel
    fslice = (fk - kmin) >> 16
    want_slice = np.bincount(fslice, minlength=S * W)
    dest = fslice % W
    del fslice
    assert int(ct.sum()) == len(fk)
    for q in range(W):
        c = ct[q * E:(q + 1) * E]
        got_slice = c.view(S, grid).sum(1).cpu().numpy()
        assert np.array_equal(got_slice, want_slice[np.arange(S) * W + q]), f"destination {q}: slice counts"
        pc = (c + 1) & ~1
        assert int(pc.sum()) == int(tot[q]), f"destination {q}: block total"
        if q == me:
            continue  # (its own block stays in phase A's regions: checked through finish below)
        region = torch.repeat_interleave(torch.arange(E, device="cuda"), pc)
        start = torch.cumsum(pc, 0) - pc
        keep = (torch.arange(int(tot[q]), device="cuda") - start[region]) < c[region]
        key16 = kt[q * bc:q * bc + int(tot[q])][keep].to(torch.int64) & 0xFFFF
        got_k = kmin + (((region[keep] // grid) * W + q) << 16) + key16
        got_v = vt[q * bc:q * bc + int(tot[q])][keep]
        del region, start, keep, key16
        m = dest == q
        want_k = torch.from_numpy(fk[m]).cuda()
        want_v = torch.from_numpy(fv[m].view(np.int64)).cuda()
        del m
        a, b = _canon(got_k, got_v), _canon(want_k, want_v)
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]), f"destination {q}: item multiset"
        del a, b, got_k, got_v, want_k, want_v
    torch.cuda.synchronize()
    uk, uv = [fk[dest == me]], [fv[dest == me]]  # the union rank 5 aggregates, source-major
    del fk, fv, dest
    own_counts = ct[me * E:(me + 1) * E].to(torch.int32).clone()

    # ---- receive side: block 5 of the seven other sources (first 1.25e8 rows of each shard) ----
    rks, rvs, rcs, pout = [], [], [], []
    for r in range(W):
        if r == me:
            rcs.append(own_counts)
            pout.append(0)
            continue
        fr = fact(r, n_src)
        hr = ctx.shuffle_items_begin(fr, 1, pred, aggs, M.data_ptr(), W, r, row_len)
        okr, kpr, vpr, cpr, bcr, Er, totr = ctx.shuffle_items_pack(hr, W)
        assert okr and Er == E
        t5 = int(totr[me])
        rks.append(torch.as_tensor(_DeviceView(kpr, W * bcr, "<i2", None))[me * bcr:me * bcr + t5].clone())
        rvs.append(torch.as_tensor(_DeviceView(vpr, W * bcr, "<i8", None))[me * bcr:me * bcr + t5].clone())
        rcs.append(torch.as_tensor(_DeviceView(cpr, W * E, "<i4", None))[me * E:(me + 1) * E].clone())
        pout.append(t5)
        torch.cuda.synchronize()
        ctx.fused_items_abort(hr)
        del fr
        hx = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n_src, 100, row0=r * n) > 49
        hk = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n_src, nd, row0=r * n)[hx]
        hv = ob.generate(abi.GEN_UNIT_F64, SEED, 3, n_src, row0=r * n)[hx]
        m = (((hk - kmin) >> 16) % W) == me
        uk.append(hk[m]), uv.append(hv[m])
        assert int(m.sum()) == int(rcs[-1].sum())
        del hx, hk, hv, m
    rk = torch.cat(rks + [torch.zeros(4, dtype=torch.int16, device="cuda")])
    rv = torch.cat(rvs + [torch.zeros(4, dtype=torch.int64, device="cuda")])
    rc = torch.cat(rcs)
    src_off = np.concatenate([[0], np.cumsum(pout)[:-1]]).astype(np.int64)
    # every rank's dimension items (built from the same device plan), concatenated rank-major
    nb, span = ctx.fused_items_shape(int(np.diff(db).max()), W)
    OW = 2 * (ctx.FUSED_ITEMS_SLICES + 1)
    gi = torch.empty(W * nb * span, dtype=torch.int32, device="cuda")
    go = torch.empty(W * nb * OW, dtype=torch.int32, device="cuda")
    for r, (dk, dg) in enumerate(dshards):
        ctx.fused_items_build(h, dk, dg, nb, span, gi[r * nb * span:].data_ptr(), go[r * nb * OW:].data_ptr())
    nl = (1 + len(aggs)) * G + 1
    lanes = torch.empty(nl, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    ctx.sync()
    ctx.shuffle_items_finish(h, rk.data_ptr(), rv.data_ptr(), rc.data_ptr(), src_off, gi.data_ptr(), span,
                             go.data_ptr(), W * nb, G, lanes.data_ptr())
    torch.cuda.synchronize()
    assert float(lanes[nl - 1]) == 0.0  # status lane: no duplicate key, no overflow
    okc, ov, g = ctx.dense_states_take(lanes.data_ptr(), len(aggs), gmin, G, 1, 0, abi.DT_INT64,
                                       [abi.DT_FLOAT64, abi.DT_INT64])
    got_k, got_a = [okc.to_numpy()], [c.to_numpy() for c in ov]
    del dshards, gi, go, rk, rv, rc
    hdk = ob.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
    hdg = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 5, nd, groups)
    uk, uv = np.concatenate(uk), np.concatenate(uv)
    wk, wa, wg = ob.join_filter_aggregate_mt([ob.HostCol(uk), ob.HostCol(uv)], 0, None, ob.HostCol(hdk),
                                             [ob.HostCol(hdg)], [(AF.Sum, 1), (AF.Count, 1)], _host_threads())
    assert g == wg
    assert_grouped_equal(got_k, got_a, wk, wa, float_aggs=[0])
    assert int(got_a[1][0].sum()) == len(uk)  # every row rank 5 received met its dimension row
