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
