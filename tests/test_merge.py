"""Merge (crates/query-distributed/src/operators.rs:75-224) on the device: qeh_concat,
qeh_sort_indices_nulls and qeh_merge_sorted vs the oracle, the Arrow golden
(tests/golden/merge_sorted.npz) and the reference's own known answer
(operators.rs:343-374: merging [3, 1] and [4, 2] sorted gives [1, 2, 3, 4])."""
import os

import numpy as np
import pytest

import oracle_bind as ob
from qe_hip import Merge, MergeStrategy, SortColumn, abi

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def host(c):
    v, m = c.to_numpy()
    return v, (np.ones(len(v), bool) if m is None else m)


@pytest.mark.gpu
def test_merge_sorted_reference_known_answer(ctx):
    m = Merge.sorted(ctx, ["value"], [SortColumn("value", True, True)])
    out = m.execute([[[ctx.upload(np.array([3, 1], np.int64))]], [[ctx.upload(np.array([4, 2], np.int64))]]])
    assert len(out) == 1
    assert out[0][0].to_numpy()[0].tolist() == [1, 2, 3, 4]


@pytest.mark.gpu
def test_merge_sorted_matches_arrow_golden(ctx):
    z = np.load(os.path.join(GOLD, "merge_sorted.npz"), allow_pickle=False)
    names = ["x", "i", "v", "f", "b", "k"]
    cols = [(z["in_" + n], z["in_" + n + "__valid"]) for n in names]
    bounds = np.concatenate([[0], np.cumsum(z["part_rows"])])
    parts = [[[ctx.upload(v[a:b], m[a:b]) for v, m in cols]] for a, b in zip(bounds[:-1], bounds[1:])]
    m = Merge.sorted(ctx, names, [SortColumn("k", False, False), SortColumn("x", True, True),
                                  SortColumn("v", True, False), SortColumn("missing", True, True)])
    out = m.execute(parts)
    perm = z["perm"]
    for j, (v, mk) in enumerate(cols):
        gv, gm = host(out[0][j])
        assert np.array_equal(gm, mk[perm]), names[j]
        assert np.array_equal(gv[gm], v[perm][mk[perm]]), names[j]


@pytest.mark.gpu
def test_merge_strategies_concat_union_and_unresolved_names(ctx):
    a = [ctx.upload(np.array([5, 6], np.int64))]
    b = [ctx.upload(np.array([1], np.int64))]
    for strat in (MergeStrategy.Concat(), MergeStrategy.UnionDistinct(["value"])):
        out = Merge(ctx, ["value"], strat).execute([[a], [b, a]])
        assert [c[0].to_numpy()[0].tolist() for c in out] == [[5, 6], [1], [5, 6]]
    out = Merge.sorted(ctx, ["value"], [SortColumn("nope")]).execute([[a], [b]])
    assert out[0][0].to_numpy()[0].tolist() == [5, 6, 1]  # no resolvable sort column: concatenation
    assert Merge.sorted(ctx, ["value"], [SortColumn("value")]).execute([[], []]) == []


@pytest.mark.gpu
@pytest.mark.parametrize("sizes", [[0, 5], [1, 1, 1], [31, 33, 64, 7], [1000, 0, 4097]])
def test_concat_all_types_with_offsets(ctx, sizes):
    r = np.random.default_rng(sum(sizes))
    kinds = []
    for n in sizes:
        kinds.append([
            (r.integers(-50, 50, n).astype(np.int64), r.random(n) > 0.2),
            (r.random(n) > 0.5, r.random(n) > 0.3),
            (r.random(n).astype(np.float32), None),
            (np.array([f"s{int(x)}" * (int(x) % 4) for x in r.integers(0, 100, n)], dtype=object), r.random(n) > 0.1),
        ])
    for j in range(4):
        parts = [ctx.upload(k[j][0], k[j][1], offset=(i * 3) % 5) if j != 3 else ctx.upload(k[j][0], k[j][1])
                 for i, k in enumerate(kinds)]
        got = ctx.concat(parts)
        want_v = np.concatenate([k[j][0] for k in kinds]) if sum(sizes) else np.zeros(0)
        want_m = np.concatenate([np.ones(len(k[j][0]), bool) if k[j][1] is None else k[j][1] for k in kinds])
        gv, gm = host(got)
        assert len(gv) == sum(sizes)
        assert np.array_equal(gm, want_m)
        if j == 3:
            assert [x for x, ok in zip(gv, gm) if ok] == [x for x, ok in zip(want_v, want_m) if ok]
        else:
            assert np.array_equal(np.asarray(gv)[gm], np.asarray(want_v)[want_m])


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["int64_nulls_last_desc", "mixed_three_keys", "full_range_nulls_last", "float_keys"])
def test_sort_indices_nulls_vs_oracle(ctx, case):
    r = np.random.default_rng(len(case))
    n = 200_003
    if case == "int64_nulls_last_desc":
        keys = [(r.integers(-1000, 1000, n).astype(np.int64), r.random(n) > 0.1)]
        asc, nf = [False], [False]
    elif case == "mixed_three_keys":
        keys = [(r.integers(0, 20, n).astype(np.int32), r.random(n) > 0.05),
                (r.integers(0, 50, n).astype(np.int64), r.random(n) > 0.2),
                (r.random(n), r.random(n) > 0.1)]
        asc, nf = [True, False, True], [False, True, False]
    elif case == "full_range_nulls_last":
        keys = [(r.integers(-(2 ** 63), 2 ** 63 - 1, n, dtype=np.int64), r.random(n) > 0.3)]
        keys[0][0][:2] = [-(2 ** 63), 2 ** 63 - 1]
        keys[0][1][:2] = True
        asc, nf = [True], [False]
    else:
        keys = [(np.round(r.standard_normal(n), 2), r.random(n) > 0.1), (r.integers(0, 9, n).astype(np.int64), None)]
        asc, nf = [False, True], [False, True]
    got = ctx.sort_indices_nulls([ctx.upload(v, m) for v, m in keys], asc, nf).to_numpy()[0]
    want = ob.sort_indices_nulls([ob.HostCol(v, m) for v, m in keys], asc, nf)
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("dt,asc,nf,nulls,key_col,span", [
    (np.int64, False, False, True, 0, 5000),   # the Merge::sorted bench shape: k DESC NULLS LAST, v payload
    (np.int64, True, True, True, 1, 5000),     # key second, NULLs first
    (np.int32, True, False, False, 0, 5000),   # Int32 key, no NULLs
    (np.int64, False, True, False, 1, 5000),
    (np.int32, False, True, True, 0, 100),     # one radix pass: encode on load and decode on store together
    (np.int64, True, False, True, 1, 2 ** 40),  # five passes
])
def test_merge_sorted_key_payload_pairs_vs_oracle(ctx, dt, asc, nf, nulls, key_col, span):
    """One sort key and one 8-byte payload: the payload rides through the radix passes (no gather)
    and the key column is decoded from the sorted codes.  Stable (ties keep the concatenation order),
    NULL placement, negative keys, several tiles and ragged partitions; equal to the oracle's stable
    sort and to the general path (QEH_NO_PAYLOAD_SORT=1)."""
    rng = np.random.default_rng(7 + key_col)
    sizes = [70_001, 0, 33_333, 9]
    n = sum(sizes)
    k = rng.integers(-span, span, n).astype(dt)  # many ties at the small spans
    kv = rng.random(n) > 0.1 if nulls else np.ones(n, bool)
    v = rng.random(n)
    bounds = np.concatenate([[0], np.cumsum(sizes)])
    parts = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        kc = ctx.upload(k[a:b], kv[a:b]) if nulls else ctx.upload(k[a:b])
        pc = ctx.upload(v[a:b])
        parts.append([kc, pc] if key_col == 0 else [pc, kc])
    cols, rows = ctx.merge_sorted(parts, [key_col], [asc], [nf])
    assert rows == n
    perm = ob.sort_indices_nulls([ob.HostCol(k.astype(np.int64), kv)], [asc], [nf])
    gk, gm = host(cols[key_col])
    gv, _ = host(cols[1 - key_col])
    assert np.array_equal(gm, kv[perm])
    assert np.array_equal(gk[gm], k[perm][kv[perm]])
    assert np.array_equal(gv, v[perm])  # bit-exact payload, stable order
    assert cols[key_col].dtype == (abi.DT_INT32 if dt == np.int32 else abi.DT_INT64)


@pytest.mark.gpu
@pytest.mark.parametrize("asc,nf,nulls", [(True, False, False), (False, True, False), (True, True, True),
                                          (False, False, True)])
def test_merge_sorted_payload_full_range_keys(ctx, asc, nf, nulls):
    """Keys spanning the whole Int64 range (INT64_MIN and INT64_MAX present): the payload sort needs all
    64 key bits (eight passes); with NULLs there is no free code left, so the permutation sort runs.
    Either way the result equals the oracle's stable sort (range + 1 used to wrap to 0)."""
    r = np.random.default_rng(11)
    n = 50_001
    k = r.integers(-(2 ** 63), 2 ** 63 - 1, n, dtype=np.int64)
    k[:4] = [-(2 ** 63), 2 ** 63 - 1, -(2 ** 63), 0]
    k[-3:] = [2 ** 63 - 1, -1, -(2 ** 63)]
    kv = r.random(n) > 0.2 if nulls else np.ones(n, bool)
    kv[:4] = True
    v = r.random(n)
    half = n // 2
    parts = [[ctx.upload(k[a:b], kv[a:b]) if nulls else ctx.upload(k[a:b]), ctx.upload(v[a:b])]
             for a, b in ((0, half), (half, n))]
    cols, rows = ctx.merge_sorted(parts, [0], [asc], [nf])
    assert rows == n
    perm = ob.sort_indices_nulls([ob.HostCol(k, kv)], [asc], [nf])
    gk, gm = host(cols[0])
    gv, _ = host(cols[1])
    assert np.array_equal(gm, kv[perm])
    assert np.array_equal(gk[gm], k[perm][kv[perm]])
    assert np.array_equal(gv, v[perm])


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["bench_shape", "ties_25_bits", "skew_redo", "constant_big", "int32_full", "asc_nulls_first",
                                  "45_bits", "repeats_40", "half_repeats"])
def test_merge_sorted_msd_payload_vs_oracle(ctx, monkeypatch, case):
    """The MSD payload sort (codes of 24..48 bits over >= 2^20 rows: two global 256-way passes on the top
    16 bits, then an LDS sort per sub-bucket): equal to the oracle's stable sort and to the LSD passes
    (QEH_NO_MSD_SORT=1) -- the Merge::sorted bench shape, many ties, a sub-bucket too large for LDS
    (the LSD redo), a large sub-bucket of one repeated key (copied through), Int32 keys over their
    whole range, NULLs first, 45-bit codes (the widest the LDS sort packs), every key 40 times and half
    the keys 40 times (sub-buckets whose counting-sort bucket overflows go to the radix LDS passes).
    Also equal to the radix LDS passes for every sub-bucket (QEH_MSD_RADIX_LDS=1)."""
    r = np.random.default_rng(23)
    n = (1 << 20) + 12_345
    dt, asc, nf, nulls = np.int64, False, False, True
    k = r.integers(0, 2 ** 40, n, dtype=np.int64)
    if case == "ties_25_bits":
        k = r.integers(-(2 ** 23), 2 ** 23, n, dtype=np.int64)
        asc = True
    elif case == "skew_redo":
        k[r.random(n) < 0.3] %= 100_000  # one sub-bucket of ~300K distinct-ish keys
    elif case == "constant_big":
        k[r.random(n) < 0.2] = 123_456_789_012
        asc = True
    elif case == "int32_full":
        k = r.integers(-(2 ** 31), 2 ** 31 - 1, n, dtype=np.int64).astype(np.int32)
        k[:2] = [-(2 ** 31), 2 ** 31 - 1]
        dt, nulls = np.int32, False
    elif case == "asc_nulls_first":
        asc, nf = True, True
    elif case == "45_bits":
        k = r.integers(-(2 ** 43), 2 ** 43, n, dtype=np.int64)
        nulls = False
    elif case == "repeats_40":
        k = r.permutation(np.repeat(r.integers(0, 2 ** 40, n // 40 + 1, dtype=np.int64), 40)[:n])
    elif case == "half_repeats":
        rep = r.permutation(np.repeat(r.integers(0, 2 ** 39, n // 80 + 1, dtype=np.int64), 40)[:n // 2])
        k = np.concatenate([rep, r.integers(2 ** 39, 2 ** 40, n - rep.size, dtype=np.int64)])[r.permutation(n)]
    kv = r.random(n) > 0.05 if nulls else np.ones(n, bool)
    v = r.random(n)
    cuts = [0, n // 3, n // 3 + 7, n]
    parts = [[ctx.upload(k[a:b], kv[a:b]) if nulls else ctx.upload(k[a:b]), ctx.upload(v[a:b])] for a, b in zip(cuts[:-1], cuts[1:])]
    perm = ob.sort_indices_nulls([ob.HostCol(k.astype(np.int64), kv)], [asc], [nf])
    outs = []
    for env in (None, "QEH_MSD_RADIX_LDS", "QEH_NO_MSD_SORT"):
        if env:
            monkeypatch.setenv(env, "1")
        cols, rows = ctx.merge_sorted(parts, [0], [asc], [nf])
        assert rows == n
        gk, gm = host(cols[0])
        gv, _ = host(cols[1])
        assert np.array_equal(gm, kv[perm])
        assert np.array_equal(gk[gm], k[perm][kv[perm]])
        assert np.array_equal(gv, v[perm])
        assert cols[0].dtype == (abi.DT_INT32 if dt == np.int32 else abi.DT_INT64)
        outs.append(gv)
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])


@pytest.mark.gpu
def test_merge_sorted_full_size_vs_oracle(ctx):
    """The Merge::sorted bench configuration at its full size (tools/bench_configs.py cfg_merge: 8
    partitions x 1.25e7 rows, k Int64 over 2^40 with 5 % NULLs, v Float64, ORDER BY k DESC NULLS LAST)
    against the oracle's stable sort of the concatenation: keys, validity and payloads bit-exact (the
    payload order pins stability: ties keep partition-major input order).  Runs the default MSD path
    (two global passes, the counting sort per sub-bucket, radix LDS passes for crowded ones)."""
    seed, per = 0x5EED, 12_500_000
    parts, hk, hv, hm = [], [], [], []
    for p in range(8):
        k = ctx.generate(abi.GEN_UNIFORM_MOD, seed + p, 7, per, 2 ** 40)
        kv, _ = k.to_numpy()
        valid = np.random.default_rng(p).random(per) > 0.05
        v = ctx.generate(abi.GEN_UNIT_F64, seed + p, 8, per)
        parts.append([ctx.upload(kv, valid), v])
        hk.append(kv)
        hm.append(valid)
        hv.append(v.to_numpy()[0])
        k.release()
    cols, rows = ctx.merge_sorted(parts, [0], [False], [False])
    n = 8 * per
    assert rows == n
    k, m, v = np.concatenate(hk), np.concatenate(hm), np.concatenate(hv)
    del hk, hm, hv
    perm = ob.sort_indices_nulls([ob.HostCol(k, m)], [False], [False])
    gk, gm = host(cols[0])
    assert np.array_equal(gm, m[perm])
    assert np.array_equal(gk[gm], k[perm][m[perm]])
    gv, _ = host(cols[1])
    assert np.array_equal(gv.view(np.uint64), v[perm].view(np.uint64))
    for c in cols:
        c.release()
    for a, b in parts:
        a.release()
        b.release()
