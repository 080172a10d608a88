#!/usr/bin/env python3
"""Secondary BASELINE configs on one MI355X (the headline metric is bench.py).

  cfg2  Filter + GROUP BY SUM/COUNT: SELECT k, SUM(v), COUNT(v), SUM(vi) FROM t
        WHERE x > 49 GROUP BY k   (1e8 rows; 32 B/row algorithmic)
  cfg3  INNER hash join 1e9 x 1e7 materialising (f.v, d.a)
        (16 B probe + 16 B output per fact row; build 16 B/dim row)
  cfg5  ROW_NUMBER() OVER (PARTITION BY k ORDER BY v), k in [0, 2^20)
        (16 B read + 8 B write per row)
  filter  the Filter operator alone: SELECT x, k, v WHERE x > 49 (24 B in + 12 B out avg per row)
  limit   the same filter under LIMIT 1000 (capped filter, early exit)
  plan    the metric query through QueryExecutor from host Arrow batches, cold vs device-cached Scan
  left / full   LEFT / FULL outer join 2e8 x 1e7, half the probe rows unmatched
  merge   Merge::sorted of 8 partitions x 1.25e7 rows, ORDER BY k DESC NULLS LAST
  encode  pgwire DataRow text encoding of 1e7 result rows
  partition  device side of a hash Exchange, 1e8 rows into 8 partitions
  cfg5leg    config 5's per-rank device leg at N = 8 (8-way exchange pass, local ROW_NUMBER over the
             received rows, the unmove pass that returns the numbers to input order)
  cfg4leg    config 4's per-rank device leg at N = 8 (fused filter + 8-way exchange pass over 1e9
             rows, the dim shard's exchange pass, the local join of what the rank receives)

Prints one JSON line per config: rows/s, ms per run, algorithmic GB/s and
fraction of 8 TB/s, and the oracle's rows/s on a bounded sample (1 thread).
usage: python tools/bench_configs.py [--only cfg2,cfg3,cfg5,window,filter,limit,plan,left,full,merge,encode,partition] [--scale 1.0]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime: torch first, see qe_hip/abi.py)

import qe_hip  # noqa: E402
import oracle_bind as ob  # noqa: E402
from qe_hip import AggregateFunction as AF, BinaryOp, abi, binop, col, lit  # noqa: E402

PEAK = 8000.0
SEED = 0x5EED


def timed(ctx, fn, reps, names):
    fn()
    ctx.sync()
    ctx.timing(True)
    ctx.timing_reset()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    ctx.sync()
    wall = (time.perf_counter() - t0) / reps
    kt = {n: ctx.kernel_time(n)[0] / reps for n in names}
    ctx.timing(False)
    return wall, kt, out


def line(cfg, rows, wall, alg_bytes, kernel_ms, kernel, cpu, extra=None):
    gbs = alg_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms and alg_bytes else None
    d = {"config": cfg, "rows": rows, "rows_per_s": rows / wall, "ms_per_run": wall * 1e3,
         "dominant_kernel": kernel, "kernel_ms": kernel_ms, "alg_bytes": alg_bytes,
         "achieved_GBs": gbs, "frac_of_8TBs": gbs / PEAK if gbs else None, "cpu_baseline": cpu}
    if extra:
        d.update(extra)
    print(json.dumps(d), flush=True)


def cfg2(ctx, scale):
    n = int(1e8 * scale)
    x = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, 1024)
    v = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n)
    vi = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 4, n, 2 ** 21, lo=-(2 ** 20))
    pred = binop(col(0), BinaryOp.Greater, lit(49))
    fn = lambda: ctx.filter_aggregate([x, k, v, vi], pred, [1], [(AF.Sum, 2), (AF.Count, 2), (AF.Sum, 3)])
    wall, kt, _ = timed(ctx, fn, 10, ["aggregate_rows", "group_insert"])
    m = 20_000_000
    hx = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 1, m, 100)
    hk = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 2, m, 1024)
    hv = ob.generate(abi.GEN_UNIT_F64, SEED, 3, m)
    hvi = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 4, m, 2 ** 21, lo=-(2 ** 20))
    t0 = time.perf_counter()
    fc, rows, _ = ob.filter([ob.HostCol(hx), ob.HostCol(hk), ob.HostCol(hv), ob.HostCol(hvi)], pred)
    fh = [ob.HostCol(a, b) for a, b in fc]
    ob.hash_aggregate([fh[1]], fh, [(AF.Sum, 2), (AF.Count, 2), (AF.Sum, 3)])
    dt = time.perf_counter() - t0
    cpu = {"value": m / dt, "unit": "rows/s", "cores": 1, "kind": "port", "sample": f"{m} rows, {dt:.2f} s"}
    kms = kt["aggregate_rows"] + kt["group_insert"]
    line("cfg2 filter+group-by 1e8", n, wall, 32.0 * n, kms, "k_group_agg_fast (LDS key hash per workgroup)", cpu)


def cfg3(ctx, scale):
    n, nd = int(1e9 * scale), 10_000_000
    fk = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, nd)
    fv = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n)
    dk = ctx.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
    da = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 6, nd, 1000)

    def fn():
        p, b, rows = ctx.hash_join_inner(fk, [fv], dk, [da])
        for c in p + b:
            c.release()
        return rows
    wall, kt, rows = timed(ctx, fn, 3, ["join_probe", "join_gather", "join_build"])
    m = 20_000_000
    hk = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 2, m, nd)
    hv = ob.generate(abi.GEN_UNIT_F64, SEED, 3, m)
    hdk = ob.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
    hda = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 6, nd, 1000)
    t0 = time.perf_counter()
    ob.hash_join_inner(ob.HostCol(hk), [ob.HostCol(hv)], ob.HostCol(hdk), [ob.HostCol(hda)])
    dt = time.perf_counter() - t0
    cpu = {"value": m / dt, "unit": "rows/s", "cores": 1, "kind": "port", "sample": f"{m} probe x {nd} build, {dt:.2f} s"}
    kms = kt["join_probe"] + kt["join_gather"]
    line("cfg3 inner join 1e9 x 1e7", n, wall, 32.0 * n, kms, "k_slice_count + k_slice_partition + k_slice_join_inplace", cpu,
         {"output_rows": rows, "build_ms": kt["join_build"]})


def cfg3_wide(ctx, scale):
    """cfg3 with a full-range Int64 build payload: the u16 frame-of-reference of the slice path
    does not apply, so the fused embedded-record join (k_join_mat) runs."""
    n, nd = int(1e9 * scale), 10_000_000
    fk = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, nd)
    fv = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n)
    dk = ctx.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
    da = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 6, nd, 1 << 62)

    def fn():
        p, b, rows = ctx.hash_join_inner(fk, [fv], dk, [da])
        for c in p + b:
            c.release()
        return rows
    wall, kt, rows = timed(ctx, fn, 3, ["join_probe", "join_gather", "join_build", "join_mat"])
    line("cfg3 inner join 1e9 x 1e7, full-range Int64 payload", n, wall, 32.0 * n, wall * 1e3,
         "k_join_mat (embedded build records)", None, {"output_rows": rows, "kernel_split_ms": kt,
                                                         "note": "kernel_ms = wall: the path has no single timer"})


def cfg_metric_shapes(ctx, scale, only=("sparse", "g17", "agg2")):
    """The metric query beyond the dense-key best case (1e9 fact rows x 1e7 dim rows):
      sparse  dim keys are sparse 64-bit values (H(i), GEN_SPARSE_KEY), fact keys drawn from them
      g17     2^17 groups (d.g uniform in [0, 2^17))
      agg2    two aggregate columns: SUM(f.v), SUM(f.w), COUNT(f.v)
    Algorithmic bytes: 24 B per fact row (x, k, v; +8 B for w) + 16 B per dim row."""
    n, nd = int(1e9 * scale), 10_000_000
    x = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100)
    v = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n)
    pred = binop(col(0), BinaryOp.Greater, lit(49))
    names = ["join_filter_aggregate", "slice_partition", "slice_probe", "slice_keyagg", "join_build", "aggregate_rows"]
    for shape in only:
        if shape == "sparse":
            k = ctx.generate(abi.GEN_SPARSE_KEY, SEED, 2, n, nd)
            dk = ctx.generate(abi.GEN_SPARSE_KEY, SEED, 0, nd, 0)
            dg = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 5, nd, 1024)
            cols, aggs, alg = [x, k, v], [(AF.Sum, 2), (AF.Count, 2)], 24.0
        elif shape == "g17":
            k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, nd)
            dk = ctx.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
            dg = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 5, nd, 1 << 17)
            cols, aggs, alg = [x, k, v], [(AF.Sum, 2), (AF.Count, 2)], 24.0
        else:
            k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, nd)
            dk = ctx.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
            dg = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 5, nd, 1024)
            w = ctx.generate(abi.GEN_UNIT_F64, SEED, 9, n)
            cols, aggs, alg = [x, k, v, w], [(AF.Sum, 2), (AF.Sum, 3), (AF.Count, 2)], 32.0

        def fn():
            gk, ga, g = ctx.join_filter_aggregate(cols, 1, pred, dk, [dg], aggs)
            for c in gk + ga:
                c.release()
            return g
        wall, kt, g = timed(ctx, fn, 5, names)
        # the slice pipeline ran when phase A holds a real share of the wall time (a declined prelaunch
        # leaves a few microseconds on its timers: r04's sparse line summed those, frac 184)
        sliced = kt["slice_partition"] > 0.1 * wall * 1e3
        kms = kt["slice_partition"] + kt["slice_probe"] + kt["slice_keyagg"] if sliced else kt["join_filter_aggregate"]
        dom = ("k_slice_partition + k_slice_keyagg" if kt["slice_keyagg"] else "k_slice_partition + k_slice_probe") \
            if sliced else "single pass (join_filter_aggregate)"
        line(f"metric shape {shape} 1e9 x 1e7", n, wall, alg * n + 16.0 * nd, kms, dom,
             None, {"groups": g, "kernel_split_ms": kt})
        del k, dk, dg


def cfg5(ctx, scale):
    n = int(1e9 * scale)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 7, n, 2 ** 20)
    v = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 8, n, 2 ** 62, lo=-(2 ** 61))

    def fn():
        rn = ctx.row_number([k], [v], [True])
        rn.release()
    wall, kt, _ = timed(ctx, fn, 2, ["radix_pass", "sort_encode", "row_number", "window_partition", "window_sort", "window_place",
                                    "w3_partition", "w3_sort", "w3_place"])
    m = 5_000_000
    hk = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 7, m, 2 ** 20)
    hv = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 8, m, 2 ** 62, lo=-(2 ** 61))
    t0 = time.perf_counter()
    ob.row_number([ob.HostCol(hk)], [ob.HostCol(hv)], [True])
    dt = time.perf_counter() - t0
    cpu = {"value": m / dt, "unit": "rows/s", "cores": 1, "kind": "port", "sample": f"{m} rows, {dt:.2f} s"}
    kms = sum(kt.values())
    line("cfg5 ROW_NUMBER 1e9", n, wall, 24.0 * n, kms, "k_window.hip partition passes + wave sort + placement (LSD sort fallback)", cpu, kt)


def cfg_window(ctx, scale):
    """RANK() and LAG(v, 1) OVER (PARTITION BY k ORDER BY v) on the cfg-5 data (1e9 rows)."""
    from qe_hip.plan import WindowFunctionType as W
    n = int(1e9 * scale)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 7, n, 2 ** 20)
    v = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 8, n, 2 ** 62, lo=-(2 ** 61))
    m = 2_000_000
    hk = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 7, m, 2 ** 20)
    hv = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 8, m, 2 ** 62, lo=-(2 ** 61))
    for name, func, arg, alg in [("RANK", W.Rank, None, 24.0), ("LAG(v,1)", W.Lag, v, 24.0)]:
        def fn():
            ctx.window(func, [k], [v], [True], arg=arg, param=1).release()
        wall, kt, _ = timed(ctx, fn, 2, ["radix_pass", "sort_encode", "window", "window_partition", "window_sort", "window_place", "w3_partition", "w3_sort", "w3_place"])
        t0 = time.perf_counter()
        ob.window(func, [ob.HostCol(hk)], [ob.HostCol(hv)], [True], arg=ob.HostCol(hv) if arg is not None else None,
                  param=1)
        dt = time.perf_counter() - t0
        cpu = {"value": m / dt, "unit": "rows/s", "cores": 1, "kind": "port", "sample": f"{m} rows, {dt:.2f} s"}
        line(f"window {name} 1e9", n, wall, alg * n, sum(kt.values()), "radix sort + k_seg_start/k_window_out", cpu, kt)


def cfg_window_lsd(ctx, scale):
    """Window shapes beyond config 5's: ROW_NUMBER() and RANK() OVER (PARTITION BY k ORDER BY v) with k
    over 2^24 values (groups of 16 consecutive keys in the partitioning path), and ROW_NUMBER over two
    PARTITION BY keys (64 x 2^16 values: their composite key takes the same path), 1e9 rows.
    QEH_WM_NO_SUB=1 / QEH_NO_WINDOW_MSD=1 give the LSD path for comparison.  Algorithmic bytes: 16 B read
    + 8 B written per row (24 B read with the second key)."""
    from qe_hip.plan import WindowFunctionType as W
    n = int(1e9 * scale)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 7, n, 2 ** 24)
    v = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 8, n, 2 ** 62, lo=-(2 ** 61))
    names = ["radix_pass", "sort_encode", "row_number", "window", "window_partition", "window_sort", "window_place", "gather",
             "w3_partition", "w3_sort", "w3_place"]
    for label, fn, alg in [
            ("ROW_NUMBER, k over 2^24", lambda: ctx.row_number([k], [v], [True]).release(), 24.0),
            ("RANK, k over 2^24", lambda: ctx.window(W.Rank, [k], [v], [True]).release(), 24.0)]:
        wall, kt, _ = timed(ctx, fn, 2, names)
        path = "partitioning path" if kt["window_sort"] else "LSD path"
        line(f"window {label} 1e9 ({path})", n, wall, alg * n, sum(kt.values()), path, None,
             {"kernel_split_ms": {q: w for q, w in kt.items() if w}})
    k2 = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 9, n, 64)
    kk = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 7, n, 2 ** 16)
    wall, kt, _ = timed(ctx, lambda: ctx.row_number([kk, k2], [v], [True]).release(), 2, names)
    path = "partitioning path, composite key" if kt["window_sort"] else "LSD path"
    line(f"window ROW_NUMBER, PARTITION BY (k, k2) 1e9 ({path})", n, wall, 32.0 * n, sum(kt.values()), path, None,
         {"kernel_split_ms": {q: w for q, w in kt.items() if w}})


def cfg_outer(ctx, scale, jt=1):
    """LEFT (jt=1) / FULL (jt=3) join, 2e8 probe rows (keys uniform over twice the dim key range,
    so half find no match) x 1e7 dim rows, materialising (f.v, d.a).  Algorithmic bytes: 16 B probe
    read + 16 B output written per output row (+ the FULL tail)."""
    n, nd = int(2e8 * scale), 10_000_000
    fk = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, 2 * nd)
    fv = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n)
    dk = ctx.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
    da = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 6, nd, 1000)

    def fn():
        lo, ro, rows = ctx.hash_join_outer(jt, fk, [fk, fv], dk, [da])
        for c in lo + ro:
            c.release()
        return rows
    wall, kt, rows = timed(ctx, fn, 5, ["join_probe", "join_count", "join_gather", "join_build"])
    m = 10_000_000
    hk = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 2, m, 2 * nd)
    hv = ob.generate(abi.GEN_UNIT_F64, SEED, 3, m)
    hdk = ob.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
    hda = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 6, nd, 1000)
    t0 = time.perf_counter()
    ob.hash_join_outer(jt, ob.HostCol(hk), [ob.HostCol(hk), ob.HostCol(hv)], ob.HostCol(hdk), [ob.HostCol(hda)])
    dt = time.perf_counter() - t0
    cpu = {"value": m / dt, "unit": "rows/s", "cores": 1, "kind": "port", "sample": f"{m} probe x {nd} build, {dt:.2f} s"}
    kms = kt["join_probe"] + kt["join_count"] + kt["join_gather"]
    name = {1: "LEFT", 3: "FULL"}[jt]
    # LEFT over the unique dim takes the embedded path: probe payloads leave as views, so only the
    # key is read and the build column (+ validity) written; FULL gathers every output column
    alg = 16.0 * n + n / 8 if jt == 1 else 16.0 * n + 24.0 * rows
    line(f"{name} outer join 2e8 x 1e7 (50% unmatched)", n, wall, alg, kms,
         "order-preserving slice probe k_os_part + k_os_probe + k_os_emit (FULL: + unmatched build rows)", cpu, {"output_rows": rows, "kernel_split_ms": kt})


def cfg_merge(ctx, scale):
    """Merge::sorted of 8 partitions x 1.25e7 rows (k Int64 with 5 % NULLs, v Float64), ORDER BY k
    DESC NULLS LAST.  Algorithmic bytes: read 16 B + write 16 B per row (+ validity)."""
    parts = []
    per = int(1.25e7 * scale)
    for p in range(8):
        k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED + p, 7, per, 2 ** 40)
        kv, _ = k.to_numpy()
        valid = np.random.default_rng(p).random(per) > 0.05
        parts.append([ctx.upload(kv, valid), ctx.generate(abi.GEN_UNIT_F64, SEED + p, 8, per)])
    n = 8 * per

    def fn():
        cols, rows = ctx.merge_sorted(parts, [0], [False], [False])
        for c in cols:
            c.release()
        return rows
    wall, kt, rows = timed(ctx, fn, 3, ["merge_concat", "radix_pass", "sort_encode", "gather"])
    hk = [p[0].to_numpy() for p in parts]
    m = 4_000_000
    hkk = np.concatenate([a for a, _ in hk])[:m]
    hkv = np.concatenate([b for _, b in hk])[:m]
    t0 = time.perf_counter()
    ob.sort_indices_nulls([ob.HostCol(hkk, hkv)], [False], [False])
    dt = time.perf_counter() - t0
    cpu = {"value": m / dt, "unit": "rows/s", "cores": 1, "kind": "port", "sample": f"{m} rows sort, {dt:.2f} s"}
    line("Merge::sorted 8 x 1.25e7 rows, ORDER BY k DESC NULLS LAST", n, wall, 32.0 * n, sum(kt.values()),
         "k_rs_hist/k_rs_scatter carrying the payload (encode on load in pass 0, decode on store in the last)", cpu, kt)


def cfg_encode(ctx, scale):
    """§8 f4: pgwire DataRow text encoding of a 1e7-row result (k Int64, sum Float64, count Int64),
    the shape of the metric query's output rows at scale.  Bytes: 24 B read per row + the encoded
    messages written."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pg_text
    n = int(1e7 * scale)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, 1 << 40)
    v = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n)
    c = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 4, n, 1000000)

    def fn():
        out = ctx.encode_pg_datarows([k, v, c])
        nb = out.c.values_bytes
        out.release()
        return nb
    wall, kt, nbytes = timed(ctx, fn, 5, ["encode_len", "encode_write"])
    m = 100_000
    hk, hv, hc = (x.to_numpy()[0][:m] for x in (k, v, c))
    t0 = time.perf_counter()
    pg_text.encode_rows([("int64", hk.tolist()), ("float64", hv.tolist()), ("int64", hc.tolist())])
    dt = time.perf_counter() - t0
    cpu = {"value": m / dt, "unit": "rows/s", "cores": 1, "kind": "port",
           "sample": f"{m} rows, oracle/pg_text.py (pure Python), {dt:.2f} s"}
    line("pgwire DataRow text encoding 1e7 x (Int64, Float64, Int64)", n, wall, 24.0 * n + nbytes,
         sum(kt.values()), "k_pg_row_len + k_pg_row_write (Schubfach shortest floats)", cpu,
         {"encoded_bytes": nbytes, "kernel_split_ms": kt})
    # Arrow IPC stream of the same batch (network.rs:56-72): device normalisation + copy to host
    reps = 5
    data = ctx.encode_arrow_ipc([k, v, c], ["k", "sum", "count"])
    t0 = time.perf_counter()
    for _ in range(reps):
        data = ctx.encode_arrow_ipc([k, v, c], ["k", "sum", "count"])
    wall = (time.perf_counter() - t0) / reps
    names, cols, _ = ctx.decode_arrow_ipc(data)
    t0 = time.perf_counter()
    for _ in range(reps):
        names, cols, _ = ctx.decode_arrow_ipc(data)
        for x in cols:
            x.release()
    wall_d = (time.perf_counter() - t0) / reps
    line("Arrow IPC stream encode 1e7 x (Int64, Float64, Int64), device -> host bytes", n, wall, None, None,
         "device normalise + D2H copies", None,
         {"stream_bytes": len(data), "host_GBs": len(data) / wall / 1e9, "decode_ms": wall_d * 1e3,
          "decode_host_GBs": len(data) / wall_d / 1e9})


def cfg_partition(ctx, scale):
    """§8 f2: the device side of a hash Exchange into 8 partitions (one per GPU of a node):
    1e8 rows x (k Int64, v Float64) -> partition-major columns + counts.  Bytes: 16 B read +
    16 B written per row (the permutation is an intermediate)."""
    from qe_hip.partition import DeviceBatch, Hash, Partitioner
    n = int(1e8 * scale)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, 1 << 40)
    v = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n)
    pt = Partitioner(ctx, Hash(["k"], 8))
    b = DeviceBatch(["k", "v"], [k, v])

    def fn():
        counts, moved = pt.batch_move(b)
        for c in moved:
            c.release()
        return counts
    wall, kt, counts = timed(ctx, fn, 5, ["partition_move"])
    line("hash Exchange 1e8 rows x (Int64, Float64) into 8 partitions (device side)", n, wall, 32.0 * n,
         sum(kt.values()), "k_hash_ids8 + k_rs_hist + k_part_scatter (columns moved in one pass)", None,
         {"kernel_split_ms": kt, "max_partition_share": float(max(counts)) / n})


def cfg4_leg(ctx, scale, world=8):
    """BASELINE config 4's per-rank device leg at N = 8, on one GPU: what one rank of the
    hash-partitioned plan runs besides the RCCL all-to-all (DistributedExecutor.
    join_filter_aggregate_shuffle; partition.rs:151-212, planner.rs:200-249):
      1. filter f.x > 49 fused into the 8-way hash exchange pass over its 1e9 fact rows
         (qeh_filter_partition_hash_move: x, k, v read once, (k, v) of the selected rows written
         partition-major);
      2. the 8-way hash exchange pass over its dim shard (1e7 / 8 rows of (k, g));
      3. the local fused join + partial aggregate over what the rank receives: the rows of ITS
         partition from all 8 ranks — stood in for by 8 copies of this rank's partition 0 (same
         size and key distribution: uniform keys send 1/8 of every rank's rows to each rank) —
         against the dim keys of partition 0 (a sparse 1/8 of the key range).
    Algorithmic bytes: 24 B read + 16 B written per selected row in (1), 32 B per dim row in (2),
    16 B per received row in (3)."""
    from qe_hip.partition import DeviceBatch  # noqa: F401  (same package the plan uses)
    n, nd = int(1e9 * scale), 10_000_000
    x = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, nd)
    v = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n)
    dn = nd // world
    dk = ctx.generate(abi.GEN_PERMUTATION, SEED, 0, dn, nd)
    dg = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 5, dn, 1024)
    pred = binop(col(0), BinaryOp.Greater, lit(49))
    aggs = [(AF.Sum, 1), (AF.Count, 1)]
    # what rank 0 receives (built once, outside the timed legs)
    pc, pm = ctx.filter_partition_hash_move([x, k, v], pred, 1, world, [1, 2])
    selected = int(pc.sum())
    recv_k = ctx.concat([ctx.slice(pm[0], 0, int(pc[0]))] * world)
    recv_v = ctx.concat([ctx.slice(pm[1], 0, int(pc[0]))] * world)
    for c in pm:
        c.release()
    full_dk = ctx.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
    full_dg = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 5, nd, 1024)
    bc, bm = ctx.partition_hash_move([full_dk], world, [full_dk, full_dg])
    bk0, bg0 = ctx.slice(bm[0], 0, int(bc[0])), ctx.slice(bm[1], 0, int(bc[0]))
    recv = len(recv_k)

    def leg1():
        c, m = ctx.filter_partition_hash_move([x, k, v], pred, 1, world, [1, 2])
        for q in m:
            q.release()
        return c

    def leg2():
        c, m = ctx.partition_hash_move([dk], world, [dk, dg])
        for q in m:
            q.release()
        return c

    def leg3():
        gk, ga, g = ctx.join_filter_aggregate([recv_k, recv_v], 0, None, bk0, [bg0], aggs)
        for q in gk + ga:
            q.release()
        return g
    names = ["partition_move", "filter", "join_filter_aggregate", "slice_partition", "slice_probe", "join_build"]
    w1, k1, _ = timed(ctx, leg1, 5, names)
    w2, k2, _ = timed(ctx, leg2, 5, names)
    w3, k3, g = timed(ctx, leg3, 5, names)
    # bytes each leg moves through HBM (intermediates included: the exchange's writes and re-reads)
    b1, b2, b3 = 24.0 * n + 16.0 * selected, 32.0 * dn, 16.0 * recv
    kms1 = k1["partition_move"] + k1["filter"]
    kms3 = k3["slice_partition"] + k3["slice_probe"] if k3["slice_partition"] else k3["join_filter_aggregate"]
    legs = {"exchange_pass_fact": {"ms": kms1, "wall_ms": w1 * 1e3, "hbm_bytes_moved": b1,
                                   "moved_GBs": b1 / (kms1 * 1e-3) / 1e9},
            "exchange_pass_dim": {"ms": k2["partition_move"], "wall_ms": w2 * 1e3, "hbm_bytes_moved": b2},
            "local_join": {"ms": kms3, "wall_ms": w3 * 1e3, "hbm_bytes_moved": b3, "rows": recv, "groups": g,
                           "build_ms": k3["join_build"], "kernels": "slice" if k3["slice_partition"] else "single pass",
                           "moved_GBs": b3 / (kms3 * 1e-3) / 1e9}}
    kms = kms1 + k2["partition_move"] + kms3
    # the per-GPU algorithmic bytes of config 4 are the metric's (24 B per fact row
    # + 16 B per dim row read once, intermediates excluded); the exchange is reported separately
    alg = 24.0 * n + 16.0 * nd
    xgmi = (world - 1) / world * (16.0 * selected + 16.0 * dn)
    line(f"cfg4 per-rank device leg at N={world} (1e9 fact rows + 1/{world} dim per rank)", n, w1 + w2 + w3,
         alg, kms, "k_hash_ids8_pred + k_part_scatter (fused filter + 8-way exchange), local fused join",
         None, {"legs": legs, "selected": selected, "exchange_hbm_bytes": b1 + b2 + b3 - 24.0 * n - 16.0 * dn,
                "xgmi_bytes_per_rank": xgmi,
                "note": "frac on SURVEY §8(d)'s 24 B / fact row + 16 B / dim row; the exchange's HBM writes and "
                        "re-reads are in exchange_hbm_bytes, the bytes leaving the rank over xGMI in "
                        "xgmi_bytes_per_rank; RCCL all-to-all time excluded (8-GPU runs are the driver's); "
                        "wall = sum of the legs"})


def cfg4_items_leg(ctx, scale, world=8, rank=5):
    """BASELINE config 4's per-rank device leg at N = 8 in the shuffle join's items form
    (DistributedExecutor._shuffle_items, include/qeh.h qeh_shuffle_items_*), on one GPU: rank `rank`'s
    phase A over its 1e9 fact rows with the regions laid out per destination, its 1/8 of the dimension
    grouped by slice (k_dim_items), the per-destination packing, and phase B over what it receives --
    stood in for by its own block for itself from each of the 8 sources (uniform keys send every rank
    the same share) -- against its slices, built from the whole dimension's items (the all-gather's
    result).  RCCL time excluded (8-GPU runs are the driver's).  Algorithmic bytes as cfg4leg."""
    import torch
    from qe_hip.distributed import _DeviceView
    n, nd = int(1e9 * scale), 10_000_000
    x = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, nd)
    v = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n)
    full_dk = ctx.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
    full_dg = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 5, nd, 1024)
    b = np.linspace(0, nd, world + 1).astype(int)
    shards = [(ctx.slice(full_dk, int(b[r]), int(b[r + 1] - b[r])), ctx.slice(full_dg, int(b[r]), int(b[r + 1] - b[r])))
              for r in range(world)]
    pred = binop(col(0), BinaryOp.Greater, lit(49))
    aggs = [(AF.Sum, 2), (AF.Count, 2)]
    row_len = 7
    rows = []
    for dk, dg in shards:
        row = torch.empty(row_len, dtype=torch.int64, device="cuda")
        ctx.broadcast_stats(dk, dg, [0, 1], row.data_ptr())
        rows.append(row)
    M = torch.cat(rows)
    ctx.sync()
    G = 1024
    nb, span = ctx.fused_items_shape(int(np.diff(b).max()), world)
    OW = 2 * 161
    # every shard's dimension items once (the all-gather's result), from throwaway handles
    gi = torch.empty(world * nb * span, dtype=torch.int32, device="cuda")
    go = torch.empty(world * nb * OW, dtype=torch.int32, device="cuda")
    tiny = [ctx.slice(x, 0, 8192), ctx.slice(k, 0, 8192), ctx.slice(v, 0, 8192)]
    for r, (dk, dg) in enumerate(shards):
        h = ctx.shuffle_items_begin(tiny, 1, pred, aggs, M.data_ptr(), world, r, row_len)
        ctx.fused_items_build(h, dk, dg, nb, span, gi.data_ptr() + r * nb * span * 4, go.data_ptr() + r * nb * OW * 4)
        ctx.fused_items_abort(h)
    ctx.sync()
    names = ["slice_partition", "shuffle_pack", "slice_probe", "fused_build"]
    nl = (1 + len(aggs)) * G + 1
    lanes = torch.empty(nl, dtype=torch.float64, device="cuda")
    best = None
    for rep in range(4):
        ctx.timing(True)
        ctx.timing_reset()
        t0 = time.perf_counter()
        h = ctx.shuffle_items_begin([x, k, v], 1, pred, aggs, M.data_ptr(), world, rank, row_len)
        it = torch.empty(nb * span, dtype=torch.int32, device="cuda")
        of = torch.empty(nb * OW, dtype=torch.int32, device="cuda")
        dk, dg = shards[rank]
        ctx.fused_items_build(h, dk, dg, nb, span, it.data_ptr(), of.data_ptr())
        ok, kp, vp, cp, bc, E, tot = ctx.shuffle_items_pack(h, world)
        assert ok
        # the receive buffers' stand-in: a packed block of this rank's (the next rank's, same size under
        # uniform keys) once per remote source; its own block is read in place by phase B
        kt = torch.as_tensor(_DeviceView(kp, world * bc, "<i2", None))
        vt = torch.as_tensor(_DeviceView(vp, world * bc, "<i8", None))
        ct = torch.as_tensor(_DeviceView(cp, world * E, "<i4", None))
        q1 = (rank + 1) % world
        t1 = int(tot[q1])
        rk = torch.cat([kt[q1 * bc:q1 * bc + t1]] * (world - 1) + [torch.zeros(4, dtype=torch.int16, device="cuda")])
        rv = torch.cat([vt[q1 * bc:q1 * bc + t1]] * (world - 1) + [torch.zeros(4, dtype=torch.int64, device="cuda")])
        rc = torch.cat([ct[q1 * E:(q1 + 1) * E] if q != rank else ct[rank * E:(rank + 1) * E] for q in range(world)])
        so, off = [], 0
        for q in range(world):
            so.append(off)
            off += t1 if q != rank else 0
        ctx.shuffle_items_finish(h, rk.data_ptr(), rv.data_ptr(), rc.data_ptr(), so, gi.data_ptr(), span, go.data_ptr(),
                                 world * nb, G, lanes.data_ptr())
        ctx.sync()
        wall = time.perf_counter() - t0
        kt_ = {nm: ctx.kernel_time(nm)[0] for nm in names}
        ctx.timing(False)
        if rep and (best is None or sum(kt_.values()) < sum(best[1].values())):
            best = (wall, kt_, int(tot.sum()), t1 * (world - 1) + int(tot[rank]))
        del rk, rv, rc
    wall, kt_, sent, recv = best
    kms = sum(kt_.values())
    alg = 24.0 * n + 16.0 * nd
    line(f"cfg4 per-rank device leg at N={world}, items form (1e9 fact rows + 1/{world} dim per rank)", n, wall, alg, kms,
         "k_slice_partition (per-destination layout) + k_region_pack + k_slice_probe (received regions)", None,
         {"kernel_split_ms": kt_, "items_packed": sent, "items_received": recv,
          "xgmi_bytes_per_rank": 10.0 * (sent - sent // world),
          "note": "frac on SURVEY §8(d)'s 24 B / fact row + 16 B / dim row; the receive side stood in by this "
                  "rank's own block x 8 (uniform keys); RCCL all-to-all time excluded; wall includes the "
                  "stand-in copies"})


def cfg5_leg(ctx, scale, world=8):
    """BASELINE config 5's per-rank device leg at N = 8, on one GPU: what one rank of the distributed
    ROW_NUMBER() OVER (PARTITION BY k ORDER BY v) runs besides the two RCCL all-to-alls
    (DistributedExecutor.row_number -> _moved_window; window.rs:32-226 on each rank):
      1. the 8-way hash exchange pass over the rank's 1.25e8 rows (qeh_partition_hash_move: k, v read
         once, written partition-major);
      2. the local ROW_NUMBER over what the rank receives: partition 0 of every rank's rows (the
         1e9-row table is generated whole and each rank's 1/8 moved, so the received rows are the real
         ones, source-rank-major);
      3. the reverse pass (qeh_partition_hash_unmove): the row numbers that come back, partition-major,
         gathered into the rank's input order.
    Algorithmic bytes: 16 B read + 8 B written per row of the rank."""
    n = int(1e9 * scale)
    nr = n // world
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 7, n, 2 ** 20)
    v = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 8, n, 2 ** 62, lo=-(2 ** 61))
    rk, rv = ctx.slice(k, 0, nr), ctx.slice(v, 0, nr)  # rank 0's rows
    recv_k, recv_v = [], []
    for r in range(world):  # what rank 0 receives: partition 0 of every rank's rows, source-rank-major
        c, m = ctx.partition_hash_move([ctx.slice(k, r * nr, nr)], world, [ctx.slice(k, r * nr, nr), ctx.slice(v, r * nr, nr)])
        recv_k.append(ctx.concat([ctx.slice(m[0], 0, int(c[0]))]))
        recv_v.append(ctx.concat([ctx.slice(m[1], 0, int(c[0]))]))
        for q in m:
            q.release()
    rk_all, rv_all = ctx.concat(recv_k), ctx.concat(recv_v)
    for q in recv_k + recv_v:
        q.release()
    recv = len(rk_all)
    counts0, m0 = ctx.partition_hash_move([rk], world, [rk])
    m0[0].release()
    back = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 9, nr, 2 ** 30)  # stands in for the returned numbers

    def leg1():
        c, m = ctx.partition_hash_move([rk], world, [rk, rv])
        for q in m:
            q.release()
        return c

    def leg2():
        rn = ctx.row_number([rk_all], [rv_all], [True])
        rn.release()

    def leg3():
        out = ctx.partition_hash_unmove(rk, world, [back])
        for q in out:
            q.release()
    names = ["partition_move", "radix_pass", "sort_encode", "row_number", "window_partition", "window_sort",
             "window_place", "w3_partition", "w3_sort", "w3_place"]
    w1, k1, _ = timed(ctx, leg1, 5, names)
    w2, k2, _ = timed(ctx, leg2, 3, names)
    w3, k3, _ = timed(ctx, leg3, 5, names)
    kms2 = sum(v_ for n_, v_ in k2.items() if n_ != "partition_move")
    legs = {"exchange_pass": {"ms": k1["partition_move"], "wall_ms": w1 * 1e3, "hbm_bytes_moved": 32.0 * nr},
            "local_row_number": {"ms": kms2, "wall_ms": w2 * 1e3, "rows": recv, "kernels": {n_: v_ for n_, v_ in k2.items() if v_}},
            "unmove_pass": {"ms": k3["partition_move"], "wall_ms": w3 * 1e3, "hbm_bytes_moved": 17.0 * nr}}
    kms = k1["partition_move"] + kms2 + k3["partition_move"]
    xgmi = (world - 1) / world * (16.0 * nr + 8.0 * recv)
    line(f"cfg5 per-rank device leg at N={world} (ROW_NUMBER, 1e9 rows, 1/{world} per rank)", nr, w1 + w2 + w3,
         24.0 * nr, kms, "k_part_scatter_small (exchange), k_window passes (local ROW_NUMBER), k_part_gather_small (unmove)",
         None, {"legs": legs, "received_rows": recv, "rank0_partition_counts": [int(q) for q in counts0],
                "xgmi_bytes_per_rank": xgmi,
                "note": "frac on SURVEY §8(d)'s 24 B per row of the rank; RCCL all-to-all time excluded (8-GPU runs "
                        "are the driver's); wall = sum of the legs"})


def cfg_filter(ctx, scale):
    n = int(5e8 * scale)
    x = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, 1024)
    v = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n)
    pred = binop(col(0), BinaryOp.Greater, lit(49))

    def fn():
        out, rows = ctx.filter([x, k, v], pred)
        for c in out:
            c.release()
        return rows
    wall, kt, rows = timed(ctx, fn, 5, ["filter"])
    line("filter 5e8 x3 cols", n, wall, 24.0 * n + 24.0 * rows, kt["filter"], "k_filter<1>", None,
         {"selected": rows})


def cfg_limit(ctx, scale):
    """SELECT x, k, v FROM t WHERE x > 49 LIMIT 1000 over 5e8 rows: qeh_filter_limit stops claiming
    tiles once 1000 rows are placed (the reference filters every row, then slices)."""
    n = int(5e8 * scale)
    x = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, 1024)
    v = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n)
    pred = binop(col(0), BinaryOp.Greater, lit(49))

    def fn():
        out, rows = ctx.filter([x, k, v], pred, max_rows=1000)
        for c in out:
            c.release()
        return rows
    wall, kt, rows = timed(ctx, fn, 20, ["filter"])
    line("filter+limit 5e8 x3 cols LIMIT 1000", n, wall, None, kt["filter"], "k_filter_fast (capped)", None,
         {"selected": rows, "note": "rows_per_s counts the table's rows; only the leading tiles are read"})


def cfg_plan(ctx, scale):
    """The metric query through QueryExecutor.execute from host Arrow batches (the reference's
    MemoryDataSource path): cold = every execute imports the Scan batches over PCIe; cached = the
    sources carry a cache key, so the device copy from the first execute is reused."""
    import pyarrow as pa
    from qe_hip import (AggregateExpr, Filter, HashAggregate, HashJoin, JoinType, MemoryDataSource,
                        QueryExecutor, Scan)
    from qe_hip.expr import Column
    n, nd = int(1e8 * scale), int(1e7 * scale)
    cols = {"f.x": (abi.GEN_UNIFORM_MOD, 1, 100), "f.k": (abi.GEN_UNIFORM_MOD, 2, nd), "f.v": (abi.GEN_UNIT_F64, 3, 0)}
    fact = pa.table({name: ctx.generate(kind, SEED, cid, n, mod).to_numpy()[0] for name, (kind, cid, mod) in cols.items()})
    dim = pa.table({"d.k": ctx.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd).to_numpy()[0],
                    "d.g": ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 5, nd, 1024).to_numpy()[0]})
    qx = QueryExecutor(ctx)
    out = {}
    for mode in ("cold", "cached"):
        cache = mode == "cached"
        fs = MemoryDataSource(fact.schema, fact.to_batches(max_chunksize=1 << 23), device_cache=cache)
        ds = MemoryDataSource(dim.schema, dim.to_batches(), device_cache=cache)
        join = HashJoin(Scan(fs), Scan(ds), JoinType.Inner, binop(Column("f.k", 1), BinaryOp.Equal, Column("d.k", 3)))
        plan = HashAggregate(Filter(join, binop(Column("f.x", 0), BinaryOp.Greater, lit(49))), [Column("d.g", 4)],
                             [AggregateExpr(AF.Sum, Column("f.v", 2)), AggregateExpr(AF.Count, Column("f.v", 2))])
        qx.execute(plan)
        reps = 3 if mode == "cold" else 10
        t0 = time.perf_counter()
        for _ in range(reps):
            res = qx.execute(plan)
        wall = (time.perf_counter() - t0) / reps
        out[mode] = wall
        line(f"plan metric query 1e8 x 1e7 from host Arrow ({mode})", n, wall, None, None, None, None,
             {"groups": res[0].num_rows, "host_bytes_per_execute": 24 * n + 16 * nd if mode == "cold" else 0,
              "pcie_inclusive_GBs": (24 * n + 16 * nd) / wall / 1e9 if mode == "cold" else None})
        qx.cache_evict()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="cfg2,cfg3,cfg5,filter")
    ap.add_argument("--scale", type=float, default=1.0)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx = qe_hip.Context(0)
    ctx.set_stream(s.cuda_stream)
    for name in args.only.split(","):
        {"cfg2": cfg2, "cfg3": cfg3, "cfg5": cfg5, "filter": cfg_filter, "limit": cfg_limit,
         "plan": cfg_plan, "left": lambda c, s: cfg_outer(c, s, 1), "full": lambda c, s: cfg_outer(c, s, 3),
         "merge": cfg_merge, "encode": cfg_encode, "shapes": cfg_metric_shapes, "partition": cfg_partition, "cfg3w": cfg3_wide, "window": cfg_window,
         "cfg4leg": cfg4_leg, "cfg4items": cfg4_items_leg, "cfg5leg": cfg5_leg,
         "window_lsd": cfg_window_lsd}[name](ctx, args.scale)
        ctx.sync()
        abi.check(ctx.lib.qeh_pool_trim(ctx.h))
    ctx.close()


if __name__ == "__main__":
    main()
