#!/usr/bin/env python3
"""BASELINE metric: rows/s of filter -> hash-join -> group-by over 1e9 fact rows.

    SELECT d.g, SUM(f.v), COUNT(f.v) FROM fact f JOIN dim d ON f.k = d.k
    WHERE f.x > 49 GROUP BY d.g

fact: x Int64 in [0,100), k Int64 uniform in [0,1e7), v Float64 in [0,1)
dim : k = a permutation of [0,1e7), g Int64 in [0,1024)        

One step = one execution of the query over device-resident synthetic columns
(data generated in HBM by the counter-based generator before timing): build
the dim hash table, probe + filter + aggregate every fact row, finalize the
groups, and for N>1 the RCCL exchanges.

Default workload (the metric, strong scaling): 1e9 fact rows in total, split
across the N GPUs (one rank per GPU); the dim is sharded too.  Inside the step
(broadcast join, DistributedExecutor.join_filter_aggregate_broadcast, the items
form first): one small all-gather of every shard's stats row, phase A of the
fused probe launched from the device-side plan over this rank's fact rows,
every rank's dim shard grouped by key slice into 4-B items and all-gathered
over RCCL, phase B builds each slice's LDS entries from every rank's items and
aggregates, and the per-group partial states (1024 bounded integer group keys)
are merged by one dense RCCL all-reduce of f64 lanes, each rank keeping the
groups it owns (the reference's partial/final aggregate stage shape,
crates/query-distributed/src/planner.rs:200-249).  Shapes outside the items
form take the table form (shard tables summed by an all-reduce) or all-gather
the dim shards; the line's "dist_build" names the form that ran.

Launch: the driver starts N > 1 under torch.distributed.run (WORLD_SIZE = N).
Run directly with --gpus N > 1, bench.py starts that launcher itself as a child
process before anything touches the GPU and exits with its code; a --gpus that
disagrees with a WORLD_SIZE already set is an error (exit 2), never a silent
N = 1 run.

--workload cfg4 (BASELINE config 4, weak scaling): 1e9 fact rows per GPU; both
sides hash-partitioned by the join key and exchanged over RCCL all-to-all
(shuffle join, partition.rs:151-212), local fused join + partial aggregate,
partial/final by group key.  Runs through a world-1 RCCL group at N = 1.

After the timed steps the result is checked at the full size: Σ COUNT over the
groups equals the device filter's count of x > 49, Σ SUM(v) equals the
device's filtered Σ v (1e-6), and every group is present.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
SEED = 0x5EED


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["metric", "cfg4"], default="metric",
                    help="metric: the BASELINE query, 1e9 fact rows in total (strong scaling); cfg4: BASELINE "
                         "config 4, hash-partitioned join + aggregate, --rows fact rows per GPU (weak scaling)")
    ap.add_argument("--rows", type=int, default=1_000_000_000,
                    help="fact rows (metric: in total; cfg4: per GPU)")
    ap.add_argument("--dim", type=int, default=10_000_000)
    ap.add_argument("--groups", type=int, default=1024)
    ap.add_argument("--threshold", type=int, default=49, help="WHERE f.x > threshold (49 = the BASELINE query)")
    ap.add_argument("--cpu-sample", type=int, default=100_000_000,
                    help="fact rows for the 1-thread CPU baseline (0 = skip the CPU baseline)")
    ap.add_argument("--cpu-sample-mt", type=int, default=400_000_000, help="fact rows for the all-cores CPU baseline")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="PMC-derived HBM bytes per launch of the probe kernel (tools/pmc_traffic.py)")
    return ap.parse_args()


def cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads() -> int:
    """Threads for the all-cores leg: this process's CPU share (the GPU box sets
    OMP_NUM_THREADS to it; os.cpu_count() there reports the whole machine)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(n, 1)


def cpu_baseline(args):
    """The metric query on the host CPU, same run, same box, two variants:
      * 1 thread: the oracle's intended-semantics hash join + filter + grouped aggregate
        (qo_join_filter_aggregate: the reference's own executor.rs would take its Cartesian join
        path and return no rows for this GROUP BY; executor.rs is single-threaded,
        rayon unused) over the full dim table and the first `cpu-sample` fact rows;
      * all cores: qo_join_filter_aggregate_mt (OpenMP) over `cpu-sample-mt` fact rows.
    Both from oracle/_native/liboracle.so built with -march=native on this host when gcc is
    available (else the portable x86-64-v2 build).  `value` is the all-cores figure."""
    if args.cpu_sample <= 0:
        return None
    import subprocess
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    native = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native"],
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL).returncode == 0
    import oracle_bind as ob
    native = native and ob.use_native()
    from qe_hip import AggregateFunction as AF, BinaryOp, abi, binop, col, lit
    pred = binop(col(0), BinaryOp.Greater, lit(args.threshold))
    aggs = [(AF.Sum, 2), (AF.Count, 2)]
    dk = ob.generate(abi.GEN_PERMUTATION, SEED, 0, args.dim, args.dim)
    dg = ob.generate(abi.GEN_UNIFORM_MOD, SEED, 5, args.dim, args.groups)

    def fact(n):
        return [ob.HostCol(ob.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100)),
                ob.HostCol(ob.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, args.dim)),
                ob.HostCol(ob.generate(abi.GEN_UNIT_F64, SEED, 3, n))]

    build = "-O3 -march=native (built on this host)" if native else "-O3 -march=x86-64-v2 (portable build)"
    threads = host_threads()
    out = {"unit": "rows/s", "kind": "port", "cpu_model": cpu_model(), "host_cpus_nproc": os.cpu_count()}
    n1 = args.cpu_sample
    f = fact(n1)
    t0 = time.perf_counter()
    ob.join_filter_aggregate(f, 1, pred, ob.HostCol(dk), [ob.HostCol(dg)], aggs)
    dt1 = time.perf_counter() - t0
    del f
    single = {"value": n1 / dt1, "cores": 1,
              "sample": f"oracle/qe_oracle.c qo_join_filter_aggregate (intended-semantics hash join + filter + "
                        f"group-by of the oracle, 1 thread), {n1} fact rows x {args.dim} dim rows, build included, {dt1:.2f} s, {build}"}
    nm = args.cpu_sample_mt
    f = fact(nm)
    ob.join_filter_aggregate_mt(f, 1, pred, ob.HostCol(dk), [ob.HostCol(dg)], aggs, threads)  # page in
    t0 = time.perf_counter()
    ob.join_filter_aggregate_mt(f, 1, pred, ob.HostCol(dk), [ob.HostCol(dg)], aggs, threads)
    dtm = time.perf_counter() - t0
    del f
    out.update({"value": nm / dtm, "cores": threads,
                "sample": f"oracle/qe_oracle.c qo_join_filter_aggregate_mt (intended-semantics hash join of the "
                          f"oracle, OpenMP, {threads} threads = the CPUs this process may use (affinity), not all "
                          f"{os.cpu_count()} host CPUs), {nm} fact rows x {args.dim} dim rows, "
                          f"build included, {dtm:.2f} s, {build}",
                "single_thread": single})
    return out


def torch_device_count():
    import torch
    return torch.cuda.device_count()


def shard(total: int, world: int, rank: int):
    """[start, start + count) of `total` rows owned by `rank` (contiguous, balanced)."""
    base, rem = divmod(total, world)
    count = base + (1 if rank < rem else 0)
    return rank * base + min(rank, rem), count


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_plan(gpus: int, env) -> str:
    """How this invocation runs: "run" (this process is the job's rank, or N = 1), "spawn" (--gpus N > 1
    outside a launcher: start torch.distributed.run with N ranks as a child) or "mismatch" (a launcher
    set WORLD_SIZE and --gpus disagrees with it)."""
    ws = env.get("WORLD_SIZE")
    if gpus < 1:
        return "mismatch"
    if ws is None:
        return "spawn" if gpus > 1 else "run"
    return "run" if int(ws) == gpus else "mismatch"


def spawn_command(argv, gpus: int, port: int):
    """The launcher command for --gpus N outside torchrun (the driver's own form of the N > 1 run)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def main():
    args = parse()
    plan = launch_plan(args.gpus, os.environ)
    if plan == "mismatch":
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE')} -- launch N > 1 as "
              "`python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`, or run bench.py --gpus N "
              "directly and it starts that launcher itself", file=sys.stderr)
        sys.exit(2)
    if plan == "spawn":  # (nothing has touched the GPU yet: the ranks are children, not an exec)
        import subprocess
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.exit(subprocess.run(spawn_command(sys.argv[1:], args.gpus, free_port()), env=env).returncode)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if os.environ.get("QEH_BENCH_LAUNCH_PROBE"):  # (tests/test_bench_launch.py: the rank's view, no GPU work)
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "world": world, "gpus": args.gpus}), flush=True)
        return
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("QEH_BENCH_SHARE_GPU"):  # rehearsal only: several ranks on one GPU
        local = local % max(torch_device_count(), 1)
    cfg4 = args.workload == "cfg4"
    # config 4 always runs the distributed plan (a world-1 RCCL group at N = 1); the metric
    # query at N = 1 is the local operator, at N > 1 the broadcast join over RCCL
    # QEH_BENCH_FORCE_DIST=1: the N > 1 plan at N = 1 (measures its fixed per-step overhead)
    dist = world > 1 or cfg4 or bool(os.environ.get("QEH_BENCH_FORCE_DIST"))
    # QEH_BENCH_RANK_OF="r/W": rehearse rank r's share of an N = W metric run on one GPU -- its fact
    # rows and its dim shard through the distributed plan at world size 1 (the RCCL table all-reduce
    # has one member, so its xGMI time is not in the step); checked against the local operator over
    # the same dim shard instead of the full-join properties
    rehearse = os.environ.get("QEH_BENCH_RANK_OF")
    if rehearse:
        rr, ww = (int(q) for q in rehearse.split("/"))
        assert world == 1 and not cfg4 and 0 <= rr < ww, "QEH_BENCH_RANK_OF: one process, metric workload, r < W"
        dist = True
        # the rank's 1/W of the dim spans the whole key range: let the table form take it, as the job's W shards would
        os.environ.setdefault("QEH_TABLE_MAX_SPARSITY", str(4 * ww))
    import torch
    if dist:
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local)
        backend = os.environ.get("QEH_BENCH_BACKEND", "nccl")  # "gloo": host-exchange rehearsal (several ranks per GPU)
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
    import qe_hip
    from qe_hip import AggregateFunction as AF, BinaryOp, abi, binop, col, lit

    torch.cuda.set_device(local)
    stream = torch.cuda.Stream(local)
    torch.cuda.set_stream(stream)  # a real stream handle: library kernels, copies and RCCL are ordered on it
    ctx = qe_hip.Context(local)
    ctx.set_stream(stream.cuda_stream)

    nd = args.dim
    if cfg4:  # weak scaling: `rows` fact rows on every GPU
        row0, n = rank * args.rows, args.rows
        total_rows = args.rows * world
    elif rehearse:
        row0, n = shard(args.rows, ww, rr)
        total_rows = n
    else:     # strong scaling: `rows` fact rows in total, split across the GPUs
        row0, n = shard(args.rows, world, rank)
        total_rows = args.rows
    x = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100, row0=row0)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, nd, row0=row0)
    v = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n, row0=row0)
    # the dimension: whole on one GPU; sharded across ranks for N > 1 / config 4 (each rank
    # holds rows [d0, d0 + dn) of the same table) and moved by RCCL inside the step
    d0, dn = shard(nd, ww, rr) if rehearse else shard(nd, world, rank) if dist else (0, nd)
    dk = ctx.generate(abi.GEN_PERMUTATION, SEED, 0, dn, nd, row0=d0)
    dg = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 5, dn, args.groups, row0=d0)
    ctx.sync()
    pred = binop(col(0, "f.x"), BinaryOp.Greater, lit(args.threshold))
    aggs = [(AF.Sum, 2), (AF.Count, 2)]

    dx = None
    if dist:
        from qe_hip.distributed import DistributedExecutor
        dx = DistributedExecutor(ctx)

    def step():
        if cfg4:  # hash-partitioned join: both sides shuffled by f.k / d.k over RCCL all-to-all
            return dx.join_filter_aggregate_shuffle([x, k, v], 1, pred, dk, [dg], aggs)
        if not dist:
            return ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], aggs)
        # broadcast join: the dim shards all-gathered over RCCL, partial states shuffled by
        # group key over RCCL all-to-all, final aggregate on the owning rank
        return dx.join_filter_aggregate_broadcast([x, k, v], 1, pred, dk, [dg], aggs, build_sharded=True)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # timed region: K steps bracketed by barrier + synchronize
    ctx.timing(True)
    ctx.timing_reset()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    names = ["join_filter_aggregate", "slice_partition", "slice_probe", "join_build", "fused_build", "filter",
             "partition_move"]
    kt = {nm: ctx.kernel_time(nm) for nm in names}
    ctx.timing(False)

    if dist:
        cdev = "cuda" if tdist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([elapsed], device=cdev, dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())

    # result checks at the full size (size-independent properties): every selected fact row
    # landed in exactly one group (Σ COUNT = rows with x > threshold, counted independently on
    # the device by the filter operator), and Σ SUM(v) over the groups = the filtered Σ v
    gk, ga, g = res
    counts, _ = ga[1].to_numpy()
    sums, _ = ga[0].to_numpy()
    counted, groups, vsum = int(counts.sum()), int(g), float(sums.sum())
    if rehearse:  # the local operator over the same fact rows and dim shard
        _, lga, lg = ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], aggs)
        want_rows, want_sum = int(lga[1].to_numpy()[0].sum()), float(lga[0].to_numpy()[0].sum())
        assert int(lg) == groups, f"{groups} groups, the local operator {int(lg)}"
        args.groups = groups  # every group of the shard, checked against the local operator above
    else:
        fx, want_rows = ctx.filter([x, v], pred, out_idx=[1])
        _, want_sum_cols, _ = ctx.hash_aggregate([], fx, [(AF.Sum, 0)])
        want_sum = float(want_sum_cols[0].to_numpy()[0][0]) if want_rows else 0.0
    if dist:
        t = torch.tensor([counted, groups, want_rows], device=cdev, dtype=torch.int64)
        tdist.all_reduce(t)
        counted, groups, want_rows = (int(q) for q in t.tolist())
        t = torch.tensor([vsum, want_sum], device=cdev, dtype=torch.float64)
        tdist.all_reduce(t)
        vsum, want_sum = (float(q) for q in t.tolist())
    assert counted == want_rows, f"Σ COUNT over groups {counted} != rows passing the filter {want_rows}"
    assert abs(vsum - want_sum) <= 1e-6 * max(abs(want_sum), 1e-300), f"Σ SUM(v) {vsum} != filtered Σ v {want_sum}"
    assert groups == args.groups, f"{groups} groups, expected {args.groups}"

    ms_per_step = elapsed * 1e3 / args.steps
    value = total_rows * args.steps / elapsed
    part_ms, part_launches = kt["slice_partition"]
    sprobe_ms, _ = kt["slice_probe"]
    probe_ms, probe_launches = kt["join_filter_aggregate"]
    if cfg4:  # the local device pipeline of the hash-partitioned plan: (filter +) exchange pass, fused join
        # the local join runs the LDS-slice pipeline when its table shape allows (then its two kernels'
        # events), else the single fused pass; at world size 1 the exchange is the identity (no pass)
        join_ms = part_ms + sprobe_ms if part_launches else probe_ms
        local_ms = (kt["filter"][0] + kt["partition_move"][0] + join_ms) / args.steps
        avg_probe_ms = local_ms
        kernel_name = ("config-4 local pipeline per step: fused filter + hash exchange passes (partition_move; "
                       "filter if not fused) + the local fused join-aggregate (slice_partition + slice_probe, or "
                       "join_filter_aggregate) (HIP events)")
        kernel_split = {"filter": kt["filter"][0] / args.steps, "partition_move": kt["partition_move"][0] / args.steps,
                        "join": join_ms / args.steps, "join_kernels": "slice" if part_launches else "single pass"}
    elif part_launches:  # LDS-slice partitioned pipeline: the two kernels' own event times per query
        q = max(part_launches // max(args.steps, 1), 1) if part_launches >= args.steps else 1
        per = part_launches / q  # queries timed (launches per query > 1 for the chunked pipeline)
        avg_probe_ms = (part_ms + sprobe_ms) / per
        kernel_name = "k_slice_partition + k_slice_probe (HIP events 'slice_partition' + 'slice_probe')"
        kernel_split = {"partition_ms": part_ms / per, "probe_ms": sprobe_ms / per, "launches_per_query": q}
    else:
        avg_probe_ms = probe_ms / max(probe_launches, 1)
        kernel_name = "k_join_agg_fast (HIP events 'join_filter_aggregate')"
        kernel_split = None
    # x, k, v read once per fact row of this GPU (24 B) + the dim's k, g read once
    # per dim row this GPU builds from (16 B; at N = 1 the whole 1e7-row dim: 24.16 GB per step)
    alg_bytes = 24.0 * n + 16.0 * dn
    achieved = alg_bytes / (avg_probe_ms * 1e-3) / 1e9
    # roofline.traffic is not measured in this run (PMC counters need their own rocprofv3 passes):
    # it is read from the committed record of such a run (tools/profile.sh -> tools/pmc_traffic.py),
    # used only when that record is for the same shape, and labelled with where it came from
    traffic, traffic_source = None, None
    if os.path.exists(args.traffic_json) and not dist:
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("rows") == n and tj.get("kernel") == "join_filter_aggregate":
                traffic = tj.get("hbm_bytes_per_launch")
                traffic_source = (f"{os.path.relpath(args.traffic_json, ROOT)}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                                  f"passes of a separate run ({tj.get('source', 'tools/profile.sh')}), FETCH_SIZE x2 "
                                  "(gfx950 wide-read correction) + WRITE_SIZE per query, not measured in this run")
        except Exception:
            traffic = None

    if rank == 0:
        cpu = cpu_baseline(args) if world == 1 and not cfg4 and not rehearse else None  # an N=1 figure
        if cfg4:
            workload = ("BASELINE config 4: hash-partitioned join + aggregate (filter f.x > 49, both sides "
                        "hash-partitioned by the join key over RCCL all-to-all, local fused join + partial "
                        "aggregate, partial states shuffled by d.g, final aggregate)")
            par = f"fact {n} rows per GPU x{world} (weak scaling), dim sharded x{world}, shuffle join over RCCL"
        else:
            workload = ("filter->hash-join->group-by (BASELINE metric query): SELECT d.g, SUM(f.v), COUNT(f.v) "
                        "FROM fact f JOIN dim d ON f.k = d.k WHERE f.x > 49 GROUP BY d.g")
            form = getattr(dx, "last_build", None) if dx is not None else None
            how = {"items": "every rank's dim shard grouped by key slice into 4-B items and all-gathered over RCCL "
                            "(broadcast join, items form)",
                   "table": "shard tables summed by RCCL all-reduce (broadcast join, table form)",
                   "allgather": "dim shards all-gathered over RCCL (broadcast join)",
                   "replicated": "dim replicated on every rank"}.get(form, f"broadcast join ({form})")
            par = (f"fact {args.rows} rows split x{world} (strong scaling)"
                   + (f", dim sharded x{world}: {how} inside the step, partial states merged by a dense RCCL "
                      "all-reduce, final aggregate per owner rank" if dist else ""))
        if rehearse:
            par = (f"rehearsal of rank {rr} of {ww} at world size 1: fact rows [{row0}, {row0 + n}), dim rows "
                   f"[{d0}, {d0 + dn}) through the broadcast join ({form} form; its RCCL collectives have one "
                   "member: their xGMI time is not in the step)")
        line = {
            "metric": "rows/sec filter->hash-join->group-by, 1B rows, 1/2/4/8 GPUs; % HBM roofline",
            "value": value,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak" if cfg4 else "strong",
            "vs_baseline": None,
            "dtype": "int64/f64",
            "data": "synthetic (counter-based splitmix64, generated in HBM; BASELINE.md §2)",
            "config": {
                "workload": workload,
                "fact_rows_total": total_rows,
                "fact_rows_per_gpu": n,
                "dim_rows": nd,
                "groups": args.groups,
                "parallelism": par,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_source,
                "kernel": kernel_name,
                "kernel_ms": avg_probe_ms,
                "kernel_split_ms": kernel_split,
                # the operator's main-queue part (phase A runs on the second queue, under the build)
                "operator_main_queue_ms": probe_ms / max(probe_launches, 1),
                "alg_bytes_per_launch": alg_bytes,
            },
            # the build: the dim grouped by slice before phase A (fused pipeline), or the table insert
            "build_ms_per_step": (kt["join_build"][0] + kt["fused_build"][0]) / args.steps,
            # N > 1 (or QEH_BENCH_FORCE_DIST): how the broadcast join got its table ("table": shard
            # tables summed by all-reduce; "allgather": dim shards all-gathered) and merged its groups
            "dist_build": getattr(dx, "last_build", None) if dx is not None and not cfg4 else None,
            "dist_final": getattr(dx, "last_final", None) if dx is not None else None,
            "result_groups": groups,
            "result_rows_counted": counted,
            "result_check": ("Σ COUNT, Σ SUM(v) (1e-6) and groups == the local operator over the same dim shard: passed"
                             if rehearse else
                             "Σ COUNT == device filter count, Σ SUM(v) == device filtered Σ v (1e-6), groups == "
                             f"{args.groups}: passed"),
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
