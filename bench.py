#!/usr/bin/env python3
"""BASELINE metric: rows/s of filter -> hash-join -> group-by over 1e9 fact rows.

    SELECT d.g, SUM(f.v), COUNT(f.v) FROM fact f JOIN dim d ON f.k = d.k
    WHERE f.x > 49 GROUP BY d.g

fact: x Int64 in [0,100), k Int64 uniform in [0,1e7), v Float64 in [0,1)
dim : k = a permutation of [0,1e7), g Int64 in [0,1024)        

One step = one execution of the query over device-resident synthetic columns
(data generated in HBM by the counter-based generator before timing): build
the dim hash table, probe + filter + aggregate every fact row, finalize the
groups, and for N>1 the partial->final aggregate exchange over RCCL.

Multi-GPU (torchrun, one rank per GPU): every rank holds its own 1e9-row fact
shard (weak scaling, BASELINE config 4) and the replicated dim (broadcast
join: each rank generates it, no data-path collective); the partial
per-group states are all-gathered over RCCL and merged on the device by a
second HashAggregate (the reference's partial/final aggregate stage shape,
crates/query-distributed/src/planner.rs:200-249).
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
    ap.add_argument("--rows", type=int, default=1_000_000_000, help="fact rows per GPU")
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
      * 1 thread: the oracle's line-by-line restatement of the reference executor
        (qo_join_filter_aggregate; executor.rs is single-threaded, rayon unused) over the full
        dim table and the first `cpu-sample` fact rows;
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
              "sample": f"oracle/qe_oracle.c qo_join_filter_aggregate (line-by-line restatement of executor.rs, "
                        f"1 thread), {n1} fact rows x {args.dim} dim rows, build included, {dt1:.2f} s, {build}"}
    nm = args.cpu_sample_mt
    f = fact(nm)
    ob.join_filter_aggregate_mt(f, 1, pred, ob.HostCol(dk), [ob.HostCol(dg)], aggs, threads)  # page in
    t0 = time.perf_counter()
    ob.join_filter_aggregate_mt(f, 1, pred, ob.HostCol(dk), [ob.HostCol(dg)], aggs, threads)
    dtm = time.perf_counter() - t0
    del f
    out.update({"value": nm / dtm, "cores": threads,
                "sample": f"oracle/qe_oracle.c qo_join_filter_aggregate_mt (OpenMP, {threads} threads = this "
                          f"process's CPU share of {os.cpu_count()} host CPUs), {nm} fact rows x {args.dim} dim rows, "
                          f"build included, {dtm:.2f} s, {build}",
                "single_thread": single})
    return out


def torch_device_count():
    import torch
    return torch.cuda.device_count()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("QEH_BENCH_SHARE_GPU"):  # rehearsal only: several ranks on one GPU
        local = local % max(torch_device_count(), 1)
    dist = world > 1
    import torch
    if dist:
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
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

    n, nd = args.rows, args.dim
    row0 = rank * n
    x = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100, row0=row0)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, nd, row0=row0)
    v = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n, row0=row0)
    dk = ctx.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
    dg = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 5, nd, args.groups)
    ctx.sync()
    pred = binop(col(0, "f.x"), BinaryOp.Greater, lit(args.threshold))
    aggs = [(AF.Sum, 2), (AF.Count, 2)]

    dx = None
    if dist:
        from qe_hip.distributed import DistributedExecutor
        dx = DistributedExecutor(ctx)

    def step():
        if not dist:
            return ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], aggs)
        # broadcast join (dim replicated), partial states shuffled by group key
        # over RCCL all-to-all, final aggregate on the owning rank
        return dx.join_filter_aggregate_broadcast([x, k, v], 1, pred, dk, [dg], aggs)

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
    probe_ms, probe_launches = ctx.kernel_time("join_filter_aggregate")
    part_ms, part_launches = ctx.kernel_time("slice_partition")
    sprobe_ms, _ = ctx.kernel_time("slice_probe")
    build_ms, _ = ctx.kernel_time("join_build")
    ctx.timing(False)

    if dist:
        cdev = "cuda" if tdist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([elapsed], device=cdev, dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())

    # sanity on the result: every selected row landed in exactly one group
    gk, ga, g = res
    counts, _ = ga[1].to_numpy()
    counted = int(counts.sum())
    groups = int(g)
    if dist:
        t = torch.tensor([counted, groups], device=cdev, dtype=torch.int64)
        tdist.all_reduce(t)
        counted, groups = int(t[0].item()), int(t[1].item())
    total_rows = n * world
    ms_per_step = elapsed * 1e3 / args.steps
    value = total_rows * args.steps / elapsed
    if part_launches:  # LDS-slice partitioned pipeline: the two kernels' own event times
        avg_probe_ms = (part_ms + sprobe_ms) / part_launches
        kernel_name = "k_slice_partition + k_slice_probe (HIP events 'slice_partition' + 'slice_probe')"
        kernel_split = {"partition_ms": part_ms / part_launches, "probe_ms": sprobe_ms / part_launches}
    else:
        avg_probe_ms = probe_ms / max(probe_launches, 1)
        kernel_name = "k_join_agg_fast (HIP events 'join_filter_aggregate')"
        kernel_split = None
    alg_bytes = 24.0 * n  # x, k, v read once per fact row
    achieved = alg_bytes / (avg_probe_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("rows") == n and tj.get("kernel") == "join_filter_aggregate":
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if rank == 0:
        cpu = cpu_baseline(args) if world == 1 else None  # the CPU baseline is an N=1 figure
        line = {
            "metric": "rows/sec filter->hash-join->group-by, 1B rows, 1/2/4/8 GPUs; % HBM roofline",
            "value": value,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64/f64",
            "data": "synthetic (counter-based splitmix64, generated in HBM; BASELINE.md §2)",
            "config": {
                "workload": "filter->hash-join->group-by (BASELINE metric query): SELECT d.g, SUM(f.v), COUNT(f.v) "
                            "FROM fact f JOIN dim d ON f.k = d.k WHERE f.x > 49 GROUP BY d.g",
                "fact_rows_per_gpu": n,
                "dim_rows": nd,
                "groups": args.groups,
                "parallelism": f"fact sharded x{world}, dim replicated (broadcast join)"
                               + (", partial states shuffled by RCCL all-to-all, final aggregate per owner rank" if dist else ""),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": kernel_name,
                "kernel_ms": avg_probe_ms,
                "kernel_split_ms": kernel_split,
                # the operator's main-queue part (phase A runs on the second queue, under the build)
                "operator_main_queue_ms": probe_ms / max(probe_launches, 1),
                "alg_bytes_per_launch": alg_bytes,
            },
            "build_ms_per_step": build_ms / args.steps,
            "result_groups": groups,
            "result_rows_counted": counted,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
