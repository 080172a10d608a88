"""Per-stage host timing of the broadcast-join step (bench.py's N > 1 plan) at world size 1 over
RCCL: where the fixed per-step overhead of the distributed plan goes.  Dev tool only."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "query-engine_amd"))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29555")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
import qe_hip  # noqa: E402
from qe_hip import AggregateFunction as AF, BinaryOp, abi, binop, col, lit  # noqa: E402
from qe_hip.distributed import DistributedExecutor  # noqa: E402

n, nd = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000, 10_000_000
stream = torch.cuda.Stream(0)
torch.cuda.set_stream(stream)
ctx = qe_hip.Context(0)
ctx.set_stream(stream.cuda_stream)
x = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 1, n, 100)
k = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 2, n, nd)
v = ctx.generate(abi.GEN_UNIT_F64, 0x5EED, 3, n)
dk = ctx.generate(abi.GEN_PERMUTATION, 0x5EED, 0, nd, nd)
dg = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 5, nd, 1024)
pred = binop(col(0), BinaryOp.Greater, lit(49))
aggs = [(AF.Sum, 2), (AF.Count, 2)]
dx = DistributedExecutor(ctx)
T = {}


def tick(name, t0):
    torch.cuda.synchronize()
    t = time.perf_counter()
    T[name] = T.get(name, 0.0) + (t - t0)
    return t


for it in range(25):
    if it == 5:
        T.clear()
    torch.cuda.synchronize()
    t = time.perf_counter()
    full = dx.allgather_columns([dk, dg])
    t = tick("allgather_columns", t)
    pk, pa, g = ctx.join_filter_aggregate([x, k, v], 1, pred, full[0], full[1:], aggs)
    t = tick("join_filter_aggregate", t)
    res = dx._final_dense(full[1:], [x, k, v], pk, pa, aggs)
    t = tick("final_dense", t)
    res2 = dx._final(pk, pa, aggs)
    t = tick("final_shuffle (not in the step)", t)
for k_, v_ in T.items():
    print(f"{k_:34s} {v_ / 20 * 1e3:8.3f} ms")
dist.destroy_process_group()
