#!/usr/bin/env python3
"""Does a collective-sized kernel on the torch stream run beside phase A's persistent grid?
The N = 8 per-rank metric shape (1.25e8 fact rows, 1e7-row dimension): phase A is prelaunched on the
library's second queue (as the broadcast join does under its dimension all-gather), then a 160 MB
device copy -- the bytes a rank receives in the all-gather, a stand-in for RCCL's kernels -- runs on
the torch stream, then the fused call adopts phase A.  Run under rocprofv3 --kernel-trace; the trace
shows whether the copy kernel's span lies inside k_slice_partition's."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
import torch  # noqa: E402
import qe_hip  # noqa: E402
from qe_hip import AggregateFunction as AF, BinaryOp, abi, binop, col, lit  # noqa: E402

n, nd, SEED = 125_000_000, 10_000_000, 0x5EED
torch.cuda.set_device(0)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
ctx = qe_hip.Context(0)
ctx.set_stream(s.cuda_stream)
x = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100)
k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, nd)
v = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n)
dk = ctx.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
dg = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 5, nd, 1024)
pred = binop(col(0), BinaryOp.Greater, lit(49))
aggs = [(AF.Sum, 2), (AF.Count, 2)]
src = torch.empty(20_000_000, dtype=torch.int64, device="cuda")
dst = torch.empty_like(src)
src.fill_(1)
ctx.sync()
for it in range(4):
    ctx.join_filter_aggregate_prelaunch([x, k, v], 1, pred, aggs, [0, nd - 1, nd], [0, 1023, nd])
    dst.copy_(src)  # 160 MB on the torch stream while phase A runs on the second queue
    gk, ga, g = ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], aggs)
    for c in gk + ga:
        c.release()
torch.cuda.synchronize()
print("ok groups", g)
