#!/usr/bin/env python3
"""Fixed host + launch overhead of one fused filter->join->group-by call:
wall time per call on tiny inputs (everything device-resident)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
import torch  # noqa: E402,F401
import qe_hip  # noqa: E402
from qe_hip import AggregateFunction as AF, BinaryOp, abi, binop, col, lit  # noqa: E402

n, nd = int(sys.argv[1]) if len(sys.argv) > 1 else 8192, int(sys.argv[2]) if len(sys.argv) > 2 else 1024
ctx = qe_hip.Context(0)
x = ctx.generate(abi.GEN_UNIFORM_MOD, 1, 1, n, 100)
k = ctx.generate(abi.GEN_UNIFORM_MOD, 1, 2, n, nd)
v = ctx.generate(abi.GEN_UNIT_F64, 1, 3, n)
dk = ctx.generate(abi.GEN_PERMUTATION, 1, 0, nd, nd)
dg = ctx.generate(abi.GEN_UNIFORM_MOD, 1, 5, nd, 64)
pred = binop(col(0), BinaryOp.Greater, lit(49))
aggs = [(AF.Sum, 2), (AF.Count, 2)]
for _ in range(20):
    ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], aggs)
ctx.sync()
reps = 200
t0 = time.perf_counter()
for _ in range(reps):
    r = ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], aggs)
ctx.sync()
dt = (time.perf_counter() - t0) / reps
print(f"n={n} dim={nd}: {dt * 1e6:.1f} us per call")
