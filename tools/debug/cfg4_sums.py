"""Debug: Σ v at each stage of the config-4 local pipeline at full size."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
import numpy as np
import qe_hip
from qe_hip import AggregateFunction as AF, BinaryOp, abi, binop, col, lit
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
nd = 10_000_000
ctx = qe_hip.Context(0)
x = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 1, n, 100)
k = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 2, n, nd)
v = ctx.generate(abi.GEN_UNIT_F64, 0x5EED, 3, n)
dk = ctx.generate(abi.GEN_PERMUTATION, 0x5EED, 0, nd, nd)
dg = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 5, nd, 1024)
def gsum(c):
    _, a, _ = ctx.hash_aggregate([], [c], [(AF.Sum, 0), (AF.Count, 0)])
    return float(a[0].to_numpy()[0][0]), int(a[1].to_numpy()[0][0])
pred = binop(col(0), BinaryOp.Greater, lit(49))
fc, rows = ctx.filter([x, k, v], pred, out_idx=[1, 2])
print("filtered rows", rows, "sum v", gsum(fc[1]), flush=True)
counts, moved = ctx.partition_hash_move([fc[0]], 1, fc)
print("moved counts", counts, "sum v", gsum(moved[1]), "sum k", gsum(moved[0]), "filtered sum k", gsum(fc[0]), flush=True)
for name, cols in (("filtered", fc), ("moved", moved)):
    gk, ga, g = ctx.join_filter_aggregate(cols, 0, None, dk, [dg], [(AF.Sum, 1), (AF.Count, 1)])
    print(name, "jfa groups", g, "Σsum", float(ga[0].to_numpy()[0].sum()), "Σcnt", int(ga[1].to_numpy()[0].sum()), flush=True)
gk, ga, g = ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], [(AF.Sum, 2), (AF.Count, 2)])
print("metric jfa groups", g, "Σsum", float(ga[0].to_numpy()[0].sum()), "Σcnt", int(ga[1].to_numpy()[0].sum()), flush=True)
