"""Host-side cost of one fused join-aggregate call: a tiny query (8192 fact rows, 1000 dim rows,
forced onto the slice pipeline) whose kernels take microseconds, timed per call over many calls,
beside the same call's kernel time (HIP events).  The difference is host work plus launch gaps."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
os.environ.setdefault("QEH_SLICE_MIN_BYTES", "0")
import qe_hip  # noqa: E402
from qe_hip import AggregateFunction as AF, BinaryOp, abi, binop, col, lit  # noqa: E402

n, nd = int(sys.argv[1]) if len(sys.argv) > 1 else 8192, 1000
ctx = qe_hip.Context(0)
x = ctx.generate(abi.GEN_UNIFORM_MOD, 1, 1, n, 100)
k = ctx.generate(abi.GEN_UNIFORM_MOD, 1, 2, n, nd)
v = ctx.generate(abi.GEN_UNIT_F64, 1, 3, n)
dk = ctx.generate(abi.GEN_PERMUTATION, 1, 0, nd, nd)
dg = ctx.generate(abi.GEN_UNIFORM_MOD, 1, 5, nd, 64)
ctx.sync()
pred = binop(col(0), BinaryOp.Greater, lit(49))
aggs = [(AF.Sum, 2), (AF.Count, 2)]
for _ in range(20):
    r = ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], aggs)
reps = 200
t0 = time.perf_counter()
for _ in range(reps):
    r = ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], aggs)
wall = (time.perf_counter() - t0) / reps * 1e6
t0 = time.perf_counter()
for _ in range(reps):
    cp = ctx._cols([x, k, v])
    e, keep = pred.to_c()
py = (time.perf_counter() - t0) / reps * 1e6
print(f"{'fused' if not os.environ.get('QEH_NO_FUSED') else 'prelaunch'} path, {n} fact rows: {wall:.1f} us per call "
      f"(python marshalling alone {py:.1f} us), groups {r[2]}", flush=True)
