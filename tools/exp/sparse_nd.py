"""How the single-pass sparse-key join-aggregate scales with the build table's footprint (1e9 fact rows,
sparse 64-bit dim keys): a smaller table (fewer dim rows) shows what a compact table layout would gain."""
import json
import sys
import time

sys.path.insert(0, "tools")
import bench_configs as b  # noqa: E402
from qe_hip import AggregateFunction as AF, BinaryOp, abi, binop, col, lit  # noqa: E402

import torch  # noqa: E402
import qe_hip  # noqa: E402

torch.cuda.set_device(0)
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
ctx = qe_hip.Context(0)
ctx.set_stream(st.cuda_stream)
n = 1_000_000_000
x = ctx.generate(abi.GEN_UNIFORM_MOD, b.SEED, 1, n, 100)
v = ctx.generate(abi.GEN_UNIT_F64, b.SEED, 3, n)
pred = binop(col(0), BinaryOp.Greater, lit(49))
for nd in [int(a) for a in sys.argv[1:]] or [10_000_000, 5_000_000, 2_500_000]:
    k = ctx.generate(abi.GEN_SPARSE_KEY, b.SEED, 2, n, nd)
    dk = ctx.generate(abi.GEN_SPARSE_KEY, b.SEED, 0, nd, 0)
    dg = ctx.generate(abi.GEN_UNIFORM_MOD, b.SEED, 5, nd, 1024)

    def fn():
        gk, ga, g = ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], [(AF.Sum, 2), (AF.Count, 2)])
        for c in gk + ga:
            c.release()
    wall, kt, _ = b.timed(ctx, fn, 3, ["join_filter_aggregate", "join_build"])
    print(json.dumps({"nd": nd, "wall_ms": wall * 1e3, **kt}), flush=True)
    del k, dk, dg
