#!/usr/bin/env python3
"""Does the metric step's time drift over a run (clock / power-state ramp)?  Runs the metric query
(1e9 x 1e7) `steps` times back to back after generating the data and prints the phase-A / phase-B
kernel times per block of 20 steps, plus the first 10 steps one by one.  Dev tool (not the product).
usage: python tools/exp/ramp.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))


def main(steps):
    import torch
    import qe_hip
    from qe_hip import abi
    from qe_hip import AggregateFunction as AF, BinaryOp, binop, col, lit
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx = qe_hip.Context(0)
    ctx.set_stream(s.cuda_stream)
    seed, n, nd = 0x5EED, 1_000_000_000, 10_000_000
    x = ctx.generate(abi.GEN_UNIFORM_MOD, seed, 1, n, 100)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, seed, 2, n, nd)
    v = ctx.generate(abi.GEN_UNIT_F64, seed, 3, n)
    dk = ctx.generate(abi.GEN_PERMUTATION, seed, 0, nd, nd)
    dg = ctx.generate(abi.GEN_UNIFORM_MOD, seed, 5, nd, 1024)
    ctx.sync()
    pred = binop(col(0), BinaryOp.Greater, lit(49))
    aggs = [(AF.Sum, 2), (AF.Count, 2)]
    ctx.timing(True)
    rows = []
    t_start = time.perf_counter()
    for i in range(steps):
        ctx.timing_reset()
        t0 = time.perf_counter()
        r = ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], aggs)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        rows.append((time.perf_counter() - t_start, wall, ctx.kernel_time("slice_partition")[0],
                     ctx.kernel_time("slice_probe")[0]))
        for c in r[0] + r[1]:
            c.release()
    for i in range(min(10, steps)):
        print(f"step {i:3d} t={rows[i][0]:6.3f}s wall {rows[i][1]:7.3f} A {rows[i][2]:6.3f} B {rows[i][3]:6.3f}")
    for b in range(0, steps, 20):
        blk = rows[b:b + 20]
        m = lambda j: sum(r[j] for r in blk) / len(blk)
        print(f"steps {b:3d}-{b + len(blk) - 1:3d} t={blk[0][0]:6.3f}s wall {m(1):7.3f} A {m(2):6.3f} B {m(3):6.3f}",
              flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 300)
