#!/usr/bin/env python3
"""Phase A / phase B kernel times of the metric query (1e9 x 1e7) for several builds of the library,
alternating builds in rounds (results are not checked: experiment builds may compute garbage).
usage: python tools/exp_slice.py [--rows N] [--steps K] [--rounds R] lib1.so[:ENV=V,ENV2=V2] ..."""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, time, json
sys.path.insert(0, os.path.join(%(root)r, "query-engine_amd"))
import torch
from qe_hip import abi
abi._lib = abi.load(%(lib)r)
import qe_hip
from qe_hip import AggregateFunction as AF, BinaryOp, binop, col, lit
n, nd, SEED = %(rows)d, 10_000_000, 0x5EED
torch.cuda.set_device(0)
s = torch.cuda.Stream(); torch.cuda.set_stream(s)
ctx = qe_hip.Context(0); ctx.set_stream(s.cuda_stream)
x = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 1, n, 100)
k = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 2, n, nd)
v = ctx.generate(abi.GEN_UNIT_F64, SEED, 3, n)
dk = ctx.generate(abi.GEN_PERMUTATION, SEED, 0, nd, nd)
dg = ctx.generate(abi.GEN_UNIFORM_MOD, SEED, 5, nd, 1024)
ctx.sync()
pred = binop(col(0), BinaryOp.Greater, lit(49))
aggs = [(AF.Sum, 2), (AF.Count, 2)]
step = lambda: ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], aggs)
for _ in range(2): step()
torch.cuda.synchronize()
ctx.timing(True); ctx.timing_reset()
t0 = time.perf_counter()
for _ in range(%(steps)d): r = step()
torch.cuda.synchronize()
el = (time.perf_counter() - t0) * 1e3 / %(steps)d
a, na = ctx.kernel_time("slice_partition"); b, nb = ctx.kernel_time("slice_probe")
print(json.dumps({"lib": os.path.basename(%(lib)r), "step_ms": round(el, 3), "A_ms": round(a / max(na, 1), 3),
                  "B_ms": round(b / max(nb, 1), 3), "launches": na}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    for r in range(a.rounds):
        for spec in a.libs:
            lib, _, envs = spec.partition(":")
            env = dict(os.environ)
            for kv in filter(None, envs.split(",")):
                k, _, v = kv.partition("=")
                env[k] = v
            p = os.path.join(ROOT, "query-engine_amd", lib) if not os.path.isabs(lib) else lib
            code = CHILD % {"root": ROOT, "lib": p, "rows": a.rows, "steps": a.steps}
            out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env)
            line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-400:]
            print(f"round {r} [{envs}] {line}", flush=True)
            if out.returncode != 0:
                sys.exit(out.returncode)


if __name__ == "__main__":
    main()
