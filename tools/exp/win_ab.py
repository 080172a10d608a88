#!/usr/bin/env python3
"""A/B of config 5 (ROW_NUMBER() OVER (PARTITION BY k ORDER BY v), 1e9 rows, k in [0, 2^20)) across
library builds, alternating builds in rounds: the window path's timer groups (partition passes, group
sort, inverse passes) per build, best of `reps` runs.  Results are not checked (experiment builds).
usage: python tools/exp/win_ab.py [--rounds R] lib1.so[:ENV=V] lib2.so ...   (dev tool, not the product)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(lib, reps=3):
    sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
    import torch
    from qe_hip import abi
    abi._lib = abi.load(os.path.join(ROOT, "query-engine_amd", lib))
    import qe_hip
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx = qe_hip.Context(0)
    ctx.set_stream(s.cuda_stream)
    n = 1_000_000_000
    k = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 7, n, 2 ** 20)
    v = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 8, n, 2 ** 62, lo=-(2 ** 61))
    ctx.row_number([k], [v], [True]).release()
    best = None
    for _ in range(reps):
        ctx.timing(True)
        ctx.timing_reset()
        ctx.row_number([k], [v], [True]).release()
        ctx.sync()
        t = {g: ctx.kernel_time(g)[0] for g in ("window_partition", "window_sort", "window_place")}
        t["total"] = sum(t.values())
        if best is None or t["total"] < best["total"]:
            best = t
    print(f"{lib:22s} {os.environ.get('QEH_AB_TAG', ''):20s} " + "  ".join(f"{g} {x:7.3f}" for g, x in best.items()),
          flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    if os.environ.get("QEH_AB_CHILD"):
        child(a[0])
        sys.exit(0)
    rounds = 2
    if a and a[0] == "--rounds":
        rounds, a = int(a[1]), a[2:]
    for r in range(rounds):
        for spec in a:
            lib, _, envs = spec.partition(":")
            env = dict(os.environ, QEH_AB_CHILD="1", QEH_AB_TAG=envs)
            for kv in filter(None, envs.split(",")):
                x, _, y = kv.partition("=")
                env[x] = y
            subprocess.run([sys.executable, __file__, lib], env=env, check=True)
