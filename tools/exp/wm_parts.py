#!/usr/bin/env python3
"""(Needs the experiments build: make -C query-engine_amd experiments, then QEH_LIB_PATH=.../libqeh_exp.so.)
Config 5's partition passes per setting (QEH_WM_EXP=16: pass 1 alone, the query then fails;
QEH_WM_LB: the digit split; QEH_WM_G1W / G1X: pass-1 workgroups): the window timers (partition =
min/max + histogram + scan + pass 1 [+ pass 2]), best of `reps`, alternating settings over rounds.
Results are not checked (dev tool, not the product).
usage: python tools/exp/wm_parts.py [--rounds R] [--rows N] [--keys K] ENV=V[,ENV=V] ...   ("-" = defaults)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(tag, n, keys, reps=3):
    sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
    import torch
    import qe_hip
    from qe_hip import abi
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx = qe_hip.Context(0)
    ctx.set_stream(s.cuda_stream)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 7, n, keys)
    v = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 8, n, 2 ** 62, lo=-(2 ** 61))
    best = None
    for _ in range(reps + 1):
        ctx.timing(True)
        ctx.timing_reset()
        try:
            ctx.row_number([k], [v], [True]).release()
        except Exception:
            pass  # experiment runs stop after the partition passes
        ctx.sync()
        t = {g: ctx.kernel_time(g)[0] for g in ("window_partition", "window_sort", "window_place")}
        t["total"] = sum(t.values())
        if best is None or t["total"] < best["total"]:
            best = t
    print(f"{tag:36s} " + "  ".join(f"{g} {x:7.3f}" for g, x in best.items()), flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    if os.environ.get("QEH_AB_CHILD"):
        child(a[0], int(a[1]), int(a[2]))
        sys.exit(0)
    rounds, n, keys = 2, 1_000_000_000, 2 ** 20
    while a and a[0].startswith("--"):
        if a[0] == "--rounds":
            rounds, a = int(a[1]), a[2:]
        elif a[0] == "--keys":
            keys, a = int(float(a[1])), a[2:]
        elif a[0] == "--rows":
            n, a = int(float(a[1])), a[2:]
    for r in range(rounds):
        for spec in a:
            env = dict(os.environ, QEH_AB_CHILD="1")
            for kv in filter(None, spec.split(",")):
                if kv == "-":
                    continue
                x, _, y = kv.partition("=")
                env[x] = y
            subprocess.run([sys.executable, __file__, spec, str(n), str(keys)], env=env, check=True)
