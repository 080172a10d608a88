#!/usr/bin/env python3
"""One config-5 query shape, repeated (for rocprofv3 kernel traces / PMC passes of the window kernels).
usage: python tools/exp/w3_run.py [rows] [keys] [reps] [func: rn|rank|lag]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
import qe_hip  # noqa: E402
from qe_hip import abi  # noqa: E402
from qe_hip.plan import WindowFunctionType as W  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
keys = int(float(sys.argv[2])) if len(sys.argv) > 2 else 1 << 20
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
func = sys.argv[4] if len(sys.argv) > 4 else "rn"
ctx = qe_hip.Context(0)
k = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 7, n, keys)
v = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 8, n, 2 ** 62, lo=-(2 ** 61))
names = ("w3_partition", "w3_sort", "w3_place", "window_partition", "window_sort", "window_place")
for _ in range(reps):
    ctx.timing(True)
    ctx.timing_reset()
    if func == "rn":
        ctx.row_number([k], [v], [True]).release()
    elif func == "rank":
        ctx.window(W.Rank, [k], [v], [True]).release()
    else:
        ctx.window(W.Lag, [k], [v], [True], arg=v, param=1).release()
    ctx.sync()
    t = {g: ctx.kernel_time(g)[0] for g in names}
    print(" ".join(f"{g} {x:.3f}" for g, x in t.items() if x), f"total {sum(t.values()):.3f}", flush=True)
