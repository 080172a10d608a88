#!/usr/bin/env python3
"""Experiment: per-row cost of the window partition passes by digit width.
Runs ROW_NUMBER() OVER (PARTITION BY k ORDER BY v) on n rows with k in [0, 2^kbits), under
the env QEH_WM_LB given per case (low-digit bits), a few repetitions each; run it under
rocprofv3 --kernel-trace to split per kernel.  usage: exp_wm_digits.py n kbits [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
import torch  # noqa: E402,F401
import qe_hip  # noqa: E402
from qe_hip import abi  # noqa: E402

n, kbits = int(float(sys.argv[1])), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
with qe_hip.Context(0) as ctx:
    k = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 7, n, 2 ** kbits)
    v = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 8, n, 2 ** 62, lo=-(2 ** 61))
    ctx.row_number([k], [v], [True]).release()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.row_number([k], [v], [True]).release()
    ctx.sync()
    print(f"n={n} kbits={kbits} lb={os.environ.get('QEH_WM_LB', '-')}: {(time.perf_counter() - t0) / reps * 1e3:.2f} ms")
