#!/usr/bin/env python3
"""Window pass-1 cost split (run under rocprofv3 --kernel-trace, QEH_WM_EXP set by the caller):
ROW_NUMBER on n rows, k in [0, 2^20), three calls; with QEH_WM_EXP != 0 the library stops after
pass 1 and raises.  usage: QEH_WM_EXP=<bits> wm_exp.py n"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
import torch  # noqa: E402,F401
import qe_hip  # noqa: E402
from qe_hip import abi  # noqa: E402

n = int(float(sys.argv[1]))
with qe_hip.Context(0) as ctx:
    k = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 7, n, 2 ** 20)
    v = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 8, n, 2 ** 62, lo=-(2 ** 61))
    for _ in range(3):
        try:
            ctx.row_number([k], [v], [True]).release()
        except abi.QehError:
            pass
    ctx.sync()
print("ok", os.environ.get("QEH_WM_EXP"))
