#!/usr/bin/env python3
"""Merge::sorted of 8 x 1.25e7 rows (tools/bench_configs.py cfg_merge's shape), repeated: for kernel traces."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
import qe_hip  # noqa: E402
from qe_hip import abi  # noqa: E402

ctx = qe_hip.Context(0)
parts, per = [], 12_500_000
for p in range(8):
    k = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED + p, 7, per, 2 ** 40)
    kv, _ = k.to_numpy()
    valid = np.random.default_rng(p).random(per) > 0.05
    parts.append([ctx.upload(kv, valid), ctx.generate(abi.GEN_UNIT_F64, 0x5EED + p, 8, per)])
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    cols, rows = ctx.merge_sorted(parts, [0], [False], [False])
    for c in cols:
        c.release()
ctx.sync()
