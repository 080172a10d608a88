#!/usr/bin/env python3
"""Per-phase shader-clock cycles of the fused phase A (k_slice_partition, EARLY) from a diagnostic
build made with -DQEH_PA_STAMPS=1 (make BUILD=build_stamps LIB=libqeh_stamps.so EXTRA=-DQEH_PA_STAMPS=1).
Runs the metric query (1e9 x 1e7) a few times and reads the stamps of the last run: per wave, the
cycles of each phase summed over its tiles.  Prints the mean per tile over waves (and over wave 0 /
waves 1-15 separately), the in-kernel clock (s_memtime / s_memrealtime) and the phase-A kernel time.
usage: python tools/exp/pa_stamps.py [lib.so ...]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))

PHASES = ["load_wait", "eval_rank", "issue_flush", "B1_wait", "scan_carry", "B2_wait", "stage_plan", "B3_wait",
          "tiles", "loop_top"]


def run(libpath, n=1_000_000_000, nd=10_000_000):
    import torch
    from qe_hip import abi
    abi._lib = abi.load(libpath)
    import qe_hip
    from qe_hip import AggregateFunction as AF, BinaryOp, binop, col, lit
    seed = 0x5EED
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx = qe_hip.Context(0)
    ctx.set_stream(s.cuda_stream)
    x = ctx.generate(abi.GEN_UNIFORM_MOD, seed, 1, n, 100)
    k = ctx.generate(abi.GEN_UNIFORM_MOD, seed, 2, n, nd)
    v = ctx.generate(abi.GEN_UNIT_F64, seed, 3, n)
    dk = ctx.generate(abi.GEN_PERMUTATION, seed, 0, nd, nd)
    dg = ctx.generate(abi.GEN_UNIFORM_MOD, seed, 5, nd, 1024)
    pred = binop(col(0), BinaryOp.Greater, lit(49))
    aggs = [(AF.Sum, 2), (AF.Count, 2)]
    for _ in range(3):
        ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], aggs)
    ctx.timing(True)
    ctx.timing_reset()
    ctx.join_filter_aggregate([x, k, v], 1, pred, dk, [dg], aggs)
    torch.cuda.synchronize()
    a_ms = ctx.kernel_time("slice_partition")[0]
    lib = C.CDLL(libpath)
    words = 512 * 16 * 16
    buf = np.zeros(words, np.uint64)
    assert lib.qeh_debug_pa_stamps(buf.ctypes.data_as(C.c_void_p), C.c_uint64(words)) == 0
    w = buf.reshape(512 * 16, 16)
    w = w[w[:, 8] > 0]
    tiles = w[:, 8].astype(np.float64)
    per = {p: float(np.mean(w[:, i] / tiles)) for i, p in enumerate(PHASES) if p != "tiles"}
    w0 = w.reshape(-1, 16, 16)[:, 0, :]
    wr = w.reshape(-1, 16, 16)[:, 1:, :].reshape(-1, 16)
    per_w0 = {p: float(np.mean(w0[:, i] / w0[:, 8])) for i, p in enumerate(PHASES) if p != "tiles"}
    per_wr = {p: float(np.mean(wr[:, i] / wr[:, 8])) for i, p in enumerate(PHASES) if p != "tiles"}
    clock = float(np.median(w[:, 10] / np.maximum(w[:, 11], 1))) * 100.0  # MHz
    out = {"lib": os.path.basename(libpath), "phaseA_ms": round(a_ms, 3), "clock_MHz": round(clock, 1),
           "tiles_per_wave": float(np.mean(tiles)), "loop_cycles_per_tile": float(np.mean(w[:, 10] / tiles)),
           "cycles_per_tile_mean": {k: round(v, 1) for k, v in per.items()},
           "wave0": {k: round(v, 1) for k, v in per_w0.items()},
           "waves1_15": {k: round(v, 1) for k, v in per_wr.items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 2 or (len(sys.argv) == 2 and sys.argv[1] == "--all"):
        import subprocess
        libs = sys.argv[1:] if sys.argv[1] != "--all" else []
        for lib in libs:
            subprocess.run([sys.executable, __file__, lib], check=True)
    else:
        run(os.path.join(ROOT, "query-engine_amd", sys.argv[1] if len(sys.argv) > 1 else "libqeh_stamps.so"))
