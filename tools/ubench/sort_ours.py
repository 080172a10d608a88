"""Time qeh_sort_indices on one Int64 column of n values in [0, 2^bits) (the LSD passes of
k_sort.hip), to set beside sort_ubench's rocPRIM number."""
import sys
import time

import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "query-engine_amd"))
import qe_hip  # noqa: E402
from qe_hip import abi  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
bits = int(sys.argv[2]) if len(sys.argv) > 2 else 40
with qe_hip.Context(0) as ctx:
    k = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 1, n, modulus=1 << bits)
    ctx.timing(True)
    for it in range(4):
        ctx.timing_reset()
        ctx.sync()
        t = time.perf_counter()
        p = ctx.sort_indices([k], [True])
        ctx.sync()
        ms = (time.perf_counter() - t) * 1e3
        names = ["sort_encode", "radix_pass"]
        print(f"qeh_sort_indices n={n} bits={bits}: {ms:.2f} ms wall;",
              ", ".join(f"{nm} {ctx.kernel_time(nm)[0]:.2f}ms/{ctx.kernel_time(nm)[1]}" for nm in names), flush=True)
        del p
