"""Where the time of qeh_encode_arrow_ipc goes (library call vs Python copy)."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
import torch  # noqa: F401,E402
import qe_hip  # noqa: E402
from qe_hip import abi  # noqa: E402

ctx = qe_hip.Context(0)
n = 10_000_000
cols = [ctx.generate(abi.GEN_UNIFORM_MOD, 1, i, n, 1 << 40) for i in range(3)]
cin = ctx._cols(cols)
nm = (C.c_char_p * 3)(b"a", b"b", b"c")
for rep in range(4):
    p, size = C.c_void_p(), C.c_int64()
    t0 = time.perf_counter()
    abi.check(ctx.lib.qeh_encode_arrow_ipc(ctx.h, cin, nm, 3, C.byref(p), C.byref(size)))
    t1 = time.perf_counter()
    b = C.string_at(p, size.value)
    t2 = time.perf_counter()
    ctx.lib.qeh_host_free(p)
    t3 = time.perf_counter()
    print(f"lib {1e3*(t1-t0):.1f} ms  copy {1e3*(t2-t1):.1f} ms  free {1e3*(t3-t2):.1f} ms  bytes {size.value}")
