"""cfg5 timing breakdown of the partitioning window path (per-timer ms), 1e9 rows by default."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "query-engine_amd"))
import qe_hip
from qe_hip import abi
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
ctx = qe_hip.Context(0)
k = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 7, n, 2 ** 20)
v = ctx.generate(abi.GEN_UNIFORM_MOD, 0x5EED, 8, n, 2 ** 62, lo=-(2 ** 61))
ctx.row_number([k], [v], [True]).release()
ctx.sync()
ctx.timing(True)
for rep in range(3):
    ctx.timing_reset()
    ctx.row_number([k], [v], [True]).release()
    t = {nm: round(ctx.kernel_time(nm)[0], 2) for nm in ("window_partition", "scan", "window_sort", "window_place")}
    print(os.environ.get("TAG", ""), t, "total", round(sum(t.values()), 2), flush=True)
