#!/bin/bash
# One-step kernel timeline of the bench (kernel trace only, no counters):
# prints every dispatch between two consecutive k_slice_partition launches with
# its start offset, duration and the gap before it.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/timeline"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o tl -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-sample 0 "$@" > "$OUT/run.log" 2>&1 || { tail "$OUT/run.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_slice_partition" in r["Kernel_Name"] or "k_join_agg_fast" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
# the step before the last probe: from the dispatch after the previous probe's finalize
seg = rows[a - 40 if a >= 40 else 0: b + 1]
t0 = int(rows[a]["Start_Timestamp"])
prev_end = None
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    print(f"{(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:9.1f} us  gap {gap:8.1f} us  {r['Kernel_Name'].split('(')[0][:70]}")
    prev_end = e
PY
