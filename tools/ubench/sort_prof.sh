#!/bin/bash
# Kernel-trace stats of our LSD sort (sort_ours.py) and rocPRIM's (sort_ubench) on 1e9 40-bit pairs.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/prof_sort"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ours" -o kt -- python3 "$ROOT/tools/ubench/sort_ours.py" 1e9 40 \
    > "$OUT/ours.log" 2>&1 || { echo "ours failed"; tail "$OUT/ours.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprim" -o kt -- "$ROOT/tools/ubench/sort_ubench" 1000000000 40 \
    > "$OUT/rocprim.log" 2>&1 || { echo "rocprim failed"; tail "$OUT/rocprim.log"; exit 1; }
for d in ours rocprim; do
  echo "== $d"
  f=$(find "$OUT/$d" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for r in sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'{r["Name"][:90]:90s} calls={r["Calls"]:>4s} avg_us={float(r["AverageNs"])/1e3:9.1f}')
PY
done
