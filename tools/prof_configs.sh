#!/bin/bash
# Per-kernel durations of tools/bench_configs.py (rocprofv3 kernel trace only).
# usage: tools/prof_configs.sh <tag> [bench_configs args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/profcfg_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o kt -- \
    python3 "$ROOT/tools/bench_configs.py" "$@" > "$OUT/run.log" 2>&1 || { echo "profile failed"; tail -20 "$OUT/run.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print("%-90s calls=%5s avg_us=%10.1f total_ms=%9.2f" % (r["Name"][:90], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                           float(r["TotalDurationNs"]) / 1e6))
PY
grep '^{' "$OUT/run.log"
