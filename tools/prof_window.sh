#!/bin/bash
# Per-kernel durations and HBM bytes of the config-5 window path (ROW_NUMBER, bench_configs cfg5):
# a kernel-trace pass, then FETCH_SIZE and WRITE_SIZE passes of their own.
# usage: tools/prof_window.sh <tag> [bench_configs args, default --only cfg5 --scale 0.25]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
ARGS=("$@"); [ ${#ARGS[@]} -eq 0 ] && ARGS=(--only cfg5 --scale 0.25)
OUT="$ROOT/gpurun_out/profwin_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
RUN=(python3 "$ROOT/tools/bench_configs.py" "${ARGS[@]}")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- "${RUN[@]}" \
    > "$OUT/kt.log" 2>&1 || { echo "kernel-trace pass failed"; tail -5 "$OUT/kt.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- "${RUN[@]}" \
    > "$OUT/fetch.log" 2>&1 || { echo "FETCH_SIZE pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- "${RUN[@]}" \
    > "$OUT/write.log" 2>&1 || { echo "WRITE_SIZE pass failed"; exit 1; }
python3 "$ROOT/tools/pmc_traffic.py" "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
