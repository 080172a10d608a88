#!/bin/bash
# rocprofv3 evidence for the bench's dominant kernel (run on the GPU box):
#   1) --kernel-trace --stats over a short bench run  -> per-kernel durations
#   2) --pmc FETCH_SIZE and 3) --pmc WRITE_SIZE, each its own pass (TCC slots;
#      never combined with other trace domains)
# then tools/pmc_traffic.py turns the CSVs into per-launch HBM bytes.
# usage: tools/profile.sh <tag> [extra bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH=(python3 "$ROOT/bench.py" --steps 5 --warmup 1 --cpu-sample 0 "$@")
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- "${BENCH[@]}" \
    > "$OUT/kt.log" 2>&1 || { echo "kernel-trace pass failed"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- "${BENCH[@]}" \
    > "$OUT/fetch.log" 2>&1 || { echo "FETCH_SIZE pass failed"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- "${BENCH[@]}" \
    > "$OUT/write.log" 2>&1 || { echo "WRITE_SIZE pass failed"; exit 1; }
python3 "$ROOT/tools/pmc_traffic.py" "$OUT" --emit "$OUT/traffic_latest.json" > "$OUT/summary.txt" 2>&1 || { echo "parse failed"; cat "$OUT/summary.txt"; exit 1; }
cat "$OUT/summary.txt"
