#!/bin/bash
# Kernel-trace of the window partition passes at several digit splits (tools/exp_wm_digits.py).
# usage: tools/exp_wm.sh <tag>
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/expwm_$1"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name n kbits lb
    QEH_WM_LB=$4 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$1" -o kt -- \
        python3 "$ROOT/tools/exp_wm_digits.py" "$2" "$3" 3 > "$OUT/$1.log" 2>&1 || { echo "$1 failed"; tail -5 "$OUT/$1.log"; exit 1; }
    grep "ms" "$OUT/$1.log" | tail -1
}
run c20 2.5e8 20 10 && run a18 2.5e8 18 8 && run b18 2.5e8 18 10 && run d16 6.25e7 16 6
