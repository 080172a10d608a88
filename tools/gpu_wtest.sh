#!/bin/bash
# Window path check on the GPU box: partitioning-window parity tests, then cfg5 (ROW_NUMBER) and the
# RANK / LAG window lines.  usage: tools/gpu_wtest.sh [full]  (full: also the LSD-path window tests)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=tests/test_window_msd.py; [ "$1" = full ] && T="$T tests/test_join_sort_window.py"
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wtest.log 2>&1 || { tail -30 gpurun_out/wtest.log; exit 1; }
tail -1 gpurun_out/wtest.log
timeout -k 10 200 python tools/bench_configs.py --only cfg5 > gpurun_out/cfg5.jsonl 2>&1 || { tail -5 gpurun_out/cfg5.jsonl; exit 1; }
timeout -k 10 300 python tools/bench_configs.py --only window > gpurun_out/window.jsonl 2>&1 || { tail -5 gpurun_out/window.jsonl; exit 1; }
grep -o '"config": "[^"]*"\|"window_[a-z]*": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/cfg5.jsonl gpurun_out/window.jsonl
