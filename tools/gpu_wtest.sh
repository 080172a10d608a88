#!/bin/bash
# Window path check on the GPU box: partitioning-window parity tests, then cfg5 with the
# workgroup-per-group counting sort and with the network only (QEH_WM_NO_COUNT=1), then RANK / LAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_window_msd.py tests/test_join_sort_window.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wtest.log 2>&1 || { tail -30 gpurun_out/wtest.log; exit 1; }
tail -1 gpurun_out/wtest.log
timeout -k 10 200 python tools/bench_configs.py --only cfg5 > gpurun_out/cfg5.jsonl 2>&1 || { tail -5 gpurun_out/cfg5.jsonl; exit 1; }
QEH_WM_NO_COUNT=1 timeout -k 10 200 python tools/bench_configs.py --only cfg5 > gpurun_out/cfg5b.jsonl 2>&1 || { tail -5 gpurun_out/cfg5b.jsonl; exit 1; }
timeout -k 10 300 python tools/bench_configs.py --only window > gpurun_out/window.jsonl 2>&1 || { tail -5 gpurun_out/window.jsonl; exit 1; }
grep -o '"config": "[^"]*"\|"window_[a-z]*": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/cfg5.jsonl gpurun_out/cfg5b.jsonl gpurun_out/window.jsonl
