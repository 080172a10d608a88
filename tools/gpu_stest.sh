#!/bin/bash
# Sort / merge check on the GPU box: sort, merge and window tests, then the Merge::sorted line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_merge.py tests/test_join_sort_window.py tests/test_window.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/stest.log 2>&1 || { tail -30 gpurun_out/stest.log; exit 1; }
tail -1 gpurun_out/stest.log
timeout -k 10 300 python tools/bench_configs.py --only merge > gpurun_out/merge.jsonl 2>&1 || { tail -5 gpurun_out/merge.jsonl; exit 1; }
grep -o '"config": "[^"]*"\|"kernel_ms": [0-9.]*\|"sort_encode": [0-9.]*\|"gather": [0-9.]*\|"radix_pass": [0-9.]*' gpurun_out/merge.jsonl
