#!/bin/bash
# Exchange + window-histogram check on the GPU box: partition / distributed / window tests, then the
# hash Exchange line and cfg5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_partition.py tests/test_distributed.py tests/test_window_msd.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ptest.log 2>&1 || { tail -30 gpurun_out/ptest.log; exit 1; }
tail -1 gpurun_out/ptest.log
timeout -k 10 300 python tools/bench_configs.py --only partition,cfg5 > gpurun_out/pcfg.jsonl 2>&1 || { tail -5 gpurun_out/pcfg.jsonl; exit 1; }
grep -o '"config": "[^"]*"\|"window_[a-z]*": [0-9.]*\|"kernel_ms": [0-9.]*\|"frac_of_8TBs": [0-9.]*' gpurun_out/pcfg.jsonl
