#!/bin/bash
# cfg5 under several window-path environment settings (one line each), one box.
# usage: tools/exp_wm_env.sh "VAR=a" "VAR=b" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for kv in "$@"; do
  env $kv timeout -k 10 200 python tools/bench_configs.py --only cfg5 > gpurun_out/wmenv.jsonl 2>&1 || { tail -5 gpurun_out/wmenv.jsonl; exit 1; }
  echo "$kv $(grep -o '"kernel_ms": [0-9.]*\|"window_[a-z]*": [0-9.]*' gpurun_out/wmenv.jsonl | tr '\n' ' ')"
done
