#!/bin/bash
# A/B of an environment switch on the metric bench, alternating on one box
# usage: tools/exp_ab.sh "<ENV=VAL for B>" [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
B="$1"; R="${2:-2}"
for i in $(seq 1 "$R"); do
  for v in A B; do
    if [ "$v" = A ]; then e=""; else e="$B"; fi
    env $e timeout -k 10 200 python bench.py --cpu-sample 0 > gpurun_out/ab/bench_$v$i.log 2>&1 || { tail -20 gpurun_out/ab/bench_$v$i.log; exit 1; }
    echo "$v$i [$e] $(tail -1 gpurun_out/ab/bench_$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), round(d["roofline"]["kernel_ms"],3), d["roofline"]["kernel_split_ms"], round(d["roofline"]["frac"],4))')"
  done
done
