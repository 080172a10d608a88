#!/bin/bash
# Same-box A/B of the metric bench: A = this tree, B = another built tree (ab_old/: a HEAD copy)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abt
for i in 1 2 3; do
  for v in A B; do
    if [ "$v" = A ]; then b=bench.py; else b=ab_old/bench.py; fi
    timeout -k 10 200 python $b --cpu-sample 0 --traffic-json profiles/traffic_latest.json > gpurun_out/abt/$v$i.log 2>&1 || { tail -20 gpurun_out/abt/$v$i.log; exit 1; }
    echo "$v$i $(tail -1 gpurun_out/abt/$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["roofline"]["kernel_split_ms"], round(d["roofline"]["frac"],4))')"
  done
done
