#!/bin/bash
# A/B of an environment switch on the metric bench, alternating runs on one box.
# usage: tools/exp_env_ab.sh VAR valueA valueB [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V="$1"; A="$2"; B="$3"; N="${4:-2}"
for r in $(seq 1 $N); do
  for x in "$A" "$B"; do
    env "$V=$x" timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/ab_$x.log 2>&1 || { tail -5 gpurun_out/ab_$x.log; exit 1; }
    tail -1 gpurun_out/ab_$x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$V=$x', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['kernel_ms'],3), d['roofline']['kernel_split_ms'])"
  done
done
