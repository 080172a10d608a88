#!/bin/bash
# pgwire DataRow encode A/B over environment settings, alternating twice:
#   bash tools/exp/encode_env_ab.sh "QEH_ENC_LDS_KB=48" "QEH_ENC_LDS_KB=16"
set -o pipefail
O=gpurun_out/eenv; mkdir -p $O
for r in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 200 python3 -u tools/bench_configs.py --only encode > $O/v${i}_$r.jsonl 2> $O/v${i}_$r.err || { tail $O/v${i}_$r.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/v${i}_$r.jsonl').readline()); print('$e', $r, round(d['kernel_ms'],3), d['kernel_split_ms'])
"
  done
done
