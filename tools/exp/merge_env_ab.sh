#!/bin/bash
# Merge::sorted A/B on one box over environment settings, alternating twice:
#   bash tools/exp/merge_env_ab.sh "QEH_MSD_HIST_SUB=1" "QEH_MSD_HIST_SUB=4" ...
set -o pipefail
O=gpurun_out/menv; mkdir -p $O
for r in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 200 python3 -u tools/bench_configs.py --only merge > $O/v${i}_$r.jsonl 2> $O/v${i}_$r.err || { tail $O/v${i}_$r.err; exit 1; }
    python3 -c "
import json
for l in open('$O/v${i}_$r.jsonl'):
    d=json.loads(l); print('$e', $r, round(d['kernel_ms'],3), round(d['ms_per_run'],3), round(d['frac_of_8TBs'],4))
"
  done
done
