#!/bin/bash
# Merge::sorted A/B on one box: the counting-sort LDS kernel (default) vs the three-pass radix LDS sort
# (QEH_MSD_RADIX_LDS=1), alternating twice.
set -o pipefail
O=gpurun_out/mcs; mkdir -p $O
for r in 1 2; do
  for mode in csort radix; do
    if [ $mode = radix ]; then export QEH_MSD_RADIX_LDS=1; else unset QEH_MSD_RADIX_LDS; fi
    timeout -k 10 200 python3 -u tools/bench_configs.py --only merge > $O/${mode}_$r.jsonl 2> $O/${mode}_$r.err || { tail $O/${mode}_$r.err; exit 1; }
    python3 -c "
import json
for l in open('$O/${mode}_$r.jsonl'):
    d=json.loads(l); print('$mode', $r, round(d['kernel_ms'],3), round(d['ms_per_run'],3), round(d['frac_of_8TBs'],4))
"
  done
done
