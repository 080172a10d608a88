#!/bin/bash
# A/B on one box: round-5 final library (libqeh_r5.so, built from 288fd1a) vs the current tree, cfg3 and
# shapes, alternating twice, so box state changes show up as both sides moving together.
set -o pipefail
O=gpurun_out/ab6; mkdir -p $O
for r in 1 2; do
  for lib in libqeh_r5.so libqeh.so; do
    QEH_LIB_PATH=$PWD/query-engine_amd/$lib timeout -k 10 300 python3 -u tools/bench_configs.py --only cfg3,left,full > $O/cfg_${lib}_$r.jsonl 2>$O/cfg_${lib}_$r.err || { tail $O/cfg_${lib}_$r.err; exit 1; }
    python3 -c "
import json,sys
for l in open('$O/cfg_${lib}_$r.jsonl'):
    d=json.loads(l); print('$lib', $r, d['config'][:40], round(d.get('kernel_ms',0),3))
"
  done
done
