#!/bin/bash
# bench.py (the metric) with library builds alternating on one box: bench_lib_ab.sh lib1 lib2 ...
set -o pipefail
O=gpurun_out/blab; mkdir -p $O
for r in 1 2 3; do
  for lib in "$@"; do
    QEH_LIB_PATH=$PWD/query-engine_amd/$lib timeout -k 10 300 python3 -u bench.py > $O/${lib}_$r.json 2> $O/${lib}_$r.err || { tail $O/${lib}_$r.err; exit 1; }
    python3 -c "
import json
d=json.load(open('$O/${lib}_$r.json')); r=d['roofline']; print('$lib', $r, round(d['ms_per_step'],3), round(r['frac'],4), {k: round(v,3) for k,v in r['kernel_split_ms'].items()})
"
  done
done
