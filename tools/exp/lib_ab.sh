#!/bin/bash
# Same-box A/B of library builds on tools/bench_configs.py configs, alternating: lib_ab.sh OUT CONFIGS lib1 lib2 ...
set -o pipefail
O=$1; CF=$2; shift 2
mkdir -p $O
for r in 1 2; do
  for lib in "$@"; do
    QEH_LIB_PATH=$PWD/query-engine_amd/$lib timeout -k 10 300 python3 -u tools/bench_configs.py --only $CF > $O/${lib}_$r.jsonl 2> $O/${lib}_$r.err || { tail $O/${lib}_$r.err; exit 1; }
    python3 -c "
import json
for l in open('$O/${lib}_$r.jsonl'):
    d=json.loads(l); print('$lib', $r, d['config'][:44], round(d.get('kernel_ms') or 0,3), {k: round(v,2) for k,v in (d.get('kernel_split_ms') or {}).items() if v})
"
  done
done
