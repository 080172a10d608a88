#!/bin/bash
# Outer-join slice probe A/B: kernel stats of LEFT / FULL per library variant (QEH_LIB_PATH), one box.
# usage: tools/exp/os_ab.sh OUTDIR lib1.so lib2.so ...
set -o pipefail
O=$1; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for lib in "$@"; do
  QEH_LIB_PATH=$PWD/query-engine_amd/$lib timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt_$lib -o run --output-format csv -- python3 tools/bench_configs.py --only left,full > $O/b_$lib.jsonl 2> $O/b_$lib.err || { tail $O/b_$lib.err; exit 1; }
  python3 - $O/kt_$lib/run_kernel_stats.csv $lib <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
    if 'k_os' in r['Name'] or 'embed32' in r['Name'] or 'tail' in r['Name']:
        print(sys.argv[2], r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
  grep '^{' $O/b_$lib.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$lib', d['config'][:30], round(d['kernel_ms'],3), round(d['frac_of_8TBs'],3))"
done
