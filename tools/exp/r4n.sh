#!/bin/bash
# Round-4 GPU session n: MSD payload sort parity + Merge::sorted kernel trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R"
O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_merge.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o kt -- python3 $R/tools/bench_configs.py --only merge > $R/$O/merge.jsonl 2>$R/$O/merge.err || { tail $R/$O/merge.err; exit 1; }
cut -c1-300 $R/$O/merge.jsonl
python3 - "$(find $R/$O/kt -name '*kernel_stats.csv' | head -1)" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:80]:80s} calls={r["Calls"]:>4s} avg_ms={float(r["AverageNs"])/1e6:8.3f}')
PY
