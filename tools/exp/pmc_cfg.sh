#!/bin/bash
# rocprofv3 counter passes over one tools/bench_configs.py config (run on the GPU box):
#   tools/exp/pmc_cfg.sh <tag> <config> <kernel-name filter regex> "COUNTERS ..." ["COUNTERS ..." ...]
# Each group is its own pass (<= 8 SQ, 4 TCC counters; never with tracing domains), under a hard time limit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
TAG="$1"; CFG="$2"; FILT="$3"; shift 3
O=$R/gpurun_out/pmc_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p -- \
        python3 $R/tools/bench_configs.py --only $CFG > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - "$O" "$FILT" > $O/summary.txt <<'PY'
import csv, glob, os, re, sys
from collections import defaultdict
d, filt = sys.argv[1], re.compile(sys.argv[2])
acc = defaultdict(lambda: defaultdict(float))
n = defaultdict(lambda: defaultdict(int))
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k][r["Counter_Name"]] += 1
for k in sorted(acc):
    if not filt.search(k):
        continue
    print(k)
    for c in sorted(acc[k]):
        print(f"   {c:28s} per dispatch {acc[k][c] / max(n[k][c], 1):.4g}")
PY
cat $O/summary.txt
