#!/bin/bash
# One rocprofv3 counter pass per argument group over a short metric bench run (run on the GPU box):
#   tools/pmc.sh <tag> "SQ_WAIT_ANY SQ_WAVE_CYCLES ..." ["GRBM_GUI_ACTIVE ..." ...]
# Each group is its own pass (<= 8 SQ, 4 TCC, 2 GRBM counters; never combined with tracing domains),
# under a hard time limit; per-kernel sums go to gpurun_out/pmc_<tag>/summary.txt.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
O=$R/gpurun_out/pmc_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p -- \
        python3 $R/bench.py --steps 3 --warmup 1 --cpu-sample 0 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - "$O" > $O/summary.txt <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
n = defaultdict(lambda: defaultdict(int))
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k][r["Counter_Name"]] += 1
for k in sorted(acc, key=lambda k: -max(acc[k].values())):
    if "slice" not in k and "probe" not in k:
        continue
    print(k)
    for c in sorted(acc[k]):
        print(f"   {c:28s} per dispatch {acc[k][c] / max(n[k][c], 1):.4g}")
PY
cat $O/summary.txt
