#!/bin/bash
# PMC counters for any command, one rocprofv3 pass per counter group (never
# combined with trace domains).  Prints per-kernel mean counter values.
# usage: tools/pmc_cmd.sh <tag> "<ctr> <ctr>" ["<ctr>" ...] -- <program> [args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
GROUPS_=()
while [ "$1" != "--" ]; do GROUPS_+=("$1"); shift; done
shift
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for g in "${GROUPS_[@]}"; do
  timeout -k 10 600 rocprofv3 --pmc $g --output-format csv -d "$OUT/p$i" -o p -- "$@" > "$OUT/p$i.log" 2>&1 \
    || { echo "pmc pass $i ($g) failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  i=$((i + 1))
done
python3 - "$OUT" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
        acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
kern = sorted({k for k, _ in acc})
for k in kern:
    vals = {c: sum(v) / len(v) for (kk, c), v in acc.items() if kk == k}
    print(k, " ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))
PY
