set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/pmc_part
mkdir -p $R
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/w -o w -- $GRAFT_REPO_ROOT/tools/ubench/part_ubench 1000000000 10000000 1 > $R/w.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/f -o f -- $GRAFT_REPO_ROOT/tools/ubench/part_ubench 1000000000 10000000 1 > $R/f.log 2>&1 || exit 1
python3 - $R <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
        acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:60s} {c:12s} n={len(v):3d} mean={sum(v)/len(v)*1024/1e9:8.3f} GB (raw KiB units)")
PY
