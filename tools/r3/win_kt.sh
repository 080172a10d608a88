#!/bin/bash
# Kernel-trace stats + FETCH_SIZE of config 5 under two env settings (per-kernel split of a window A/B).
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG=${1:-wkt}; O=$R/gpurun_out/r3/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for mode in "QEH_X=0" "${AB:-QEH_WM_INV2C=0}"; do
  i=$((i+1))
  env $mode timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$i -o kt -- \
      python3 $R/tools/bench_configs.py --only cfg5 > $O/kt$i.log 2>&1 || { tail -5 $O/kt$i.log; exit 1; }
  env $mode timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$i -o f -- \
      python3 $R/tools/bench_configs.py --only cfg5 > $O/f$i.log 2>&1 || { tail -5 $O/f$i.log; exit 1; }
  echo "== [$mode]"
  python3 - $O/kt$i/kt_kernel_stats.csv $O/f$i/f_counter_collection.csv <<'PY'
import csv, sys, collections
f = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[2])):
    f[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0]
    if "wm" in n:
        fb = sum(f[n]) / len(f[n]) * 2 / 1e9 if f[n] else -1
        print(f"{n[:44]:44s} avg {float(r['AverageNs'])/1e6:7.3f} ms  fetch x2 {fb:6.2f} GB")
PY
done
