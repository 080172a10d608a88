#!/bin/bash
# Window passes: non-temporal run stores (QEH_WM_NTS bits) vs cached, kernel trace at 2.5e8 rows.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p $R/gpurun_out/r3/wmnts
cd /tmp && export TMPDIR=/tmp
for e in 0 1 2 3; do
  QEH_WM_NTS=$e timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3/wmnts/n$e -o kt -- \
      python3 $R/tools/r3/wm_exp.py 2.5e8 > $R/gpurun_out/r3/wmnts/n$e.log 2>&1 || { tail -5 $R/gpurun_out/r3/wmnts/n$e.log; exit 1; }
  python3 - "$R/gpurun_out/r3/wmnts/n$e" "$e" <<'PY'
import csv, glob, sys
p = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(p)):
    if "pass" in r["Name"] or "inv" in r["Name"]:
        print(f"nts={sys.argv[2]:3s} {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']}  {r['Name'][:60]}")
PY
done
