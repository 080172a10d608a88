#!/bin/bash
# Kernel-trace split of config 3 (INNER join 1e9 x 1e7) for the in-tree library and an old build.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r3/${1:-cfg3ab}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for lib in "" "$R/query-engine_amd/${OLD:-libqeh_old.so}"; do
  i=$((i+1))
  QEH_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$i -o kt -- \
      python3 $R/tools/bench_configs.py --only ${CFG:-cfg3} > $O/kt$i.log 2>&1 || { tail -5 $O/kt$i.log; exit 1; }
  echo "== lib [${lib:-in-tree}]"; grep "${CFGK:-cfg3}" $O/kt$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel_ms'],2))"
  python3 - $O/kt$i/kt_kernel_stats.csv <<'PY'
import csv, sys, os
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0]
    if any(s in n for s in (os.environ.get("KPAT") or "slice").split(",")): print(f"{n[:60]:60s} avg {float(r['AverageNs'])/1e6:7.3f} ms x{r['Calls']}")
PY
done
