#!/bin/bash
# Round-4 GPU session r: the LSD window path's shapes (bench_configs window_lsd) and SQ counters of the
# partitioning path's kernels (config 5 at 2.5e8 rows, one counter pass each group).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R"
O=gpurun_out/r4r; mkdir -p $O
timeout -k 10 600 python3 -u tools/bench_configs.py --only window_lsd > $O/window_lsd.jsonl 2>$O/window_lsd.err || { tail $O/window_lsd.err; exit 1; }
cut -c1-260 $O/window_lsd.jsonl
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $R/$O/p$i -o p -- python3 $R/tools/bench_configs.py --only cfg5 --scale 0.25 > $R/$O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/$O/p$i.log; exit 1; }
done
python3 - "$R/$O" > $R/$O/sq_window.txt <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(lambda: defaultdict(int))
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
for k in sorted(acc):
    if "wm" not in k: continue
    c = {q: acc[k][q] / max(n[k][q], 1) for q in acc[k]}
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k[:60]:60s} wait_any {c.get('SQ_WAIT_ANY',0)/wc:6.1%} wait_inst {c.get('SQ_WAIT_INST_ANY',0)/wc:6.1%} active {c.get('SQ_ACTIVE_INST_ANY',0)/wc:6.1%} lds_conflict/idx {c.get('SQ_LDS_BANK_CONFLICT',0)/max(c.get('SQ_LDS_IDX_ACTIVE',1),1):6.1%}")
    for q in sorted(c): print(f"    {q:26s} {c[q]:.4g}")
PY
head -80 $R/$O/sq_window.txt
