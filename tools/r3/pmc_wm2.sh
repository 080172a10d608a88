#!/bin/bash
# SQ counters of the window passes (ROW_NUMBER, 2.5e8 rows, k in [0, 2^20)): two passes of <= 8 SQ
# counters each, then per-kernel averages.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT=$R/gpurun_out/r3/pmcwm; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS \
    --output-format csv -d $OUT/a -o sq -- python3 $R/tools/exp_wm_digits.py 2.5e8 20 1 > $OUT/a.log 2>&1 || { tail -5 $OUT/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE \
    --output-format csv -d $OUT/b -o sq -- python3 $R/tools/exp_wm_digits.py 2.5e8 20 1 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "wm" in k:
        print(k[:48], {c: round(sum(v) / len(v) / 1e6, 2) for c, v in sorted(d.items())})
PY
