#!/bin/bash
# SQ counters of the radix-sort kernels on the Merge::sorted config (tools/bench_configs.py --only merge):
# two passes of <= 8 SQ counters, then per-dispatch averages per kernel (millions).
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT=$R/gpurun_out/r3/${1:-pmcsort}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B=(python3 $R/tools/bench_configs.py --only ${CFG:-merge})
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS \
    --output-format csv -d $OUT/a -o sq -- "${B[@]}" > $OUT/a.log 2>&1 || { tail -5 $OUT/a.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE \
    --output-format csv -d $OUT/b -o sq -- "${B[@]}" > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
python3 - "$OUT" <<'PY' | tee $OUT/summary.txt
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if any(s in k for s in ("k_rs", "encode", "decode", "k_wm")):
        print(k[:60], {c: round(sum(v) / len(v) / 1e6, 3) for c, v in sorted(d.items())})
PY
