#!/bin/bash
# Round-3 evidence on one GPU (after tools/r3/check.sh): rocprof kernel-trace stats + PMC traffic of
# the metric bench, the secondary configurations (incl. config 4's per-rank leg), the N = 8 per-rank
# metric shape through the local / table-form / all-gather-form plans with a kernel trace, the
# co-scheduling trace, and the LDS-atomic ordering microbenchmark.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
TAG="${1:-ev}"
O=gpurun_out/r3/$TAG
mkdir -p $O
T="timeout -k 10"
bash tools/profile.sh "r3_$TAG" > /dev/null || exit 1
cp gpurun_out/prof_r3_$TAG/summary.txt $O/pmc_summary.txt
cp gpurun_out/prof_r3_$TAG/traffic_latest.json $O/traffic.json
cp gpurun_out/prof_r3_$TAG/kt/kt_kernel_stats.csv $O/kernel_stats.csv 2>/dev/null || cp $(ls gpurun_out/prof_r3_$TAG/kt/*kernel_stats.csv | head -1) $O/kernel_stats.csv
echo profile-ok
$T 900 python tools/bench_configs.py --only ${CONFIGS:-cfg2,cfg3,cfg5,window,filter,left,merge,partition,shapes,cfg4leg} \
    > $O/configs.jsonl 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
echo configs-ok
for mode in "QEH_X=0" "QEH_BENCH_FORCE_DIST=1" "QEH_BENCH_FORCE_DIST=1 QEH_NO_TABLE_BCAST=1"; do
  env $mode $T 300 python bench.py --rows 125000000 --steps 20 --warmup 3 --cpu-sample 0 > $O/b125.log 2>&1 || { tail -20 $O/b125.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/b125.log').read().strip().splitlines()[-1]);print('125M [$mode]', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), d['roofline']['kernel_split_ms'], round(d['build_ms_per_step'],3))" | tee -a $O/n8_per_rank.txt
done
cd /tmp && export TMPDIR=/tmp
QEH_BENCH_FORCE_DIST=1 $T 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace_125m_table -o kt -- \
    python3 $R/bench.py --rows 125000000 --steps 5 --warmup 2 --cpu-sample 0 > $R/$O/trace_125m_table.log 2>&1 || { tail -5 $R/$O/trace_125m_table.log; exit 1; }
$T 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace_cosched -o kt -- \
    python3 $R/tools/r3/cosched.py > $R/$O/trace_cosched.log 2>&1 || { tail -5 $R/$O/trace_cosched.log; exit 1; }
cd $R
python3 tools/trace_step.py $(ls $O/trace_125m_table/*kernel_trace.csv | head -1) k_slice_probe > $O/trace_125m_table.txt
python3 tools/trace_step.py $(ls $O/trace_cosched/*kernel_trace.csv | head -1) k_slice_probe > $O/trace_cosched.txt
$T 120 tools/ubench/lds_order_ubench > $O/lds_order.log 2>&1 || { tail -5 $O/lds_order.log; exit 1; }
tail -3 $O/lds_order.log
echo evidence-ok
