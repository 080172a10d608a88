#!/bin/bash
# One rank's share of the N = 8 metric run on one GPU (bench.py QEH_BENCH_RANK_OF=r/8: 1.25e8 fact rows,
# 1.25e6 dim rows through the table-form broadcast join at world size 1), beside the same fact rows with the
# whole dim (QEH_BENCH_FORCE_DIST=1), then a kernel trace of the rehearsal.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r3/${1:-rankof}; mkdir -p $O
T="timeout -k 10"
for r in 0 7; do
  QEH_BENCH_RANK_OF=$r/8 $T 300 python bench.py --rows 1000000000 --steps 20 --warmup 3 --cpu-sample 0 > $O/rank$r.log 2>&1 || { tail -20 $O/rank$r.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/rank$r.log').read().strip().splitlines()[-1]);print('rank $r of 8', round(d['ms_per_step'],3), 'ms/step; kernels', round(d['roofline']['kernel_ms'],3), d['roofline']['kernel_split_ms'], 'build', round(d['build_ms_per_step'],3), d['dist_build'], '|', d['result_check'])"
done
QEH_BENCH_FORCE_DIST=1 $T 300 python bench.py --rows 125000000 --steps 20 --warmup 3 --cpu-sample 0 > $O/full_dim.log 2>&1 || { tail -20 $O/full_dim.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/full_dim.log').read().strip().splitlines()[-1]);print('1.25e8 rows, whole dim', round(d['ms_per_step'],3), 'ms/step; kernels', round(d['roofline']['kernel_ms'],3), 'build', round(d['build_ms_per_step'],3))"
cd /tmp && export TMPDIR=/tmp
QEH_BENCH_RANK_OF=0/8 $T 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o kt -- \
    python3 $R/bench.py --rows 1000000000 --steps 5 --warmup 2 --cpu-sample 0 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
cd $R
python3 tools/trace_step.py $(ls $O/trace/*kernel_trace.csv | head -1) k_slice_probe > $O/trace_step.txt
head -30 $O/trace_step.txt
