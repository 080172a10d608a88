#!/bin/bash
# Kernel trace of the metric bench (5 steps) + one step's timeline, and the SQ counters of the pipeline.
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG=${1:-ps}; OUT=$R/gpurun_out/r3/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 \
    > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 1; }
python3 $R/tools/trace_step.py $OUT/kt/kt_kernel_trace.csv k_slice_probe > $OUT/step.txt
tail -28 $OUT/step.txt
bash $R/tools/r3/pmc_slice.sh $TAG/pmc > /dev/null || exit 1
grep -E "slice_partition|slice_probe" $OUT/pmc/summary.txt
