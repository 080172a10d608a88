#!/bin/bash
# Round-4 GPU session e: kernel trace of the fused pipeline's step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=$R/gpurun_out/r4e; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
    python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
f=$(find $O/kt -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_step.py $f > $O/trace.txt; cat $O/trace.txt | head -60
