#!/bin/bash
# Kernel-trace stats of a short metric bench run.  usage: tools/trace_bench.sh <tag> [bench args]
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="$1"; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tb_$TAG -o kt -- \
    python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 "$@" > $R/gpurun_out/tb_$TAG.log 2>&1 || { tail -5 $R/gpurun_out/tb_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/tb_$TAG.log | cut -c1-300
