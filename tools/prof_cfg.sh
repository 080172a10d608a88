#!/bin/bash
# Kernel-trace stats of tools/bench_configs.py lines.  usage: tools/prof_cfg.sh <tag> <--only list>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="$1"; ONLY="$2"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profcfg_$TAG -o kt -- \
    python3 $R/tools/bench_configs.py --only "$ONLY" > $R/gpurun_out/profcfg_$TAG.log 2>&1 || { tail -5 $R/gpurun_out/profcfg_$TAG.log; exit 1; }
grep -o '"config": "[^"]*"\|"kernel_ms": [0-9.]*' $R/gpurun_out/profcfg_$TAG.log
