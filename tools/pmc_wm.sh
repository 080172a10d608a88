#!/bin/bash
# SQ counters of the window partition passes (cfg5 shape at 2.5e8 rows): instruction mix and waits.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT=$R/gpurun_out/pmcwm; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
    --output-format csv -d $OUT -o sq -- python3 $R/tools/exp_wm_digits.py 2.5e8 20 1 > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
echo ok
