#!/bin/bash
# pass-1 translation counters: digit-major (EXP=16) vs workgroup-major (EXP=80) run layout
# (QEH_WM_EXP bit 64, the workgroup-major layout, was an experiment-only kernel path, since removed)
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_wm
for ex in 80 16; do
  QEH_AB_CHILD=1 QEH_WM_EXP=$ex timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_PENDING_STALL_CYCLES_sum -d gpurun_out/pmc_wm/tlb2_$ex -o run --output-format csv -- python3 tools/exp/wm_parts.py tlb2_$ex 1000000000 1048576 > gpurun_out/pmc_wm/tlb2_$ex.log 2>&1
done
echo done
