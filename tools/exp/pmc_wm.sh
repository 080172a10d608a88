#!/bin/bash
# pass-1 counters, scattered (EXP=16) vs coalesced (EXP=48) run writes
# (the coalesced variant, QEH_WM_EXP bit 32, and the workgroup-major layout, bit 64, were experiment-only
#  kernel paths, removed after this measurement: profiles/r05/cfg5_pass1_counters.txt holds the results)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { # tag exp counters...
  local tag=$1 ex=$2; shift 2
  QEH_AB_CHILD=1 QEH_WM_EXP=$ex timeout -s KILL 90 rocprofv3 --pmc "$@" -d gpurun_out/pmc_wm/$tag -o run --output-format csv -- python3 tools/exp/wm_parts.py $tag 1000000000 1048576 > gpurun_out/pmc_wm/$tag.log 2>&1
}
mkdir -p gpurun_out/pmc_wm
for ex in 16 48; do
  run tlb_$ex $ex TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum
  run tcc_$ex $ex TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_WRITE_sum TCC_EA0_WRREQ_STALL_sum
  run ta_$ex $ex TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
  run tcp_$ex $ex TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCR_TCP_STALL_CYCLES_sum
  run tcc2_$ex $ex TCC_TAG_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum
done
echo done
