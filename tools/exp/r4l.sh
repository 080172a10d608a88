#!/bin/bash
# Round-4 GPU session l: the whole GPU suite, then evidence -- config 5's kernel trace, the metric's
# kernel trace + PMC traffic (tools/profile.sh) and SQ counters (tools/pmc.sh) for both phase-A kernels.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R"
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/cfg5_kt -o kt -- python3 $R/tools/bench_configs.py --only cfg5 > $R/$O/cfg5_kt.log 2>&1 || { echo "cfg5 trace failed"; tail $R/$O/cfg5_kt.log; exit 1; }
cd "$R"
timeout -k 10 900 bash tools/profile.sh r04 > $O/profile.txt 2>&1 || { echo "profile failed"; tail -20 $O/profile.txt; exit 1; }
tail -12 $O/profile.txt
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
timeout -k 10 300 bash tools/pmc.sh r04_staged "$SQ" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" > $O/pmc_staged.txt 2>&1 || { echo "pmc staged failed"; tail $O/pmc_staged.txt; exit 1; }
QEH_FUSED_RING=1 timeout -k 10 300 bash tools/pmc.sh r04_ring "$SQ" > $O/pmc_ring.txt 2>&1 || { echo "pmc ring failed"; tail $O/pmc_ring.txt; exit 1; }
cat $O/pmc_staged.txt $O/pmc_ring.txt | grep -v "^ *$" | head -60
QEH_BENCH_RANK_OF=0/8 timeout -k 10 300 bash tools/trace_bench.sh rank08 > $O/trace_rank08.txt 2>&1 || { echo "rank08 trace failed"; cat $O/trace_rank08.txt; exit 1; }
f=$(ls gpurun_out/tb_rank08/*/kt_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find gpurun_out/tb_rank08 -name "*kernel_trace.csv" | head -1)
python3 tools/trace_step.py "$f" > $O/step_rank08.txt 2>&1; cat $O/step_rank08.txt | head -60
timeout -k 10 300 bash tools/trace_bench.sh metric > $O/trace_metric.txt 2>&1 || { echo "metric trace failed"; cat $O/trace_metric.txt; exit 1; }
f=$(find gpurun_out/tb_metric -name "*kernel_trace.csv" | head -1)
python3 tools/trace_step.py "$f" > $O/step_metric.txt 2>&1; cat $O/step_metric.txt | head -40
