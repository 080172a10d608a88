#!/bin/bash
# Table-form broadcast join: tests, the N = 8 per-rank metric shape (1.25e8 rows) through the
# distributed plan at world size 1 (table form vs all-gather form vs the local operator), trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_distributed.py tests/test_abi.py \
  "tests/test_pipeline.py::test_table_form_broadcast_join_vs_oracle" "tests/test_pipeline.py::test_prelaunch_adopted_only_when_the_hint_matches" \
  > gpurun_out/r3/pytest7.log 2>&1 || { tail -60 gpurun_out/r3/pytest7.log; exit 1; }
tail -2 gpurun_out/r3/pytest7.log
for mode in "QEH_X=0" "QEH_BENCH_FORCE_DIST=1" "QEH_BENCH_FORCE_DIST=1 QEH_NO_TABLE_BCAST=1"; do
  env $mode $T 300 python bench.py --rows 125000000 --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/r3/bench_125m.log 2>&1 || { tail -20 gpurun_out/r3/bench_125m.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r3/bench_125m.log').read().strip().splitlines()[-1]);print('125M [$mode]', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), d['roofline']['kernel_split_ms'], round(d['build_ms_per_step'],3))"
done
cd /tmp && export TMPDIR=/tmp
QEH_BENCH_FORCE_DIST=1 $T 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r3/trace_125m_table -o kt -- \
    python3 $R/bench.py --rows 125000000 --steps 5 --warmup 2 --cpu-sample 0 > $R/gpurun_out/r3/trace_125m_table.log 2>&1 || { tail -5 $R/gpurun_out/r3/trace_125m_table.log; exit 1; }
cd $R
python3 tools/trace_step.py $(ls gpurun_out/r3/trace_125m_table/*kernel_trace.csv | head -1) k_slice_probe > gpurun_out/r3/trace_125m_table.txt
cat gpurun_out/r3/trace_125m_table.txt | head -40
