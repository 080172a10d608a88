#!/bin/bash
# Distributed-path check on one GPU: pipeline / distributed / ABI tests, then the N = 8 per-rank metric
# shape (1.25e8 fact rows) through the local operator and the table-form plan at world size 1, and a
# kernel trace of the table form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; TAG=${1:-n8}; O=gpurun_out/r3/$TAG; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_distributed.py tests/test_abi.py \
  tests/test_pipeline.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for mode in "QEH_X=0" "QEH_BENCH_FORCE_DIST=1" "QEH_BENCH_FORCE_DIST=1 QEH_NO_TABLE_LANES=1"; do
  env $mode $T 300 python bench.py --rows 125000000 --steps 20 --warmup 3 --cpu-sample 0 > $O/b125.log 2>&1 || { tail -20 $O/b125.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/b125.log').read().strip().splitlines()[-1]);print('125M [$mode]', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), d['roofline']['kernel_split_ms'])" | tee -a $O/n8.txt
done
cd /tmp && export TMPDIR=/tmp
QEH_BENCH_FORCE_DIST=1 $T 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace -o kt -- \
    python3 $R/bench.py --rows 125000000 --steps 5 --warmup 2 --cpu-sample 0 > $R/$O/trace.log 2>&1 || { tail -5 $R/$O/trace.log; exit 1; }
cd $R && python3 tools/trace_step.py $O/trace/kt_kernel_trace.csv k_slice_probe > $O/trace_step.txt && tail -40 $O/trace_step.txt
