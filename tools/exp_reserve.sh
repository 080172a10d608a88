#!/bin/bash
# bench the metric query with 0/8/16/32 CUs left to the build under the prelaunched phase A,
# then a kernel trace at the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/reserve
timeout -k 10 300 python -u -m pytest tests/test_pipeline.py tests/test_aggregate.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/reserve/pytest.log 2>&1 || { tail -30 gpurun_out/reserve/pytest.log; exit 1; }
tail -2 gpurun_out/reserve/pytest.log
for r in 0 4 8; do
  QEH_SLICE_RESERVE_CUS=$r timeout -k 10 200 python bench.py --cpu-sample 0 > gpurun_out/reserve/bench_$r.log 2>&1 || { tail -20 gpurun_out/reserve/bench_$r.log; exit 1; }
  echo "reserve=$r $(tail -1 gpurun_out/reserve/bench_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), round(d["roofline"]["kernel_ms"],3), d["roofline"]["kernel_split_ms"], round(d["roofline"]["frac"],4))')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/reserve/kt" -o kt -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --cpu-sample 0 > "$GRAFT_REPO_ROOT/gpurun_out/reserve/kt.log" 2>&1 || { echo kt failed; exit 1; }
echo done
