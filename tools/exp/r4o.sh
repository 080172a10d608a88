#!/bin/bash
# Round-4 GPU session o: distributed tests, then the N = 8 rank rehearsal (bench + kernel trace of a step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_distributed.py tests/test_pipeline.py -k "dist or table or rank" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for m in "" "QEH_SYNC_TABLE_CHECK=1"; do
  env $m QEH_BENCH_RANK_OF=0/8 timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --cpu-sample 0 > $O/rank08.out 2>$O/rank08.err || { tail $O/rank08.err; exit 1; }
  echo "[$m] $(tail -1 $O/rank08.out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["roofline"]["kernel_split_ms"])')"
done
QEH_BENCH_RANK_OF=0/8 timeout -k 10 300 bash tools/trace_bench.sh rank08o > $O/trace_rank08.txt 2>&1 || { echo "rank08 trace failed"; cat $O/trace_rank08.txt; exit 1; }
f=$(find gpurun_out/tb_rank08o -name "*kernel_trace.csv" | head -1)
python3 tools/trace_step.py "$f" > $O/step_rank08.txt 2>&1; cat $O/step_rank08.txt | head -50
