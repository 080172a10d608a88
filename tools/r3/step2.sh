#!/bin/bash
# Round 3: tests touched by the atomic ranking (window passes, radix sort, partition scatter), the
# multi-rank device-tensor rehearsal, then A/B timings.  Each GPU step time-limited; stop at first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_partition.py tests/test_distributed.py \
  tests/test_window_msd.py tests/test_window.py tests/test_join_sort_window.py tests/test_merge.py \
  "tests/test_pipeline.py::test_prelaunch_adopted_only_when_the_hint_matches" > gpurun_out/r3/pytest2.log 2>&1 \
  || { tail -60 gpurun_out/r3/pytest2.log; exit 1; }
tail -2 gpurun_out/r3/pytest2.log
$T 300 python tools/bench_configs.py --only cfg5,window,merge > gpurun_out/r3/cfg_atomic.jsonl 2> gpurun_out/r3/cfg.err || { tail -20 gpurun_out/r3/cfg.err; exit 1; }
cut -c1-600 gpurun_out/r3/cfg_atomic.jsonl
QEH_WM_BALLOT=1 QEH_RS_BALLOT=1 $T 300 python tools/bench_configs.py --only cfg5,merge > gpurun_out/r3/cfg_ballot.jsonl 2> gpurun_out/r3/cfg.err || { tail -20 gpurun_out/r3/cfg.err; exit 1; }
cut -c1-600 gpurun_out/r3/cfg_ballot.jsonl
$T 400 python tools/bench_configs.py --only cfg4leg,partition > gpurun_out/r3/cfg4leg.jsonl 2> gpurun_out/r3/cfg4leg.err || { tail -20 gpurun_out/r3/cfg4leg.err; exit 1; }
cut -c1-900 gpurun_out/r3/cfg4leg.jsonl
for mode in 1 2 1 2; do
  QEH_INSERT_XCD=$mode $T 300 python bench.py --cpu-sample 0 > gpurun_out/r3/bench_xcd$mode.log 2>&1 || { tail -20 gpurun_out/r3/bench_xcd$mode.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r3/bench_xcd$mode.log').read().strip().splitlines()[-1]);print('xcd$mode', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel_split_ms'], d['build_ms_per_step'])"
done
