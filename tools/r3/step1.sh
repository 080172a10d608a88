#!/bin/bash
# Round 3, first GPU call: gloo-with-CUDA-tensor probe, the changed / new GPU tests, config 4's
# per-rank device leg, one metric bench line.  Each GPU step is time-limited; stop at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
timeout -k 10 120 ./tools/ubench/lds_order_ubench > gpurun_out/r3/lds_order.log 2>&1 || { tail -20 gpurun_out/r3/lds_order.log; exit 1; }
cat gpurun_out/r3/lds_order.log
timeout -k 10 180 python tools/debug/gloo_cuda_probe.py > gpurun_out/r3/gloo_probe.log 2>&1 || { tail -20 gpurun_out/r3/gloo_probe.log; exit 1; }
cat gpurun_out/r3/gloo_probe.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_partition.py \
  "tests/test_pipeline.py::test_prelaunch_adopted_only_when_the_hint_matches" tests/test_distributed.py \
  > gpurun_out/r3/pytest1.log 2>&1 || { tail -40 gpurun_out/r3/pytest1.log; exit 1; }
tail -3 gpurun_out/r3/pytest1.log
timeout -k 10 400 python tools/bench_configs.py --only cfg4leg > gpurun_out/r3/cfg4leg.jsonl 2> gpurun_out/r3/cfg4leg.err \
  || { tail -20 gpurun_out/r3/cfg4leg.err; exit 1; }
cat gpurun_out/r3/cfg4leg.jsonl
timeout -k 10 300 python bench.py > gpurun_out/r3/bench.log 2>&1 || { tail -20 gpurun_out/r3/bench.log; exit 1; }
tail -1 gpurun_out/r3/bench.log
if grep -q "RESULT: stable" gpurun_out/r3/lds_order.log; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_window_msd.py \
    > gpurun_out/r3/pytest_wm.log 2>&1 || { tail -40 gpurun_out/r3/pytest_wm.log; exit 1; }
  tail -2 gpurun_out/r3/pytest_wm.log
  timeout -k 10 300 python tools/bench_configs.py --only cfg5 > gpurun_out/r3/cfg5_atomic.jsonl 2> gpurun_out/r3/cfg5.err || { tail -20 gpurun_out/r3/cfg5.err; exit 1; }
  cat gpurun_out/r3/cfg5_atomic.jsonl
  QEH_WM_BALLOT=1 timeout -k 10 300 python tools/bench_configs.py --only cfg5 > gpurun_out/r3/cfg5_ballot.jsonl 2> gpurun_out/r3/cfg5.err || { tail -20 gpurun_out/r3/cfg5.err; exit 1; }
  cat gpurun_out/r3/cfg5_ballot.jsonl
fi
QEH_INSERT_XCD=1 timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/r3/bench_xcd1.log 2>&1 || { tail -20 gpurun_out/r3/bench_xcd1.log; exit 1; }
tail -1 gpurun_out/r3/bench_xcd1.log | cut -c1-400
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/r3/bench_xcd2.log 2>&1 || { tail -20 gpurun_out/r3/bench_xcd2.log; exit 1; }
tail -1 gpurun_out/r3/bench_xcd2.log | cut -c1-400
