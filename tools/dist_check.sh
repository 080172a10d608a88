#!/bin/bash
# GPU-box check of the distributed layer: RCCL world-1 + two-rank gloo tests, then the bench's
# config-4 mode (world-1 RCCL group) and a two-rank rehearsal of the metric's broadcast path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_distributed.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/dist_tests.log 2>&1 || { tail -40 gpurun_out/dist_tests.log; exit 1; }
tail -3 gpurun_out/dist_tests.log
timeout -k 10 300 python bench.py --workload cfg4 --rows 200000000 --steps 3 --warmup 1 > gpurun_out/bench_cfg4_small.log 2>&1 \
  || { tail -20 gpurun_out/bench_cfg4_small.log; exit 1; }
tail -1 gpurun_out/bench_cfg4_small.log | cut -c1-600
timeout -k 10 300 python bench.py --workload cfg4 --steps 5 --warmup 2 > gpurun_out/bench_cfg4.log 2>&1 \
  || { tail -20 gpurun_out/bench_cfg4.log; exit 1; }
tail -1 gpurun_out/bench_cfg4.log
QEH_BENCH_SHARE_GPU=1 QEH_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 \
    --rows 400000000 > gpurun_out/bench2_metric.log 2>&1 || { tail -20 gpurun_out/bench2_metric.log; exit 1; }
tail -1 gpurun_out/bench2_metric.log | cut -c1-700
echo dist-check-ok
