#!/bin/bash
# End-of-round GPU evidence: parity suite, smoke, bench (metric + config 4), rocprof profile with
# PMC traffic, the secondary configurations, and two-rank rehearsals of the N>1 bench paths on one
# GPU (gloo).  Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG="${1:-final}"
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit 1
timeout -k 10 300 python bench.py --workload cfg4 --steps 5 --warmup 2 > gpurun_out/bench_cfg4_$TAG.log 2>&1 \
  || { tail -20 gpurun_out/bench_cfg4_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_cfg4_$TAG.log | cut -c1-300
bash tools/profile.sh "$TAG" > /dev/null || exit 1
timeout -k 10 900 python tools/bench_configs.py --only cfg2,cfg3,cfg5,window,filter,left,merge,partition,shapes \
    > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err || { tail -5 gpurun_out/configs_$TAG.err; exit 1; }
QEH_BENCH_SHARE_GPU=1 QEH_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 \
    --rows 400000000 --cpu-sample 0 > gpurun_out/bench2_$TAG.log 2>&1 || { tail -20 gpurun_out/bench2_$TAG.log; exit 1; }
tail -1 gpurun_out/bench2_$TAG.log | cut -c1-200
QEH_BENCH_SHARE_GPU=1 QEH_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --workload cfg4 --steps 3 \
    --warmup 1 --rows 200000000 > gpurun_out/bench2_cfg4_$TAG.log 2>&1 || { tail -20 gpurun_out/bench2_cfg4_$TAG.log; exit 1; }
tail -1 gpurun_out/bench2_cfg4_$TAG.log | cut -c1-200
echo final-check-ok
