#!/bin/bash
# End-of-round GPU evidence: parity suite, smoke, bench, rocprof profile, the secondary
# configurations, and a two-rank rehearsal of the N>1 bench path on one GPU (gloo).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG="${1:-final}"
bash tools/gpu_check.sh || exit 1
bash tools/profile.sh "$TAG" > /dev/null || exit 1
timeout -k 10 600 python tools/bench_configs.py --only cfg2,cfg3,cfg5,window,filter,left,merge,partition \
    > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err || { tail -5 gpurun_out/configs_$TAG.err; exit 1; }
QEH_BENCH_SHARE_GPU=1 QEH_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 \
    --rows 200000000 > gpurun_out/bench2_$TAG.log 2>&1 || { tail -20 gpurun_out/bench2_$TAG.log; exit 1; }
tail -1 gpurun_out/bench2_$TAG.log | cut -c1-200
echo final-check-ok
