#!/bin/bash
# Round 3 regression check on one GPU: the whole -m gpu suite, smoke, the metric and config-4 bench
# lines, the two-rank (gloo, one GPU) rehearsals of both bench plans.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG="${1:-check}"
O=gpurun_out/r3/$TAG
mkdir -p $O
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
$T 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print('metric', round(d['ms_per_step'],3), round(d['value']/1e9,1), 'G rows/s frac', round(d['roofline']['frac'],4), d['roofline']['kernel_split_ms'])"
$T 300 python bench.py --workload cfg4 --steps 5 --warmup 2 --cpu-sample 0 > $O/bench_cfg4.log 2>&1 || { tail -20 $O/bench_cfg4.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_cfg4.log').read().strip().splitlines()[-1]);print('cfg4', round(d['ms_per_step'],3), round(d['value']/1e9,1))"
QEH_BENCH_SHARE_GPU=1 QEH_BENCH_BACKEND=gloo $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --rows 400000000 --cpu-sample 0 \
    > $O/bench2.log 2>&1 || { tail -20 $O/bench2.log; exit 1; }
tail -1 $O/bench2.log | cut -c1-200
QEH_BENCH_SHARE_GPU=1 QEH_BENCH_BACKEND=gloo $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --workload cfg4 --steps 3 --warmup 1 --rows 200000000 \
    > $O/bench2_cfg4.log 2>&1 || { tail -20 $O/bench2_cfg4.log; exit 1; }
tail -1 $O/bench2_cfg4.log | cut -c1-200
echo check-ok
