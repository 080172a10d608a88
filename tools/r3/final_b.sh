#!/bin/bash
# Round-3 final evidence, part 2: secondary configurations, the N = 8 per-rank metric shape (local /
# table form / all-gather form) with a kernel trace, two-rank gloo rehearsals of both bench plans.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; TAG=${1:-fin}; O=gpurun_out/r3/$TAG; mkdir -p $O
T="timeout -k 10"
$T 900 python tools/bench_configs.py --only cfg2,cfg3,cfg5,window,filter,left,merge,partition,shapes,cfg4leg \
    > $O/configs.jsonl 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
echo configs-ok
for mode in "QEH_X=0" "QEH_BENCH_FORCE_DIST=1" "QEH_BENCH_FORCE_DIST=1 QEH_NO_TABLE_BCAST=1"; do
  env $mode $T 300 python bench.py --rows 125000000 --steps 20 --warmup 3 --cpu-sample 0 > $O/b125.log 2>&1 || { tail -20 $O/b125.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/b125.log').read().strip().splitlines()[-1]);print('125M [$mode]', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), d['roofline']['kernel_split_ms'])" | tee -a $O/n8_per_rank.txt
done
cd /tmp && export TMPDIR=/tmp
QEH_BENCH_FORCE_DIST=1 $T 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace_125m_table -o kt -- \
    python3 $R/bench.py --rows 125000000 --steps 5 --warmup 2 --cpu-sample 0 > $R/$O/trace_125m_table.log 2>&1 || { tail -5 $R/$O/trace_125m_table.log; exit 1; }
cd $R
python3 tools/trace_step.py $O/trace_125m_table/kt_kernel_trace.csv k_slice_probe > $O/trace_125m_table.txt
QEH_BENCH_SHARE_GPU=1 QEH_BENCH_BACKEND=gloo $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --rows 400000000 --cpu-sample 0 \
    > $O/bench2.log 2>&1 || { tail -20 $O/bench2.log; exit 1; }
tail -1 $O/bench2.log | cut -c1-200
QEH_BENCH_SHARE_GPU=1 QEH_BENCH_BACKEND=gloo $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --workload cfg4 --steps 3 --warmup 1 --rows 200000000 \
    > $O/bench2_cfg4.log 2>&1 || { tail -20 $O/bench2_cfg4.log; exit 1; }
tail -1 $O/bench2_cfg4.log | cut -c1-200
echo final-b-ok
