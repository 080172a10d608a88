#!/bin/bash
# Round-3 final evidence, part 1: GPU suite, smoke, metric bench (with the CPU baseline), config-4
# bench, rocprof kernel-trace stats + PMC traffic (FETCH / WRITE passes) + SQ counters of the metric.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=${1:-fin}; O=gpurun_out/r3/$TAG; mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/profile.sh "r3_$TAG" > /dev/null || exit 1
cp gpurun_out/prof_r3_$TAG/summary.txt $O/summary.txt
cp gpurun_out/prof_r3_$TAG/traffic_latest.json $O/traffic.json
cp gpurun_out/prof_r3_$TAG/kt/kt_kernel_stats.csv $O/kernel_stats.csv
python3 tools/trace_step.py gpurun_out/prof_r3_$TAG/kt/kt_kernel_trace.csv k_slice_probe > $O/trace_metric_step.txt
cp gpurun_out/prof_r3_$TAG/traffic_latest.json profiles/traffic_latest.json
echo profile-ok
$T 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print('metric', round(d['ms_per_step'],3), round(d['value']/1e9,1), 'G rows/s frac', round(d['roofline']['frac'],4), d['roofline']['kernel_split_ms'], 'traffic', d['roofline'].get('traffic'))"
$T 300 python bench.py --workload cfg4 --steps 5 --warmup 2 --cpu-sample 0 > $O/bench_cfg4.log 2>&1 || { tail -20 $O/bench_cfg4.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_cfg4.log').read().strip().splitlines()[-1]);print('cfg4', round(d['ms_per_step'],3), round(d['value']/1e9,1))"
bash tools/r3/pmc_slice.sh $TAG/pmc > /dev/null || exit 1
cp gpurun_out/r3/$TAG/pmc/summary.txt $O/sq_counters_metric.txt
echo final-a-ok
