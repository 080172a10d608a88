#!/bin/bash
# Round 3: sparse DIRECT rule (joins / pipeline tests), config 4's per-rank leg with and without it,
# kernel-trace splits of the config-4 leg and config 5, one metric bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pipeline.py tests/test_executor.py \
  tests/test_aggregate.py tests/test_join_predicates.py tests/test_join_sort_window.py tests/test_partition.py tests/test_window_msd.py \
  tests/test_window.py > gpurun_out/r3/pytest3.log 2>&1 \
  || { tail -60 gpurun_out/r3/pytest3.log; exit 1; }
tail -2 gpurun_out/r3/pytest3.log
$T 300 python tools/bench_configs.py --only cfg4leg > gpurun_out/r3/cfg4leg_sparse.jsonl 2> gpurun_out/r3/cfg4leg.err || { tail -20 gpurun_out/r3/cfg4leg.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r3/cfg4leg_sparse.jsonl').readline());print(d['kernel_ms'], json.dumps(d['legs']))"
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3/prof_cfg4leg -o kt -- \
    python3 $R/tools/bench_configs.py --only cfg4leg --scale 0.25 > $R/gpurun_out/r3/prof_cfg4leg.log 2>&1 || { tail -5 $R/gpurun_out/r3/prof_cfg4leg.log; exit 1; }
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3/prof_cfg5 -o kt -- \
    python3 $R/tools/bench_configs.py --only cfg5,window --scale 0.25 > $R/gpurun_out/r3/prof_cfg5.log 2>&1 || { tail -5 $R/gpurun_out/r3/prof_cfg5.log; exit 1; }
cd $R
for f in gpurun_out/r3/prof_cfg4leg gpurun_out/r3/prof_cfg5; do
  python3 - "$f" <<'PY'
import csv, glob, sys
p = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(p)))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:10.1f} us  {r['Name'][:110]}")
PY
done
$T 300 python bench.py --cpu-sample 0 > gpurun_out/r3/bench3.log 2>&1 || { tail -20 gpurun_out/r3/bench3.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r3/bench3.log').read().strip().splitlines()[-1]);print('metric', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['kernel_split_ms'], d['build_ms_per_step'])"
bash tools/r3/pmc_wm2.sh || exit 1
