#!/bin/bash
# Round 3: fused filter/ids/histogram exchange pass (tests + cfg4 leg + partition), HBM traffic of the
# window passes (FETCH_SIZE / WRITE_SIZE at 2.5e8 rows), the N = 8 per-rank metric shape on one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_partition.py tests/test_distributed.py \
  > gpurun_out/r3/pytest4.log 2>&1 || { tail -60 gpurun_out/r3/pytest4.log; exit 1; }
tail -2 gpurun_out/r3/pytest4.log
$T 300 python tools/bench_configs.py --only cfg4leg,partition > gpurun_out/r3/cfg4leg_fused.jsonl 2> gpurun_out/r3/cfg4leg.err || { tail -20 gpurun_out/r3/cfg4leg.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r3/cfg4leg_fused.jsonl'):
    d=json.loads(l); print(d['config'][:50], round(d['kernel_ms'],3), round(d['frac_of_8TBs'],3), json.dumps(d.get('legs', d.get('kernel_split_ms'))))"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/r3/pmcwm_$c -o p -- python3 $R/tools/exp_wm_digits.py 2.5e8 20 1 \
    > $R/gpurun_out/r3/pmcwm_$c.log 2>&1 || { tail -5 $R/gpurun_out/r3/pmcwm_$c.log; exit 1; }
done
cd $R
python3 - <<'PY'
import csv, glob, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/r3/pmcwm_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        if "wm" in k:
            print(c, k[:50], round(sum(v) / len(v) / 1024 / 1024, 3), "GiB per dispatch (raw KiB counter)")
PY
for mode in "" "QEH_BENCH_FORCE_DIST=1"; do
  env $mode $T 300 python bench.py --rows 125000000 --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/r3/bench_125m.log 2>&1 || { tail -20 gpurun_out/r3/bench_125m.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r3/bench_125m.log').read().strip().splitlines()[-1]);print('125M [$mode]', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel_split_ms'], d['build_ms_per_step'])"
done
