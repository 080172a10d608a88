#!/bin/bash
# Round-4 GPU sessions, one function each (the runs the profiles/r04 records and DESIGN.md quote).
# usage (on the GPU box, from the repo root): bash tools/exp/round4.sh <session>, e.g. r4k
set -o pipefail

r4a() {
# Round-4 first GPU session: phase-A traffic floor, early-issue A/B, the new parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 120 tools/ubench/floor_ubench 1000000000 5 > $O/floor.txt 2>&1 || { echo floor failed; cat $O/floor.txt; exit 1; }
cat $O/floor.txt
timeout -k 10 400 python3 tools/exp_slice.py --rounds 3 libqeh.so libqeh_exp1.so > $O/early.txt 2>&1 || { echo ab failed; cat $O/early.txt; exit 1; }
cat $O/early.txt
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_lds_rank.py \
    tests/test_merge.py "tests/test_pipeline.py::test_config2_full_size_vs_oracle" \
    "tests/test_pipeline.py::test_metric_full_size_vs_oracle" > $O/tests.txt 2>&1
rc=$?; tail -30 $O/tests.txt; exit $rc
}

r4b() {
# Round-4 GPU session b: write-layout floor (interleaved slots) + the payload-sort fix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 180 tools/ubench/floor_ubench 1000000000 5 > $O/floor.txt 2>&1 || { echo floor failed; cat $O/floor.txt; exit 1; }
cat $O/floor.txt
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_lds_rank.py \
    tests/test_merge.py "tests/test_pipeline.py::test_config2_full_size_vs_oracle" \
    "tests/test_pipeline.py::test_metric_full_size_vs_oracle" > $O/tests.txt 2>&1
rc=$?; tail -30 $O/tests.txt; exit $rc
}

r4c() {
# Round-4 GPU session c: phase A with / without the build beside it, early-issue variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 500 python3 tools/exp_slice.py --rounds 2 libqeh.so libqeh.so:QEH_NO_OVERLAP=1 libqeh_exp1.so \
    libqeh_exp1.so:QEH_NO_OVERLAP=1 > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
}

r4d() {
# Round-4 GPU session d: the fused pipeline -- parity tests, then A/B against the prelaunch path, then the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pipeline.py \
    > $O/tests.txt 2>&1 || { echo tests failed; tail -40 $O/tests.txt; exit 1; }
tail -5 $O/tests.txt
timeout -k 10 400 python3 tools/exp_slice.py --rounds 2 libqeh.so libqeh.so:QEH_NO_FUSED=1 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --cpu-sample 0 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
}

r4e() {
# Round-4 GPU session e: kernel trace of the fused pipeline's step.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=$R/gpurun_out/r4e; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
    python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
f=$(find $O/kt -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_step.py $f > $O/trace.txt; cat $O/trace.txt | head -60
}

r4f() {
# Round-4 GPU session f: trace + SQ counters of the fused pipeline's step.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
$R/tools/exp/r4e.sh > /dev/null || exit 1
tail -32 $R/gpurun_out/r4e/trace.txt
$R/tools/pmc.sh r4f "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
    "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"
}

r4g() {
# Round-4 GPU session g: box calibration + phase B / shard A/B of the fused pipeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 180 tools/ubench/floor_ubench 1000000000 3 > $O/floor.txt 2>&1 || { echo floor failed; cat $O/floor.txt; exit 1; }
head -12 $O/floor.txt
timeout -k 10 500 python3 tools/exp_slice.py --rounds 2 libqeh.so libqeh.so:QEH_NO_SHARDS=1 libqeh.so:QEH_FUSED_PV=1 \
    libqeh.so:QEH_NO_FUSED=1 > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python3 tools/probes/host_overhead.py > $O/host.txt 2>&1 && QEH_NO_FUSED=1 timeout -k 10 120 python3 tools/probes/host_overhead.py >> $O/host.txt 2>&1
cat $O/host.txt
}

r4h() {
# Round-4 GPU session h: parity of the chunk / carry variants, then A/B on one box (+ calibration).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4h; mkdir -p $O
for v in c32 c64; do
  QEH_LIB_PATH=$PWD/query-engine_amd/libqeh_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
      tests/test_pipeline.py -k "fused or slice_partitioned or metric_shape" > $O/tests_$v.txt 2>&1 || { echo "tests $v failed"; tail -30 $O/tests_$v.txt; exit 1; }
  tail -2 $O/tests_$v.txt
done
timeout -k 10 180 tools/ubench/floor_ubench 1000000000 3 > $O/floor.txt 2>&1 || { echo floor failed; cat $O/floor.txt; exit 1; }
head -12 $O/floor.txt
timeout -k 10 600 python3 tools/exp_slice.py --rounds 3 libqeh_base.so libqeh_c32.so libqeh_c64.so libqeh_c64.so:QEH_NO_SHARDS=1 \
    libqeh_c64.so:QEH_FUSED_PV=1 > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python3 tools/probes/host_overhead.py > $O/host.txt 2>&1 && QEH_NO_FUSED=1 timeout -k 10 120 python3 tools/probes/host_overhead.py >> $O/host.txt 2>&1
cat $O/host.txt
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_distributed.py tests/test_partition.py > $O/dist.txt 2>&1 || { echo dist tests failed; tail -30 $O/dist.txt; exit 1; }
tail -2 $O/dist.txt
for m in "" "QEH_SYNC_TABLE_CHECK=1"; do
  env $m QEH_BENCH_RANK_OF=0/8 timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --cpu-sample 0 > $O/rank08.json 2>$O/rank08.err || { tail $O/rank08.err; exit 1; }
  echo "[$m] $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(round(d["ms_per_step"],3), d["roofline"]["kernel_split_ms"])' $O/rank08.json)"
done
}

r4i() {
# Round-4 GPU session i: the new fused defaults (64-item chunks, paired phase-B loads, one state copy),
# the bench line, and the N = 8 per-rank rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pipeline.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(round(d["ms_per_step"],3), round(d["roofline"]["frac"],3), d["roofline"]["kernel_split_ms"])' $O/bench.json
QEH_BENCH_RANK_OF=0/8 PYTHONFAULTHANDLER=1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --cpu-sample 0 > $O/rank08.json 2>$O/rank08.err
echo "rank08 rc=$?"; cat $O/rank08.json; tail -5 $O/rank08.err
timeout -k 10 300 python3 -u tools/bench_configs.py --only cfg5leg,cfg5 > $O/cfg5.jsonl 2>$O/cfg5.err || { tail $O/cfg5.err; exit 1; }
cat $O/cfg5.jsonl
}

r4j() {
# Round-4 GPU session j: phase A as two 512-thread workgroups per CU (QEH_FUSED_2WG=1) -- parity, then
# A/B against the one-workgroup default on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4j; mkdir -p $O
QEH_FUSED_2WG=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pipeline.py -k "fused or slice_partitioned or metric_shape" > $O/tests_2wg.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests_2wg.txt; exit 1; }
tail -2 $O/tests_2wg.txt
timeout -k 10 600 python3 tools/exp_slice.py --rounds 3 libqeh.so libqeh.so:QEH_FUSED_2WG=1 > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; [ $rc = 0 ] || exit $rc
}

r4k() {
# Round-4 GPU session k: phase A without staging (ring kernel, default) -- parity, then A/B against the
# staged kernel (QEH_FUSED_RING=0) and the ring kernel with 8192-row tiles (libqeh_r4.so) on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pipeline.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
QEH_LIB_PATH=$PWD/query-engine_amd/libqeh_r4.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pipeline.py -k "fused or metric_shape" > $O/tests_r4.txt 2>&1 || { echo "tests r4 failed"; tail -30 $O/tests_r4.txt; exit 1; }
tail -2 $O/tests_r4.txt
timeout -k 10 600 python3 tools/exp_slice.py --rounds 3 libqeh.so libqeh.so:QEH_FUSED_RING=0 libqeh_r4.so > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; [ $rc = 0 ] || exit $rc
}

r4l() {
# Round-4 GPU session l: the whole GPU suite, then evidence -- config 5's kernel trace, the metric's
# kernel trace + PMC traffic (tools/profile.sh) and SQ counters (tools/pmc.sh) for both phase-A kernels.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R"
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/cfg5_kt -o kt -- python3 $R/tools/bench_configs.py --only cfg5 > $R/$O/cfg5_kt.log 2>&1 || { echo "cfg5 trace failed"; tail $R/$O/cfg5_kt.log; exit 1; }
cd "$R"
timeout -k 10 900 bash tools/profile.sh r04 > $O/profile.txt 2>&1 || { echo "profile failed"; tail -20 $O/profile.txt; exit 1; }
tail -12 $O/profile.txt
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
timeout -k 10 300 bash tools/pmc.sh r04_staged "$SQ" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" > $O/pmc_staged.txt 2>&1 || { echo "pmc staged failed"; tail $O/pmc_staged.txt; exit 1; }
QEH_FUSED_RING=1 timeout -k 10 300 bash tools/pmc.sh r04_ring "$SQ" > $O/pmc_ring.txt 2>&1 || { echo "pmc ring failed"; tail $O/pmc_ring.txt; exit 1; }
cat $O/pmc_staged.txt $O/pmc_ring.txt | grep -v "^ *$" | head -60
QEH_BENCH_RANK_OF=0/8 timeout -k 10 300 bash tools/trace_bench.sh rank08 > $O/trace_rank08.txt 2>&1 || { echo "rank08 trace failed"; cat $O/trace_rank08.txt; exit 1; }
f=$(ls gpurun_out/tb_rank08/*/kt_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find gpurun_out/tb_rank08 -name "*kernel_trace.csv" | head -1)
python3 tools/trace_step.py "$f" > $O/step_rank08.txt 2>&1; cat $O/step_rank08.txt | head -60
timeout -k 10 300 bash tools/trace_bench.sh metric > $O/trace_metric.txt 2>&1 || { echo "metric trace failed"; cat $O/trace_metric.txt; exit 1; }
f=$(find gpurun_out/tb_metric -name "*kernel_trace.csv" | head -1)
python3 tools/trace_step.py "$f" > $O/step_metric.txt 2>&1; cat $O/step_metric.txt | head -40
}

r4m() {
# Round-4 GPU session m: the MSD payload sort (parity, then Merge::sorted A/B against the LSD passes) and
# the N = 8 rank rehearsal with the stats copy queued ahead of phase A.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_merge.py tests/test_executor.py \
    > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for m in "" "QEH_NO_MSD_SORT=1"; do
  env $m timeout -k 10 300 python3 -u tools/bench_configs.py --only merge > $O/merge.jsonl 2>$O/merge.err || { tail $O/merge.err; exit 1; }
  echo "[$m] $(cut -c1-400 $O/merge.jsonl)"
done
QEH_BENCH_RANK_OF=0/8 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --cpu-sample 0 > $O/rank08.json 2>$O/rank08.err || { tail $O/rank08.err; exit 1; }
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print("rank08", round(d["ms_per_step"],3), d["roofline"]["kernel_split_ms"])' $O/rank08.json
}

r4n() {
# Round-4 GPU session n: MSD payload sort parity + Merge::sorted kernel trace.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R"
O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_merge.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o kt -- python3 $R/tools/bench_configs.py --only merge > $R/$O/merge.jsonl 2>$R/$O/merge.err || { tail $R/$O/merge.err; exit 1; }
cut -c1-300 $R/$O/merge.jsonl
python3 - "$(find $R/$O/kt -name '*kernel_stats.csv' | head -1)" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:80]:80s} calls={r["Calls"]:>4s} avg_ms={float(r["AverageNs"])/1e6:8.3f}')
PY
}

r4o() {
# Round-4 GPU session o: distributed tests, then the N = 8 rank rehearsal (bench + kernel trace of a step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_distributed.py tests/test_pipeline.py -k "dist or table or rank" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for m in "" "QEH_SYNC_TABLE_CHECK=1"; do
  env $m QEH_BENCH_RANK_OF=0/8 timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --cpu-sample 0 > $O/rank08.out 2>$O/rank08.err || { tail $O/rank08.err; exit 1; }
  echo "[$m] $(tail -1 $O/rank08.out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["roofline"]["kernel_split_ms"])')"
done
QEH_BENCH_RANK_OF=0/8 timeout -k 10 300 bash tools/trace_bench.sh rank08o > $O/trace_rank08.txt 2>&1 || { echo "rank08 trace failed"; cat $O/trace_rank08.txt; exit 1; }
f=$(find gpurun_out/tb_rank08o -name "*kernel_trace.csv" | head -1)
python3 tools/trace_step.py "$f" > $O/step_rank08.txt 2>&1; cat $O/step_rank08.txt | head -50
}

r4p() {
# Round-4 GPU session p: the secondary configs on the current tree + the bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4p; mkdir -p $O
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(round(d["ms_per_step"],3), round(d["roofline"]["frac"],3), d["roofline"]["kernel_split_ms"])' $O/bench.json
timeout -k 10 900 python3 -u tools/bench_configs.py --only cfg2,cfg3,filter,limit,left,full,shapes,partition,merge,window,cfg4leg,cfg5leg,cfg5 > $O/configs.jsonl 2>$O/configs.err || { tail $O/configs.err; exit 1; }
python3 - $O/configs.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    f=d.get("frac_of_8TBs")
    print(f'{d["config"][:70]:70s} {d["ms_per_run"]:8.2f} ms  kernel {d.get("kernel_ms") or 0:8.2f}  frac {f if f is None else round(f,3)}')
PY
}

r4q() {
# Round-4 GPU session q: window pass-1 histogram folded into the key min/max read -- parity, then
# config 5 A/B against the separate histogram (QEH_WM_NO_FOLD=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4q; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_window_msd.py tests/test_join_sort_window.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for m in "" "QEH_WM_NO_FOLD=1" "" "QEH_WM_NO_FOLD=1"; do
  env $m timeout -k 10 300 python3 -u tools/bench_configs.py --only cfg5 > $O/cfg5.jsonl 2>$O/cfg5.err || { tail $O/cfg5.err; exit 1; }
  echo "[$m] $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(round(d["ms_per_run"],2), round(d["kernel_ms"],2), round(d["window_partition"],2), round(d["window_sort"],2), round(d["window_place"],2))' $O/cfg5.jsonl)"
done
}

r4r() {
# Round-4 GPU session r: the LSD window path's shapes (bench_configs window_lsd) and SQ counters of the
# partitioning path's kernels (config 5 at 2.5e8 rows, one counter pass each group).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R"
O=gpurun_out/r4r; mkdir -p $O
timeout -k 10 600 python3 -u tools/bench_configs.py --only window_lsd > $O/window_lsd.jsonl 2>$O/window_lsd.err || { tail $O/window_lsd.err; exit 1; }
cut -c1-260 $O/window_lsd.jsonl
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $R/$O/p$i -o p -- python3 $R/tools/bench_configs.py --only cfg5 --scale 0.25 > $R/$O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/$O/p$i.log; exit 1; }
done
python3 - "$R/$O" > $R/$O/sq_window.txt <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(lambda: defaultdict(int))
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
for k in sorted(acc):
    if "wm" not in k: continue
    c = {q: acc[k][q] / max(n[k][q], 1) for q in acc[k]}
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k[:60]:60s} wait_any {c.get('SQ_WAIT_ANY',0)/wc:6.1%} wait_inst {c.get('SQ_WAIT_INST_ANY',0)/wc:6.1%} active {c.get('SQ_ACTIVE_INST_ANY',0)/wc:6.1%} lds_conflict/idx {c.get('SQ_LDS_BANK_CONFLICT',0)/max(c.get('SQ_LDS_IDX_ACTIVE',1),1):6.1%}")
    for q in sorted(c): print(f"    {q:26s} {c[q]:.4g}")
PY
head -80 $R/$O/sq_window.txt
}

r4s() {
# Round-4 GPU session s: window groups of 2^sb keys (key ranges up to 2^24) -- parity, then the wide-key shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_window_msd.py tests/test_lds_rank.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 600 python3 -u tools/bench_configs.py --only window_lsd,cfg5 > $O/window.jsonl 2>$O/window.err || { tail $O/window.err; exit 1; }
python3 - $O/window.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d['config'], round(d['ms_per_run'],2), round(d['kernel_ms'],2), round(d['frac_of_8TBs'],4), d.get('kernel_split_ms'))
PY
}

r4t() {
# Round-4 GPU session t: the whole GPU suite + smoke on the current tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4t; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
}

r4u() {
# the status lane written by the lanes kernel (no torch ops between the probe and the lanes all-reduce)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4u; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_distributed.py tests/test_pipeline.py -k "dist or table or rank" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for m in "" "QEH_SYNC_TABLE_CHECK=1" "" "QEH_SYNC_TABLE_CHECK=1"; do
  env $m QEH_BENCH_RANK_OF=0/8 timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 --cpu-sample 0 > $O/rank08.out 2>$O/rank08.err || { tail $O/rank08.err; exit 1; }
  echo "[$m] $(tail -1 $O/rank08.out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["roofline"]["kernel_split_ms"])')"
done
}

r4v() {
# the window path's pipelined inverse pass 1: parity, then config 5 / LAG A/B against the serial kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_window_msd.py tests/test_lds_rank.py tests/test_join_sort_window.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for m in "" "QEH_WM_INV1_SERIAL=1" "" "QEH_WM_INV1_SERIAL=1"; do
  env $m timeout -k 10 300 python3 -u tools/bench_configs.py --only cfg5,window > $O/cfg5.jsonl 2>$O/cfg5.err || { tail $O/cfg5.err; exit 1; }
  echo "[$m] $(python3 -c 'import json,sys; print([(json.loads(l)["config"][:22], round(json.loads(l)["kernel_ms"],2), round(json.loads(l).get("window_place",0),2)) for l in open(sys.argv[1])])' $O/cfg5.jsonl)"
done
}

r4w() {
# the final tree: bench line (default run, as the driver runs it), twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4w; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python3 bench.py > $O/bench_$i.json 2>$O/bench_$i.err || { tail $O/bench_$i.err; exit 1; }
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(round(d["ms_per_step"],3), round(d["value"]/1e9,1), round(d["roofline"]["frac"],3), d["roofline"]["kernel_split_ms"], d["cpu_baseline"]["value"])' $O/bench_$i.json
done
}

r4x() {
# the fused pipeline with two aggregate columns: parity, then the agg2 shape A/B against the prelaunch path
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4x; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pipeline.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for m in "" "QEH_NO_FUSED_AGG2=1" "" "QEH_NO_FUSED_AGG2=1"; do
  env $m timeout -k 10 300 python3 -u -c "import sys; sys.argv=['x','--only','shapes']; sys.path.insert(0,'tools'); import bench_configs as b; b.cfg_metric_shapes.__defaults__ = (('agg2',),); b.main()" > $O/agg2.jsonl 2>$O/agg2.err || { tail $O/agg2.err; exit 1; }
  echo "[$m] $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(round(d["ms_per_run"],2), round(d["kernel_ms"],2), round(d["frac_of_8TBs"],3), d["dominant_kernel"])' $O/agg2.jsonl)"
done
}

r4y() {
# key-window slices (k_slice_keyagg) for the 2^17-group shape: parity, then A/B against the group-range slices
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4y; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pipeline.py -k "group_range or widened" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for m in "" "QEH_NO_KEY_SLICES=1" ""; do
  env $m timeout -k 10 300 python3 -u -c "import sys; sys.argv=['x','--only','shapes']; sys.path.insert(0,'tools'); import bench_configs as b; b.cfg_metric_shapes.__defaults__ = (('g17',),); b.main()" > $O/g17.jsonl 2>$O/g17.err || { tail $O/g17.err; exit 1; }
  echo "[$m] $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(round(d["ms_per_run"],2), round(d["kernel_ms"],2), round(d["frac_of_8TBs"],3), d["dominant_kernel"], {k: round(v, 3) for k, v in d["kernel_split_ms"].items()})' $O/g17.jsonl)"
done
}

r4z() {
# k_slice_keyagg variants (LS: workgroup walks regions in turn, PF: prefetch) on the 2^17-group shape, then L2 hits
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4z; mkdir -p $O
G17="import sys; sys.argv=['x','--only','shapes']; sys.path.insert(0,'tools'); import bench_configs as b; b.cfg_metric_shapes.__defaults__ = (('g17',),); b.main()"
for v in ${R4Z_VARS:-0 1 2 3 0}; do
  QEH_KEYAGG_C16=$v timeout -k 10 300 python3 -u -c "$G17" > $O/g17.jsonl 2>$O/g17.err || { tail $O/g17.err; exit 1; }
  echo "[var $v] $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(round(d["ms_per_run"],2), round(d["kernel_ms"],2), round(d["frac_of_8TBs"],3), {k: round(v, 3) for k, v in d["kernel_split_ms"].items() if v})' $O/g17.jsonl)"
done
[ -n "$R4Z_NOPMC" ] && return 0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $O/pmc -o pmc --output-format csv -- python3 -u -c "$G17" > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for path in f:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"][:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "TCC_HIT_sum": n[k] += 1
for k, d in acc.items():
    if "slice" in k:
        print(k, n[k], {c: round(v / n[k] / 1e6, 2) for c, v in d.items()}, "hit", round(d["TCC_HIT_sum"] / max(1, d["TCC_HIT_sum"] + d["TCC_MISS_sum"]), 3))
PY
}

r4f2() {
# full GPU suite on the final tree, the three widened metric shapes, and the 2^17-group shape's kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4f2; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python3 -u tools/bench_configs.py --only shapes > $O/shapes.jsonl 2>$O/shapes.err || { tail $O/shapes.err; exit 1; }
python3 -c 'import json,sys; [print(d["config"], round(d["ms_per_run"],2), round(d["kernel_ms"],2), round(d["frac_of_8TBs"],3), d["dominant_kernel"]) for d in map(json.loads, open(sys.argv[1]))]' $O/shapes.jsonl
G17="import sys; sys.argv=['x','--only','shapes']; sys.path.insert(0,'tools'); import bench_configs as b; b.cfg_metric_shapes.__defaults__ = (('g17',),); b.main()"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/g17prof -o g17 --output-format csv -- python3 -u -c "$G17" > $O/g17prof.log 2>&1 || { tail $O/g17prof.log; exit 1; }
find $O/g17prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/g17_kernel_stats.csv
head -6 $O/g17_kernel_stats.csv | cut -c1-200
}

r4end() {
# last tree: GPU suite, smoke, the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4end; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 400 python3 bench.py > $O/bench.out 2>$O/bench.err || { tail $O/bench.err; exit 1; }
tail -1 $O/bench.out | cut -c1-400
}

[ -n "$1" ] || { echo "usage: $0 <session: r4a r4b r4c r4d r4e r4f r4g r4h r4i r4j r4k r4l r4m r4n r4o r4p r4q r4r r4s r4t r4u r4v r4w r4x r4y r4z r4f2 r4end>"; exit 2; }
"$1"
