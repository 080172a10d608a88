#!/bin/bash
# Round-5 GPU sessions, one function each (the runs the profiles/r05 records and DESIGN.md quote).
# usage (on the GPU box, from the repo root): bash tools/exp/round5.sh <session>, e.g. r5a
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"

run_tests() {  # $1 = output file, rest = pytest targets
    local out=$1; shift
    timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu "$@" > "$out" 2>&1
    local rc=$?; tail -25 "$out"; return $rc
}

r5a() {
# phase A: flush after rank (no store round trip in front of the loop head's vmcnt wait) and the
# branch-free predicate, A/B against the round-4 library; then the new parity tests
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 500 python3 tools/exp_slice.py --rounds 3 libqeh_base.so libqeh_late0.so libqeh.so > $O/ab.txt 2>&1 \
    || { echo ab failed; cat $O/ab.txt; exit 1; }
cat $O/ab.txt
run_tests $O/tests.txt tests/test_employees_departments.py tests/test_config4.py \
    "tests/test_distributed.py::test_device_tensor_collectives_several_ranks_on_one_gpu" tests/test_pipeline.py
}

r5b() {
# phase-A cycle stamps (diagnostic builds): flush late (default) and the round-4 order
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 300 python3 tools/exp/pa_stamps.py libqeh_stamps.so libqeh_stamps0.so > $O/stamps.txt 2>&1 \
    || { echo stamps failed; cat $O/stamps.txt; exit 1; }
cat $O/stamps.txt
}

r5c() {
# items form of the distributed broadcast join: parity on one device (simulated ranks) and over gloo
# device tensors (world 2 / 3 / 8), then the rank-share rehearsal of an N = 8 step (1.10 ms in r04)
O=gpurun_out/r5c; mkdir -p $O
run_tests $O/tests.txt "tests/test_pipeline.py::test_items_form_vs_oracle" \
    "tests/test_distributed.py::test_device_tensor_collectives_several_ranks_on_one_gpu" \
    "tests/test_distributed.py::test_rccl_world_size_one" || exit 1
for r in 0 3; do
  QEH_BENCH_RANK_OF=$r/8 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 > $O/rank${r}of8.json 2> $O/rank${r}of8.err \
      || { tail -20 $O/rank${r}of8.err; exit 1; }
  tail -1 $O/rank${r}of8.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("dist_build"), d.get("dist_final"))'
done
QEH_NO_ITEMS_BCAST=1 QEH_BENCH_RANK_OF=0/8 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 > $O/rank0of8_table.json 2> $O/rank0of8_table.err \
    || { tail -20 $O/rank0of8_table.err; exit 1; }
tail -1 $O/rank0of8_table.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("table form", d["ms_per_step"], d.get("dist_build"))'
}

r5d() {
# kernel trace of the rank-share rehearsal step (items form) and of the N = 1 metric step
O=gpurun_out/r5d; mkdir -p $O
QEH_BENCH_RANK_OF=0/8 bash tools/trace_bench.sh r5d_rank0 || exit 1
f=$(ls gpurun_out/tb_r5d_rank0/*/kt_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find gpurun_out/tb_r5d_rank0 -name '*kernel_trace.csv' | head -1)
python3 tools/trace_step.py "$f" k_slice_probe > $O/rank0_step_trace.txt; cat $O/rank0_step_trace.txt
}

r5h() {
# config 5 (ROW_NUMBER over 1e9 rows): kernel trace and per-kernel HBM bytes (FETCH_SIZE, WRITE_SIZE, one
# pass each), the window path's first traffic record
O=$PWD/gpurun_out/r5h; mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
B=(python3 "$R/tools/bench_configs.py" --only cfg5)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- "${B[@]}" > "$O/kt.log" 2>&1 || { tail -20 "$O/kt.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o fetch -- "${B[@]}" > "$O/fetch.log" 2>&1 || { tail -20 "$O/fetch.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o write -- "${B[@]}" > "$O/write.log" 2>&1 || { tail -20 "$O/write.log"; exit 1; }
python3 "$R/tools/pmc_traffic.py" "$O" > "$O/summary.txt" 2>&1 || { cat "$O/summary.txt"; exit 1; }
cat "$O/summary.txt"
grep -h cfg5 "$O/kt.log" | tail -2
}

r5i() {
# one box, three views of phase A: the traffic floor (no LDS work), the metric step, and the stamped
# phase A (diagnostic build) -- run on several boxes to see which phases grow on a slow one
O=gpurun_out/r5i_$(date +%H%M%S); mkdir -p $O
rocm-smi --showclocks > $O/clocks.txt 2>&1 || true
timeout -k 10 180 tools/ubench/floor_ubench 1000000000 5 > $O/floor.txt 2>&1 || { echo floor failed; cat $O/floor.txt; exit 1; }
timeout -k 10 300 python3 tools/exp_slice.py --rounds 2 libqeh.so > $O/step.txt 2>&1 || { cat $O/step.txt; exit 1; }
timeout -k 10 200 python3 tools/exp/pa_stamps.py libqeh_stamps.so > $O/stamps.txt 2>&1 || { cat $O/stamps.txt; exit 1; }
rocm-smi --showclocks >> $O/clocks.txt 2>&1 || true
cat $O/floor.txt $O/step.txt; grep -v amdgpu.ids $O/stamps.txt | cut -c1-400
}

r5j() {
# phase-A time over a long run (clock / power ramp?), with the SMU's view before and after
O=gpurun_out/r5j_$(date +%H%M%S); mkdir -p $O
rocm-smi --showclocks --showpower > $O/smi_before.txt 2>&1 || true
timeout -k 10 300 python3 -u tools/exp/ramp.py 400 > $O/ramp.txt 2>&1 || { cat $O/ramp.txt; exit 1; }
rocm-smi --showclocks --showpower > $O/smi_after.txt 2>&1 || true
grep -v amdgpu.ids $O/ramp.txt; grep -i "mclk\|fclk\|sclk\|socclk\|Power" $O/smi_before.txt $O/smi_after.txt | head -20
}

r5k() {
# config 5's partition / inverse passes with one LDS word per staged row (pass 1) and the run bases
# folded into one array (pass 1, inverse passes): A/B against the previous build, then window parity
O=gpurun_out/r5k; mkdir -p $O
timeout -k 10 400 python3 tools/exp/win_ab.py --rounds 2 libqeh_wbase.so libqeh.so > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
run_tests $O/tests.txt tests/test_window_msd.py
}

r5l() {
# the shuffle join's items form (config 4): simulated ranks on one device, then gloo device-tensor
# ranks (world 2 / 3 / 8) through DistributedExecutor, then the per-rank leg
O=gpurun_out/r5l; mkdir -p $O
run_tests $O/tests.txt "tests/test_pipeline.py::test_shuffle_items_form_vs_oracle" \
    "tests/test_pipeline.py::test_items_form_vs_oracle" \
    "tests/test_distributed.py::test_device_tensor_collectives_several_ranks_on_one_gpu" \
    "tests/test_distributed.py::test_config4_shuffle_join_two_ranks_on_one_gpu" || exit 1
}

r5m() {
# config 4's per-rank device leg at N = 8: the two-pass exchange form and the items form, one box
O=gpurun_out/r5m; mkdir -p $O
timeout -k 10 400 python3 tools/bench_configs.py --only cfg4leg,cfg4items > $O/cfg4.txt 2>&1 || { tail -30 $O/cfg4.txt; exit 1; }
grep -v amdgpu.ids $O/cfg4.txt | cut -c1-700
}

r5t() {
# the whole GPU suite (the driver's round-end tier)
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 1080 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -15 $O/tests.txt; exit $rc
}

r5b2() {
# the bench line (driver contract), then the profile of the same command (kernel trace + PMC passes)
O=gpurun_out/r5b2; mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
timeout -k 10 900 bash tools/profile.sh r05 > $O/profile.txt 2>&1 || { tail -20 $O/profile.txt; exit 1; }
tail -25 $O/profile.txt
}

r5n() {
# phase A's key stores non-temporal (as the value stores) vs cached, alternating builds
O=gpurun_out/r5n_$(date +%H%M%S); mkdir -p $O
timeout -k 10 500 python3 tools/exp_slice.py --rounds 3 libqeh_base.so libqeh.so > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
}

r5o() {
# config 5: the partition passes' run writes non-temporal (QEH_WM_NTS bit 0 pass 1, bit 1 pass 2) vs cached
O=gpurun_out/r5o_$(date +%H%M%S); mkdir -p $O
timeout -k 10 600 python3 tools/exp/win_ab.py --rounds 2 libqeh.so libqeh.so:QEH_WM_NTS=1 libqeh.so:QEH_WM_NTS=2 \
    libqeh.so:QEH_WM_NTS=3 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
}

r5p() {
# non-temporal result stores of the group sort (QEH_WM_NTS=4) and of the small exchange scatter
# (QEH_PM_NT=1: config 4's two-pass exchange and the window leg's move) vs cached
O=gpurun_out/r5p_$(date +%H%M%S); mkdir -p $O
timeout -k 10 600 python3 tools/exp/win_ab.py --rounds 2 libqeh.so libqeh.so:QEH_WM_NTS=4 > $O/ab_win.txt 2>&1 || { cat $O/ab_win.txt; exit 1; }
grep -v amdgpu.ids $O/ab_win.txt
for e in 0 1; do
  QEH_NO_ITEMS_SHUFFLE=1 QEH_PM_NT=$e timeout -k 10 300 python3 tools/bench_configs.py --only cfg4leg > $O/cfg4_nt$e.txt 2>&1 || { tail -5 $O/cfg4_nt$e.txt; exit 1; }
  grep -v amdgpu.ids $O/cfg4_nt$e.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("PM_NT='$e'", d["kernel_ms"], d["legs"]["exchange_pass_fact"]["ms"], d["legs"]["local_join"]["ms"])'
done
}

r5q() {
# the configs table of this round (one box), then the N = 8 rank-share rehearsal (items form)
O=gpurun_out/r5q; mkdir -p $O
timeout -k 10 1000 python3 -u tools/bench_configs.py --only cfg2,cfg3,filter,limit,left,full,shapes,partition,merge,window,cfg4leg,cfg4items,cfg5leg,cfg5 > $O/configs.jsonl 2>$O/configs.err || { tail $O/configs.err; exit 1; }
python3 -c 'import json,sys
for l in open(sys.argv[1]):
    l=l.strip()
    if not l.startswith("{"): continue
    d=json.loads(l); print(str(d["config"])[:70], round(d["kernel_ms"] or 0,3), d["frac_of_8TBs"])' $O/configs.jsonl
for r in 0 3; do
  QEH_BENCH_RANK_OF=$r/8 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 > $O/rank${r}of8.json 2> $O/rank${r}of8.err || { tail -20 $O/rank${r}of8.err; exit 1; }
  tail -1 $O/rank${r}of8.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rank-share", d["ms_per_step"], d.get("dist_build"), d.get("dist_final"))'
done
}

r5r() {
# non-temporal key stores in the fused pipeline only: cfg3 / g17 / agg2 and the metric, base (cached
# keys everywhere) vs this build, one box
O=gpurun_out/r5r; mkdir -p $O
for lib in libqeh_base.so libqeh.so; do
  QEH_LIB_PATH=$PWD/query-engine_amd/$lib timeout -k 10 400 python3 -u tools/bench_configs.py --only cfg3,shapes > $O/cfg_$lib.jsonl 2>$O/cfg_$lib.err || { tail $O/cfg_$lib.err; exit 1; }
  python3 -c 'import json,sys
for l in open(sys.argv[1]):
    l=l.strip()
    if l.startswith("{"): d=json.loads(l); print(sys.argv[2], str(d["config"])[:40], round(d["kernel_ms"] or 0,3))' $O/cfg_$lib.jsonl $lib
done
timeout -k 10 500 python3 tools/exp_slice.py --rounds 2 libqeh_base.so libqeh.so > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
}

r5s() {
# own block read in place (not packed, not copied): shuffle items-form parity, then the per-rank leg
O=gpurun_out/r5s; mkdir -p $O
run_tests $O/tests.txt "tests/test_pipeline.py::test_shuffle_items_form_vs_oracle" \
    "tests/test_distributed.py::test_device_tensor_collectives_several_ranks_on_one_gpu" || exit 1
timeout -k 10 300 python3 tools/bench_configs.py --only cfg4items > $O/cfg4.txt 2>&1 || { tail -20 $O/cfg4.txt; exit 1; }
grep -v amdgpu.ids $O/cfg4.txt | cut -c1-600
}

"$@"
