#!/bin/bash
# Round-4 GPU session h: parity of the chunk / carry variants, then A/B on one box (+ calibration).
set -o pipefail
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
