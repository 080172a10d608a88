set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -q -x > gpurun_out/pytest16.log 2>&1; rc=$?
tail -3 gpurun_out/pytest16.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest16.log; exit $rc; }
for V in fused nosh part partchunk; do
  case $V in
    fused) E="";; nosh) E="QEH_NO_SHARDS=1";; part) E="QEH_PART_MIN_BYTES=0";; partchunk) E="QEH_PART_MIN_BYTES=0 QEH_PART_CHUNK=8388608";;
  esac
  env $E timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/b16_$V.log 2>&1 || { tail gpurun_out/b16_$V.log; exit 1; }
  echo "$V $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b16_$V.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/b16_$V.log)"
done
timeout -k 10 600 python tools/bench_configs.py --only cfg2,filter > gpurun_out/configs16.log 2>&1 || { tail gpurun_out/configs16.log; exit 1; }
grep -o '"config": "[^"]*"\|"kernel_ms": [0-9.]*\|"frac_of_8TBs": [0-9.]*' gpurun_out/configs16.log
