set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export QEH_PART_MIN_BYTES=0
timeout -k 10 600 python -m pytest tests/test_pipeline.py -m gpu -q -x > gpurun_out/pytest15.log 2>&1 || { tail -30 gpurun_out/pytest15.log; exit 1; }
QEH_PART_CHUNK=8388608 timeout -k 10 600 python -m pytest tests/test_pipeline.py -m gpu -q -x >> gpurun_out/pytest15.log 2>&1 || { tail -30 gpurun_out/pytest15.log; exit 1; }
tail -2 gpurun_out/pytest15.log
for CH in 0 2097152 4194304 8388608 16777216 67108864; do
  QEH_PART_CHUNK=$CH timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/b15_$CH.log 2>&1 || { tail gpurun_out/b15_$CH.log; exit 1; }
  echo "chunk=$CH $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b15_$CH.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/b15_$CH.log)"
done
unset QEH_PART_MIN_BYTES
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/b15_fused.log 2>&1 || exit 1
echo "fused $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b15_fused.log)"
