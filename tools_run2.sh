set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_pipeline.py -m gpu -x -q > gpurun_out/pytest2.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest2.log; exit 1; }
for nt in 0 1; do
  QEH_NT_LOADS=$nt timeout -k 10 600 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/bench2_nt$nt.log 2>&1 || { echo "bench failed"; exit 1; }
done
QEH_NO_FAST=1 timeout -k 10 600 python bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/bench2_nofast.log 2>&1 || { echo "bench nofast failed"; exit 1; }
grep -h -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"frac": [0-9.]*' gpurun_out/bench2_*.log
bash tools/profile.sh r1a || exit 1
