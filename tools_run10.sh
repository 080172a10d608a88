set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -q -x > gpurun_out/pytest10.log 2>&1; rc=$?
tail -5 gpurun_out/pytest10.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest10.log; exit $rc; }
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench10.log 2>&1 || { tail gpurun_out/bench10.log; exit 1; }
tail -1 gpurun_out/bench10.log
QEH_PART_MIN_BYTES=0 timeout -k 10 600 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/bench10_part.log 2>&1 || { tail gpurun_out/bench10_part.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench10_part.log
QEH_PART_MIN_BYTES=0 bash tools/profile.sh r1c > /dev/null 2>&1 || { echo "profile failed"; exit 1; }
head -8 gpurun_out/prof_r1c/summary.txt
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/configs10.log 2>&1 || { tail -20 gpurun_out/configs10.log; exit 1; }
cat gpurun_out/configs10.log
