set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_pipeline.py -m gpu -x -q > gpurun_out/pytest5.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest5.log; exit 1; }
tail -2 gpurun_out/pytest5.log
for cfg in "part 1" "part 0" "nopart 1"; do
  set -- $cfg
  if [ "$1" = nopart ]; then export QEH_NO_PART=1; else unset QEH_NO_PART; fi
  QEH_NT_LOADS=$2 timeout -k 10 600 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/bench5_$1_$2.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench5_$1_$2.log; exit 1; }
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench5_$1_$2.log)"
done
unset QEH_NO_PART
QEH_NT_LOADS=1 bash tools/profile.sh r1b > /dev/null 2>&1 || { echo "profile failed"; exit 1; }
head -12 gpurun_out/prof_r1b/summary.txt
