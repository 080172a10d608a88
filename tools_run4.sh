set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { tag=$1; shift; env "$@" > /dev/null; }
for cfg in "1000000 0" "10000000 0" "10000000 1" "30000000 0" "100000000 0"; do
  set -- $cfg
  QEH_NO_U16=$( [ "$2" = 1 ] && echo 1 ) 
  if [ "$2" = 1 ]; then export QEH_NO_U16=1; else unset QEH_NO_U16; fi
  QEH_NT_LOADS=1 timeout -k 10 600 python bench.py --steps 10 --warmup 2 --cpu-sample 0 --dim $1 > gpurun_out/bench4_d$1_$2.log 2>&1 || { echo "bench failed"; cat gpurun_out/bench4_d$1_$2.log | tail; exit 1; }
  echo "dim=$1 nou16=$2 $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/bench4_d$1_$2.log)"
done
