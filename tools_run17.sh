set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export QEH_PART_MIN_BYTES=0
bash tools/prof_configs.sh d --only filter --scale 0.01 > /dev/null 2>&1
for V in base exp1 b4k b64k; do
  case $V in base) E="X=1";; exp1) E="QEH_PART_EXP=1";; b4k) E="QEH_PART_BATCH=4096";; b64k) E="QEH_PART_BATCH=65536";; esac
  cd /tmp
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/p17_$V -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --cpu-sample 0 > $GRAFT_REPO_ROOT/gpurun_out/p17_$V.log 2>&1 || { tail $GRAFT_REPO_ROOT/gpurun_out/p17_$V.log; exit 1; }
  cd "$GRAFT_REPO_ROOT"
  python3 - gpurun_out/p17_$V $V <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "join" in r["Name"]:
        print(sys.argv[2], r["Name"].split("(")[0][:60], "avg_us=%.1f" % (float(r["AverageNs"]) / 1e3))
PY
done
bash tools/pmc_cmd.sh partB "TCC_HIT_sum TCC_MISS_sum" "TCC_REQ_sum TCC_EA0_RDREQ_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --cpu-sample 0 2>&1 | grep -i "join"
