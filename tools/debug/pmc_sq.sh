set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d "$R/gpurun_out/pmc_sq" -o sq -- python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-sample 0 > "$R/gpurun_out/pmc_sq.log" 2>&1 || { tail -5 "$R/gpurun_out/pmc_sq.log"; exit 1; }
python3 - <<'PY'
import csv, glob, os, collections
R = os.environ["GRAFT_REPO_ROOT"]
f = glob.glob(R + "/gpurun_out/pmc_sq/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "slice" in k:
        print(k, {c: round(sum(v) / len(v) / 1e6, 2) for c, v in d.items()}, "(millions, avg per dispatch)")
PY
