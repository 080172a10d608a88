#!/bin/bash
# Window pass 1: cost split by experiment switches (QEH_WM_EXP), kernel trace per setting.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p $R/gpurun_out/r3/wmexp
cd /tmp && export TMPDIR=/tmp
for e in 0 1 2 3 4 12; do
  QEH_WM_EXP=$e timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3/wmexp/e$e -o kt -- \
      python3 $R/tools/r3/wm_exp.py 2.5e8 > $R/gpurun_out/r3/wmexp/e$e.log 2>&1 || { tail -5 $R/gpurun_out/r3/wmexp/e$e.log; exit 1; }
  python3 - "$R/gpurun_out/r3/wmexp/e$e" "$e" <<'PY'
import csv, glob, sys
p = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(p)):
    if "wm" in r["Name"]:
        print(f"exp={sys.argv[2]:3s} {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']}  {r['Name'][:60]}")
PY
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r3/cosched -o kt -- \
    python3 $R/tools/r3/cosched.py > $R/gpurun_out/r3/cosched.log 2>&1 || { tail -5 $R/gpurun_out/r3/cosched.log; exit 1; }
python3 - "$R/gpurun_out/r3/cosched" <<'PY'
import csv, glob, sys
p = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(p)), key=lambda r: int(r["Start_Timestamp"]))
parts = [r for r in rows if "k_slice_partition" in r["Kernel_Name"]]
for a in parts[-3:]:
    s0, e0 = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
    print(f"phase A {s0} .. {e0} ({(e0 - s0) / 1e3:.1f} us)")
    for r in rows:
        s1, e1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s1 < e0 + 200_000 and e1 > s0 - 50_000 and r is not a:
            print(f"   {(s1 - s0) / 1e3:9.1f} {(e1 - s0) / 1e3:9.1f} {(e1 - s1) / 1e3:8.1f} q{r['Queue_Id']} {r['Kernel_Name'][:60]}")
PY
