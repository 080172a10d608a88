"""Print the last two steps of a rocprofv3 kernel trace as a timeline (us from the step start)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_slice_probe"
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
s, e = idx[-3] + 1, idx[-1] + 3
t0 = int(rows[s]["Start_Timestamp"])
for r in rows[s:e]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(st - t0) / 1e3:9.1f} {(en - t0) / 1e3:9.1f} {(en - st) / 1e3:8.1f} q{r['Queue_Id']} {r['Kernel_Name'][:60]}")
