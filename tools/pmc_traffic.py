#!/usr/bin/env python3
"""Summarise a tools/profile.sh run: per-kernel stats from the kernel-trace
pass and per-dispatch HBM bytes from the FETCH_SIZE / WRITE_SIZE passes.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per
128-B fabric request of a wide streaming read, i.e. reads exactly half the
bytes of a 16-B-per-lane coalesced stream -> doubled here; WRITE_SIZE is
exact for 16-B streaming stores.  Units of both counters are KiB.
Writes <dir>/traffic.json and prints a table.  With --emit FILE --rows N it
also writes the bench-readable per-step HBM bytes of the metric query's probe
pipeline (k_slice_partition + k_slice_probe, or the single-pass
k_join_agg_fast, plus the ragged-tail k_agg_rows) to FILE."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def main(d):
    stats = rows(os.path.join(d, "kt", "**", "*kernel_stats.csv"))
    print("== kernel stats (kernel-trace pass) ==")
    stats.sort(key=lambda r: -float(r.get("TotalDurationNs", 0) or 0))
    for r in stats[:15]:
        print(f"{short(r['Name'])[:80]:80s} calls={r.get('Calls')} avg_us={float(r.get('AverageNs', 0)) / 1e3:10.1f} "
              f"total_ms={float(r.get('TotalDurationNs', 0)) / 1e6:9.2f} pct={r.get('Percentage')}")
    res = {}
    for ctr, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        per = defaultdict(list)
        for r in rows(os.path.join(d, sub, "**", "*counter_collection.csv")):
            if r.get("Counter_Name") != ctr:
                continue
            per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        res[ctr] = {k: sum(v) / len(v) for k, v in per.items()}
    print("== per-dispatch HBM bytes (FETCH x2 gfx950 correction, WRITE exact) ==")
    summary = {}
    for k in sorted(set(res["FETCH_SIZE"]) | set(res["WRITE_SIZE"])):
        f = res["FETCH_SIZE"].get(k, 0.0) * 1024
        w = res["WRITE_SIZE"].get(k, 0.0) * 1024
        summary[k] = {"fetch_raw_bytes": f, "fetch_corrected_bytes": 2 * f, "write_bytes": w,
                      "hbm_bytes": 2 * f + w}
        print(f"{k[:80]:80s} fetch_raw={f / 1e9:8.3f} GB  fetch_x2={2 * f / 1e9:8.3f} GB  write={w / 1e9:8.3f} GB")
    json.dump({"kernels": summary, "stats": stats}, open(os.path.join(d, "traffic.json"), "w"), indent=1)
    return summary, stats


PIPELINE = ("k_slice_partition", "k_slice_probe", "k_join_agg_fast", "k_agg_rows<1")


def emit(summary, stats, path, rows, source):
    """Per-launch HBM bytes and average durations of the probe pipeline's kernels."""
    comp, dur = {}, {}
    for k, v in summary.items():
        if any(p in k for p in PIPELINE):
            comp[k] = v["hbm_bytes"]
    for r in stats:
        k = short(r["Name"])
        if any(p in k for p in PIPELINE):
            dur[k] = float(r.get("AverageNs", 0) or 0) / 1e6
    out = {"rows": rows, "kernel": "join_filter_aggregate", "hbm_bytes_per_launch": sum(comp.values()),
           "source": source,
           "components_hbm_bytes": comp, "components_avg_ms": dur,
           "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, mean per dispatch, summed over the "
                   "pipeline's kernels (one dispatch each per query)"}
    json.dump(out, open(path, "w"), indent=1)
    print("emitted", path, json.dumps(out))


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--emit")
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    a = ap.parse_args()
    summary, stats = main(a.dir)
    if a.emit:
        emit(summary, stats, a.emit, a.rows, "tools/profile.sh run " + os.path.basename(os.path.abspath(a.dir)))
