"""Summarise a profiles_run.sh output dir: per-launch averages of the sweep kernel."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
out = {}
for f in glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv")):
    acc = {}
    for r in csv.DictReader(open(f)):
        if "sweep_kernel" in r["Kernel_Name"]:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in acc.items():
        out[k] = sum(v) / len(v)
st = os.path.join(d, "trace", "run_kernel_stats.csv")
if os.path.exists(st):
    for r in csv.DictReader(open(st)):
        if "sweep_kernel" in r["Name"]:
            out["sweep_avg_ns"] = float(r["AverageNs"])
            out["sweep_calls"] = int(r["Calls"])
print(json.dumps(out, indent=1))
