#!/usr/bin/env python3
"""Per-wave averages of the SQ counters collected by tools/sq_counters.sh (diagnostic)."""
import csv
import glob
import statistics
import sys
from collections import defaultdict

out = sys.argv[1]
vals = defaultdict(list)
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    per = defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "ms_step_kernel" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] = per[r["Dispatch_Id"]].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for d in per.values():
        for k, v in d.items():
            vals[k].append(v)
med = {k: statistics.median(v) for k, v in vals.items()}
waves = med.get("SQ_WAVES", 1.0)
for k in sorted(med):
    print(f"{k:32s} {med[k]:16.0f} {med[k] / waves:12.1f} /wave")
