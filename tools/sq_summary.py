#!/usr/bin/env python3
"""Per-wave SQ counters of the env-step kernels from the passes of `tools/gpu.sh sq` (diagnostic).

    python tools/sq_summary.py <dir> [--last K] [--json out.json]

Each pass directory <dir>/p*/ holds one rocprofv3 counter_collection.csv. Every step-kernel
dispatch (ms_step_kernel, ms_step_group_kernel, ms_step_pair_kernel and the K-step *_n_kernel launches) is a
row group; the last K dispatches of the step kernel (the bench's timed window) are kept and the
median of each counter over them is reported, per dispatch and per wave. SQ cycle counters are
quad-cycles (x4 = clock cycles). WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES.
"""
import argparse
import csv
import glob
import json
import statistics
from collections import defaultdict

STEP = ("ms_step_kernel", "ms_step_group_kernel", "ms_step_pair_kernel",
        "ms_step_pair_n_kernel", "ms_step_group_n_kernel")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=100)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    vals = defaultdict(list)
    kernels = set()
    for f in sorted(glob.glob(f"{a.dir}/p*/**/*counter_collection.csv", recursive=True)):
        per = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not any(k in name for k in STEP):
                continue
            kernels.add(name.split("(")[0])
            d = per[int(r["Dispatch_Id"])]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for did in sorted(per)[-a.last:]:
            for k, v in per[did].items():
                vals[k].append(v)
    med = {k: statistics.median(v) for k, v in vals.items()}
    waves = med.get("SQ_WAVES", 1.0)
    out = {"kernels": sorted(kernels), "dispatches": a.last, "per_dispatch": med,
           "per_wave": {k: v / waves for k, v in med.items()}}
    print("kernels:", ", ".join(sorted(kernels)))
    for k in sorted(med):
        print(f"{k:32s} {med[k]:16.0f} {med[k] / waves:12.1f} /wave")
    pw = out["per_wave"]
    if "SQ_WAVE_CYCLES" in pw and "SQ_ACTIVE_INST_ANY" in pw:
        wc = pw["SQ_WAVE_CYCLES"]
        print(f"issuing {pw['SQ_ACTIVE_INST_ANY'] / wc:.3f}  waitcnt {pw.get('SQ_WAIT_ANY', 0) / wc:.3f}  "
              f"issue-stall {pw.get('SQ_WAIT_INST_ANY', 0) / wc:.3f} of wave cycles")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
