#!/usr/bin/env python3
"""HBM-side request split of the step kernel (diagnostic): which part of the write and read traffic
goes out as whole 64-B requests and which as 32-B (partial) ones, per env-step.

    python tools/tcc_split.py gpurun_out/<tag>/tcc_<lib> <kernel> <envs> <steps>

Reads the rocprofv3 --pmc passes written by `tools/gpu.sh tcc` (TCC_EA0_WRREQ / _64B, TCC_EA0_RDREQ /
_32B, TCC_EA0_WRREQ_DRAM / TCC_EA0_RDREQ_DRAM, TCC_BUBBLE, summed over the TCC channels) and reports the
medians over the last <steps> dispatches of <kernel>: write bytes = 64 x WRREQ_64B + 32 x (WRREQ -
WRREQ_64B) (WRITE_SIZE's own formula), read bytes = 128 x BUBBLE + 64 x (RDREQ - BUBBLE - RDREQ_32B)
+ 32 x RDREQ_32B (FETCH_SIZE's), and the share of requests that reach DRAM rather than the
Infinity Cache.
"""
import csv
import glob
import json
import os
import statistics
import sys


def main(d, kernel, envs, steps):
    vals = {}
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        rows = [r for r in csv.DictReader(open(f)) if kernel in r["Kernel_Name"].split("<")[0].split("(")[0]]
        by = {}
        for r in rows:
            by.setdefault(r["Counter_Name"], {}).setdefault(int(r["Dispatch_Id"]), 0.0)
            by[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        for c, dd in by.items():
            ids = sorted(dd)[-steps:]
            vals[c] = statistics.median(dd[i] for i in ids)
    g = lambda n: vals.get(n, vals.get(n + "_sum"))  # noqa: E731
    out = {"dir": d, "kernel": kernel, "envs": envs, "counters_median_per_launch": vals}
    wr, wr64 = g("TCC_EA0_WRREQ"), g("TCC_EA0_WRREQ_64B")
    if wr is not None and wr64 is not None:
        out["write"] = {"bytes_per_env_step": (64 * wr64 + 32 * (wr - wr64)) / envs,
                        "in_64B_requests": 64 * wr64 / envs, "in_32B_requests": 32 * (wr - wr64) / envs,
                        "partial_request_share": (wr - wr64) / wr}
    rd, rd32, bub = g("TCC_EA0_RDREQ"), g("TCC_EA0_RDREQ_32B"), g("TCC_BUBBLE")
    if rd is not None and rd32 is not None:
        b = bub or 0.0
        out["read"] = {"bytes_per_env_step": (128 * b + 64 * (rd - b - rd32) + 32 * rd32) / envs,
                       "in_32B_requests": 32 * rd32 / envs, "requests": rd / envs}
    wd, rdd = g("TCC_EA0_WRREQ_DRAM"), g("TCC_EA0_RDREQ_DRAM")
    if wd is not None and wr:
        out["write_requests_to_dram_share"] = wd / wr
    if rdd is not None and rd:
        out["read_requests_to_dram_share"] = rdd / rd
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
