#!/usr/bin/env python3
"""Summarise a rocprofv3 run of tools/bench_frame_ring.py (kernel trace + FETCH_SIZE and
WRITE_SIZE passes) per step kernel: average duration and HBM bytes per launch, read with the
gfx950 correction of tools/pmc_summary.py. Runs where the CSVs are (the GPU box).

    python tools/ring_pmc.py <dir> <envs> > summary.json
"""
import csv
import json
import os
import statistics
import sys


def main(d, envs):
    out = {}
    trace = "ring_trace" if os.path.isdir(os.path.join(d, "ring_trace")) else "trace"
    fetch_dir = "ring_FETCH_SIZE" if trace == "ring_trace" else "pmc_fetch"
    write_dir = "ring_WRITE_SIZE" if trace == "ring_trace" else "pmc_write"
    stats = list(csv.DictReader(open(os.path.join(d, trace, "run_kernel_stats.csv"))))
    for kernel in ("ms_step_kernel", "ms_step_ring_kernel", "ms_step_pair_kernel", "ms_step_pair_ring_kernel"):
        ks = [r for r in stats if kernel + "<" in r["Name"]]
        fetch = [float(r["Counter_Value"]) for r in csv.DictReader(open(os.path.join(d, fetch_dir, "run_counter_collection.csv")))
                 if kernel + "<" in r["Kernel_Name"]]
        write = [float(r["Counter_Value"]) for r in csv.DictReader(open(os.path.join(d, write_dir, "run_counter_collection.csv")))
                 if kernel + "<" in r["Kernel_Name"]]
        if not ks or not fetch or not write:
            continue
        rd = 2.0 * statistics.median(fetch) * 1024
        wr = statistics.median(write) * 1024
        out[kernel] = {"names": [r["Name"] for r in ks], "calls": sum(int(r["Calls"]) for r in ks),
                       "avg_ns": sum(float(r["TotalDurationNs"]) for r in ks) / sum(int(r["Calls"]) for r in ks),
                       "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                       "hbm_bytes_per_env_step": (rd + wr) / envs, "pmc_launches": len(fetch)}
    out["correction"] = "read = 2 x FETCH_SIZE KiB (gfx950 half-count), write = WRITE_SIZE KiB; medians over launches"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
