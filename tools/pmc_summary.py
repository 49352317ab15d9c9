#!/usr/bin/env python3
"""Summarise a gpurun_out/<tag>/ profiling run into profiles/ (tracked).

Reads rocprofv3 CSVs written by `tools/gpu.sh profile`:
  trace/run_kernel_stats.csv          -> profiles/<tag>_kernel_stats.csv (copied verbatim)
  pmc_fetch|pmc_write/run_counter_collection.csv -> profiles/<tag>_pmc.json
FETCH_SIZE / WRITE_SIZE are KiB per dispatch (TCC_EA0 request counters). Per
MI355X_MICROARCH.md §HBM, FETCH_SIZE reads 1/2 of the bytes of wide coalesced streams on
gfx950, so hbm_read_bytes = 2 x FETCH_SIZE x 1024 (upper estimate for narrower accesses);
WRITE_SIZE is taken as is.
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, kernel):
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    return [float(r["Counter_Value"]) for r in rows], rows


def compiler_usage(tag, kernel):
    """The step kernel's block of profiles/<tag>_resource_usage.txt (tools/resource_usage.py)."""
    path = os.path.join(ROOT, "profiles", f"{tag}_resource_usage.txt")
    if not os.path.exists(path):
        return None
    out, cur = {}, None
    for ln in open(path):
        k, _, v = ln.strip().partition(": ")
        if k == "Function Name":
            cur = v
            if out:
                break
        elif cur and kernel in cur and "ILb1E" in cur and v:
            out[k] = v
    return dict(out, source=f"profiles/{tag}_resource_usage.txt", kernel=f"{kernel}<true> (default physics)") if out else None


def window_pmc(src, kernel, envs, warmup, steps, pass_w=None, pass_s=None, per_launch_steps=1):
    """HBM bytes per launch over dispatches [warmup, warmup + steps) of `kernel` in the
    FETCH_SIZE and WRITE_SIZE passes of one bench window (medians over the window). pass_w /
    pass_s name the bench pass when the kernel's own window differs from it (the K-step leg);
    hbm_bytes_per_env_step divides by envs x per_launch_steps."""
    out = {}
    vals = {}
    pw, ps = (warmup if pass_w is None else pass_w), (steps if pass_s is None else pass_s)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        path = os.path.join(src, f"pmc_{c}_w{pw}_s{ps}", "run_counter_collection.csv")
        if not os.path.exists(path):
            return None
        _, rows = per_kernel(path, kernel)
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        if not rows:
            return None
        win = rows[warmup:warmup + steps]
        vals[c] = [float(r["Counter_Value"]) for r in win]
        out["dispatches"] = [warmup, warmup + len(win)]
        out["rocprof_vgpr_field"] = int(rows[0]["VGPR_Count"])
        out["rocprof_accum_vgpr_field"] = int(rows[0]["Accum_VGPR_Count"])
        out["sgpr"] = int(rows[0]["SGPR_Count"])
        out["scratch_bytes_per_lane"] = int(rows[0]["Scratch_Size"])
        out["lds_bytes_per_block"] = int(rows[0]["LDS_Block_Size"])
        out["kernel"] = rows[0]["Kernel_Name"].split("<")[0].split("(")[0].replace("void ", "").strip()
    fetch_kib, write_kib = statistics.median(vals["FETCH_SIZE"]), statistics.median(vals["WRITE_SIZE"])
    rd, wr = 2.0 * fetch_kib * 1024, write_kib * 1024
    out.update({"FETCH_SIZE_KiB_median": fetch_kib, "WRITE_SIZE_KiB_median": write_kib,
                "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
                "hbm_bytes_per_env_step": (rd + wr) / (envs * per_launch_steps)})
    return out


def fused_summary(tag, src, dst, envs, kernel, K, max_steps):
    """profiles/pmc_fused_kernel.json: the K-step leg's (bench.py `fused_steps`) launches in the same
    PMC passes: its own window is the pass's warm-up and steps rounded up to whole K-step launches
    (at least one warm-up and four timed launches), as bench.py computes it."""
    nk = kernel.replace("_kernel", "_n_kernel")
    out = {"tag": tag, "kernel": nk, "envs": envs, "K": K,
           "correction": "read = 2 x FETCH_SIZE (gfx950 half-count, MI355X_MICROARCH.md HBM); write = WRITE_SIZE",
           "regimes": {}}
    for w, s in ((5, 20), (1000, 1000)):
        fw, fs = K * max(1, -(-w // K)), K * max(4, -(-s // K))
        r = window_pmc(src, nk, envs, fw // K, fs // K, pass_w=w, pass_s=s, per_launch_steps=K)
        if r is not None:
            out["regimes"][f"e{envs}_ms{max_steps}_K{K}_w{fw}_s{fs}"] = r
    if out["regimes"]:
        with open(os.path.join(dst, "pmc_fused_kernel.json"), "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out, indent=1))
    return out


def main(tag, envs=65536, kernel="ms_step_kernel", warmup=1000, steps=1000, max_steps=1000):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    ks = [r for r in stats if kernel in r["Name"]][0]
    out = {
        "tag": tag, "kernel": kernel, "envs": envs,
        "kernel_avg_ns": float(ks["AverageNs"]), "kernel_calls": int(ks["Calls"]),
        "compiler": compiler_usage(tag, kernel),
        "correction": "read = 2 x FETCH_SIZE (gfx950 half-count, MI355X_MICROARCH.md HBM); write = WRITE_SIZE",
        # rocprofv3's dispatch fields (vgpr/accum_vgpr) do not match the compiler's allocation on
        # gfx950; the compiler's own resource usage is "compiler"
        "regimes": {},
    }
    for w, s in ((5, 20), (1000, 200), (1000, 1000)):
        r = window_pmc(src, kernel, envs, w, s)
        if r is not None:
            out["regimes"][f"e{envs}_ms{max_steps}_w{w}_s{s}"] = r
    # the bench's timed window alone (its event timing covers only those launches): dispatches
    # [warmup, warmup + steps) of the step kernel in the kernel trace
    tr = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))) if kernel in r["Kernel_Name"]]
    tr.sort(key=lambda r: int(r["Dispatch_Id"]))
    win = tr[warmup:warmup + steps]
    if win:
        out["kernel_avg_ns_timed_window"] = statistics.mean(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win)
        out["timed_window_dispatches"] = [warmup, warmup + len(win)]
    for name in (f"{tag}_pmc.json", "pmc_step_kernel.json"):
        with open(os.path.join(dst, name), "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
    fused_summary(tag, src, dst, envs, kernel, 50, max_steps)


if __name__ == "__main__":
    # tag [envs [kernel]]: bench.py's default window of the named step kernel
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 65536, sys.argv[3] if len(sys.argv) > 3 else "ms_step_kernel")
