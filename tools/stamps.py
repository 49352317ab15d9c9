#!/usr/bin/env python3
"""Per-phase wave timeline of ms_step_kernel (diagnostic; not part of the product path).

    python tools/stamps.py --build            # here: hipcc -DMS_STAMPS -> lib/libmarlsoccer_stamps.so
    python tools/stamps.py [--envs N] [--steps K] [--every M]   # on the GPU box

The stamps build writes s_memtime at the STAMP(k) points of ms_env.hip into a
[wave][NS] buffer. For every M-th launch of a K-step episode this tool reads the buffer
and reports, per phase, the mean cycles over all waves and over the slowest 5 % of waves
(the ones that set the launch time), plus the launch span in cycles.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "marl-soccer_amd")
STAMP_LIB = os.path.join(PKG, "lib", "libmarlsoccer_stamps.so")
NS = 48  # MS_NSTAMP: [0, 24) s_memtime cycles and accumulators, [24, 48) s_memrealtime (100 MHz) of stamps 0..23
RT = 24
# accumulated narrowphase sub-phase cycles and iteration counts (wave max over lanes)
ACC = {16: "AA test", 17: "AA insert", 18: "AA iterations", 19: "SA test", 20: "SA insert", 21: "SA iterations"}

# (label, from, to) in kernel order; a stamp inside a branch no lane took is carried forward
ORDER = [0, 1, 2, 11, 13, 3, 14, 4, 15, 22, 5, 6, 7, 8, 9, 10]
# --fine (lane-pair kernel): the narrowphase split by pair class (stamps 16-18 instead of the
# per-lane kernel's accumulators)
ORDER_FINE = [0, 1, 2, 11, 16, 17, 18, 13, 3, 14, 4, 15, 22, 5, 6, 7, 8, 9, 10]
LABELS_FINE = {16: "nphase agent-agent", 17: "nphase ball-agent", 18: "nphase static-agent shared tests",
               13: "nphase static-agent insert"}
LABELS = {1: "load+actions", 2: "integrate+transforms", 11: "bp+nphase AA/BA", 13: "nphase static-agent",
          3: "nphase ball-wall+cache age", 14: "prestep", 4: "velocity", 15: "warm start",
          22: "solver schedule (lane groups)", 5: "solver x10",
          6: "cache write", 7: "meta", 8: "goal+reward+outputs", 9: "obs frames+snap", 10: "state stores"}


def timeline(st):
    """One launch on the shared 100-MHz clock: when waves start and end, and how many waves are in
    the load, physics (narrowphase .. solver), and output (goal .. state stores) phases per 1-us bin."""
    import numpy as np
    rt = st[:, RT:RT + 16].astype(np.float64) * 0.01  # us
    ok = rt[:, 0] > 0
    rt = rt[ok]
    t0 = rt[:, 0].min()
    rt = rt - t0
    start, end = rt[:, 0], rt[:, 10]
    nb = int(np.ceil(end.max())) + 1
    def occ(a, b):
        h = np.zeros(nb)
        for x, y in zip(rt[:, a], rt[:, b]):
            i0, i1 = int(x), int(y)
            for i in range(i0, min(i1, nb - 1) + 1):
                h[i] += max(0.0, min(y, i + 1) - max(x, i))  # wave-us inside bin i
        return h
    return {"span_us": float(end.max()), "start_us": np.percentile(start, [50, 95, 100]).tolist(),
            "end_us": np.percentile(end, [5, 50, 95, 100]).tolist(),
            "dur_us": np.percentile(end - start, [50, 95, 100]).tolist(),
            "load": occ(0, 1), "physics": occ(2, 5), "outputs": occ(6, 10)}


def summarise_timeline(tl):
    import numpy as np
    nb = max(len(t["load"]) for t in tl)
    pad = lambda v: np.pad(v, (0, nb - len(v)))  # noqa: E731
    return {"span_us_mean": float(np.mean([t["span_us"] for t in tl])),
            "wave_start_us_p50_p95_max": np.mean([t["start_us"] for t in tl], axis=0).round(2).tolist(),
            "wave_end_us_p5_p50_p95_max": np.mean([t["end_us"] for t in tl], axis=0).round(2).tolist(),
            "wave_duration_us_p50_p95_max": np.mean([t["dur_us"] for t in tl], axis=0).round(2).tolist(),
            "waves_in_phase_per_us_bin": {k: np.mean([pad(t[k]) for t in tl], axis=0).round(0).tolist()
                                          for k in ("load", "physics", "outputs")}}


def build(extra=()):
    import build_native
    os.makedirs(os.path.dirname(STAMP_LIB), exist_ok=True)
    build_native.compile_and_link(STAMP_LIB, build_native.SOURCES, extra=["-DMS_STAMPS", *extra], verbose=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--every", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=0, help="untimed steps first (1000: steady state)")
    ap.add_argument("--out", default="")
    ap.add_argument("--lane-group", type=int, default=None, help="SoccerBatch.set_lane_group(G) (ms_set_lane_group)")
    ap.add_argument("--lib", default=STAMP_LIB, help="a -DMS_STAMPS library (default: the product stamps build)")
    ap.add_argument("--fine", action="store_true", help="the lane-pair kernel's narrowphase by pair class")
    a, extra = ap.parse_known_args()
    if a.fine:
        global ORDER
        ORDER = ORDER_FINE
        LABELS.update(LABELS_FINE)
    sys.path.insert(0, PKG)
    if a.build:
        build(extra)
        return
    os.environ["MARL_SOCCER_LIB"] = a.lib
    import numpy as np
    import torch
    from marlsoccer import SoccerBatch, _native

    L = _native.lib()
    L.ms_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
    L.ms_debug_stamps.restype = C.c_int
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    env = SoccerBatch(a.envs, device=0)
    if a.lane_group is not None:
        env.set_lane_group(a.lane_group)
    env.reset(seed=19)
    ptr, nw = C.c_void_p(), C.c_int64()
    L.ms_debug_stamps(env._h, C.byref(ptr), C.byref(nw))
    nw = nw.value
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    acts = torch.empty((a.envs, 4, 3), device="cuda")
    seg = {k: [] for k in ORDER[1:]}
    seg_slow = {k: [] for k in ORDER[1:]}
    spans, totals, slow_tot, maxnc, worst, accs = [], [], [], [], [], []
    tl = []  # per sampled launch: the real-time timeline (every XCD's waves on one clock)
    for t in range(a.warmup):
        acts.uniform_(-1.0, 1.0, generator=g)
        env.step(acts)
    for t in range(a.steps):
        acts.uniform_(-1.0, 1.0, generator=g)
        sample = t % a.every == 0 and t > 0
        if sample:
            torch.cuda.synchronize()
            hip.hipMemset(ptr, 0, nw * NS * 8)
            torch.cuda.synchronize()
        env.step(acts)
        if sample:
            torch.cuda.synchronize()
            buf = np.zeros((nw, NS), np.uint64)
            hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
            hip.hipMemcpy(buf.ctypes.data, ptr, nw * NS * 8, 2)
            st = buf.astype(np.int64)
            maxnc.append(st[:, 12].copy())
            for i in range(1, len(ORDER)):  # carry forward stamps of untaken branches
                k, prev = ORDER[i], ORDER[i - 1]
                st[:, k] = np.where(st[:, k] == 0, st[:, prev], st[:, k])
                st[:, RT + k] = np.where(st[:, RT + k] == 0, st[:, RT + prev], st[:, RT + k])
            tl.append(timeline(st))
            tot = st[:, 10] - st[:, 0]
            slow = tot >= np.quantile(tot, 0.95)
            totals.append(tot.mean())
            slow_tot.append(tot[slow].mean())
            spans.append(st[:, 10].max() - st[st[:, 0] > 0, 0].min())
            w = int(np.argmax(tot))
            accs.append(st[:, 16:22].copy())
            worst.append({"cycles": int(tot[w]), "max_contacts": int(maxnc[-1][w]),
                          "acc": {ACC[16 + j]: int(st[w, 16 + j]) for j in range(6)},
                          "phases": {LABELS[ORDER[i]]: int(st[w, ORDER[i]] - st[w, ORDER[i - 1]]) for i in range(1, len(ORDER))}})
            for i in range(1, len(ORDER)):
                d = st[:, ORDER[i]] - st[:, ORDER[i - 1]]
                seg[ORDER[i]].append(d.mean())
                seg_slow[ORDER[i]].append(d[slow].mean())
    mnc = np.concatenate(maxnc)
    res = {"envs": a.envs, "steps": a.steps, "warmup": a.warmup, "samples": len(totals),
           "launch": f"lane groups, {env.lane_group} lanes per env" if env.lane_group > 0 else "one wave per 64-env block",
           "wave_cycles_mean": float(np.mean(totals)), "wave_cycles_slowest5pct": float(np.mean(slow_tot)),
           "launch_span_cycles_note": "s_memtime counters differ between XCDs: see timeline (real time)",
           "timeline": summarise_timeline(tl),
           "worst_wave_cycles_mean": float(np.mean([w["cycles"] for w in worst])),
           "worst_wave_max_contacts": {str(v): sum(1 for w in worst if w["max_contacts"] == v) for v in sorted({w["max_contacts"] for w in worst})},
           "narrowphase_acc_mean": {ACC[16 + j]: round(float(np.mean(np.concatenate(accs)[:, j])), 1) for j in range(6)},
           "worst_wave_acc_mean": {k: round(float(np.mean([w["acc"][k] for w in worst])), 1) for k in ACC.values()},
           "worst_wave_phases_mean": {k: round(float(np.mean([w["phases"][k] for w in worst])), 1) for k in worst[0]["phases"]},
           "max_contacts_per_wave": {str(int(v)): int((mnc == v).sum()) for v in np.unique(mnc)},
           "phases": {LABELS[k]: {"mean": round(float(np.mean(seg[k])), 1),
                                  "slow5": round(float(np.mean(seg_slow[k])), 1)} for k in ORDER[1:]}}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
