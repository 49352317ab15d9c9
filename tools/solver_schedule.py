#!/usr/bin/env python3
"""Rounds of the contact solve under a dependency-level schedule (design study; CPU only).

    python tools/solver_schedule.py [--envs 2048] [--steps 1300] [--from 1000]

Steps the fp32 oracle (test infrastructure) with uniform(-1, 1) actions, as bench.py does, and
after each step of the window reads every env's contact list back from its arbiter cache (the
touched arbiters, idle 0, in pair order = the canonical solve order). For each env it computes:

  serial    11 n      (warm start + 10 Gauss-Seidel passes over n contacts, one lane)
  levels    the ASAP level of each contact in one pass (1 + the latest level of its two
            dynamic bodies; the static body never changes), lmax the deepest level, and the
            period P = max over dynamic bodies of (last level - first level + 1): pass it of
            contact k runs at round lv(k) - 1 + it * P, which keeps every pair of solves that
            share a body in sequence order, so
  sched     lmax + 9 P + lmax   (warm start by levels, then the 10 passes)

and reports per-env and per-wave (8 envs, the lane-group kernel's wave) distributions of
both, the worst wave's figures first.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def bodies(p: int):
    if p < 6:
        i = 0 if p < 3 else (1 if p < 5 else 2)
        j = p + 1 if p < 3 else (p - 1 if p < 5 else 3)
        return i, j
    if p < 10:
        return 4, p - 6
    if p < 42:
        return 5, (p - 10) >> 3
    return 4, 5


def schedule(contacts):
    last = [0] * 6
    first = [0] * 6
    lmax = 0
    for a, b in contacts:
        lv = 1 + max(last[a] if a < 5 else 0, last[b] if b < 5 else 0)
        for x in (a, b):
            if x < 5:
                last[x] = lv
                if first[x] == 0:
                    first[x] = lv
        lmax = max(lmax, lv)
    P = max([last[x] - first[x] + 1 for x in range(5) if first[x]] or [0])
    return lmax, P


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=1300)
    ap.add_argument("--from", dest="start", type=int, default=1000)
    ap.add_argument("--wave", type=int, default=8)
    a = ap.parse_args()
    import oracle as orc
    n = a.envs
    ref = orc.OracleBatch(n, "f32")
    ref.reset(np.stack([orc.pcg_from_seed(19 + i) for i in range(n)]), 0)
    rng = np.random.default_rng(7)
    ser_w, sch_w, ser_e, sch_e, worst = [], [], [], [], None
    for t in range(a.steps):
        ref.step(rng.uniform(-1, 1, (n, 4, 3)).astype(np.float32))
        if t < a.start:
            continue
        st = ref.export_state()
        ser = np.zeros(n, np.int64)
        sch = np.zeros(n, np.int64)
        for e in range(n):
            k = int(st["n_arb"][e])
            arb = st["arb"][e, :k]
            cl = []
            for x in arb:
                if x["idle"] == 0:
                    cl += [bodies(int(x["pair"]))] * int(x["count"])
            lmax, P = schedule(cl)
            ser[e] = 11 * len(cl)
            sch[e] = 2 * lmax + 9 * P
        ser_e.append(ser)
        sch_e.append(sch)
        sw = ser.reshape(-1, a.wave).max(1)
        cw = sch.reshape(-1, a.wave).max(1)
        ser_w.append(sw)
        sch_w.append(cw)
        w = int(np.argmax(sw))
        if worst is None or sw[w] > worst[0]:
            worst = (int(sw[w]), int(cw[w]), t, w)
    ser_w, sch_w = np.concatenate(ser_w), np.concatenate(sch_w)
    ser_e, sch_e = np.concatenate(ser_e), np.concatenate(sch_e)
    q = [0.5, 0.95, 0.99, 0.999, 1.0]
    print(f"worst wave (by serial rounds): serial {worst[0]}, scheduled {worst[1]} (step {worst[2]}, wave {worst[3]})")
    print("per wave  serial   ", [int(np.quantile(ser_w, x)) for x in q])
    print("per wave  scheduled", [int(np.quantile(sch_w, x)) for x in q])
    print("per env   serial   ", [int(np.quantile(ser_e, x)) for x in q])
    print("per env   scheduled", [int(np.quantile(sch_e, x)) for x in q])
    print("max over waves of the scheduled rounds:", int(sch_w.max()), " of the serial:", int(ser_w.max()))


if __name__ == "__main__":
    main()
