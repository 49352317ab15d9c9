#!/usr/bin/env python3
"""Contiguous (N, 4, 66) observations vs the frame ring (FrameRingBatch), one GPU.

    python tools/bench_frame_ring.py [--envs 65536] [--rings 8 32 128] [--steps 2000] [--warmup 1000]

Same protocol as bench.py (seeds 19 + env index, uniform actions, one distinct buffer per step,
W untimed steps, K timed steps between synchronisations). The ring variant writes one 88-B
frame per agent per step (three on a wrap, every R - 2 steps) instead of the 264-B stacked
row: 2,289 + 2C algorithmic bytes per env-step become 1,585 + 2C. Prints one JSON line per
variant.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-soccer_amd"))


def run(n: int, ring: int, steps: int, warmup: int, sets: int):
    import torch
    from marlsoccer import FrameRingBatch, SoccerBatch

    gen = torch.Generator(device="cuda")
    gen.manual_seed(1000)
    acts = [torch.rand((n, 4, 3), device="cuda", generator=gen) * 2 - 1 for _ in range(sets)]
    if ring:
        b = FrameRingBatch(n, ring=ring)
        b.reset(seed=19)
        f = b.launcher(acts, b.rew, b.term, b.trunc, b.goal, b.score)
    else:
        b = SoccerBatch(n)
        b.reset(seed=19)
        f = b.launcher(acts, b.obs, b.rew, b.term, b.trunc, b.goal, b.score)
    for i in range(warmup):
        f(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        f(warmup + i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    b.close()
    return {"layout": f"ring{ring}" if ring else "contiguous", "envs": n, "steps": steps, "warmup": warmup,
            "action_sets": sets, "us_per_step": el * 1e6 / steps, "env_steps_per_s": n * steps / el}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--rings", type=int, nargs="+", default=[8, 32, 128])
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--action-sets", type=int, default=0, help="distinct action buffers (0: steps + warmup)")
    a = ap.parse_args()
    sets = a.action_sets or a.steps + a.warmup
    for r in [0, *a.rings, 0]:  # contiguous before and after, to bound drift
        print(json.dumps(run(a.envs, r, a.steps, a.warmup, sets)), flush=True)


if __name__ == "__main__":
    main()
