#!/usr/bin/env python3
"""A GPU's envs as K sub-batches on K streams (diagnostic).

    python tools/bench_streams.py [--envs 262144] [--parts 1 2 4] [--steps 500] [--warmup 1000]

With more waves than SIMDs (more than 65,536 envs per MI355X), one launch runs its waves in
rounds that start together and drain their stores together; sub-batches on separate streams
let the SIMDs a finished wave frees start a wave of another launch, so memory phases and
physics of different waves overlap. Each sub-batch is an ordinary SoccerBatch (global seeds
19 + env index, as bench.py); one step = every sub-batch stepped once. Prints one JSON line
per K.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-soccer_amd"))


def run(total: int, parts: int, steps: int, warmup: int, max_steps: int, join: bool):
    import torch
    from marlsoccer import SoccerBatch
    from marlsoccer.config import load_config

    cfg = None
    if max_steps != 1000:
        cfg = load_config()
        cfg["simulation"]["max_steps"] = max_steps
    per = total // parts
    batches, launches = [], []
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1000)
    nsets = min(steps + warmup, max(1, int(6 * (1 << 30) // (total * 48))))
    for p in range(parts):
        s = torch.cuda.Stream()
        b = SoccerBatch(per, config=cfg, stream=s)
        b.reset(seed=19 + p * per)
        acts = [torch.rand((per, 4, 3), device="cuda", generator=gen) * 2 - 1 for _ in range(nsets)]
        batches.append(b)
        launches.append(b.launcher(acts, b.obs, b.rew, b.term, b.trunc, b.goal, b.score))
    main_s = torch.cuda.current_stream()
    streams = [b.stream for b in batches]
    fork = [torch.cuda.Event() for _ in range(2)]
    done = [torch.cuda.Event() for _ in batches]

    def step(i):
        if join:  # every part waits for the caller's stream, the caller waits for every part
            e = fork[i & 1]
            e.record(main_s)
            for s in streams:
                s.wait_event(e)
        for k, f in enumerate(launches):
            f(i)
            if join:
                done[k].record(streams[k])
        if join:
            for d in done:
                main_s.wait_event(d)

    torch.cuda.synchronize()
    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    for b in batches:
        b.close()
    return {"envs": total, "parts": parts, "join": join, "envs_per_part": per, "max_steps": max_steps, "steps": steps,
            "warmup": warmup, "us_per_step": el * 1e6 / steps, "env_steps_per_s": total * steps / el}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=262144)
    ap.add_argument("--parts", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--max-steps", type=int, default=1000)
    ap.add_argument("--join", action="store_true", help="fork/join every step (the RL-loop contract)")
    a = ap.parse_args()
    for k in a.parts:
        print(json.dumps(run(a.envs, k, a.steps, a.warmup, a.max_steps, a.join)), flush=True)


if __name__ == "__main__":
    main()
