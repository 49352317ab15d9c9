#!/usr/bin/env python3
"""BASELINE.json configs[0]: ONE env through the PettingZoo surface, random actions, 10k steps.

    python tools/bench_single_env.py [--steps 10000] [--out gpurun_out/single_env.json]

The reference's `soccerenv()` loop (soccer_env.py:181; the notebook's random-play cell and
test_rewards.py drive it this way): dict actions sampled from the action space, step, reset
when the agents list empties (truncation). Here every step is one ms_step launch on a
one-env batch plus ONE host copy of the packed outputs, so the rate is launch- and
PCIe-latency bound, not a throughput figure; SURVEY.md §6 quotes ≈3.4 k steps/s for the
reference's glue alone (pymunk excluded), measured on the survey host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-soccer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import numpy as np
    from soccer_env import soccerenv

    env = soccerenv()
    rng = np.random.default_rng(0)
    env.reset(seed=19)
    episodes = 0

    def run(k):
        nonlocal episodes
        for _ in range(k):
            acts = {ag: rng.uniform(-1, 1, 3).astype(np.float32) for ag in env.possible_agents}
            env.step(acts)
            if not env.agents:
                episodes += 1
                env.reset()

    run(a.warmup)
    t0 = time.perf_counter()
    run(a.steps)
    dt = time.perf_counter() - t0
    line = {"config": "BASELINE.json configs[0]: 1 env via soccerenv(), random actions",
            "steps": a.steps, "seconds": dt, "steps_per_s": a.steps / dt, "us_per_step": dt * 1e6 / a.steps,
            "episodes_finished": episodes,
            "per_step": "validate dict actions, pinned upload, one ms_step launch, ONE packed D2H copy, dict build",
            "reference_context": "SURVEY.md §6: ~3.4 k steps/s for the reference's Python glue alone"}
    print(json.dumps(line), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(line, f, indent=1)
    env.close()


if __name__ == "__main__":
    main()
