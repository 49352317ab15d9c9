#!/usr/bin/env python3
"""Host-boundary throughput: SyncMultiAgentVecEnv with numpy actions in and numpy obs / rewards /
flags / lazy infos out (marl_vecenv.py's API), i.e. the PCIe-inclusive rate of the drop-in, next
to the device-resident step_tensors rate on the same envs.

    python tools/bench_vecenv.py [--envs 4096 65536] [--steps 50] [--warmup 5]

Prints one JSON line per env count.
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
    ap.add_argument("--envs", type=int, nargs="+", default=[4096, 65536])
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import torch
    from marl_vecenv import SyncMultiAgentVecEnv
    from soccer_env import soccerenv

    for n in a.envs:
        venv = SyncMultiAgentVecEnv([lambda: soccerenv() for _ in range(n)])
        venv.reset(seed=19)
        rng = np.random.default_rng(7)
        acts = [rng.uniform(-1, 1, (n, 4, 3)).astype(np.float32) for _ in range(8)]
        for i in range(a.warmup):
            venv.step(acts[i % 8])
        t0 = time.perf_counter()
        for i in range(a.steps):
            obs, rew, term, trunc, infos = venv.step(acts[i % 8])
        host_s = (time.perf_counter() - t0) / a.steps
        dacts = [torch.from_numpy(x).to(venv.batch.device) for x in acts]
        for i in range(a.warmup):
            venv.step_tensors(dacts[i % 8])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            venv.step_tensors(dacts[i % 8])
        torch.cuda.synchronize()
        dev_s = (time.perf_counter() - t0) / a.steps
        print(json.dumps({"envs": n, "numpy_step_ms": host_s * 1e3, "numpy_env_steps_per_s": n / host_s,
                          "device_step_ms": dev_s * 1e3, "device_env_steps_per_s": n / dev_s,
                          "host_bytes_per_step": n * (48 + 1056 + 4 * 8 + 4 + 4 + 1 + 8),
                          "note": "numpy path: actions H2D, obs/rew/flags/score/goal D2H every step"}), flush=True)
        venv.close()


if __name__ == "__main__":
    main()
