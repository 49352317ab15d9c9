#!/usr/bin/env python3
"""Throughput of the device-resident PPO rollout: env + policy.

    python tools/bench_rollout.py [--envs 65536] [--steps 64] [--warmup 8] [--graph] [--bf16]

One rollout step = normalise the blue agents' obs, actor + critic MLP forward (the
reference's 66-512-256-128-64 tanh networks, fp32, random init), sample actions, draw the red
agents' uniform actions, ms_step — everything on the GPU, as marlsoccer.rollout.DeviceRollout
runs it. Prints one JSON line: env-steps/s of the whole rollout, the share of the env kernel
(HIP events around each ms_step launch), and the reference's host rollout rate for context
(≈930-1,430 env-steps/s training-inclusive on one CPU).
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
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--graph", action="store_true",
                    help="DeviceRollout(graph=True): time a replay of the captured rollout graph")
    ap.add_argument("--bf16", action="store_true", help="DeviceRollout(policy_dtype=torch.bfloat16) (opt-in)")
    ap.add_argument("--policy", choices=("fused", "torch"), default=None,
                    help="DeviceRollout(policy=...): the fused ms_policy_forward kernel (fp32 default) or torch")
    a = ap.parse_args()
    import torch
    from marlsoccer import SoccerBatch
    from marlsoccer.rollout import Agent, DeviceRollout, RunningMeanStd

    b = SoccerBatch(a.envs)
    b.reset(seed=19)
    torch.manual_seed(0)
    agent = Agent().cuda().eval()
    rms = RunningMeanStd((66,), device="cuda")
    warm = DeviceRollout(b, agent, rms, a.warmup, seed=1, update_normalizer=False)
    warm.collect()
    if a.graph:
        ro = DeviceRollout(b, agent, rms, a.steps, seed=2, graph=True,
                           policy_dtype=torch.bfloat16 if a.bf16 else torch.float32, policy=a.policy)
        ro.collect()  # eager
        ro.collect()  # capture + first replay
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ro.collect()  # replay
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({
            "metric": "rollout env-steps/s (policy + env on device, one HIP graph per rollout)",
            "value": a.envs * a.steps / dt, "unit": "env-steps/s", "envs": a.envs, "steps": a.steps,
            "ms_per_step": dt * 1e3 / a.steps,
            "policy": "Agent 66-512-256-128-64-{3,1} tanh x2, " + ("bf16 autocast GEMMs" if a.bf16 else "fp32")
                      + f" ({ro.policy}), sampled actions; red uniform(-1,1)",
            "timed": "third collect(): a replay of the graph captured by the second (normaliser update included)",
        }))
        b.close()
        return
    ro = DeviceRollout(b, agent, rms, a.steps, seed=2, policy_dtype=torch.bfloat16 if a.bf16 else torch.float32,
                       policy=a.policy)
    # env-kernel share: events around every ms_step of the timed rollout
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    step_into = b.step_into

    def timed_step_into(*args, _i=[0]):
        s, e = ev[_i[0]]
        s.record()
        step_into(*args)
        e.record()
        _i[0] += 1
    b.step_into = timed_step_into
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ro.collect()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    env_ms = sum(s.elapsed_time(e) for s, e in ev)
    print(json.dumps({
        "metric": "rollout env-steps/s (policy + env on device)", "value": a.envs * a.steps / dt,
        "unit": "env-steps/s", "envs": a.envs, "steps": a.steps, "ms_per_step": dt * 1e3 / a.steps,
        "env_kernel_ms_per_step": env_ms / a.steps, "env_share": env_ms / (dt * 1e3),
        "policy": f"Agent 66-512-256-128-64-{{3,1}} tanh x2, fp32 ({ro.policy}), sampled actions; red uniform(-1,1)",
        "reference_host_rollout_env_steps_per_s": "≈930-1430 (SURVEY.md §6, training-inclusive)",
    }))
    b.close()


if __name__ == "__main__":
    main()
