#!/usr/bin/env python3
"""Policy forward variants for the device rollout (diagnostic): the reference's actor + critic
(66-512-256-128-64-{3,1} tanh) on M = 2 x envs rows, timed with HIP events.

    python tools/bench_policy.py [--envs 65536] [--iters 20]

a) nn.Sequential fp32 (hipBLASLt GEMMs + tanh passes), b) both MLPs as one 66->1024 GEMM +
batched (2, M, k) GEMMs per layer (fp32), c) a) under bf16 autocast, d) b) in bf16, e) the
fused gfx950 kernel ms_policy_forward (f32-input MFMA, activations in registers; marlsoccer.policy),
f) e) with the RunningMeanStd normalisation fused (raw rows in, float64 normalisation in-kernel),
g) ms_policy_run as DeviceRollout launches it: the env's (N, 4, 66) obs rows of the blue agents,
sampling, log-prob, obs storage copy and the env's action rows.
Prints ms per forward and the max |difference| of the action mean and value against a).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-soccer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch
    from marlsoccer.rollout import Agent

    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    agent = Agent().to(dev)
    M = 2 * a.envs
    x = torch.randn(M, 66, device=dev).clamp(-10, 10)

    def seq():
        return agent.actor_mean(x), agent.critic(x)

    lin_c = [m for m in agent.critic if isinstance(m, torch.nn.Linear)]
    lin_a = [m for m in agent.actor_mean if isinstance(m, torch.nn.Linear)]

    def pack(dtype):
        W1 = torch.cat([lin_c[0].weight, lin_a[0].weight]).t().contiguous().to(dtype)
        b1 = torch.cat([lin_c[0].bias, lin_a[0].bias]).to(dtype)
        mids = [(torch.stack([lin_c[i].weight.t(), lin_a[i].weight.t()]).contiguous().to(dtype),
                 torch.stack([lin_c[i].bias, lin_a[i].bias])[:, None, :].to(dtype)) for i in (1, 2, 3)]
        lasts = [(lin_c[4].weight.t().contiguous().to(dtype), lin_c[4].bias.to(dtype)),
                 (lin_a[4].weight.t().contiguous().to(dtype), lin_a[4].bias.to(dtype))]
        return W1, b1, mids, lasts

    def fused(p, dtype):
        W1, b1, mids, lasts = p
        h = torch.tanh(torch.addmm(b1, x.to(dtype), W1))           # (M, 1024)
        h = h.view(M, 2, 512).transpose(0, 1)                       # (2, M, 512)
        for W, b in mids:
            h = torch.tanh(torch.baddbmm(b, h, W))
        v = torch.addmm(lasts[0][1], h[0], lasts[0][0])
        mu = torch.addmm(lasts[1][1], h[1], lasts[1][0])
        return mu.float(), v.float()

    p32, p16 = pack(torch.float32), pack(torch.bfloat16)
    from marlsoccer.policy import FusedPolicy
    fp = FusedPolicy(agent)
    am = torch.empty((M, 3), device=dev)
    vv = torch.empty((M,), device=dev)
    mean0 = torch.zeros(66, dtype=torch.float64, device=dev)
    den1 = torch.full((66,), 1.0 + 1e-8, dtype=torch.float64, device=dev)

    def kern():
        fp.forward(x, act_mean=am, value=vv)
        return am, vv[:, None]

    def kern_norm():
        fp.forward(x, mean0, den1, act_mean=am, value=vv)
        return am, vv[:, None]

    # the rollout step's launch (DeviceRollout): (N, 4, 66) env obs rows, sampling, every output
    xo = torch.randn(a.envs, 4, 66, device=dev).clamp(-10, 10)
    eps = torch.randn(M, 3, device=dev)
    red = torch.rand(M, 3, device=dev)
    act, lp, obs_copy = torch.empty((M, 3), device=dev), torch.empty((M,), device=dev), torch.empty((M, 66), device=dev)
    env_act = torch.empty((a.envs, 4, 3), device=dev)

    def kern_rollout():
        fp.run(xo, M, 2, 264, 66, mean0, den1, eps=eps, act_mean=am, action=act, logprob=lp, value=vv,
               obs_copy=obs_copy, env_actions=env_act, red_uniform=red)
        return am, vv[:, None]

    variants = {
        "sequential_fp32": seq,
        "fused_fp32": lambda: fused(p32, torch.float32),
        "sequential_bf16_autocast": lambda: torch.autocast("cuda", dtype=torch.bfloat16)(seq)(),
        "fused_bf16": lambda: fused(p16, torch.bfloat16),
        "ms_policy_forward": kern,
        "ms_policy_forward_normalising": kern_norm,
        "ms_policy_run_rollout_io": kern_rollout,
    }
    with torch.no_grad():
        ref_mu, ref_v = seq()
        xb = xo[:, :2].reshape(M, 66)
        refs = {"ms_policy_run_rollout_io": (agent.actor_mean(xb), agent.critic(xb))}
        for name, fn in variants.items():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                mu, v = fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            print(json.dumps({"variant": name, "rows": M, "ms_per_forward": ms, "tflops": 824192 * 2 * M / 2 / ms / 1e9,
                              "max_abs_diff_mean": float((mu.float() - refs.get(name, (ref_mu,))[0]).abs().max()),
                              "max_abs_diff_value": float((v.float() - refs.get(name, (0, ref_v))[1]).abs().max())}),
                  flush=True)


if __name__ == "__main__":
    main()
