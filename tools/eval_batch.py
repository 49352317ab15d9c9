#!/usr/bin/env python3
"""eval.py, batched on the GPU: load a checkpoint and normaliser in the reference's formats
(runs/<run>/ppo_pettingzoo_soccer.ppo_model, latest_normalizer_stats.npz) and play N episodes
at once (blue: actor mean, red: uniform random), printing per-episode returns and scores as
eval.py does; optionally PNG frames of episode 0.

    python tools/eval_batch.py --model RUN/ppo_pettingzoo_soccer.ppo_model \
        --normalizer RUN/latest_normalizer_stats.npz [--episodes 5] [--seed S] [--png-dir DIR] [--graph]
Without --model the policy is randomly initialised (a smoke run). --graph replays one captured
step (evaluate(graph=True)); the wall time of the evaluation is printed last.
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-soccer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default=None)
    ap.add_argument("--normalizer", default=None)
    ap.add_argument("--episodes", type=int, default=5)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--png-dir", default=None)
    ap.add_argument("--png-every", type=int, default=60)
    ap.add_argument("--graph", action="store_true", help="evaluate(graph=True) (no PNG frames)")
    ap.add_argument("--quiet", action="store_true", help="print only the summary lines")
    a = ap.parse_args()
    import numpy as np
    import torch
    from marlsoccer.evaluate import evaluate
    from marlsoccer.render import write_png
    from marlsoccer.rollout import Agent, RunningMeanStd

    agent = Agent().cuda()
    if a.model:
        agent.load_state_dict(torch.load(a.model, map_location="cuda", weights_only=True))
    agent.eval()
    rms = RunningMeanStd.load_npz(a.normalizer, device="cuda") if a.normalizer else RunningMeanStd(device="cuda")
    import time
    if a.quiet:  # a timing run: initialise the GEMM libraries and kernels outside the timed call
        evaluate(agent, rms, 8, seed=0, graph=a.graph)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = evaluate(agent, rms, a.episodes, seed=a.seed, frames_every=a.png_every if a.png_dir else 0, graph=a.graph)
    wall = time.perf_counter() - t0
    for ep in range(0 if a.quiet else a.episodes):
        r = res["returns"][ep]
        print(f"Episode {ep + 1}: steps={res['steps']} return agent_0={r[0]:.4f} agent_1={r[1]:.4f} "
              f"score blue={int(res['score'][ep, 0])} red={int(res['score'][ep, 1])}")
    print(f"mean return {float(np.mean(res['returns'])):.4f} over {a.episodes} episodes")
    print(f"wall {wall:.3f} s for {a.episodes} episodes x {res['steps']} steps "
          f"({a.episodes * res['steps'] / wall / 1e6:.3f} M env-steps/s{', graph' if a.graph else ''})")
    if a.png_dir:
        os.makedirs(a.png_dir, exist_ok=True)
        for t, imgs in res["frames"]:
            write_png(os.path.join(a.png_dir, f"ep0_step{t:04d}.png"), imgs[0])


if __name__ == "__main__":
    main()
