"""Policy evaluation, batched: the reference's eval.py loop (eval.py:69-120) with its episodes
run as parallel envs on the GPU instead of one after another on the CPU.

eval.py plays `num_episodes` episodes: the blue agents (agent_0, agent_1) take the actor mean of
the normalised observation (`np.clip((obs - mean) / (std + 1e-8), -10, 10)`, float32), the red
agents uniform(-1, 1) actions; it sums each blue agent's rewards over the episode and reads
the final score from the infos of the last step. Every episode ends at `max_steps` (there are
no terminations), so the episodes here are one batch of envs stepped `max_steps` times,
without auto-reset.
"""
from __future__ import annotations

import torch

from .batch import SoccerBatch
from .rollout import ACT_DIM, OBS_DIM, TRAINABLE, Agent, RunningMeanStd


@torch.no_grad()
def evaluate(agent: Agent, normalizer: RunningMeanStd, num_episodes: int, seed=None, config: dict | None = None,
             device=None, red: str = "uniform", generator_seed: int = 0, frames_every: int = 0,
             frame_envs=(0,)) -> dict:
    """Returns {"returns": (E, 2) float64 per-episode reward sums of agent_0/agent_1,
    "score": (E, 2) int (blue, red) at the end, "steps": episode length, "frames": list of
    (step, uint8 (K, 600, 800, 3)) rasters of `frame_envs` every `frames_every` steps}.

    seed: None (OS entropy, like eval.py's env.reset()) or int s (episode i seeded s + i).
    red: "uniform" (eval.py) or "zero" (deterministic, for tests)."""
    batch = SoccerBatch(int(num_episodes), config=config, device=device, autoreset=False)
    try:
        dev = batch.device
        n = batch.num_envs
        max_steps = int(batch.config["simulation"]["max_steps"])
        if max_steps <= 0:
            raise ValueError("evaluate() needs a config with max_steps > 0 (episodes end by truncation)")
        gen = torch.Generator(device=dev)
        gen.manual_seed(generator_seed)
        batch.reset(seed=seed)
        acts = torch.zeros((n, 4, ACT_DIM), dtype=torch.float32, device=dev)
        returns = torch.zeros((n, 2), dtype=torch.float64, device=dev)
        frames = []
        if frames_every:
            from .render import render_batch
        for t in range(max_steps):
            x = normalizer.normalize(batch.obs[:, list(TRAINABLE)].reshape(-1, OBS_DIM))
            acts[:, :2] = agent.get_deterministic_action(x).reshape(n, 2, ACT_DIM)
            if red == "uniform":
                acts[:, 2:] = torch.rand((n, 2, ACT_DIM), generator=gen, device=dev) * 2.0 - 1.0
            elif red != "zero":
                raise ValueError(f"red must be 'uniform' or 'zero', got {red!r}")
            out = batch.step(acts)
            returns += out.rew[:, :2].to(torch.float64)
            if frames_every and (t % frames_every == 0 or t == max_steps - 1):
                frames.append((t, render_batch(batch, list(frame_envs)).cpu().numpy()))
        score = batch.score.clone()
        return {"returns": returns.cpu().numpy(), "score": score.cpu().numpy(), "steps": max_steps,
                "frames": frames}
    finally:
        batch.close()
