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


GRAPH_CHUNK = 25  # env steps per captured graph (evaluate(graph=True)): fewer graph launches


@torch.no_grad()
def evaluate(agent: Agent, normalizer: RunningMeanStd, num_episodes: int, seed=None, config: dict | None = None,
             device=None, red: str = "uniform", generator_seed: int = 0, frames_every: int = 0,
             frame_envs=(0,), graph: bool = False) -> dict:
    """Returns {"returns": (E, 2) float64 per-episode reward sums of agent_0/agent_1,
    "score": (E, 2) int (blue, red) at the end, "steps": episode length, "frames": list of
    (step, uint8 (K, 600, 800, 3)) rasters of `frame_envs` every `frames_every` steps}.

    seed: None (OS entropy, like eval.py's env.reset()) or int s (episode i seeded s + i).
    red: "uniform" (eval.py) or "zero" (deterministic, for tests).
    graph: run the first steps eagerly, capture GRAPH_CHUNK steps (policy, red actions, ms_step,
    return sums; the loop body does not depend on t) as one HIP graph and replay it for the rest
    of the episode; same results as the eager loop. Not combined with frames_every (host
    rasters)."""
    if red not in ("uniform", "zero"):
        raise ValueError(f"red must be 'uniform' or 'zero', got {red!r}")
    if graph and frames_every:
        raise ValueError("evaluate(): graph=True cannot take frames (frames_every > 0)")
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
        blue = torch.tensor(TRAINABLE, dtype=torch.int64, device=dev)  # on the device: a host index would copy per step

        def body():
            x = normalizer.normalize(batch.obs.index_select(1, blue).reshape(-1, OBS_DIM))
            acts[:, :2] = agent.get_deterministic_action(x).reshape(n, 2, ACT_DIM)
            if red == "uniform":
                acts[:, 2:] = torch.rand((n, 2, ACT_DIM), generator=gen, device=dev) * 2.0 - 1.0
            out = batch.step(acts)
            returns.add_(out.rew[:, :2].to(torch.float64))

        if graph:
            chunk = min(GRAPH_CHUNK, max_steps - 1) if max_steps > 1 else 1
            # eager steps first: step 0 initialises the GEMM libraries before the capture, and the
            # rest of the episode is then a whole number of chunks
            eager = max_steps - chunk * ((max_steps - 1) // chunk) if max_steps > 1 else 1
            for _ in range(eager):
                body()
            replays = (max_steps - eager) // chunk
        if graph and replays > 0:
            g = torch.cuda.CUDAGraph()
            g.register_generator_state(gen)
            cur = torch.cuda.current_stream(dev)
            s = torch.cuda.Stream(dev)
            s.wait_stream(cur)
            old = batch.stream
            batch.set_stream(s)  # ms_step launches on the capture stream
            try:
                with torch.cuda.graph(g, stream=s):
                    for _ in range(chunk):
                        body()  # recorded, not run
            finally:
                batch.set_stream(old)
            cur.wait_stream(s)
            for _ in range(replays):
                g.replay()
        elif not graph:
            for t in range(max_steps):
                body()
                if frames_every and (t % frames_every == 0 or t == max_steps - 1):
                    frames.append((t, render_batch(batch, list(frame_envs)).cpu().numpy()))
        score = batch.score.clone()
        return {"returns": returns.cpu().numpy(), "score": score.cpu().numpy(), "steps": max_steps,
                "frames": frames}
    finally:
        batch.close()
