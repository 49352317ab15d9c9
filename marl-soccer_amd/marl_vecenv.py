"""Drop-in for soccer_simulation/marl_vecenv.py: SyncMultiAgentVecEnv, batched on the MI355X.

The reference steps its envs one by one in a Python loop (marl_vecenv.py:39-60). Here the
N envs built by `env_fns` are folded into one SoccerBatch and every reset/step is a
single kernel launch. Return values keep the reference's types and shapes:
    reset(options=None, seed=None)  -> obs float32 (N, 4, 66)
    step(actions (N, 4, 3))         -> obs float32 (N, 4, 66), rewards float64 (N, 4),
                                       terminations bool (N, 4), truncations bool (N, 4),
                                       infos: sequence of N {agent: {"score": {...},
                                       ["goal_scored_by": "blue"|"red"]}} (built lazily)
A finished env is reset inside step with the full-random spawn and its returned obs is
the reset obs, while its rewards and infos are the terminal step's (marl_vecenv.py:45-56).

Device-resident fast path (no host copies): reset_tensors / step_tensors / .batch.

Difference (documented): a non-finite action raises ValueError before ANY env is stepped;
the reference raises from the failing env after stepping the envs before it.
"""
from __future__ import annotations

from collections.abc import Sequence

import numpy as np


class LazyInfos(Sequence):
    """infos list of the reference (one dict per env), materialised on access."""

    def __init__(self, score: np.ndarray, goal: np.ndarray, agents):
        self._score = score
        self._goal = goal
        self._agents = list(agents)

    def __len__(self):
        return len(self._goal)

    def _one(self, i: int) -> dict:
        info = {"score": {"blue": int(self._score[i, 0]), "red": int(self._score[i, 1])}}
        g = int(self._goal[i])
        if g:
            info["goal_scored_by"] = "blue" if g == 1 else "red"
        return {a: dict(info) for a in self._agents}

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self._one(k) for k in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        return self._one(i)

    def __eq__(self, other):
        return list(self) == list(other)


class SyncMultiAgentVecEnv:
    """Synchronous multi-agent vector env over N SoccerEnv instances (marl_vecenv.py:3-80)."""

    def __init__(self, env_fns, device=None):
        from marlsoccer.batch import SoccerBatch

        self.envs = [fn() for fn in env_fns]
        if not self.envs:
            raise ValueError("SyncMultiAgentVecEnv needs at least one env")
        cfg = getattr(self.envs[0], "_config", None)
        if cfg is None:
            raise TypeError("env_fns must build marl-soccer SoccerEnv instances (soccer_env.soccerenv)")
        for e in self.envs[1:]:
            if getattr(e, "_config", None) != cfg:
                raise ValueError("all envs of one SyncMultiAgentVecEnv must share one config")
        self.num_envs = len(self.envs)
        a0 = self.envs[0].possible_agents[0]
        self.single_observation_space = self.envs[0].observation_space(a0)
        self.single_action_space = self.envs[0].action_space(a0)
        self.possible_agents = self.envs[0].possible_agents
        self.config = cfg
        self.batch = SoccerBatch(self.num_envs, config=cfg, device=device, autoreset=True)

    # ---- reference API (numpy in / numpy out) ------------------------------------------
    def reset(self, options=None, seed=None):
        """Env i reset with seed + i (or its continuing stream when seed is None)."""
        return self.reset_tensors(options=options, seed=seed).cpu().numpy()

    def step(self, actions):
        import torch

        act = np.asarray(actions, dtype=np.float32)
        if act.ndim != 3 or act.shape[0] != self.num_envs or act.shape[1] != len(self.possible_agents):
            raise ValueError(f"actions must have shape ({self.num_envs}, {len(self.possible_agents)}, 3), "
                             f"got {act.shape}")
        if act.shape[2] != 3:
            raise ValueError(f"Action for agent '{self.possible_agents[0]}' must have shape (3,), got {act.shape[2:]}.")
        bad = ~np.isfinite(act)
        if bad.any():
            e, a, _ = np.argwhere(bad)[0]
            agent = self.possible_agents[a]
            raise ValueError(f"Action contains non-finite values for agent '{agent}': {act[e, a].tolist()}")
        # One round trip per step: the actions go up from a pinned staging copy and every output
        # comes down into fresh pinned buffers (torch's caching host allocator recycles them once
        # the caller drops the arrays), all ordered on the env's stream, then ONE synchronise.
        # rewards are widened to float64 and the flags to bool on the device.
        dev, st = self.batch.device, self.batch.stream
        n = self.num_envs
        with torch.cuda.device(dev), torch.cuda.stream(st):
            a_h = torch.from_numpy(np.ascontiguousarray(act)).pin_memory()
            out = self.batch.step(a_h.to(dev, non_blocking=True))
            obs = torch.empty((n, 4, 66), dtype=torch.float32, pin_memory=True)
            rew = torch.empty((n, 4), dtype=torch.float64, pin_memory=True)
            term = torch.empty((n, 4), dtype=torch.bool, pin_memory=True)
            trunc = torch.empty((n, 4), dtype=torch.bool, pin_memory=True)
            score = torch.empty((n, 2), dtype=torch.int32, pin_memory=True)
            goal = torch.empty((n,), dtype=torch.int8, pin_memory=True)
            obs.copy_(out.obs, non_blocking=True)
            rew.copy_(out.rew.to(torch.float64), non_blocking=True)
            term.copy_(out.term.bool(), non_blocking=True)
            trunc.copy_(out.trunc.bool(), non_blocking=True)
            score.copy_(out.score, non_blocking=True)
            goal.copy_(out.goal, non_blocking=True)
            st.synchronize()
        infos = LazyInfos(score.numpy(), goal.numpy(), self.possible_agents)
        return obs.numpy(), rew.numpy(), term.numpy(), trunc.numpy(), infos

    def close(self):
        for e in self.envs:
            e.close()
        self.batch.close()

    # ---- device-resident fast path ----------------------------------------------------
    def reset_tensors(self, options=None, seed=None):
        return self.batch.reset(seed=seed, options=options)

    def step_tensors(self, actions):
        """actions: torch float32 (N, 4, 3) on the env's device; returns device tensors
        (obs, rew f32, term u8, trunc u8, goal i8, score i32), overwritten by the next step."""
        return self.batch.step(actions)

    def step_n_tensors(self, actions):
        """K steps with the actions given up front (open loop: random or scripted actions):
        actions torch float32 (K, N, 4, 3) on the env's device; returns the K steps' device
        tensors with a leading K dimension, bit-identical to K step_tensors calls (one launch
        for the default kernels: SoccerBatch.step_n, ms_step_n)."""
        return self.batch.step_n(actions)

    def _dict_to_array(self, data_dict):
        return np.array([data_dict[a] for a in self.possible_agents])

    def _array_to_dict(self, data_array):
        return {a: data_array[i] for i, a in enumerate(self.possible_agents)}
