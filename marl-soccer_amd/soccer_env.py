"""Drop-in for soccer_simulation/soccer_env.py (PettingZoo ParallelEnv surface), backed by the
MI355X kernel.

Same names, arguments, return structures and ValueError conditions as the reference
(soccer_env.py:16-221); the env's physics and bookkeeping run on the GPU (a one-env
SoccerBatch with SoccerEnv semantics: no auto-reset, the agent list empties on truncation).
For many envs use marl_vecenv.SyncMultiAgentVecEnv or marlsoccer.SoccerBatch, which step
the whole batch in one kernel launch.
"""
from __future__ import annotations

import numpy as np

from marlsoccer.config import resolve
from marlsoccer.spaces import Box

try:  # pragma: no cover - pettingzoo is not installed in the build image
    from pettingzoo import ParallelEnv  # type: ignore
except Exception:  # noqa: BLE001
    ParallelEnv = object

FRAME_SKIPS = 6  # kept for API parity; unused, as in the reference (soccer_env.py:12)

AGENTS = [f"agent_{i}" for i in range(4)]


class SoccerEnv(ParallelEnv):
    metadata = {"render_modes": ["human", "rgb_array"], "name": "soccer_sim_v1"}

    def __init__(self, render_mode=None, config=None, device=None, **kwargs):
        if "env" in kwargs and kwargs["env"] != 1:
            raise ValueError("SoccerEnv supports only a single environment (env must be 1).")
        if "num_envs" in kwargs and kwargs["num_envs"] != 1:
            raise ValueError("SoccerEnv supports only a single environment (num_envs must be 1).")
        self.render_mode = render_mode
        self.possible_agents = list(AGENTS)
        self.agents = self.possible_agents[:]
        self.agent_name_mapping = {a: i for i, a in enumerate(self.possible_agents)}
        self._action_space = Box(low=-1.0, high=1.0, shape=(3,), dtype=np.float32)
        self._stack_size = 3
        self._frame_size = 22
        self._observation_space = Box(low=-np.inf, high=np.inf, shape=(self._frame_size * self._stack_size,),
                                      dtype=np.float32)
        self._config = resolve(config)
        physics = self._config.get("physics", {})
        self._force_max = float(physics.get("action_force_max", 150000.0))
        self._torque_max = float(physics.get("action_torque_max", 100000.0))
        self._device = device
        self._batch = None  # created on first use: constructing many envs stays cheap
        self._host = None

    # -- lazily bound GPU env ---------------------------------------------------------------
    @property
    def batch(self):
        if self._batch is None:
            from marlsoccer.batch import SoccerBatch
            self._batch = SoccerBatch(1, config=self._config, device=self._device, autoreset=False)
        return self._batch

    def observation_space(self, agent):
        return self._observation_space

    def action_space(self, agent):
        return self._action_space

    def reset(self, seed=None, options=None):
        """Game.reset + 3 identical stacked frames (soccer_env.py:81-98)."""
        self.agents = self.possible_agents[:]
        if seed is not None:
            try:
                seed = int(seed)
                if seed < 0:
                    raise ValueError
            except Exception:  # game.py:84-85: an unusable seed falls back to OS entropy
                from marlsoccer import _native as N
                seed = N.pcg_state_for_seed(None)[None]
        obs = self.batch.reset(seed=seed, options=options).cpu().numpy()[0]
        observations = {a: obs[i].copy() for i, a in enumerate(self.possible_agents)}
        infos = {a: {} for a in self.possible_agents}
        return observations, infos

    def _validate(self, actions) -> np.ndarray:
        expected = list(self.possible_agents)
        missing = [a for a in expected if a not in actions]
        if missing:
            raise ValueError(f"Missing actions for agents: {missing}. Expected actions for {expected}.")
        extra = [a for a in actions.keys() if a not in expected]
        if extra:
            raise ValueError(f"Received actions for unknown agents: {extra}. Expected only {expected}.")
        out = np.zeros((1, 4, 3), np.float32)
        for i, a in enumerate(expected):
            arr = np.asarray(actions.get(a), dtype=np.float32)
            if arr.shape != (3,):
                raise ValueError(f"Action for agent '{a}' must have shape (3,), got {arr.shape}.")
            if not np.all(np.isfinite(arr)):
                raise ValueError(f"Action contains non-finite values for agent '{a}': {arr.tolist()}")
            out[0, i] = arr
        return out

    def step(self, actions):
        """One env step (soccer_env.py:100-154); clipping/scaling happen in the kernel."""
        import torch

        act = self._validate(actions)
        b = self.batch
        if self._host is None:  # pinned staging: actions up, the packed step outputs down
            from marlsoccer.batch import output_views
            self._act_h = torch.empty((1, 4, 3), dtype=torch.float32, pin_memory=True)
            self._host = torch.empty(b.outputs.shape, dtype=torch.uint8, pin_memory=True)
            self._host_views = output_views(self._host.numpy(), 1)
        with torch.cuda.device(b.device), torch.cuda.stream(b.stream):
            self._act_h.numpy()[:] = act
            b.step(self._act_h.to(b.device, non_blocking=True))
            self._host.copy_(b.outputs, non_blocking=True)  # ONE device-to-host copy per step
            b.stream.synchronize()
        hv = self._host_views
        obs = hv["obs"][0]
        r = float(hv["rew"][0, 0])
        done = bool(hv["trunc"][0, 0])
        goal = int(hv["goal"][0])
        sb, sr = (int(x) for x in hv["score"][0])
        observations = {a: obs[i].copy() for i, a in enumerate(self.possible_agents)}
        rewards = {"agent_0": r, "agent_1": r, "agent_2": 0.0, "agent_3": 0.0}
        terminations = {a: False for a in self.possible_agents}
        truncations = {a: done for a in self.possible_agents}
        info = {"score": {"blue": sb, "red": sr}}
        if goal:
            info["goal_scored_by"] = "blue" if goal == 1 else "red"
        infos = {a: dict(info) for a in self.possible_agents}
        if done:
            self.agents = []
        return observations, rewards, terminations, truncations, infos

    def state(self) -> np.ndarray:
        """Full env state record (marl_soccer.h ms_env_state) — not part of the reference."""
        return self.batch.export_state()[0]

    def render(self):
        """soccer_env.py:156-162. "rgb_array" returns the (600, 800, 3) uint8 frame; "human"
        shows it in a pygame window when pygame is installed (the reference's renderer.py
        draws with pygame too), else raises — there is no silent no-op."""
        if self.render_mode is None:
            return None
        from marlsoccer.render import render_state
        img = render_state(self.batch.export_state()[0])
        if self.render_mode == "rgb_array":
            return img
        try:
            import pygame
        except ImportError as exc:
            raise RuntimeError("render_mode='human' needs pygame, which is not installed; use "
                               "render_mode='rgb_array' (and marlsoccer.render.write_png)") from exc
        if getattr(self, "_screen", None) is None:
            pygame.init()
            self._screen = pygame.display.set_mode((img.shape[1], img.shape[0]))
            pygame.display.set_caption("Soccer Simulation")
        for _ in pygame.event.get():
            pass
        pygame.surfarray.blit_array(self._screen, img.transpose(1, 0, 2))
        pygame.display.flip()
        return None

    def close(self):
        if getattr(self, "_screen", None) is not None:
            import pygame
            pygame.display.quit()
            self._screen = None
        if self._batch is not None:
            self._batch.close()
            self._batch = None


def soccer_raw_env(**kwargs):
    """The raw, unwrapped environment (soccer_env.py:174-178)."""
    return SoccerEnv(**kwargs)


def soccerenv(**kwargs):
    """soccer_env.py:181-187 (no wrapper is applied there either)."""
    return soccer_raw_env(**kwargs)


def make_env(**kwargs):
    return soccerenv(**kwargs)


def get_observation_scalers(env):
    """Scales used by the observation encoding (soccer_env.py:200-221)."""
    cfg = env._config if hasattr(env, "_config") else env.config
    physics = cfg.get("physics", {})
    max_velocity = float(physics.get("max_velocity", 400.0))
    max_ang_vel = float(physics.get("max_angular_velocity", physics.get("action_torque_max", 100000.0) / 100.0))
    return {
        "max_velocity": max_velocity,
        "max_angular_velocity": max_ang_vel,
        "field_diagonal": float((800 ** 2 + 600 ** 2) ** 0.5),
        "stack_size": getattr(env, "_stack_size", 3),
        "frame_size": getattr(env, "_frame_size", 22),
    }
