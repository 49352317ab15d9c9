"""Deterministic action sources shared by the oracle/GPU parity tests."""
import numpy as np


def hash_actions(n_envs: int, step: int, env0: int = 0, seed: int = 1234) -> np.ndarray:
    """uniform(-1, 1) float32 actions (n_envs, 4, 3), a pure function of (global env, step).

    Integer splitmix64 in numpy: the same values for any sharding of the env range.
    """
    e = (np.arange(n_envs, dtype=np.uint64) + np.uint64(env0))[:, None]
    k = np.arange(12, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) + e * np.uint64(0xD1B54A32D192ED03)
             + np.uint64(step) * np.uint64(0x8CB92BA72F3D8DD7) + k * np.uint64(0x94D049BB133111EB))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(40)).astype(np.float64) * (2.0 / 16777216.0) - 1.0
    return u.astype(np.float32).reshape(n_envs, 4, 3)


def chase_actions(pos: np.ndarray, angle: np.ndarray, rng: np.random.Generator, chaser: np.ndarray) -> np.ndarray:
    """Goal-seeking actions for agent `chaser[e]` of each env (others random).

    pos (n, 5, 2) positions, angle (n, 4). Blue chasers push the ball toward x=790, red
    toward x=10; produces frequent goals, soft resets and agent-ball/agent-wall contacts.
    """
    n = pos.shape[0]
    acts = rng.uniform(-1, 1, (n, 4, 3)).astype(np.float32)
    idx = np.arange(n)
    p = pos[idx, chaser].astype(np.float64)
    ball = pos[:, 4].astype(np.float64)
    goal = np.where((chaser < 2)[:, None], np.array([790.0, 300.0]), np.array([10.0, 300.0]))
    tg = goal - ball
    tg /= np.linalg.norm(tg, axis=1, keepdims=True) + 1e-9
    behind = ball - 24.0 * tg
    d = behind - p
    close = (np.linalg.norm(d, axis=1) < 6.0) | ((np.sum((ball - p) * tg, axis=1) > 0) & (np.linalg.norm(ball - p, axis=1) < 30))
    d = np.where(close[:, None], ball - p + 20 * tg, d)
    d /= np.linalg.norm(d, axis=1, keepdims=True) + 1e-9
    a = angle[idx, chaser].astype(np.float64)
    c, s = np.cos(a), np.sin(a)
    local = np.stack([c * d[:, 0] + s * d[:, 1], -s * d[:, 0] + c * d[:, 1]], axis=1)
    acts[idx, chaser, :2] = np.clip(local * 1.2, -1, 1).astype(np.float32)
    acts[idx, chaser, 2] = 0.0
    return acts
