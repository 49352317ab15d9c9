"""ctypes wrapper of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker. The product (marl-soccer_amd/) never imports this module.

The oracle restates the reference's hot path (see soccer_oracle.c's header for the
file:line map). Two builds:
  precision="f64"  reference precision; pinned against tests/golden/ fixtures
  precision="f32"  the HIP kernel's arithmetic contract (bit-exact target)
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


class MsConfig(C.Structure):
    """Mirror of include/marl_soccer.h ms_config."""

    _fields_ = [(n, C.c_double) for n in (
        "max_velocity", "agent_mass", "ball_mass", "agent_moment", "ball_moment",
        "agent_friction", "ball_friction", "agent_elasticity", "agent_surface_friction",
        "ball_elasticity", "ball_surface_friction", "action_force_max", "action_torque_max",
        "max_angular_velocity", "ball_proximity_multiplier", "move_ball_to_goal_multiplier",
        "alive_penalty", "goal_scored_reward", "goal_conceded_penalty",
        "score_difference_multiplier")] + [("max_steps", C.c_int32), ("autoreset", C.c_int32)]


# numpy mirror of ms_env_state (include/marl_soccer.h)
BODY_DTYPE = np.dtype([(n, "<f4") for n in ("px", "py", "vx", "vy", "angle", "w", "vbx", "vby", "wb")])
ARB_DTYPE = np.dtype([("pair", "u1"), ("count", "u1"), ("idle", "u1"), ("pad0", "u1"),
                      ("hash", "u1", (2,)), ("pad1", "u1", (2,)), ("jn", "<f4", (2,)), ("jt", "<f4", (2,))])
MAX_ARB = 32
ENV_STATE_DTYPE = np.dtype([
    ("body", BODY_DTYPE, (5,)), ("snap", "<f4", (2, 26)),
    ("steps", "<i4"), ("score_blue", "<i4"), ("score_red", "<i4"),
    ("mode", "u1"), ("hist_empty", "u1"), ("n_arb", "u1"), ("has_uint32", "u1"),
    ("uinteger", "<u4"), ("pad", "<u4"),
    ("pcg_state_hi", "<u8"), ("pcg_state_lo", "<u8"), ("pcg_inc_hi", "<u8"), ("pcg_inc_lo", "<u8"),
    ("arb", ARB_DTYPE, (MAX_ARB,)),
], align=True)


def default_config(**overrides) -> MsConfig:
    cfg = MsConfig()
    lib = load("f64")
    lib.orc_config_default(C.byref(cfg))
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg


_LIBS: dict = {}


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load(precision: str):
    if precision in _LIBS:
        return _LIBS[precision]
    path = os.path.join(HERE, f"liborc_{precision}.so")
    if not os.path.exists(path):
        build()
    _LIBS[precision] = load_path(path)
    return _LIBS[precision]


def load_path(path: str):
    """Bind an oracle build at `path` (tests/test_precision.py's mutant builds use this)."""
    lib = C.CDLL(path)
    P = C.c_void_p
    lib.orc_config_default.argtypes = [P]
    lib.orc_params_init.argtypes = [P, P]
    for fn in ("orc_sizeof_params", "orc_sizeof_space", "orc_sizeof_env", "orc_sizeof_body"):
        getattr(lib, fn).restype = C.c_int
    lib.orc_space_phase1.argtypes = [P, P]
    lib.orc_space_phase2.argtypes = [P, P]
    lib.orc_space_update_velocities.argtypes = [P, P]
    lib.orc_space_step.argtypes = [P, P]
    lib.orc_space_clear_arbiters.argtypes = [P]
    lib.orc_observe_space.argtypes = [P, P, P]
    lib.orc_debug_rewards.argtypes = [P, C.c_int, P, P, P, P, P, P]
    lib.orc_env_reset.argtypes = [P, P, P, C.c_int, P]
    lib.orc_env_step.argtypes = [P, P, P, P, P, P, P, P]
    lib.orc_env_step.restype = C.c_int
    lib.orc_batch_reset.argtypes = [P, C.c_int, P, P, C.c_int, P]
    lib.orc_batch_step.argtypes = [P, C.c_int, P, P, P, P, P, P, P]
    lib.orc_batch_step.restype = C.c_int
    lib.orc_batch_export.argtypes = [P, C.c_int, P]
    lib.orc_batch_import.argtypes = [P, C.c_int, P]
    lib.orc_batch_observe.argtypes = [P, C.c_int, P, P]
    lib.orc_batch_overflow.argtypes = [P, C.c_int]
    lib.orc_batch_overflow.restype = C.c_ulonglong
    lib.orc_batch_positions.argtypes = [P, C.c_int, P]
    lib.orc_batch_rng.argtypes = [P, C.c_int, P]
    lib.orc_batch_soft_reset.argtypes = [P, C.c_int]
    lib.orc_batch_ncontacts.argtypes = [P, C.c_int, P]
    lib.orc_cpu_baseline.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_uint64]
    lib.orc_cpu_baseline.restype = C.c_double
    lib.orc_precision.restype = C.c_char_p
    return lib


def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data) if a is not None else None


class OracleBatch:
    """N independent oracle envs with the batched (SyncMultiAgentVecEnv) interface."""

    def __init__(self, n: int, precision: str = "f32", config: MsConfig | None = None, lib=None):
        self.lib = load(precision) if lib is None else lib
        self.n = n
        self.cfg = config if config is not None else default_config()
        self.params = (C.c_char * self.lib.orc_sizeof_params())()
        self.lib.orc_params_init(C.byref(self.cfg), self.params)
        self.envs = (C.c_char * (self.lib.orc_sizeof_env() * n))()

    def reset(self, pcg: np.ndarray | None, mode: int = 0) -> np.ndarray:
        obs = np.zeros((self.n, 4, 66), np.float32)
        pcg_arr = None if pcg is None else np.ascontiguousarray(pcg, dtype=np.uint64).reshape(self.n, 4)
        self.lib.orc_batch_reset(self.envs, self.n, self.params, _ptr(pcg_arr), mode, _ptr(obs))
        return obs

    def step(self, actions: np.ndarray):
        act = np.ascontiguousarray(actions, dtype=np.float32).reshape(self.n, 4, 3)
        obs = np.zeros((self.n, 4, 66), np.float32)
        rew = np.zeros((self.n, 4), np.float64)
        trunc = np.zeros((self.n, 4), np.uint8)
        goal = np.zeros((self.n,), np.int8)
        score = np.zeros((self.n, 2), np.int32)
        bad = self.lib.orc_batch_step(self.envs, self.n, self.params, _ptr(act), _ptr(obs), _ptr(rew),
                                      _ptr(trunc), _ptr(goal), _ptr(score))
        return obs, rew, trunc.astype(bool), goal, score, bad

    def export_state(self) -> np.ndarray:
        out = np.zeros((self.n,), ENV_STATE_DTYPE)
        self.lib.orc_batch_export(self.envs, self.n, _ptr(out))
        return out

    def import_state(self, st: np.ndarray) -> None:
        st = np.ascontiguousarray(st, dtype=ENV_STATE_DTYPE)
        assert st.shape == (self.n,)
        self.lib.orc_batch_import(self.envs, self.n, _ptr(st))

    def observe(self) -> np.ndarray:
        out = np.zeros((self.n, 4, 22), np.float32)
        self.lib.orc_batch_observe(self.envs, self.n, self.params, _ptr(out))
        return out

    def positions(self) -> np.ndarray:
        out = np.zeros((self.n, 5, 2), np.float64)
        self.lib.orc_batch_positions(self.envs, self.n, _ptr(out))
        return out

    def rng_state(self) -> np.ndarray:
        out = np.zeros((self.n, 6), np.uint64)
        self.lib.orc_batch_rng(self.envs, self.n, _ptr(out))
        return out

    def soft_reset(self) -> None:
        self.lib.orc_batch_soft_reset(self.envs, self.n)

    def ncontacts(self) -> np.ndarray:
        out = np.zeros((self.n,), np.int32)
        self.lib.orc_batch_ncontacts(self.envs, self.n, _ptr(out))
        return out

    def overflow(self) -> int:
        return int(self.lib.orc_batch_overflow(self.envs, self.n))

    def debug_rewards(self, prev_pos, cur_pos, goal, terminal, score) -> np.ndarray:
        n = len(goal)
        pv = np.ascontiguousarray(prev_pos, np.float32)
        cu = np.ascontiguousarray(cur_pos, np.float32)
        g = np.ascontiguousarray(goal, np.int8)
        t = np.ascontiguousarray(terminal, np.uint8)
        s = np.ascontiguousarray(score, np.int32)
        rew = np.zeros((n, 2), np.float64)
        self.lib.orc_debug_rewards(self.params, n, _ptr(pv), _ptr(cu), _ptr(g), _ptr(t), _ptr(s), _ptr(rew))
        return rew


def pcg_from_seed(seed: int) -> np.ndarray:
    """numpy default_rng(seed) PCG64 state as (state_hi, state_lo, inc_hi, inc_lo)."""
    st = np.random.default_rng(seed).bit_generator.state["state"]
    s, i = int(st["state"]), int(st["inc"])
    m = (1 << 64) - 1
    return np.array([s >> 64, s & m, i >> 64, i & m], dtype=np.uint64)


def cpu_baseline(n_envs: int, n_steps: int, threads: int, precision: str = "f64", seed: int = 19) -> float:
    """Wall seconds for n_envs x n_steps oracle env-steps on `threads` host threads."""
    lib = load(precision)
    cfg = default_config()
    params = (C.c_char * lib.orc_sizeof_params())()
    lib.orc_params_init(C.byref(cfg), params)
    return float(lib.orc_cpu_baseline(params, n_envs, n_steps, threads, seed))
