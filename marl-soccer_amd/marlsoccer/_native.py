"""ctypes binding of libmarlsoccer.so (include/marl_soccer.h).

The library is the ONLY compute path: there is no CPU fallback. Loading fails loudly
when the .so is missing, and every handle needs a HIP device.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MARL_SOCCER_LIB", os.path.join(PKG_ROOT, "lib", "libmarlsoccer.so"))

MS_OK = 0
MS_ERR_INVALID_ARGUMENT = 1
MS_ERR_HIP = 2
MS_ERR_OUT_OF_MEMORY = 3
MS_ERR_NONFINITE_ACTION = 4
MS_ERR_NO_DEVICE = 5

SPAWN_RANDOM, SPAWN_FULL_RANDOM, SPAWN_FIXED = 0, 1, 2
MAX_ARBITERS = 32

CONFIG_FIELDS = (
    "max_velocity", "agent_mass", "ball_mass", "agent_moment", "ball_moment",
    "agent_friction", "ball_friction", "agent_elasticity", "agent_surface_friction",
    "ball_elasticity", "ball_surface_friction", "action_force_max", "action_torque_max",
    "max_angular_velocity", "ball_proximity_multiplier", "move_ball_to_goal_multiplier",
    "alive_penalty", "goal_scored_reward", "goal_conceded_penalty", "score_difference_multiplier",
)


class MsConfig(C.Structure):
    _fields_ = [(n, C.c_double) for n in CONFIG_FIELDS] + [("max_steps", C.c_int32), ("autoreset", C.c_int32)]

    def as_dict(self) -> dict:
        return {n: getattr(self, n) for n, _ in self._fields_}


class MsStats(C.Structure):
    _fields_ = [("arbiter_overflow", C.c_uint64), ("nonfinite_envs", C.c_uint64),
                ("first_nonfinite_env", C.c_int64), ("env_steps", C.c_uint64), ("cache_entries_read", C.c_uint64),
                ("cache_entries_written", C.c_uint64)]


class MsPolicyIO(C.Structure):
    """ms_policy_io (include/marl_soccer.h): device pointers of one policy-kernel launch."""
    _fields_ = [("obs", C.c_void_p), ("rows", C.c_int64), ("group_rows", C.c_int32), ("pad0", C.c_int32),
                ("group_stride", C.c_int64), ("row_stride", C.c_int64), ("mean", C.c_void_p), ("den", C.c_void_p),
                ("actor", C.c_void_p), ("critic", C.c_void_p), ("logstd", C.c_void_p), ("eps", C.c_void_p),
                ("act_mean", C.c_void_p), ("action", C.c_void_p), ("logprob", C.c_void_p), ("value", C.c_void_p),
                ("obs_copy", C.c_void_p), ("env_actions", C.c_void_p), ("red_uniform", C.c_void_p)]


# numpy view of ms_env_state (include/marl_soccer.h), for export/import
BODY_DTYPE = np.dtype([(n, "<f4") for n in ("px", "py", "vx", "vy", "angle", "w", "vbx", "vby", "wb")])
ARB_DTYPE = np.dtype([("pair", "u1"), ("count", "u1"), ("idle", "u1"), ("pad0", "u1"),
                      ("hash", "u1", (2,)), ("pad1", "u1", (2,)), ("jn", "<f4", (2,)), ("jt", "<f4", (2,))])
ENV_STATE_DTYPE = np.dtype([
    ("body", BODY_DTYPE, (5,)), ("snap", "<f4", (2, 26)),
    ("steps", "<i4"), ("score_blue", "<i4"), ("score_red", "<i4"),
    ("mode", "u1"), ("hist_empty", "u1"), ("n_arb", "u1"), ("has_uint32", "u1"),
    ("uinteger", "<u4"), ("pad", "<u4"),
    ("pcg_state_hi", "<u8"), ("pcg_state_lo", "<u8"), ("pcg_inc_hi", "<u8"), ("pcg_inc_lo", "<u8"),
    ("arb", ARB_DTYPE, (MAX_ARBITERS,)),
], align=True)

EXPORTED = (
    "ms_config_default", "ms_create", "ms_destroy", "ms_set_stream", "ms_num_envs", "ms_seed_pcg64",
    "ms_seed_pcg64_range", "ms_reset", "ms_step", "ms_observe", "ms_export_state", "ms_import_state",
    "ms_debug_rewards", "ms_get_stats", "ms_reset_stats", "ms_last_error", "ms_abi_version",
    "ms_config_specialised", "ms_step_ring", "ms_reset_ring", "ms_step_n",
    "ms_set_lane_group", "ms_get_lane_group", "ms_set_group_solve", "ms_get_group_solve", "ms_step_kernel_name",
    "ms_policy_forward", "ms_policy_last_error", "ms_policy_run", "ms_rollout_record",
)

_lib = None


class NativeError(RuntimeError):
    pass


def lib():
    """Load libmarlsoccer.so (HIP runtime shared with torch: import torch first)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"marl-soccer MI355X library not found at {LIB_PATH}; build it with "
            "`python marl-soccer_amd/build_native.py` (hipcc, gfx950)")
    try:  # share torch's HIP runtime (same SONAME) when torch is present
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is a hard dependency of the batch API
        pass
    L = C.CDLL(LIB_PATH)
    P, I64 = C.c_void_p, C.c_int64
    L.ms_config_default.argtypes = [C.POINTER(MsConfig)]
    L.ms_config_default.restype = None
    L.ms_create.argtypes = [C.POINTER(MsConfig), I64, C.c_int, P, C.POINTER(P)]
    L.ms_destroy.argtypes = [P]
    L.ms_set_stream.argtypes = [P, P]
    L.ms_num_envs.argtypes = [P]
    L.ms_num_envs.restype = I64
    L.ms_seed_pcg64.argtypes = [P, C.c_int, P]
    L.ms_seed_pcg64_range.argtypes = [C.c_uint64, I64, P]
    L.ms_reset.argtypes = [P, P, P, C.c_int, P]
    L.ms_step.argtypes = [P, P, P, P, P, P, P, P]
    L.ms_observe.argtypes = [P, P]
    L.ms_export_state.argtypes = [P, P]
    L.ms_import_state.argtypes = [P, P]
    L.ms_debug_rewards.argtypes = [P, P, P, P, P, P, P]
    L.ms_get_stats.argtypes = [P, C.POINTER(MsStats)]
    L.ms_reset_stats.argtypes = [P]
    L.ms_last_error.restype = C.c_char_p
    L.ms_abi_version.restype = C.c_int
    if hasattr(L, "ms_config_specialised"):  # absent only in older builds timed by tools/variants.py
        L.ms_config_specialised.argtypes = [C.POINTER(MsConfig)]
        L.ms_config_specialised.restype = C.c_int
    if hasattr(L, "ms_step_ring"):  # likewise
        L.ms_step_ring.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int, P, P, P, P, P]
        L.ms_step_ring.restype = C.c_int
        L.ms_reset_ring.argtypes = [P, P, P, C.c_int, P, C.c_int, C.c_int]
        L.ms_reset_ring.restype = C.c_int
    if hasattr(L, "ms_step_n"):  # likewise (ABI 4)
        L.ms_step_n.argtypes = [P, C.c_int, P, P, P, P, P, P, P]
        L.ms_step_n.restype = C.c_int
    if hasattr(L, "ms_set_lane_group"):  # likewise
        L.ms_set_lane_group.argtypes = [P, C.c_int]
        L.ms_set_lane_group.restype = C.c_int
        L.ms_get_lane_group.argtypes = [P]
        L.ms_get_lane_group.restype = C.c_int
    if hasattr(L, "ms_step_kernel_name"):
        L.ms_step_kernel_name.argtypes = [P]
        L.ms_step_kernel_name.restype = C.c_char_p
    if hasattr(L, "ms_set_group_solve"):
        L.ms_set_group_solve.argtypes = [P, C.c_int]
        L.ms_set_group_solve.restype = C.c_int
        L.ms_get_group_solve.argtypes = [P]
        L.ms_get_group_solve.restype = C.c_int
    if hasattr(L, "ms_policy_forward"):  # likewise
        L.ms_policy_forward.argtypes = [P, I64, C.c_int, I64, I64, P, P, P, P, P, P, P]
        L.ms_policy_forward.restype = C.c_int
        L.ms_policy_last_error.restype = C.c_char_p
        L.ms_policy_run.argtypes = [C.POINTER(MsPolicyIO), P]
        L.ms_policy_run.restype = C.c_int
        L.ms_rollout_record.argtypes = [I64, P, P, P, P, P, P, P, P, P, P]
        L.ms_rollout_record.restype = C.c_int
    for fn in ("ms_create", "ms_destroy", "ms_set_stream", "ms_seed_pcg64", "ms_seed_pcg64_range", "ms_reset",
               "ms_step", "ms_observe", "ms_export_state", "ms_import_state", "ms_debug_rewards",
               "ms_get_stats", "ms_reset_stats"):
        getattr(L, fn).restype = C.c_int
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc == MS_OK:
        return
    msg = lib().ms_last_error().decode(errors="replace")
    if rc in (MS_ERR_INVALID_ARGUMENT, MS_ERR_NONFINITE_ACTION):
        raise ValueError(f"{what}: {msg}")
    if rc == MS_ERR_NO_DEVICE:
        raise RuntimeError(f"{what}: no HIP device ({msg}); the MI355X env has no CPU fallback")
    raise NativeError(f"{what}: {msg} (status {rc})")


def default_config() -> MsConfig:
    cfg = MsConfig()
    lib().ms_config_default(C.byref(cfg))
    return cfg


def config_specialised(cfg: MsConfig) -> int:
    """The step-kernel specialisation `cfg` selects (ms_config_specialised): 1 = the reference's
    default physics and rewards as compile-time constants, 2 = the default physics with runtime
    reward multipliers (lane-pair and lane-group kernels), 0 = the generic kernel. Same results
    in every case."""
    rc = lib().ms_config_specialised(C.byref(cfg))
    if rc < 0:
        check(-rc, "ms_config_specialised")
    return int(rc)


def _seed_words(seed: int) -> np.ndarray:
    """numpy's _coerce_to_uint32_array for a non-negative Python int."""
    seed = int(seed)
    if seed < 0:
        raise ValueError("seed must be non-negative")
    words = []
    while True:
        words.append(seed & 0xFFFFFFFF)
        seed >>= 32
        if seed == 0:
            break
    return np.array(words, dtype=np.uint32)


def pcg_state_for_seed(seed) -> np.ndarray:
    """np.random.default_rng(seed) -> PCG64 (state_hi, state_lo, inc_hi, inc_lo), computed by
    the library's SeedSequence restatement. seed=None draws OS entropy (128 bits) like
    default_rng()."""
    if seed is None:
        w = np.frombuffer(os.urandom(16), dtype=np.uint32).copy()
    else:
        w = _seed_words(seed)
    out = np.zeros(4, np.uint64)
    check(lib().ms_seed_pcg64(w.ctypes.data, len(w), out.ctypes.data), "ms_seed_pcg64")
    return out


def pcg_states_for_range(seed0: int, n: int) -> np.ndarray:
    """Seeds seed0 + i for i < n (SyncMultiAgentVecEnv.reset, marl_vecenv.py:23)."""
    out = np.zeros((n, 4), np.uint64)
    if seed0 < 0:
        raise ValueError("seed must be non-negative")
    if seed0 + n < (1 << 64):
        check(lib().ms_seed_pcg64_range(C.c_uint64(seed0), n, out.ctypes.data), "ms_seed_pcg64_range")
    else:
        for i in range(n):
            out[i] = pcg_state_for_seed(seed0 + i)
    return out


def symbols_present() -> list:
    """Names of the C-ABI entry points resolvable in the .so (no device needed)."""
    L = C.CDLL(LIB_PATH)
    return [n for n in EXPORTED if hasattr(L, n)]
