"""SoccerBatch: N soccer envs resident on one MI355X, stepped by one fused HIP kernel.

This is the GPU-native form of the reference's batched boundary
(SyncMultiAgentVecEnv over SoccerEnv over Game; marl_vecenv.py:3-80, soccer_env.py:16-171,
game/game.py:10-437). Inputs and outputs are torch tensors on the env's device; nothing
is copied to the host unless the caller asks.

    batch = SoccerBatch(65536, device=0)
    obs = batch.reset(seed=19)                       # (N, 4, 66) f32, seeds 19 + i
    obs, rew, term, trunc, goal, score = batch.step(actions)   # actions (N, 4, 3) f32
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _native as N
from .config import resolve, to_ms_config

MODE_BY_OPTION = {"use_fixed_positions": N.SPAWN_FIXED, "use_full_random_positions": N.SPAWN_FULL_RANDOM}


def spawn_mode(options) -> int:
    """SoccerEnv.reset options -> spawn mode (soccer_env.py:83-89, game.py:109-114)."""
    if isinstance(options, dict):
        if bool(options.get("use_fixed_positions", False)):
            return N.SPAWN_FIXED
        if bool(options.get("use_full_random_positions", False)):
            return N.SPAWN_FULL_RANDOM
    return N.SPAWN_RANDOM


class StepOutput(tuple):
    """(obs, rew, term, trunc, goal, score) device tensors."""

    __slots__ = ()
    obs = property(lambda s: s[0])
    rew = property(lambda s: s[1])
    term = property(lambda s: s[2])
    trunc = property(lambda s: s[3])
    goal = property(lambda s: s[4])
    score = property(lambda s: s[5])


# (name, dtype, per-env shape) of the packed step-output buffer, in order
OUTPUT_LAYOUT = (("obs", torch.float32, (4, 66)), ("rew", torch.float32, (4,)), ("term", torch.uint8, (4,)),
                 ("trunc", torch.uint8, (4,)), ("score", torch.int32, (2,)), ("goal", torch.int8, ()))


def _region_bytes(n: int, dtype, shape) -> int:
    k = n * dtype.itemsize
    for d in shape:
        k *= d
    return (k + 15) // 16 * 16


def output_bytes(n: int) -> int:
    return sum(_region_bytes(n, dt, sh) for _, dt, sh in OUTPUT_LAYOUT)


def output_views(buf, n: int) -> dict:
    """Typed views of a packed output buffer (a torch uint8 tensor or a numpy uint8 array)."""
    out, off = {}, 0
    for name, dt, sh in OUTPUT_LAYOUT:
        k = _region_bytes(n, dt, sh)
        size = n * dt.itemsize * int(np.prod(sh, dtype=np.int64))
        part = buf[off:off + size]
        if isinstance(buf, torch.Tensor):
            out[name] = part.view(dt).view((n,) + sh)
        else:
            out[name] = part.view(torch.empty((), dtype=dt).numpy().dtype).reshape((n,) + sh)
        off += k
    return out


class SoccerBatch:
    """N independent 2v2 soccer envs on one HIP device.

    autoreset=True gives SyncMultiAgentVecEnv semantics (a finished env restarts with the
    full-random spawn inside step and returns its reset obs); autoreset=False gives
    SoccerEnv semantics (the caller resets).
    """

    def __init__(self, num_envs: int, config: dict | None = None, device=None, autoreset: bool = True,
                 stream: torch.cuda.Stream | None = None):
        if not torch.cuda.is_available():
            raise RuntimeError("SoccerBatch needs a HIP device (MI355X); there is no CPU fallback")
        self.config = resolve(config)
        self.num_envs = int(num_envs)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   (device if isinstance(device, int) else torch.device(device).index or 0))
        self.autoreset = bool(autoreset)
        self._L = N.lib()
        self._cfg = to_ms_config(self.config, self.autoreset)
        with torch.cuda.device(self.device):
            self.stream = stream if stream is not None else torch.cuda.current_stream(self.device)
            h = C.c_void_p()
            N.check(self._L.ms_create(C.byref(self._cfg), self.num_envs, self.device.index,
                                      C.c_void_p(self.stream.cuda_stream), C.byref(h)), "ms_create")
        self._h = h
        n, dev = self.num_envs, self.device
        # The step outputs are views of ONE device buffer (OUTPUT_LAYOUT), so a host copy of a
        # whole step is one transfer (SoccerEnv.step). Every region starts 16-B aligned (the
        # obs region is a multiple of 16 B for any n).
        self.outputs = torch.zeros((output_bytes(n),), dtype=torch.uint8, device=dev)
        v = output_views(self.outputs, n)
        self.obs, self.rew, self.term, self.trunc = v["obs"], v["rew"], v["term"], v["trunc"]
        self.score, self.goal = v["score"], v["goal"]
        self._out_ptrs = None

    # ---- lifecycle ---------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.ms_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order varies
        try:
            self.close()
        except Exception:
            pass

    def _ptr(self, t: torch.Tensor | None):
        if t is None:
            return None
        if t.device != self.device:
            raise ValueError(f"tensor on {t.device}, env on {self.device}")
        if not t.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return C.c_void_p(t.data_ptr())

    # ---- stream ordering ---------------------------------------------------------------
    # Kernels run on self.stream. Inputs are produced, and outputs consumed, on the caller's
    # current stream; when the two differ the env's stream waits for the caller's work before a
    # launch and the caller's stream waits for the launch after it, and temporaries made for
    # the launch are recorded on the env's stream so the caching allocator cannot hand their
    # blocks out while the kernel still reads them.
    def _enter(self):
        cur = torch.cuda.current_stream(self.device)
        if cur != self.stream:
            self.stream.wait_stream(cur)
            return cur
        return None

    def _leave(self, cur, *temps):
        if cur is not None:
            for t in temps:
                if t is not None:
                    t.record_stream(self.stream)
            cur.wait_stream(self.stream)

    # ---- API ---------------------------------------------------------------------------
    def reset(self, seed=None, options=None, mask: torch.Tensor | None = None, out: torch.Tensor | None = None):
        """Game.reset for every env (or the envs selected by `mask`).

        seed: None (keep each env's RNG stream; reset(seed=None)), an int s (env i gets
        default_rng(s + i), marl_vecenv.py:23) or an (N, 4) uint64 array of PCG64 states.
        """
        mode = spawn_mode(options)
        pcg_t = None
        if seed is not None:
            if isinstance(seed, (int, np.integer)):
                pcg = N.pcg_states_for_range(int(seed), self.num_envs)
            else:
                pcg = np.ascontiguousarray(seed, dtype=np.uint64).reshape(self.num_envs, 4)
            pcg_t = torch.from_numpy(pcg.view(np.int64)).to(self.device)
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        obs = self.obs if out is None else out
        with torch.cuda.device(self.device):
            cur = self._enter()
            N.check(self._L.ms_reset(self._h, self._ptr(pcg_t), self._ptr(m), mode, self._ptr(obs)), "ms_reset")
            self._leave(cur, pcg_t, m)
        return obs

    def step(self, actions: torch.Tensor, check: bool = False) -> StepOutput:
        """One env.step for all envs; actions (N, 4, 3) float32 on the env's device.

        An env whose actions are not all finite is not stepped: its reward and observation come
        back NaN, its term / trunc / goal 0 and its score unchanged (defined values, so no stale
        episode end is read), and the library counts it (ms_get_stats). check=True synchronises and raises the
        reference's ValueError (soccer_env.py:116-117) for the first such env; otherwise call
        raise_if_nonfinite() at a point that synchronises anyway (DeviceRollout does, once
        per rollout)."""
        if actions.shape != (self.num_envs, 4, 3):
            raise ValueError(f"actions must have shape ({self.num_envs}, 4, 3), got {tuple(actions.shape)}")
        if actions.dtype != torch.float32:
            actions = actions.float()
        if actions.device != self.device:
            raise ValueError(f"tensor on {actions.device}, env on {self.device}")
        actions = actions.contiguous()
        if self._out_ptrs is None:  # the output tensors live as long as the batch
            self._out_ptrs = tuple(self._ptr(t) for t in (self.obs, self.rew, self.term, self.trunc, self.goal,
                                                           self.score))
        # ms_step launches on the handle's stream; the HIP calls inside need the env's device
        # current (switch only when it is not)
        if torch.cuda.current_device() == self.device.index:
            cur = self._enter()
            rc = self._L.ms_step(self._h, C.c_void_p(actions.data_ptr()), *self._out_ptrs)
            self._leave(cur, actions)
        else:
            with torch.cuda.device(self.device):
                cur = self._enter()
                rc = self._L.ms_step(self._h, C.c_void_p(actions.data_ptr()), *self._out_ptrs)
                self._leave(cur, actions)
        if rc:
            N.check(rc, "ms_step")
        if check:
            self.raise_if_nonfinite(actions)
        return StepOutput((self.obs, self.rew, self.term, self.trunc, self.goal, self.score))

    def step_n(self, actions: torch.Tensor, out: dict | None = None, check: bool = False) -> StepOutput:
        """K consecutive steps with the actions given up front (ms_step_n): actions (K, N, 4, 3)
        float32 on the env's device, e.g. a random-action rollout. Returns the K steps' outputs
        with a leading K dimension (obs (K, N, 4, 66), rew (K, N, 4), term / trunc (K, N, 4),
        goal (K, N), score (K, N, 2)); `out` may hold any of those tensors to write into. Bit for
        bit what K step() calls return; with the lane-pair and lane-group kernels (the defaults) the K
        steps are one launch. An env-step skipped for a non-finite action writes step()'s defined
        values into its slot (NaN obs and rewards, term / trunc / goal 0, the current score);
        check=True synchronises and raises the reference's ValueError for the first such env, as
        step(check=True) does. The check covers every env-step since the last check (or
        reset_stats()), as raise_if_nonfinite does: a non-finite action handed to an earlier
        unchecked step() / step_n() raises here too, and the message then says that the action
        was not in this call's tensor."""
        if actions.dim() != 4 or actions.shape[1:] != (self.num_envs, 4, 3):
            raise ValueError(f"actions must have shape (K, {self.num_envs}, 4, 3), got {tuple(actions.shape)}")
        K = int(actions.shape[0])
        if K < 1:
            raise ValueError("step_n: K >= 1 steps")
        if actions.dtype != torch.float32:
            actions = actions.float()
        if actions.device != self.device:
            raise ValueError(f"tensor on {actions.device}, env on {self.device}")
        actions = actions.contiguous()
        o = dict(out or {})
        n, dev = self.num_envs, self.device
        for name, dt, sh in OUTPUT_LAYOUT:
            t = o.get(name)
            if t is None:
                o[name] = torch.empty((K, n) + sh, dtype=dt, device=dev)
            elif t.shape != (K, n) + sh or t.dtype != dt or t.device != dev or not t.is_contiguous():
                raise ValueError(f"out[{name!r}] must be a contiguous {dt} tensor of shape {(K, n) + sh} on {dev}")
        with torch.cuda.device(self.device):
            cur = self._enter()
            rc = self._L.ms_step_n(self._h, K, self._ptr(actions), self._ptr(o["obs"]), self._ptr(o["rew"]),
                                   self._ptr(o["term"]), self._ptr(o["trunc"]), self._ptr(o["goal"]),
                                   self._ptr(o["score"]))
            self._leave(cur, actions)
        N.check(rc, "ms_step_n")
        if check:
            st = self.stats()
            if st["nonfinite_envs"]:
                e = st["first_nonfinite_env"]
                bad = (~torch.isfinite(actions[:, e]).all(dim=-1)).any(dim=-1).nonzero()
                if bad.numel():
                    self.raise_if_nonfinite(actions[int(bad[0, 0])])
                self.reset_stats()
                raise ValueError(f"Action contains non-finite values (env {e}, in an earlier unchecked step, "
                                 f"not in this step_n call's actions; {st['nonfinite_envs']} env-step(s) not stepped)")
        return StepOutput((o["obs"], o["rew"], o["term"], o["trunc"], o["goal"], o["score"]))

    def raise_if_nonfinite(self, actions: torch.Tensor | None = None) -> None:
        """Raise the reference's ValueError (soccer_env.py:116-117) if any env was handed a
        non-finite action since the last check (synchronises the env's stream), then clear
        the count. `actions`, when given, is the step's action tensor, used to name the agent
        and its values as the reference's message does."""
        st = self.stats()
        if st["nonfinite_envs"] == 0:
            return
        self.reset_stats()
        e = st["first_nonfinite_env"]
        agent, vals = "agent_?", None
        if actions is not None:
            row = actions[e].detach().float().cpu().numpy()
            bad = np.flatnonzero(~np.isfinite(row).all(axis=1))
            a = int(bad[0]) if bad.size else 0
            agent, vals = f"agent_{a}", row[a].tolist()
        raise ValueError(f"Action contains non-finite values for agent '{agent}': {vals}"
                         f" (env {e}; {st['nonfinite_envs']} env(s) not stepped)")

    def step_into(self, actions: torch.Tensor, obs: torch.Tensor, rew=None, term=None, trunc=None, goal=None,
                  score=None) -> None:
        """ms_step with caller-owned output tensors (any may be None except obs)."""
        with torch.cuda.device(self.device):
            cur = self._enter()
            N.check(self._L.ms_step(self._h, self._ptr(actions), self._ptr(obs), self._ptr(rew), self._ptr(term),
                                    self._ptr(trunc), self._ptr(goal), self._ptr(score)), "ms_step")
            self._leave(cur, actions)

    def launcher(self, actions: list, obs: torch.Tensor, rew=None, term=None, trunc=None, goal=None, score=None):
        """Pre-bound ms_step for a hot loop: returns f(i) that steps with actions[i % len]
        into the given tensors. All argument conversion happens once, here; each call is
        one ctypes call (no device switch: call from the env's current device)."""
        if torch.cuda.current_device() != self.device.index:
            raise RuntimeError("launcher(): make the env's device current (torch.cuda.set_device)")
        fn, h = self._L.ms_step, self._h
        outs = tuple(self._ptr(t) for t in (obs, rew, term, trunc, goal, score))
        acts = [self._ptr(a.contiguous()) for a in actions]
        keep = (actions, obs, rew, term, trunc, goal, score)
        n = len(acts)

        def step(i: int) -> None:
            rc = fn(h, acts[i % n], *outs)
            if rc:
                N.check(rc, "ms_step")

        step._keepalive = keep  # the tensors must outlive the pointers
        return step

    def observe(self) -> torch.Tensor:
        """Current frame of every agent, (N, 4, 22) (Game._get_observations)."""
        out = torch.empty((self.num_envs, 4, 22), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            cur = self._enter()
            N.check(self._L.ms_observe(self._h, self._ptr(out)), "ms_observe")
            self._leave(cur)
        return out

    @property
    def specialised(self) -> int:
        """The step kernel's specialisation (ms_config_specialised): 1 = compiled for the reference's
        default physics and rewards, 2 = default physics with runtime reward multipliers, 0 = generic."""
        return N.config_specialised(self._cfg)

    def export_state_raw(self) -> torch.Tensor:
        """Full per-env state as raw ms_env_state records on the device: uint8 (N, itemsize),
        ordered on the batch's stream (no synchronisation)."""
        buf = torch.empty((self.num_envs, N.ENV_STATE_DTYPE.itemsize), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            cur = self._enter()
            N.check(self._L.ms_export_state(self._h, self._ptr(buf)), "ms_export_state")
            self._leave(cur)
        return buf

    def export_state(self) -> np.ndarray:
        """Full per-env state as a numpy ms_env_state record array (synchronises)."""
        host = self.export_state_raw().cpu().numpy()
        return host.view(N.ENV_STATE_DTYPE).reshape(self.num_envs)

    def import_state(self, state: np.ndarray) -> None:
        st = np.ascontiguousarray(state, dtype=N.ENV_STATE_DTYPE).reshape(self.num_envs)
        buf = torch.from_numpy(st.view(np.uint8).reshape(self.num_envs, -1).copy()).to(self.device)
        with torch.cuda.device(self.device):
            cur = self._enter()
            N.check(self._L.ms_import_state(self._h, self._ptr(buf)), "ms_import_state")
            self._leave(cur, buf)
        self.synchronize()

    def debug_rewards(self, prev_pos, cur_pos, goal, terminal, score) -> torch.Tensor:
        d = self.device
        pv = torch.as_tensor(np.ascontiguousarray(prev_pos, np.float32)).to(d)
        cu = torch.as_tensor(np.ascontiguousarray(cur_pos, np.float32)).to(d)
        g = torch.as_tensor(np.ascontiguousarray(goal, np.int8)).to(d)
        t = torch.as_tensor(np.ascontiguousarray(terminal, np.uint8)).to(d)
        s = torch.as_tensor(np.ascontiguousarray(score, np.int32)).to(d)
        out = torch.empty((self.num_envs, 2), dtype=torch.float32, device=d)
        with torch.cuda.device(self.device):
            cur = self._enter()
            N.check(self._L.ms_debug_rewards(self._h, *(self._ptr(x) for x in (pv, cu, g, t, s, out))),
                    "ms_debug_rewards")
            self._leave(cur, pv, cu, g, t, s)
        return out

    def stats(self) -> dict:
        st = N.MsStats()
        N.check(self._L.ms_get_stats(self._h, C.byref(st)), "ms_get_stats")
        return {"arbiter_overflow": int(st.arbiter_overflow), "nonfinite_envs": int(st.nonfinite_envs),
                "first_nonfinite_env": int(st.first_nonfinite_env), "env_steps": int(st.env_steps),
                "cache_entries_read": int(st.cache_entries_read),
                "cache_entries_written": int(st.cache_entries_written)}

    def reset_stats(self) -> None:
        N.check(self._L.ms_reset_stats(self._h), "ms_reset_stats")

    def set_lane_group(self, lanes: int = -1) -> None:
        """ms_step's kernel (ms_set_lane_group): lanes = 8 or 16 steps each env with a group of
        that many lanes (small batches: loads, per-body work, pair tests, prestep and frames
        spread over the group); 2: a lane pair per env, two waves per SIMD (batches that fill
        the device); 0: one lane per env; -1: automatic (the library's choice by batch size,
        `step_kernel` names it). Results are identical either way."""
        N.check(self._L.ms_set_lane_group(self._h, int(lanes)), "ms_set_lane_group")

    @property
    def lane_group(self) -> int:
        return int(self._L.ms_get_lane_group(self._h))

    def set_group_solve(self, mode: int = 0) -> None:
        """The lane-group kernel's contact-solve schedule (ms_set_group_solve): 0 automatic, 1
        serial in canonical order, 2 rounds by dependency level. Results are identical in every
        mode (the GPU parity tests run each)."""
        N.check(self._L.ms_set_group_solve(self._h, int(mode)), "ms_set_group_solve")

    @property
    def group_solve(self) -> int:
        return int(self._L.ms_get_group_solve(self._h))

    @property
    def step_kernel(self) -> str:
        """Name of the kernel the next step launches (ms_step_kernel_name), as rocprofv3 lists it.
        A library without that symbol (an older build timed by tools/variants.py) is named from
        its lane group instead."""
        if not hasattr(self._L, "ms_step_kernel_name"):
            g = self.lane_group
            return "ms_step_pair_kernel" if g == 2 else ("ms_step_group_kernel" if g > 2 else "ms_step_kernel")
        return self._L.ms_step_kernel_name(self._h).decode()

    def synchronize(self) -> None:
        self.stream.synchronize()

    def set_stream(self, stream: torch.cuda.Stream) -> None:
        """Launch subsequent calls on `stream` (e.g. a graph-capture stream; ms_set_stream)."""
        N.check(self._L.ms_set_stream(self._h, C.c_void_p(stream.cuda_stream)), "ms_set_stream")
        self.stream = stream


class FrameRingBatch(SoccerBatch):
    """SoccerBatch whose stacked observation is a window into a per-agent ring of R frames
    (ms_step_ring / ms_reset_ring): a step writes 352 B of obs per env instead of 1,056 B.

    The step's observation is `self.obs`, an (N, 4, 66) view of `self.frames` (N, 4, R, 22)
    with a row stride of R * 22 floats: frames pos..pos+2 = t-2, t-1, t, the same values the
    contiguous layout holds (soccer_env.py:130-140). The view is valid until the next step or
    reset moves the window; copy it (or index the ring with `window_index`) to keep it. Every
    R - 2 steps the window moves back to the ring's start and that step writes all three
    frames. An env not stepped because of a non-finite action writes no frame, and the window
    still advances: its window holds a stale frame (zeros or one from R - 2 steps back) until two
    more valid steps have pushed it out, whereas SoccerBatch's contiguous step writes defined
    values for such an env (ABI 5: an all-NaN obs row, NaN rewards, term / trunc / goal 0 and the
    current score). Both raise via raise_if_nonfinite; after catching that ValueError, call
    reset(mask=...) for that env before reading its window again.
    """

    def __init__(self, num_envs: int, ring: int = 32, **kw):
        super().__init__(num_envs, **kw)
        ring = int(ring)
        if ring < 4 or ring % 2:
            raise ValueError(f"ring must be even and >= 4, got {ring}")
        if not hasattr(self._L, "ms_step_ring"):
            raise RuntimeError("libmarlsoccer.so predates ms_step_ring; rebuild it")
        self.ring = ring
        self.frames = torch.zeros((self.num_envs, 4, ring, 22), dtype=torch.float32, device=self.device)
        self._rows = self.frames.view(self.num_envs, 4, ring * 22)
        self.pos = 0
        self.obs = self._window(0)
        # the packed buffer's obs region is not written by the ring kernels
        self._ring_ptrs = None

    def _window(self, pos: int) -> torch.Tensor:
        return self._rows[:, :, 22 * pos:22 * pos + 66]

    def window_index(self) -> int:
        """Ring slot of frame t-2 of the current observation."""
        return self.pos

    def next_window(self, pos: int) -> tuple[int, int]:
        """(pos, wrap) of the step after one whose window starts at `pos`."""
        return (pos + 1, 0) if pos + 4 <= self.ring else (0, 1)

    def reset(self, seed=None, options=None, mask: torch.Tensor | None = None, out=None):
        """SoccerBatch.reset; the reset frame fills the current window (all envs: the window
        moves to the ring's start)."""
        if out is not None:
            raise ValueError("FrameRingBatch.reset writes into the ring (out= is not supported)")
        mode = spawn_mode(options)
        pcg_t = None
        if seed is not None:
            if isinstance(seed, (int, np.integer)):
                pcg = N.pcg_states_for_range(int(seed), self.num_envs)
            else:
                pcg = np.ascontiguousarray(seed, dtype=np.uint64).reshape(self.num_envs, 4)
            pcg_t = torch.from_numpy(pcg.view(np.int64)).to(self.device)
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        else:
            self.pos = 0
        with torch.cuda.device(self.device):
            cur = self._enter()
            N.check(self._L.ms_reset_ring(self._h, self._ptr(pcg_t), self._ptr(m), mode,
                                          C.c_void_p(self.frames.data_ptr()), self.ring, self.pos), "ms_reset_ring")
            self._leave(cur, pcg_t, m)
        self.obs = self._window(self.pos)
        return self.obs

    def step(self, actions: torch.Tensor, check: bool = False) -> StepOutput:
        if actions.shape != (self.num_envs, 4, 3):
            raise ValueError(f"actions must have shape ({self.num_envs}, 4, 3), got {tuple(actions.shape)}")
        if actions.dtype != torch.float32:
            actions = actions.float()
        if actions.device != self.device:
            raise ValueError(f"tensor on {actions.device}, env on {self.device}")
        actions = actions.contiguous()
        if self._ring_ptrs is None:
            self._ring_ptrs = tuple(self._ptr(t) for t in (self.rew, self.term, self.trunc, self.goal, self.score))
        pos, wrap = self.next_window(self.pos)
        with torch.cuda.device(self.device):
            cur = self._enter()
            rc = self._L.ms_step_ring(self._h, C.c_void_p(actions.data_ptr()), C.c_void_p(self.frames.data_ptr()),
                                      self.ring, pos, wrap, *self._ring_ptrs)
            self._leave(cur, actions)
        if rc:
            N.check(rc, "ms_step_ring")
        self.pos = pos
        self.obs = self._window(pos)
        if check:
            self.raise_if_nonfinite(actions)
        return StepOutput((self.obs, self.rew, self.term, self.trunc, self.goal, self.score))

    def step_into(self, *a, **kw):
        raise NotImplementedError("FrameRingBatch writes observations into its ring; use step()")

    def launcher(self, actions: list, rew=None, term=None, trunc=None, goal=None, score=None):
        """Pre-bound ms_step_ring for a hot loop (SoccerBatch.launcher without obs): f(i)
        steps with actions[i % len] and advances the window (self.pos and the self.obs view,
        as step() does)."""
        if torch.cuda.current_device() != self.device.index:
            raise RuntimeError("launcher(): make the env's device current (torch.cuda.set_device)")
        fn, h, R, fr = self._L.ms_step_ring, self._h, self.ring, C.c_void_p(self.frames.data_ptr())
        outs = tuple(self._ptr(t) for t in (rew, term, trunc, goal, score))
        acts = [self._ptr(a.contiguous()) for a in actions]
        keep = (actions, rew, term, trunc, goal, score)
        n = len(acts)

        def step(i: int) -> None:
            pos, wrap = self.next_window(self.pos)
            rc = fn(h, acts[i % n], fr, R, pos, wrap, *outs)
            if rc:
                N.check(rc, "ms_step_ring")
            self.pos = pos
            self.obs = self._window(pos)

        step._keepalive = keep
        return step
