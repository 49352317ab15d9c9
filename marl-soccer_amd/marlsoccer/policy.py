"""Fused policy forward on the GPU (ms_policy_forward, csrc/ms_policy.hip).

The reference's rollout (marl-soccer.ipynb train cell L299-313) normalises the blue agents'
observations with RunningMeanStd and runs the notebook Agent's actor and critic MLPs
(66-512-256-128-64-{3, 1}, tanh; eval.py:17-47). ms_policy_forward does the normalisation and
both MLPs in one gfx950 kernel on the f32-input MFMA with every activation in registers;
this module packs an Agent's nets into the kernel's weight layout and calls it.

Packed net (MS_POLICY_NET_FLOATS floats): for each Linear layer L (T = 32-feature output tiles,
G = groups of four MFMA k-steps of two input features each):
    W_L[T][G][64 lanes][4]: lane l, k-step s = 4g + j holds W[32T + (l & 31)][in_feature(s, l >> 5)]
    b_L[T][2][16]:          half h, register r holds b[32T + (r & 3) + 8 (r >> 2) + 4h]
with in_feature(s, h) = 2s + h for layer 1 (66 inputs, k-steps 33-35 zero) and
32 (s >> 4) + (s & 3) + 8 ((s & 15) >> 2) + 4h for the later layers (the order in which the
previous layer's 32x32 accumulator tiles hold their features); rows past the layer's width
(the last layer's 3 or 1 outputs) are zero.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _native as N

NET_FLOATS = 211936  # MS_POLICY_NET_FLOATS
_LAYERS = ((66, 512, 16, 9), (512, 256, 8, 64), (256, 128, 4, 32), (128, 64, 2, 16), (64, None, 1, 8))


def _in_feature(layer: int, s: np.ndarray, h: np.ndarray) -> np.ndarray:
    if layer == 0:
        return 2 * s + h
    r = s & 15
    return 32 * (s >> 4) + (r & 3) + 8 * (r >> 2) + 4 * h


def _index_map(n_out: int) -> np.ndarray:
    """Source index of every packed float into the net's flat parameters
    [W1.ravel(), b1, W2.ravel(), b2, ..., W5.ravel(), b5], -1 for zeros."""
    parts, base = [], 0
    for li, (n_in, width, T, G) in enumerate(_LAYERS):
        out = n_out if width is None else width
        t = np.arange(T)[:, None, None, None]
        g = np.arange(G)[None, :, None, None]
        lane = np.arange(64)[None, None, :, None]
        j = np.arange(4)[None, None, None, :]
        s = 4 * g + j
        o = 32 * t + (lane & 31)
        f = _in_feature(li, s, lane >> 5)
        ok = (o < out) & (f < n_in) & (s < (33 if li == 0 else G * 4))
        w = np.where(ok, base + o * n_in + f, -1)
        parts.append(w.reshape(-1))
        base += out * n_in
        tt = np.arange(T)[:, None, None]
        hh = np.arange(2)[None, :, None]
        r = np.arange(16)[None, None, :]
        ob = 32 * tt + (r & 3) + 8 * (r >> 2) + 4 * hh
        parts.append(np.where(ob < out, base + ob, -1).reshape(-1))
        base += out
    idx = np.concatenate(parts)
    assert idx.size == NET_FLOATS, idx.size
    return idx


_MAPS: dict = {}


def pack_net(seq: torch.nn.Sequential) -> torch.Tensor:
    """An Agent MLP (critic or actor_mean: Linear/Tanh x 4, Linear) in the kernel's layout, on
    the parameters' device (a device gather: re-run after every parameter update, or inside a
    captured graph)."""
    lin = [m for m in seq if isinstance(m, torch.nn.Linear)]
    assert len(lin) == 5 and lin[0].in_features == 66, "not the reference Agent's MLP"
    n_out = lin[-1].out_features
    dev = lin[0].weight.device
    key = (n_out, str(dev))
    if key not in _MAPS:
        idx = torch.from_numpy(_index_map(n_out)).to(dev)
        _MAPS[key] = (idx.clamp(min=0), idx >= 0)
    src, ok = _MAPS[key]
    flat = torch.cat([t.reshape(-1) for m in lin for t in (m.weight, m.bias)]).to(torch.float32)
    return torch.where(ok, flat[src], torch.zeros((), dtype=torch.float32, device=dev))


class FusedPolicy:
    """ms_policy_forward for one Agent: pack() after every parameter change (DeviceRollout
    does it once per collect, inside its graph), then forward()."""

    def __init__(self, agent):
        self.agent = agent
        self._L = N.lib()
        dev = agent.critic[0].weight.device
        self.packed = torch.zeros((2, NET_FLOATS), dtype=torch.float32, device=dev)
        self.pack()

    def pack(self) -> None:
        with torch.no_grad():
            self.packed[0].copy_(pack_net(self.agent.actor_mean))
            self.packed[1].copy_(pack_net(self.agent.critic))

    def forward(self, x: torch.Tensor, mean: torch.Tensor | None = None, den: torch.Tensor | None = None,
                act_mean: torch.Tensor | None = None, value: torch.Tensor | None = None,
                group_rows: int = 1, group_stride: int = 66, row_stride: int = 66, rows: int | None = None):
        """Actor mean (rows, 3) and value (rows,) of the rows of x (see include/marl_soccer.h for
        the row addressing); mean/den: float64 (66,) normaliser mean and sqrt(var) + 1e-8, or None
        when x is normalised already."""
        if rows is None:
            rows = x.numel() // 66
        dev = self.packed.device
        if act_mean is None:
            act_mean = torch.empty((rows, 3), dtype=torch.float32, device=dev)
        if value is None:
            value = torch.empty((rows,), dtype=torch.float32, device=dev)
        for t in (x, act_mean, value, mean, den):
            if t is not None and (t.device != dev or not t.is_contiguous()):
                raise ValueError("ms_policy_forward: tensors must be contiguous on the policy's device")
        if x.dtype != torch.float32 or (mean is not None and (mean.dtype != torch.float64 or den.dtype != torch.float64)):
            raise ValueError("ms_policy_forward: x float32, mean/den float64")
        stream = torch.cuda.current_stream(dev).cuda_stream
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        rc = self._L.ms_policy_forward(p(x), rows, group_rows, group_stride, row_stride, p(mean), p(den),
                                       C.c_void_p(self.packed[0].data_ptr()), C.c_void_p(self.packed[1].data_ptr()),
                                       p(act_mean), p(value), C.c_void_p(stream))
        if rc:
            raise (ValueError if rc == N.MS_ERR_INVALID_ARGUMENT else N.NativeError)(
                self._L.ms_policy_last_error().decode(errors="replace"))
        return act_mean, value

    def run(self, obs: torch.Tensor, rows: int, group_rows: int, group_stride: int, row_stride: int = 66,
            mean: torch.Tensor | None = None, den: torch.Tensor | None = None, eps: torch.Tensor | None = None,
            act_mean=None, action=None, logprob=None, value=None, obs_copy=None, env_actions=None,
            red_uniform: torch.Tensor | None = None) -> None:
        """ms_policy_run: one launch with every output of a rollout step (include/marl_soccer.h);
        the output tensors are written in place (None: not written). eps: standard-normal draws
        (rows, 3) for sampled actions (Agent.sample with the agent's actor_logstd), or None for the
        deterministic mean. red_uniform: uniform [0, 1) draws (rows, 3) written as 2u - 1 into the
        red agents' rows of env_actions."""
        dev = self.packed.device
        for t in (obs, mean, den, eps, act_mean, action, logprob, value, obs_copy, env_actions, red_uniform):
            if t is not None and (t.device != dev or not t.is_contiguous()):
                raise ValueError("ms_policy_run: tensors must be contiguous on the policy's device")
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        io = N.MsPolicyIO(obs=p(obs), rows=int(rows), group_rows=int(group_rows), pad0=0, group_stride=int(group_stride),
                          row_stride=int(row_stride), mean=p(mean), den=p(den), actor=self.packed[0].data_ptr(),
                          critic=self.packed[1].data_ptr(),
                          logstd=None if eps is None else self.logstd.data_ptr(), eps=p(eps),
                          act_mean=p(act_mean), action=p(action), logprob=p(logprob), value=p(value),
                          obs_copy=p(obs_copy), env_actions=p(env_actions), red_uniform=p(red_uniform))
        rc = self._L.ms_policy_run(C.byref(io), C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
        if rc:
            raise (ValueError if rc == N.MS_ERR_INVALID_ARGUMENT else N.NativeError)(
                self._L.ms_policy_last_error().decode(errors="replace"))

    @property
    def logstd(self) -> torch.Tensor:
        """The agent's actor_logstd (1, 3) float32, contiguous (read in place)."""
        return self.agent.actor_logstd


def rollout_record(rew: torch.Tensor, term: torch.Tensor, trunc: torch.Tensor, score: torch.Tensor,
                   rewards: torch.Tensor, next_done: torch.Tensor, dones_next: torch.Tensor | None,
                   episodes: torch.Tensor, score_sum: torch.Tensor) -> None:
    """ms_rollout_record (include/marl_soccer.h): a rollout step's storage and episode counters
    from ms_step's (N, 4) outputs in one launch — rewards (N, 2) = rew[:, :2], next_done (and
    dones_next) = float(term | trunc)[:, :2], and for every env whose episode ended
    (trunc[:, 0]) episodes += 1, score_sum += score (int64)."""
    n = rew.shape[0]
    shapes = ((rew, (n, 4), torch.float32), (term, (n, 4), torch.uint8), (trunc, (n, 4), torch.uint8),
              (score, (n, 2), torch.int32), (rewards, (n, 2), torch.float32), (next_done, (n, 2), torch.float32),
              (dones_next, (n, 2), torch.float32), (episodes, (), torch.int64), (score_sum, (2,), torch.int64))
    for t, shape, dtype in shapes:
        if t is None:
            continue
        if tuple(t.shape) != shape or t.dtype != dtype or not t.is_contiguous() or t.device != rew.device:
            raise ValueError(f"ms_rollout_record: expected a contiguous {dtype} {shape} tensor on {rew.device}")
    L = N.lib()
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    rc = L.ms_rollout_record(n, p(rew), p(term), p(trunc), p(score), p(rewards), p(next_done), p(dones_next),
                             p(episodes), p(score_sum), C.c_void_p(torch.cuda.current_stream(rew.device).cuda_stream))
    if rc:
        raise (ValueError if rc == N.MS_ERR_INVALID_ARGUMENT else N.NativeError)(
            L.ms_policy_last_error().decode(errors="replace"))
