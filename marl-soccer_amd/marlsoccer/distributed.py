"""Env sharding across GPUs: one process per GPU, contiguous global env ranges.

Envs are independent, so the step has no data-path collective: every rank steps its own
shard with one kernel launch. Env g (global index) is always seeded seed + g, so results
are bit-identical for any world size. The only collective is the optional whole-batch
obs concatenation for a policy that lives on one device (RCCL all-gather over xGMI,
BASELINE configs[3]); it runs outside the step.
"""
from __future__ import annotations

import os


def shard_range(global_envs: int, world: int, rank: int) -> tuple:
    """(start, count) of rank's contiguous shard; the first global_envs % world ranks get
    one extra env."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(int(global_envs), int(world))
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def dist_env() -> tuple:
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


# per-env step-output record for the whole-batch gather: obs (4, 66) f32, rew (4,) f32,
# term (4,) u8, trunc (4,) u8, goal () i8, score (2,) i32 — 1,089 bytes, packed as raw bytes so
# that one collective moves all of them
_FIELDS = (("obs", (4, 66), "float32"), ("rew", (4,), "float32"), ("term", (4,), "uint8"),
           ("trunc", (4,), "uint8"), ("goal", (), "int8"), ("score", (2,), "int32"))


def _nbytes(shape, dtype):
    import numpy as np
    return int(np.prod(shape, dtype=np.int64)) * np.dtype(dtype).itemsize


RECORD_BYTES = sum(_nbytes(sh, dt) for _, sh, dt in _FIELDS)


def pack_step_outputs(out: dict):
    """{obs, rew, term, trunc, goal, score} tensors of n envs -> uint8 (n, RECORD_BYTES), one
    device copy per field."""
    import torch
    n = out["obs"].shape[0]
    parts = [out[name].contiguous().view(torch.uint8).reshape(n, -1) for name, _, _ in _FIELDS]
    return torch.cat(parts, dim=1)


def unpack_step_outputs(buf) -> dict:
    """Inverse of pack_step_outputs: views into buf (m, RECORD_BYTES)."""
    import torch
    m, off, out = buf.shape[0], 0, {}
    for name, shape, dt in _FIELDS:
        nb = _nbytes(shape, dt)
        out[name] = buf[:, off:off + nb].contiguous().view(getattr(torch, dt)).reshape((m,) + tuple(shape))
        off += nb
    return out


def all_gather_rows(buf, world: int, group=None):
    """Concatenate every rank's (n, k) tensor along dim 0 (equal n): all_gather_into_tensor on
    RCCL, the list form on backends without it (gloo: the CPU tests and the shared-GPU
    rehearsal, whose device tensors are staged through host memory because gloo's all_gather
    takes CPU tensors only). The result is on buf's device."""
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        dst = torch.empty((world * buf.shape[0],) + tuple(buf.shape[1:]), dtype=buf.dtype, device=buf.device)
        dist.all_gather_into_tensor(dst, buf, group=group)
        return dst
    src = buf.cpu() if buf.is_cuda else buf
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src, group=group)
    out = torch.cat(parts, dim=0)
    return out.to(buf.device) if buf.is_cuda else out


class ShardedSoccerEnv:
    """This rank's shard of a global batch of envs on its own GPU.

    global_envs envs are split with shard_range; rank r owns [start, start + count), each
    env seeded with its GLOBAL index (marl_vecenv.py:18-28: env i gets seed + i), so the
    union of the shards is the single-process batch bit for bit.

    batch_factory(count, config, device_index, autoreset) builds the rank's batch; the default
    is SoccerBatch on GPU `device` (default: local_rank, one GPU per rank; a one-GPU rehearsal
    passes 0 so that every rank shares cuda:0). Tests inject a CPU stand-in with the same
    interface.
    """

    def __init__(self, global_envs: int, config: dict | None = None, autoreset: bool = True, group=None,
                 batch_factory=None, device: int | None = None):
        import torch.distributed as dist

        self.world, self.rank, self.local_rank = dist_env()
        if self.world > 1 and not dist.is_initialized():
            raise RuntimeError("initialise torch.distributed (backend 'nccl' = RCCL) first")
        self.group = group
        self.global_envs = int(global_envs)
        self.start, self.count = shard_range(self.global_envs, self.world, self.rank)
        if batch_factory is None:
            from .batch import SoccerBatch

            def batch_factory(count, cfg, dev, ar):
                return SoccerBatch(count, config=cfg, device=dev, autoreset=ar)
        self.batch = batch_factory(self.count, config, self.local_rank if device is None else int(device), autoreset)
        self.device = self.batch.device

    def reset(self, seed: int | None = None, options=None):
        return self.batch.reset(seed=None if seed is None else int(seed) + self.start, options=options)

    def step(self, actions):
        return self.batch.step(actions)

    def gather_obs(self):
        """All-gather of every rank's obs -> (global_envs, 4, 66) on every rank (RCCL
        all_gather_into_tensor over xGMI; gloo's list form on CPU). Requires equal shard sizes
        (global_envs % world == 0)."""
        if self.world == 1:
            return self.batch.obs
        if self.global_envs % self.world:
            raise ValueError("gather_obs needs global_envs divisible by the world size")
        return all_gather_rows(self.batch.obs, self.world, self.group)

    def gather_outputs(self) -> dict:
        """Every rank's last step outputs (obs, rew, term, trunc, goal, score) for the whole
        batch, in global env order, on every rank: ONE all-gather over a packed 1,089-B-per-env
        record instead of one collective per tensor. Requires equal shard sizes."""
        if self.world > 1 and self.global_envs % self.world:
            raise ValueError("gather_outputs needs global_envs divisible by the world size")
        b = self.batch
        buf = pack_step_outputs({"obs": b.obs, "rew": b.rew, "term": b.term, "trunc": b.trunc, "goal": b.goal,
                                 "score": b.score})
        if self.world > 1:
            buf = all_gather_rows(buf, self.world, self.group)
        return unpack_step_outputs(buf)

    def close(self):
        self.batch.close()
