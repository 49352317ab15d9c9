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


class ShardedSoccerEnv:
    """This rank's shard of a global batch of envs on its own GPU.

    global_envs envs are split with shard_range; rank r owns [start, start + count).
    """

    def __init__(self, global_envs: int, config: dict | None = None, autoreset: bool = True, group=None):
        import torch
        import torch.distributed as dist

        from .batch import SoccerBatch

        self.world, self.rank, self.local_rank = dist_env()
        if self.world > 1 and not dist.is_initialized():
            raise RuntimeError("initialise torch.distributed (backend 'nccl' = RCCL) first")
        self.group = group
        self.global_envs = int(global_envs)
        self.start, self.count = shard_range(self.global_envs, self.world, self.rank)
        self.device = torch.device("cuda", self.local_rank)
        self.batch = SoccerBatch(self.count, config=config, device=self.local_rank, autoreset=autoreset)
        self._gathered = None

    def reset(self, seed: int | None = None, options=None):
        return self.batch.reset(seed=None if seed is None else int(seed) + self.start, options=options)

    def step(self, actions):
        return self.batch.step(actions)

    def gather_obs(self):
        """All-gather of every rank's obs -> (global_envs, 4, 66) on every rank (RCCL).
        Requires equal shard sizes (global_envs % world == 0)."""
        import torch
        import torch.distributed as dist

        if self.world == 1:
            return self.batch.obs
        if self.global_envs % self.world:
            raise ValueError("gather_obs needs global_envs divisible by the world size")
        if self._gathered is None:
            self._gathered = torch.empty((self.global_envs, 4, 66), dtype=torch.float32, device=self.device)
        dist.all_gather_into_tensor(self._gathered, self.batch.obs, group=self.group)
        return self._gathered

    def close(self):
        self.batch.close()
