"""Multi-process (world_size 2, gloo, CPU) tests of the env-sharding contract.

The GPU path shards envs across ranks with no data-path collective; env g is seeded
seed + g and driven by actions that are a function of its global index, so a sharded run
must equal a single-process run bit for bit. Here the fp32 oracle stands in for each
rank's GPU batch (no GPU on this host) and gloo stands in for RCCL; the shard arithmetic
and the gather layout are the product's (marlsoccer.distributed).
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from marlsoccer.distributed import shard_range  # noqa: E402


def test_shard_range_partitions_exactly():
    for g in (1, 7, 64, 65536, 262144, 100003):
        for w in (1, 2, 3, 4, 8):
            spans = [shard_range(g, w, r) for r in range(w)]
            assert spans[0][0] == 0
            for (s0, c0), (s1, _) in zip(spans, spans[1:]):
                assert s0 + c0 == s1
            assert sum(c for _, c in spans) == g
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, G, steps, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "tests"), os.path.join(root, "oracle"), os.path.join(root, "marl-soccer_amd")]
    import oracle as orc
    import sim_helpers as sh
    from marlsoccer.distributed import all_gather_rows, pack_step_outputs, shard_range as sr

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, count = sr(G, world, rank)
    env = orc.OracleBatch(count, "f32", orc.default_config(max_steps=40))
    env.reset(np.stack([orc.pcg_from_seed(19 + start + i) for i in range(count)]), 0)
    for t in range(steps):
        obs, rew, trunc, goal, score, _ = env.step(sh.hash_actions(count, t, env0=start))
    parts = [torch.empty((count, 4, 66)) for _ in range(world)]
    dist.all_gather(parts, torch.from_numpy(obs))
    # ShardedSoccerEnv.gather_outputs' packed single collective (gloo form of all_gather_rows)
    packed = pack_step_outputs({
        "obs": torch.from_numpy(obs), "rew": torch.from_numpy(np.asarray(rew, np.float32)),
        "term": torch.zeros((count, 4), dtype=torch.uint8), "trunc": torch.from_numpy(np.asarray(trunc, np.uint8)),
        "goal": torch.from_numpy(np.asarray(goal, np.int8)), "score": torch.from_numpy(np.asarray(score, np.int32))})
    packed_all = all_gather_rows(packed, world)
    elapsed = torch.tensor([float(rank + 1)])
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)  # bench.py's max-over-ranks timing
    if rank == 0:
        q.put((torch.cat(parts).numpy(), float(elapsed), packed_all.numpy()))
    dist.barrier()
    dist.destroy_process_group()


class OracleShardBatch:
    """CPU stand-in for SoccerBatch (the fp32 oracle behind SoccerBatch's interface: reset with an
    int seed meaning env i gets seed + i, step, the output tensors), injected into the
    product's ShardedSoccerEnv through its batch_factory."""

    def __init__(self, count, config, device_index, autoreset):
        import oracle as orc
        self._orc = orc
        self.num_envs = count
        self.device = torch.device("cpu")
        self.env = orc.OracleBatch(count, "f32", orc.default_config(max_steps=config["max_steps"]))
        self.obs = torch.zeros((count, 4, 66))
        self.rew = torch.zeros((count, 4))
        self.term = torch.zeros((count, 4), dtype=torch.uint8)
        self.trunc = torch.zeros((count, 4), dtype=torch.uint8)
        self.goal = torch.zeros((count,), dtype=torch.int8)
        self.score = torch.zeros((count, 2), dtype=torch.int32)

    def reset(self, seed=None, options=None):
        pcg = np.stack([self._orc.pcg_from_seed(int(seed) + i) for i in range(self.num_envs)])
        self.obs[:] = torch.from_numpy(self.env.reset(pcg, 0))
        return self.obs

    def step(self, actions):
        obs, rew, trunc, goal, score, bad = self.env.step(actions.numpy())
        assert bad == 0
        self.obs[:] = torch.from_numpy(obs)
        self.rew[:] = torch.from_numpy(np.asarray(rew, np.float32))
        self.trunc[:] = torch.from_numpy(np.asarray(trunc, np.uint8))
        self.goal[:] = torch.from_numpy(np.asarray(goal, np.int8))
        self.score[:] = torch.from_numpy(np.asarray(score, np.int32))
        return self.obs, self.rew, self.term, self.trunc, self.goal, self.score

    def close(self):
        pass


def _sharded_worker(rank, world, port, G, steps, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "tests"), os.path.join(root, "oracle"), os.path.join(root, "marl-soccer_amd")]
    import sim_helpers as sh
    from marlsoccer.distributed import ShardedSoccerEnv
    from test_distributed import OracleShardBatch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    env = ShardedSoccerEnv(G, config={"max_steps": 40}, batch_factory=OracleShardBatch)
    obs0 = env.gather_obs().clone()
    env.reset(seed=19)
    obs_reset = env.gather_obs().clone()
    for t in range(steps):
        env.step(torch.from_numpy(sh.hash_actions(env.count, t, env0=env.start)))
    obs = env.gather_obs()
    outs = env.gather_outputs()
    if rank == 0:
        q.put((env.start, env.count, obs_reset.numpy(), obs.numpy(), {k: v.numpy() for k, v in outs.items()},
               obs0.shape))
    dist.barrier()
    env.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("G", [64, 66])
def test_gloo_world2_sharded_soccer_env(G):
    """The product's ShardedSoccerEnv on two gloo ranks (oracle-backed batches): reset(seed)
    seeds each rank's envs with their global indices, gather_obs and gather_outputs return the
    whole batch in global order, equal to one process stepping all G envs (60 steps of 40-step
    episodes: every env crosses its auto-reset)."""
    import oracle as orc
    import sim_helpers as sh

    steps, world = 60, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, G, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    start, count, obs_reset, obs, outs, shape0 = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert start == 0 and count == G // 2 and shape0 == (G, 4, 66)
    single = orc.OracleBatch(G, "f32", orc.default_config(max_steps=40))
    ro = single.reset(np.stack([orc.pcg_from_seed(19 + i) for i in range(G)]), 0)
    np.testing.assert_array_equal(obs_reset, ro)
    for t in range(steps):
        o, rew, trunc, goal, score, _ = single.step(sh.hash_actions(G, t))
    np.testing.assert_array_equal(obs, o)
    np.testing.assert_array_equal(outs["obs"], o)
    np.testing.assert_array_equal(outs["rew"], np.asarray(rew, np.float32))
    np.testing.assert_array_equal(outs["trunc"], np.asarray(trunc, np.uint8))
    np.testing.assert_array_equal(outs["goal"], goal)
    np.testing.assert_array_equal(outs["score"], score)


def test_gloo_world2_sharded_equals_single_process():
    import oracle as orc
    import sim_helpers as sh

    G, steps, world = 64, 90, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, G, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, tmax, packed_all = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert tmax == 2.0
    single = orc.OracleBatch(G, "f32", orc.default_config(max_steps=40))
    single.reset(np.stack([orc.pcg_from_seed(19 + i) for i in range(G)]), 0)
    for t in range(steps):
        obs, rew, trunc, goal, score, _ = single.step(sh.hash_actions(G, t))
    np.testing.assert_array_equal(gathered, obs)
    from marlsoccer.distributed import RECORD_BYTES, unpack_step_outputs
    assert packed_all.shape == (G, RECORD_BYTES) and RECORD_BYTES == 1089
    got = unpack_step_outputs(torch.from_numpy(packed_all))
    np.testing.assert_array_equal(got["obs"].numpy(), obs)
    np.testing.assert_array_equal(got["rew"].numpy(), np.asarray(rew, np.float32))
    np.testing.assert_array_equal(got["trunc"].numpy(), np.asarray(trunc, np.uint8))
    np.testing.assert_array_equal(got["goal"].numpy(), np.asarray(goal, np.int8))
    np.testing.assert_array_equal(got["score"].numpy(), np.asarray(score, np.int32))
    assert not got["term"].numpy().any()


@pytest.mark.parametrize("shape,dtype", [((6, 4, 66), torch.float32), ((6, 1089), torch.uint8)],
                         ids=["obs", "packed-outputs"])
def test_all_gather_rows_rccl_branch_builds_the_gathered_tensor(monkeypatch, shape, dtype):
    """all_gather_rows' RCCL branch (backend "nccl", distributed.py:72-75), which no CPU run
    reaches: with torch.distributed's backend query and all_gather_into_tensor replaced by stand-ins,
    the destination handed to the collective is (world x n, ...) of the input's dtype and device,
    the input is passed unchanged, and the tensor returned is that destination (rank r's rows at
    [r n, (r + 1) n))."""
    from marlsoccer import distributed as D

    world, calls = 4, []

    def fake_all_gather_into_tensor(dst, src, group=None):
        calls.append((tuple(dst.shape), dst.dtype, dst.device, src, group))
        n = src.shape[0]
        for r in range(world):  # what RCCL writes: rank r's buffer at rows [r n, (r + 1) n)
            dst[r * n:(r + 1) * n] = src + r if dtype != torch.uint8 else src ^ r

    monkeypatch.setattr(dist, "get_backend", lambda group=None: "nccl")
    monkeypatch.setattr(dist, "all_gather_into_tensor", fake_all_gather_into_tensor)
    src = (torch.arange(int(np.prod(shape))) % 251).reshape(shape).to(dtype)
    group = object()
    out = D.all_gather_rows(src, world, group)
    assert len(calls) == 1
    dshape, ddtype, ddev, csrc, cgroup = calls[0]
    assert dshape == (world * shape[0],) + shape[1:] and ddtype == dtype and ddev == src.device
    assert csrc is src and cgroup is group
    assert out.shape == dshape and out.dtype == dtype
    for r in range(world):
        want = src + r if dtype != torch.uint8 else src ^ r
        assert torch.equal(out[r * shape[0]:(r + 1) * shape[0]], want)
