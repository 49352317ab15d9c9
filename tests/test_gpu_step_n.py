"""ms_step_n (SoccerBatch.step_n): K steps with the actions given up front. With the lane-pair
and lane-group kernels the K steps are ONE launch (ms_step_pair_n_kernel / ms_step_group_n_kernel:
each wave steps its envs K times back to back); with the one-lane-per-env kernel K ms_step
launches. Either way the results must be those of K ms_step calls, bit for bit, and those of the
fp32 oracle (marl_vecenv.py:30-68 driven by a pre-drawn action sequence)."""
import numpy as np
import pytest

import oracle as orc
import sim_helpers as sh
from test_gpu_parity import assert_state_equal, cfg_dict, oracle_cfg

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ms():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    import marlsoccer
    return marlsoccer


def chase_sequence(ref, n, K, rng, chaser):
    """K steps of the oracle under the chase policy (goals, respawns, pile-ups): the actions it
    took and its outputs per step."""
    acts, outs = [], []
    for _ in range(K):
        st = ref.export_state()
        pos = np.stack([st["body"]["px"], st["body"]["py"]], -1)
        act = sh.chase_actions(pos, st["body"]["angle"][:, :4], rng, chaser)
        o = ref.step(act)
        assert o[5] == 0
        acts.append(act)
        outs.append(o)
    return np.stack(acts), outs


@pytest.mark.parametrize("lanes", [2, 8, 16, 0], ids=["lane-pair-fused", "lanes8-fused", "lanes16-fused", "per-lane"])
@pytest.mark.parametrize("n", [1000, 4096])
def test_step_n_chase_bitexact_vs_oracle(ms, lanes, n):
    """Three step_n calls of K = 48 under the chase policy (episodes of 60 steps: auto-resets
    inside a launch, goals and their respawns) against the fp32 oracle at every step, and the
    whole exported state after each launch. n = 1,000 leaves the last wave partly empty."""
    K, seed = 48, 23
    config = cfg_dict(max_steps=60)
    gpu = ms.SoccerBatch(n, config=config)
    gpu.set_lane_group(lanes)
    ref = orc.OracleBatch(n, "f32", oracle_cfg(ms.to_ms_config(config, True)))
    np.testing.assert_array_equal(gpu.reset(seed=seed).cpu().numpy(),
                                  ref.reset(np.stack([orc.pcg_from_seed(seed + i) for i in range(n)]), 0))
    rng = np.random.default_rng(seed)
    chaser = np.arange(n) % 4
    goals = dones = 0
    for call in range(3):
        acts, outs = chase_sequence(ref, n, K, rng, chaser)
        res = gpu.step_n(torch.from_numpy(acts).to(gpu.device))
        g = {f: getattr(res, f).cpu().numpy() for f in ("obs", "rew", "term", "trunc", "goal", "score")}
        for k, (obs, rew, trunc, goal, score, _) in enumerate(outs):
            w = f"call {call} step {k}"
            np.testing.assert_array_equal(g["obs"][k], obs, err_msg=f"obs {w}")
            np.testing.assert_array_equal(g["rew"][k], rew.astype(np.float32), err_msg=f"rew {w}")
            np.testing.assert_array_equal(g["trunc"][k].astype(bool), trunc, err_msg=f"trunc {w}")
            np.testing.assert_array_equal(g["goal"][k], goal, err_msg=f"goal {w}")
            np.testing.assert_array_equal(g["score"][k], score, err_msg=f"score {w}")
            assert not g["term"][k].any()
            goals += int((goal != 0).sum())
            dones += int(trunc[:, 0].sum())
        assert_state_equal(gpu.export_state(), ref.export_state(), f"after call {call}")
    assert goals > 0 and dones >= n  # goals and auto-resets happened inside the launches
    st = gpu.stats()
    assert st["env_steps"] == 3 * K * n and st["arbiter_overflow"] == 0
    gpu.close()


def test_step_n_full_size_equals_step(ms):
    """configs[2]'s 65,536 envs: two step_n launches of K = 64 against 128 step() calls of a second
    batch on the same uniform random actions, every output of every step compared on the device,
    the exported states at the end."""
    n, K = 65536, 64
    a = ms.SoccerBatch(n)
    b = ms.SoccerBatch(n)
    assert a.lane_group == b.lane_group == 2
    a.reset(seed=19)
    b.reset(seed=19)
    gen = torch.Generator(device=a.device)
    gen.manual_seed(5)
    for call in range(2):
        acts = torch.rand((K, n, 4, 3), generator=gen, device=a.device) * 2.0 - 1.0
        res = b.step_n(acts)
        for k in range(K):
            o = a.step(acts[k])
            for f in ("obs", "rew", "term", "trunc", "goal", "score"):
                assert torch.equal(getattr(o, f), getattr(res, f)[k]), f"{f} call {call} step {k}"
    assert_state_equal(b.export_state(), a.export_state(), "end")
    assert b.stats()["env_steps"] == a.stats()["env_steps"] == 2 * K * n
    a.close()
    b.close()


def test_step_n_rejects_bad_arguments(ms):
    gpu = ms.SoccerBatch(64)
    gpu.reset(seed=1)
    with pytest.raises(ValueError):
        gpu.step_n(torch.zeros((64, 4, 3), device=gpu.device))  # no K dimension
    with pytest.raises(ValueError):
        gpu.step_n(torch.zeros((0, 64, 4, 3), device=gpu.device))
    with pytest.raises(ValueError):
        gpu.step_n(torch.zeros((2, 64, 4, 3), device=gpu.device), out={"obs": torch.zeros((1, 64, 4, 66), device=gpu.device)})
    gpu.close()


def test_vec_env_step_n_tensors_matches_oracle(ms):
    """The vec-env wrapper's open-loop entry (SyncMultiAgentVecEnv.step_n_tensors, marl_vecenv.py's
    step driven by pre-drawn uniform actions) against the fp32 oracle step by step."""
    from marl_vecenv import SyncMultiAgentVecEnv
    from soccer_env import soccerenv
    n, K = 16, 40
    envs = SyncMultiAgentVecEnv([lambda: soccerenv() for _ in range(n)])
    envs.reset(seed=19)
    ref = orc.OracleBatch(n, "f32")
    ref.reset(np.stack([orc.pcg_from_seed(19 + i) for i in range(n)]), 0)
    act = np.random.default_rng(3).uniform(-1, 1, (K, n, 4, 3)).astype(np.float32)
    res = envs.step_n_tensors(torch.from_numpy(act).to(envs.batch.device))
    obs, rew = res.obs.cpu().numpy(), res.rew.cpu().numpy()
    for k in range(K):
        r_obs, r_rew = ref.step(act[k])[:2]
        np.testing.assert_array_equal(obs[k], r_obs, err_msg=f"obs step {k}")
        np.testing.assert_array_equal(rew[k], r_rew.astype(np.float32), err_msg=f"rew step {k}")
    envs.close()


@pytest.mark.parametrize("lanes", [2, 8], ids=["lane-pair-fused", "lanes8-fused"])
def test_step_n_nonfinite_actions_skip_like_step(ms, lanes):
    """A non-finite action inside a K-step launch skips that env for that step only (reward NaN,
    state untouched; soccer_env.py:101-117's check, counted in ms_stats), exactly as the same
    action sequence through K step() calls does."""
    n, K = 256, 12
    a = ms.SoccerBatch(n)
    b = ms.SoccerBatch(n)
    a.set_lane_group(lanes)
    b.set_lane_group(lanes)
    a.reset(seed=7)
    b.reset(seed=7)
    gen = torch.Generator(device=a.device)
    gen.manual_seed(11)
    acts = torch.rand((K, n, 4, 3), generator=gen, device=a.device) * 2.0 - 1.0
    acts[3, 5, 1, 0] = float("nan")
    acts[3, 200, 3, 2] = float("inf")
    acts[7, 5, 0, 1] = float("-inf")
    # a slot full of garbage: a skipped env-step must overwrite it with defined values (ABI 5)
    out = {"obs": torch.full((K, n, 4, 66), 7.0, device=a.device),
           "term": torch.full((K, n, 4), 1, dtype=torch.uint8, device=a.device),
           "trunc": torch.full((K, n, 4), 1, dtype=torch.uint8, device=a.device),
           "goal": torch.full((K, n), 3, dtype=torch.int8, device=a.device),
           "score": torch.full((K, n, 2), -5, dtype=torch.int32, device=a.device)}
    res = b.step_n(acts, out=out)
    skipped = {(3, 5), (3, 200), (7, 5)}
    for k in range(K):
        score_before = a.score.clone()
        o = a.step(acts[k])
        # every env bit for bit, the skipped ones included (NaN obs and rewards, term / trunc / goal
        # 0, the score unchanged: ms_step's and ms_step_n's defined values)
        for f in ("obs", "rew"):
            x, y = getattr(o, f), getattr(res, f)[k]
            assert torch.equal(x.view(torch.int32), y.view(torch.int32)), f"{f} step {k}"
        for f in ("term", "trunc", "goal", "score"):
            assert torch.equal(getattr(o, f), getattr(res, f)[k]), f"{f} step {k}"
        for (ks, e) in skipped:
            if ks != k:
                continue
            assert torch.isnan(res.obs[k, e]).all() and torch.isnan(res.rew[k, e, :2]).all()
            assert (res.term[k, e] == 0).all() and (res.trunc[k, e] == 0).all() and int(res.goal[k, e]) == 0
            assert torch.equal(res.score[k, e], score_before[e])
    assert torch.isnan(res.rew[3, 5]).any() and torch.isnan(res.rew[3, 200]).any() and torch.isnan(res.rew[7, 5]).any()
    assert not torch.isnan(res.rew[4]).any()
    assert_state_equal(b.export_state(), a.export_state(), "end")
    sa, sb = a.stats(), b.stats()
    assert sa["nonfinite_envs"] == sb["nonfinite_envs"] == 3
    # step_n(check=True) raises the reference's ValueError for the first such env (and clears the count)
    with pytest.raises(ValueError, match=r"non-finite values for agent 'agent_1'.*env 5"):
        b.step_n(acts[:4], check=True)
    b.step_n(acts[4:6], check=True)
    a.close()
    b.close()
