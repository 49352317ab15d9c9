"""Boundary compliance of the drop-in surfaces (GPU-backed):
soccer_env.SoccerEnv / soccerenv / get_observation_scalers (soccer_env.py:16-221) and
marl_vecenv.SyncMultiAgentVecEnv (marl_vecenv.py:3-80), including the checks PettingZoo's
parallel_api_test(env, num_cycles=50) performs in pz_api_lint.py:5-7 (pettingzoo itself is
not installed here, so its checks are restated)."""
import math

import numpy as np
import pytest

import oracle as orc

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def cfg(**over):
    from marlsoccer.config import load_config
    c = load_config()
    for k, v in over.items():
        sect = "simulation" if k == "max_steps" else ("physics" if k in c["physics"] else "rewards")
        c[sect][k] = v
    return c


def test_parallel_api_contract():
    from soccer_env import soccerenv
    env = soccerenv()
    assert env.possible_agents == ["agent_0", "agent_1", "agent_2", "agent_3"]
    obs, infos = env.reset(seed=3)
    assert set(obs) == set(env.agents) == set(infos)
    for a in env.agents:
        sp = env.observation_space(a)
        assert obs[a].shape == sp.shape == (66,) and obs[a].dtype == np.float32
        assert env.action_space(a).shape == (3,) and env.action_space(a).dtype == np.float32
    cycles = 0
    while env.agents and cycles < 50:
        acts = {a: env.action_space(a).sample() for a in env.agents}
        obs, rew, term, trunc, infos = env.step(acts)
        for d in (obs, rew, term, trunc, infos):
            assert set(d) == set(env.possible_agents)
        assert all(isinstance(r, float) for r in rew.values())
        assert all(isinstance(x, bool) for x in list(term.values()) + list(trunc.values()))
        assert rew["agent_2"] == 0.0 and rew["agent_3"] == 0.0 and rew["agent_0"] == rew["agent_1"]
        assert infos["agent_0"]["score"] == {"blue": 0, "red": 0} or "score" in infos["agent_0"]
        cycles += 1
    env.close()


def test_validation_errors_match_reference():
    from soccer_env import SoccerEnv, soccerenv
    with pytest.raises(ValueError, match="single environment"):
        SoccerEnv(num_envs=2)
    env = soccerenv()
    env.reset(seed=0)
    good = {a: [0.0, 0.0, 0.0] for a in env.possible_agents}
    with pytest.raises(ValueError, match="Missing actions"):
        env.step({k: v for k, v in good.items() if k != "agent_3"})
    with pytest.raises(ValueError, match="unknown agents"):
        env.step({**good, "agent_9": [0, 0, 0]})
    with pytest.raises(ValueError, match=r"must have shape \(3,\)"):
        env.step({**good, "agent_1": [0.0, 1.0]})
    with pytest.raises(ValueError, match="non-finite"):
        env.step({**good, "agent_2": [0.0, math.nan, 0.0]})
    env.close()


def test_truncation_at_max_steps_and_agents_cleared():
    from soccer_env import soccerenv
    env = soccerenv(config=cfg(max_steps=7))
    env.reset(seed=4)
    zero = {a: np.zeros(3, np.float32) for a in env.possible_agents}
    for t in range(1, 8):
        obs, rew, term, trunc, infos = env.step(zero)
        assert all(trunc.values()) == (t == 7) and not any(term.values())
    assert env.agents == []
    obs, _ = env.reset()
    assert env.agents == env.possible_agents
    env.close()


def test_reset_seed_matches_oracle_and_is_deterministic():
    from soccer_env import soccerenv
    env = soccerenv()
    o1, _ = env.reset(seed=19)
    o2, _ = env.reset(seed=19)
    ref = orc.OracleBatch(1, "f32")
    ro = ref.reset(orc.pcg_from_seed(19)[None], 0)[0]
    for i, a in enumerate(env.possible_agents):
        np.testing.assert_array_equal(o1[a], o2[a])
        np.testing.assert_array_equal(o1[a], ro[i])
        np.testing.assert_array_equal(o1[a][:22], o1[a][44:])  # 3 identical frames
    env.close()


def test_observation_scalers():
    from soccer_env import get_observation_scalers, soccerenv
    s = get_observation_scalers(soccerenv())
    assert s == {"max_velocity": 200.0, "max_angular_velocity": 10.0, "field_diagonal": 1000.0,
                 "stack_size": 3, "frame_size": 22}


def test_vec_env_shapes_dtypes_and_oracle_parity():
    from marl_vecenv import SyncMultiAgentVecEnv
    from soccer_env import soccerenv
    n = 8
    envs = SyncMultiAgentVecEnv([lambda: soccerenv() for _ in range(n)])
    assert envs.num_envs == n and envs.single_observation_space.shape == (66,)
    assert envs.single_action_space.shape == (3,)
    obs = envs.reset(seed=19)
    ref = orc.OracleBatch(n, "f32")
    np.testing.assert_array_equal(obs, ref.reset(np.stack([orc.pcg_from_seed(19 + i) for i in range(n)]), 0))
    rng = np.random.default_rng(0)
    for t in range(40):
        act = rng.uniform(-1, 1, (n, 4, 3)).astype(np.float32)
        obs, rew, term, trunc, infos = envs.step(act)
        r_obs, r_rew, r_tr, r_g, r_s, _ = ref.step(act)
        assert obs.dtype == np.float32 and obs.shape == (n, 4, 66)
        assert rew.dtype == np.float64 and rew.shape == (n, 4)
        assert term.dtype == bool and trunc.dtype == bool and term.shape == trunc.shape == (n, 4)
        assert len(infos) == n and set(infos[0]) == set(envs.possible_agents)
        np.testing.assert_array_equal(obs, r_obs)
        np.testing.assert_array_equal(rew, r_rew.astype(np.float32).astype(np.float64))
        assert (rew[:, 2:] == 0).all()
        for i in range(n):
            assert infos[i]["agent_0"]["score"] == {"blue": int(r_s[i, 0]), "red": int(r_s[i, 1])}
    envs.close()


def test_vec_env_auto_reset_returns_reset_obs():
    from marl_vecenv import SyncMultiAgentVecEnv
    from soccer_env import soccerenv
    c = cfg(max_steps=5)
    envs = SyncMultiAgentVecEnv([lambda: soccerenv(config=c) for _ in range(4)])
    envs.reset(seed=1)
    zero = np.zeros((4, 4, 3), np.float32)
    for t in range(1, 6):
        obs, rew, term, trunc, infos = envs.step(zero)
        assert trunc.all() == (t == 5)
    np.testing.assert_array_equal(obs[:, :, :22], obs[:, :, 44:])
    st = envs.batch.export_state()
    assert (st["steps"] == 0).all() and (st["mode"] == 1).all()  # full-random from now on
    with pytest.raises(ValueError, match="non-finite"):
        bad = zero.copy()
        bad[2, 1, 0] = np.inf
        envs.step(bad)
    envs.close()


def test_lazy_infos_goal_entries():
    from marl_vecenv import LazyInfos
    infos = LazyInfos(np.array([[1, 0], [0, 2]]), np.array([1, 0], np.int8), ["agent_0", "agent_1"])
    assert infos[0]["agent_0"] == {"score": {"blue": 1, "red": 0}, "goal_scored_by": "blue"}
    assert infos[1]["agent_1"] == {"score": {"blue": 0, "red": 2}}
    assert len(infos) == 2 and infos[-1] == infos[1]


def test_render_rgb_array():
    from soccer_env import soccerenv
    env = soccerenv(render_mode="rgb_array")
    env.reset(seed=0)
    img = env.render()
    assert img.shape == (600, 800, 3) and img.dtype == np.uint8
    assert (img == [0, 0, 255]).all(-1).sum() > 500 and (img == [255, 0, 0]).all(-1).sum() > 500
    env.close()
