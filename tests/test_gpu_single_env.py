"""BASELINE configs[0] at its own workload: ONE env through the reference's dict API
(soccerenv(), soccer_env.py:100-154), seed 19, 10,000 steps of uniform random actions, reset with
the full-random spawn whenever an episode truncates (what marl_vecenv.py:45-51 does for each of its
envs), against the fp32 oracle at every step: observations, rewards, truncations and
infos['goal_scored_by'] bit for bit, the full state (bodies, history, arbiter cache, RNG) every
1,000 steps."""
import numpy as np
import pytest

import oracle as orc

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

AGENTS = [f"agent_{i}" for i in range(4)]


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def test_configs0_single_env_10k_steps_dict_api_bitexact():
    from soccer_env import soccerenv
    from marlsoccer.batch import spawn_mode
    from test_gpu_parity import assert_state_equal

    env = soccerenv()
    obs, infos = env.reset(seed=19)
    ocfg = orc.default_config()
    ocfg.autoreset = 0  # the dict API does not auto-reset: the caller resets, as below
    ref = orc.OracleBatch(1, "f32", ocfg)
    robs = ref.reset(orc.pcg_from_seed(19)[None], 0)
    for i, a in enumerate(AGENTS):
        np.testing.assert_array_equal(obs[a], robs[0, i])
    full_random = spawn_mode({"use_full_random_positions": True})
    rng = np.random.default_rng(19 + 10 ** 6)
    episodes = goals = 0
    for t in range(10_000):
        act = rng.uniform(-1.0, 1.0, (4, 3)).astype(np.float32)
        obs, rew, term, trunc, infos = env.step({a: act[i] for i, a in enumerate(AGENTS)})
        robs, rrew, rtrunc, rgoal, rscore, bad = ref.step(act[None])
        assert bad == 0
        for i, a in enumerate(AGENTS):
            np.testing.assert_array_equal(obs[a], robs[0, i], err_msg=f"obs {a} t={t}")
            assert np.float32(rew[a]) == np.float32(rrew[0, i]), (t, a, rew[a], rrew[0, i])
            assert trunc[a] == bool(rtrunc[0, i]) and term[a] is False
        g = int(rgoal[0])
        want = {1: "blue", 2: "red"}.get(g)
        assert infos["agent_0"].get("goal_scored_by") == want, (t, infos["agent_0"], g)
        assert infos["agent_0"]["score"] == {"blue": int(rscore[0, 0]), "red": int(rscore[0, 1])}
        goals += g != 0
        if trunc["agent_0"]:
            episodes += 1
            assert env.agents == []
            obs, _ = env.reset(options={"use_full_random_positions": True})  # marl_vecenv.py:48-51
            robs = ref.reset(None, full_random)
            for i, a in enumerate(AGENTS):
                np.testing.assert_array_equal(obs[a], robs[0, i], err_msg=f"reset obs {a} t={t}")
        if t % 1000 == 999:
            assert_state_equal(env.state()[None], ref.export_state(), f"t={t}")
    assert episodes == 10, episodes  # (random actions rarely score: goals are checked wherever they occur)
    env.close()
