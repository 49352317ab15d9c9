"""Policy-side formats and the device rollout.

CPU: marlsoccer.rollout.Agent and RunningMeanStd against golden vectors produced by the
reference notebook's own classes (tests/golden/make_policy_fixture.py), and compatibility
with the reference's run5 checkpoint / normaliser formats.
GPU: DeviceRollout drives SoccerBatch with the policy on the device.
"""
import json
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from make_policy_fixture import rms_batches  # noqa: E402  (the batch generator, no reference code)

from marlsoccer.rollout import Agent, DeviceRollout, RunningMeanStd  # noqa: E402

FX = np.load(os.path.join(HERE, "golden", "policy.npz"))


def test_agent_matches_reference_network():
    torch.manual_seed(0)
    agent = Agent()
    x, a = torch.from_numpy(FX["x"]), torch.from_numpy(FX["a"])
    with torch.no_grad():
        np.testing.assert_array_equal(agent.actor_mean(x).numpy(), FX["mean"])
        np.testing.assert_array_equal(agent.get_value(x).numpy(), FX["value"])
        _, logprob, entropy, _ = agent.get_action_and_value(x, a)
    np.testing.assert_array_equal(logprob.numpy(), FX["logprob"])
    np.testing.assert_array_equal(entropy.numpy(), FX["entropy"])


def test_agent_state_dict_matches_reference_checkpoint():
    sd = Agent().state_dict()
    keys = [str(k) for k in FX["ckpt_keys"]]
    shapes = json.loads(str(FX["ckpt_shapes"]))
    assert sorted(sd.keys()) == keys
    assert [list(sd[k].shape) for k in keys] == shapes


def test_running_mean_std_matches_notebook():
    rms = RunningMeanStd((66,))
    for b, m, v in zip(rms_batches(), FX["rms_means"], FX["rms_vars"]):
        rms.update(torch.from_numpy(b))
        np.testing.assert_allclose(rms.mean.numpy(), m, rtol=0, atol=1e-12)
        np.testing.assert_allclose(rms.var.numpy(), v, rtol=1e-12, atol=1e-12)
    assert rms.count == int(FX["rms_batch_sizes"].sum())


def test_normaliser_npz_roundtrip_and_formula(tmp_path):
    rms = RunningMeanStd((66,))
    rms.mean = torch.from_numpy(FX["run5_mean"].copy())
    rms.var = torch.from_numpy(FX["run5_var"].copy())
    path = str(tmp_path / "latest_normalizer_stats.npz")
    rms.save_npz(path)
    with np.load(path) as d:
        assert sorted(d.files) == ["mean", "var"] and d["mean"].dtype == np.float64 and d["mean"].shape == (66,)
    back = RunningMeanStd.load_npz(path)
    np.testing.assert_array_equal(back.var.numpy(), FX["run5_var"])
    obs = np.random.default_rng(3).normal(size=(16, 66)).astype(np.float32) * 2
    # eval.py:63-64, notebook L301: numpy float64 normalisation, clipped, then float32
    want = np.clip((obs - FX["run5_mean"]) / (np.sqrt(FX["run5_var"]) + 1e-8), -10, 10).astype(np.float32)
    np.testing.assert_array_equal(back.normalize(torch.from_numpy(obs)).numpy(), want)


@pytest.mark.gpu
def test_device_rollout_drives_env_on_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from marlsoccer import SoccerBatch
    N, T = 512, 40
    b = SoccerBatch(N)
    b.reset(seed=19)
    torch.manual_seed(0)
    agent = Agent().cuda()
    rms = RunningMeanStd((66,), device="cuda")
    ro = DeviceRollout(b, agent, rms, T, seed=5)
    first_obs = b.obs[:, :2].clone()
    out = ro.collect()
    torch.cuda.synchronize()
    assert out["obs"].shape == (T, N, 2, 66) and out["actions"].shape == (T, N, 2, 3)
    assert torch.equal(out["obs"][0], first_obs)
    assert torch.equal(out["next_obs"], b.obs[:, :2])
    assert torch.equal(out["rewards"][-1], b.rew[:, :2])
    red = ro.full_actions[:, 2:]
    assert float(red.min()) >= -1.0 and float(red.max()) <= 1.0 and float(red.std()) > 0.3
    assert torch.isfinite(out["values"]).all() and torch.isfinite(out["logprobs"]).all()
    assert rms.count == T * N * 2
    # the policy saw exactly the normalised stored observations
    with torch.no_grad():
        x = RunningMeanStd((66,), device="cuda").normalize(out["obs"][3].reshape(-1, 66))
        assert torch.allclose(agent.get_value(x).reshape(N, 2), out["values"][3], atol=1e-5, rtol=1e-5)
    b.close()


@pytest.mark.gpu
def test_graph_rollout_matches_eager_rollout():
    """DeviceRollout(graph=True) (eager first collect, then one captured graph per rollout) ==
    the eager rollout from the same state and seeds: storage, env outputs, normaliser, counters,
    across three collects (eager, capture + replay, replay) with the normaliser updated between."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from marlsoccer import SoccerBatch
    N, T = 256, 16
    torch.manual_seed(0)
    agent = Agent().cuda()
    # the capturable sampling (standard normal x std + mean) draws what torch.normal draws
    m = torch.randn((4096, 3), device="cuda")
    s = torch.rand((4096, 3), device="cuda") + 0.1
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    want = torch.normal(m, s, generator=g)
    g.manual_seed(3)
    assert torch.equal(torch.randn(m.shape, device="cuda", generator=g) * s + m, want)
    runs = []
    for graph in (False, True):
        b = SoccerBatch(N)
        b.reset(seed=23)
        rms = RunningMeanStd((66,), device="cuda")
        ro = DeviceRollout(b, agent, rms, T, seed=11, graph=graph)
        outs = []
        for _ in range(3):
            out = ro.collect()
            outs.append({k: v.clone() for k, v in out.items()})
        torch.cuda.synchronize()
        runs.append((outs, rms.mean.clone(), rms.var.clone(), b.obs.clone(), b.score.clone(), b))
    (oe, me, ve, obe, se, be), (og, mg, vg, obg, sg, bg) = runs
    for a, g in zip(oe, og):
        for k in a:
            assert torch.equal(a[k], g[k]), k
    assert torch.equal(me, mg) and torch.equal(ve, vg)
    assert torch.equal(obe, obg) and torch.equal(se, sg)
    assert bg._h is not None and bg.stream == torch.cuda.current_stream()
    be.close()
    bg.close()


@pytest.mark.gpu
def test_device_rollout_deterministic_matches_host_loop():
    """Deterministic rollout (torch policy) == the eval.py-style host loop (policy mean for blue,
    the same red actions) step for step; the fused-kernel rollout's first actions are within
    1e-5 of the same loop's."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from marlsoccer import SoccerBatch
    N, T = 64, 12
    torch.manual_seed(0)
    agent = Agent().cuda()
    rms = RunningMeanStd((66,), device="cuda")
    b1, b2 = SoccerBatch(N), SoccerBatch(N)
    b1.reset(seed=7)
    b2.reset(seed=7)
    # the torch policy, so that the host loop below can use the same modules bit for bit (the
    # fused kernel's outputs are within 1e-5 of them: test_fused_policy_*)
    ro = DeviceRollout(b1, agent, rms, T, seed=9, deterministic=True, update_normalizer=False, policy="torch")
    out = ro.collect()
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    for t in range(T):
        with torch.no_grad():
            mean = agent.actor_mean(rms.normalize(b2.obs[:, :2].reshape(-1, 66))).reshape(N, 2, 3)
        acts = torch.empty((N, 4, 3), device="cuda")
        acts[:, :2] = mean
        acts[:, 2:] = torch.rand((N, 2, 3), generator=g, device="cuda") * 2.0 - 1.0
        assert torch.equal(mean, out["actions"][t])
        b2.step(acts)
    assert torch.equal(b1.obs, b2.obs) and torch.equal(b1.rew, b2.rew)
    b1.close()
    b2.close()
    b3 = SoccerBatch(N)
    b3.reset(seed=7)
    first = b3.obs[:, :2].clone()
    ro = DeviceRollout(b3, agent, rms, 2, seed=9, deterministic=True, update_normalizer=False)
    assert ro.policy == "fused"
    out = ro.collect()
    with torch.no_grad():
        mean = agent.actor_mean(rms.normalize(first.reshape(-1, 66))).reshape(N, 2, 3)
    assert float((out["actions"][0] - mean).abs().max()) <= 1e-5
    b3.close()


@pytest.mark.gpu
def test_batched_eval_matches_sequential_eval_loop():
    """marlsoccer.evaluate (eval.py's loop, episodes as parallel envs) == eval.py's own
    sequential loop over single SoccerEnv episodes with the same seeds. The actor's last layer is
    set to a constant so the actions do not depend on the GEMM batch size; the red agents are
    zero (eval.py draws them from numpy's global RNG)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from marlsoccer.config import load_config
    from marlsoccer.evaluate import evaluate
    from soccer_env import soccerenv
    torch.manual_seed(0)
    agent = Agent().cuda()
    with torch.no_grad():
        agent.actor_mean[-1].weight.zero_()
        agent.actor_mean[-1].bias.copy_(torch.tensor([0.6, -0.4, 0.2]))
    rms = RunningMeanStd(device="cuda")
    cfg = load_config()
    cfg["simulation"]["max_steps"] = 80
    res = evaluate(agent, rms, 4, seed=7, config=cfg, red="zero", frames_every=40)
    assert res["returns"].shape == (4, 2) and res["score"].shape == (4, 2) and res["steps"] == 80
    assert [t for t, _ in res["frames"]] == [0, 40, 79] and res["frames"][0][1].shape == (1, 600, 800, 3)
    for i in range(4):
        env = soccerenv(config=cfg)
        obs, _ = env.reset(seed=7 + i)
        ret = np.zeros(2)
        score = None
        while env.agents:
            x = rms.normalize(torch.tensor(np.stack([obs["agent_0"], obs["agent_1"]])).cuda())
            mu = agent.get_deterministic_action(x).detach().cpu().numpy()
            acts = {"agent_0": mu[0], "agent_1": mu[1], "agent_2": np.zeros(3, np.float32),
                    "agent_3": np.zeros(3, np.float32)}
            obs, rew, term, trunc, infos = env.step(acts)
            ret += [np.float32(rew["agent_0"]), np.float32(rew["agent_1"])]
            score = infos["agent_0"]["score"]
        env.close()
        np.testing.assert_array_equal(res["returns"][i], ret)
        assert (int(res["score"][i, 0]), int(res["score"][i, 1])) == (score["blue"], score["red"])


@pytest.mark.gpu
def test_bf16_policy_rollout_within_bound_and_graph_equal():
    """DeviceRollout(policy_dtype=bfloat16) (opt-in): the first step's actor mean and value are
    within 2e-4 / 2e-2 of the fp32 rollout's on the same observations (bound stated in
    DeviceRollout's docstring; measured ≈5e-5 / 5e-3 in DESIGN §10a), and its graph replay is
    bit-identical to its eager loop."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from marlsoccer import SoccerBatch
    N, T = 256, 8
    torch.manual_seed(0)
    agent = Agent().cuda()
    firsts = {}
    for dt in (torch.float32, torch.bfloat16):
        b = SoccerBatch(N)
        b.reset(seed=31)
        ro = DeviceRollout(b, agent, RunningMeanStd((66,), device="cuda"), T, seed=4, deterministic=True,
                           update_normalizer=False, policy_dtype=dt)
        out = ro.collect()
        firsts[dt] = (out["actions"][0].clone(), out["values"][0].clone())
        b.close()
    a32, v32 = firsts[torch.float32]
    a16, v16 = firsts[torch.bfloat16]
    assert a16.dtype == torch.float32 and v16.dtype == torch.float32
    assert float((a16 - a32).abs().max()) <= 2e-4
    assert float((v16 - v32).abs().max()) <= 2e-2
    runs = []
    for graph in (False, True):
        b = SoccerBatch(N)
        b.reset(seed=31)
        ro = DeviceRollout(b, agent, RunningMeanStd((66,), device="cuda"), T, seed=4, graph=graph,
                           policy_dtype=torch.bfloat16)
        runs.append([{k: v.clone() for k, v in ro.collect().items()} for _ in range(3)])
        b.close()
    for a, g in zip(*runs):
        for k in a:
            assert torch.equal(a[k], g[k]), k
    b = SoccerBatch(64)
    with pytest.raises(ValueError):
        DeviceRollout(b, agent, RunningMeanStd((66,), device="cuda"), 2, policy_dtype=torch.float16)
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("max_steps", [120, 37, 10, 1])
def test_graph_eval_matches_eager_eval(max_steps):
    """evaluate(graph=True) returns exactly what the eager loop returns, red agents drawn from
    the generator included. The graph path runs the first steps eagerly, then replays a graph of
    min(GRAPH_CHUNK, max_steps - 1) captured steps for the rest of the episode: 120 steps
    (20 eager, 4 replays of 25), 37 (12 eager, 1 replay: not a multiple of the chunk), 10
    (1 eager, 1 replay of 9: shorter than a chunk), 1 (eager only: nothing is captured)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from marlsoccer.config import load_config
    from marlsoccer.evaluate import evaluate
    torch.manual_seed(0)
    agent = Agent().cuda()
    rms = RunningMeanStd(device="cuda")
    cfg = load_config()
    cfg["simulation"]["max_steps"] = max_steps
    eager = evaluate(agent, rms, 96, seed=5, config=cfg, generator_seed=3)
    graph = evaluate(agent, rms, 96, seed=5, config=cfg, generator_seed=3, graph=True)
    np.testing.assert_array_equal(graph["returns"], eager["returns"])
    np.testing.assert_array_equal(graph["score"], eager["score"])
    assert graph["steps"] == eager["steps"] == max_steps
    with pytest.raises(ValueError):
        evaluate(agent, rms, 4, config=cfg, graph=True, frames_every=10)


def test_evaluate_argument_errors_before_any_device_work():
    """evaluate() rejects an unknown red policy and graph=True with frames before it creates
    an env (so on CPU too)."""
    from marlsoccer.evaluate import evaluate
    agent, rms = Agent(), RunningMeanStd()
    with pytest.raises(ValueError, match="red must be"):
        evaluate(agent, rms, 4, red="greedy")
    with pytest.raises(ValueError, match="graph=True cannot take frames"):
        evaluate(agent, rms, 4, graph=True, frames_every=10)


@pytest.mark.gpu
def test_fused_policy_kernel_matches_reference_network():
    """ms_policy_forward (csrc/ms_policy.hip: both MLPs in one gfx950 kernel on the f32-input
    MFMA) on the notebook Agent's golden vectors: the actor mean and the value within 1e-5 of
    the reference network's outputs (policy.npz, produced by the notebook's own class); and on
    131 random rows (a ragged last tile) within 1e-5 of the same Agent run by torch on the GPU."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from marlsoccer.policy import FusedPolicy
    torch.manual_seed(0)
    agent = Agent().cuda()
    fp = FusedPolicy(agent)
    x = torch.from_numpy(FX["x"]).cuda()
    mean, value = fp.forward(x)
    np.testing.assert_allclose(mean.cpu().numpy(), FX["mean"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(value.cpu().numpy(), FX["value"][:, 0], rtol=0, atol=1e-5)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    x = (torch.randn((131, 66), generator=g, device="cuda") * 3).clamp(-10, 10)
    with torch.no_grad():
        rm, rv = agent.actor_mean(x), agent.critic(x)[:, 0]
    mean, value = fp.forward(x)
    np.testing.assert_allclose(mean.cpu().numpy(), rm.cpu().numpy(), rtol=0, atol=1e-5)
    np.testing.assert_allclose(value.cpu().numpy(), rv.cpu().numpy(), rtol=0, atol=1e-5)


@pytest.mark.gpu
def test_fused_policy_kernel_normalises_like_running_mean_std():
    """The kernel's fused normalisation of raw (N, 4, 66) env observations (blue agents: rows
    2N, row 2e + a at obs[e, a]) equals RunningMeanStd.normalize followed by the torch Agent,
    within 1e-5, with the run5 normaliser stats of the reference (policy.npz) and after a
    parameter update (pack() re-reads the parameters)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from marlsoccer import SoccerBatch
    from marlsoccer.policy import FusedPolicy
    n = 1000
    env = SoccerBatch(n)
    env.reset(seed=7)
    for t in range(5):
        env.step(torch.rand((n, 4, 3), device=env.device) * 2 - 1)
    torch.manual_seed(1)
    agent = Agent().to(env.device)
    rms = RunningMeanStd(device=env.device)
    rms.mean.copy_(torch.from_numpy(FX["run5_mean"]))
    rms.var.copy_(torch.from_numpy(FX["run5_var"]))
    fp = FusedPolicy(agent)
    for it in range(2):
        obs = env.obs
        den = rms.std + 1e-8
        mean, value = fp.forward(obs, rms.mean, den, group_rows=2, group_stride=264, row_stride=66, rows=2 * n)
        with torch.no_grad():
            xn = rms.normalize(obs[:, :2].reshape(-1, 66))
            rm, rv = agent.actor_mean(xn), agent.critic(xn)[:, 0]
        np.testing.assert_allclose(mean.cpu().numpy(), rm.cpu().numpy(), rtol=0, atol=1e-5)
        np.testing.assert_allclose(value.cpu().numpy(), rv.cpu().numpy(), rtol=0, atol=1e-5)
        with torch.no_grad():  # a parameter update, then re-pack
            for p in agent.parameters():
                p.add_(0.01 * torch.randn_like(p))
        fp.pack()
    env.close()


@pytest.mark.gpu
def test_fused_rollout_step_matches_torch_policy_rollout():
    """DeviceRollout's fused step (one ms_policy_run launch: normalisation, both MLPs, sampling,
    log-prob, storage and the env's blue actions) against the torch-module rollout from the same
    state and generator seed: the first step's stored actions, log-probs and values within 1e-5
    (same random draws: the kernel consumes eps from the same generator calls), obs and dones
    equal."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from marlsoccer import SoccerBatch
    N, T = 512, 1
    torch.manual_seed(0)
    agent = Agent().cuda()
    with torch.no_grad():
        agent.actor_logstd.copy_(torch.tensor([[-0.3, 0.1, 0.4]]))
    rms = RunningMeanStd((66,), device="cuda")
    rms.mean.copy_(torch.from_numpy(FX["run5_mean"]))
    rms.var.copy_(torch.from_numpy(FX["run5_var"]))
    outs = {}
    for pol in ("torch", "fused"):
        b = SoccerBatch(N)
        b.reset(seed=41)
        ro = DeviceRollout(b, agent, rms, T, seed=6, update_normalizer=False, policy=pol)
        assert ro.policy == pol
        outs[pol] = {k: v.clone() for k, v in ro.collect().items()}
        outs[pol]["full_actions"] = ro.full_actions.clone()
        b.close()
    a, f = outs["torch"], outs["fused"]
    assert torch.equal(a["obs"], f["obs"]) and torch.equal(a["dones"], f["dones"])
    for k in ("actions", "logprobs", "values"):
        assert float((a[k] - f[k]).abs().max()) <= 1e-5, k
    assert torch.equal(f["full_actions"][:, :2], f["actions"][0])
    assert torch.equal(a["full_actions"][:, 2:], f["full_actions"][:, 2:])  # the same red draws


@pytest.mark.gpu
def test_rollout_record_matches_torch_bookkeeping():
    """ms_rollout_record (one launch) == the torch ops of the torch-policy step (rewards, dones,
    finished-episode count and scores) on random env outputs, including ragged n (not a
    multiple of the wave) and accumulation over two calls; bad shapes raise before launching."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from marlsoccer.policy import rollout_record
    g = torch.Generator(device="cuda")
    g.manual_seed(4)
    for n in (1, 63, 4099):
        episodes = torch.zeros((), dtype=torch.int64, device="cuda")
        score_sum = torch.zeros((2,), dtype=torch.int64, device="cuda")
        want_ep, want_sc = 0, torch.zeros(2, dtype=torch.int64, device="cuda")
        for _ in range(2):
            rew = torch.randn((n, 4), generator=g, device="cuda")
            term = (torch.rand((n, 4), generator=g, device="cuda") < 0.2).to(torch.uint8)
            trunc = (torch.rand((n, 4), generator=g, device="cuda") < 0.3).to(torch.uint8)
            score = torch.randint(0, 7, (n, 2), generator=g, device="cuda", dtype=torch.int32)
            rewards = torch.full((n, 2), 7.0, device="cuda")
            next_done = torch.full((n, 2), 7.0, device="cuda")
            dones_next = torch.full((n, 2), 7.0, device="cuda")
            rollout_record(rew, term, trunc, score, rewards, next_done, dones_next, episodes, score_sum)
            assert torch.equal(rewards, rew[:, :2])
            done = (term[:, :2] | trunc[:, :2]).to(torch.float32)
            assert torch.equal(next_done, done) and torch.equal(dones_next, done)
            finished = trunc[:, 0].to(torch.bool)
            want_ep += int(finished.sum())
            want_sc += (score * finished[:, None]).sum(dim=0)
        assert int(episodes) == want_ep and torch.equal(score_sum, want_sc)
    with pytest.raises(ValueError):
        rollout_record(rew, term, trunc, score.to(torch.int64), rewards, next_done, None, episodes, score_sum)


@pytest.mark.gpu
def test_fused_rollout_episode_bookkeeping():
    """A fused-policy rollout across episode ends (max_steps 5, 12 steps): dones rows mark the
    truncation steps (the step after an episode's last one starts with done = 1), every env
    finishes two episodes, and the score sum equals the scores the env reported at those ends."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from marlsoccer import SoccerBatch
    from marlsoccer.config import load_config
    N, T = 300, 12
    cfg = load_config()
    cfg["simulation"]["max_steps"] = 5
    b = SoccerBatch(N, config=cfg)
    b.reset(seed=3)
    torch.manual_seed(0)
    agent = Agent().cuda()
    rms = RunningMeanStd((66,), device="cuda")
    ro = DeviceRollout(b, agent, rms, T, seed=2, update_normalizer=False)
    assert ro.policy == "fused"
    out = ro.collect()
    torch.cuda.synchronize()
    want = torch.zeros((T, N, 2), device="cuda")
    want[5] = 1.0   # steps 4 and 9 end the episodes: dones of the following steps
    want[10] = 1.0
    assert torch.equal(out["dones"], want)
    assert int(out["episodes"]) == 2 * N
    assert torch.equal(out["next_done"], torch.zeros((N, 2), device="cuda"))
    assert torch.isfinite(out["rewards"]).all() and float(out["rewards"].abs().sum()) > 0
    assert int(out["score_sum"].sum()) >= 0
    b.close()


@pytest.mark.gpu
def test_fused_rollout_ppo_first_epoch_ratio_near_one():
    """The fused rollout's stored log-probs and values are the kernel's (tanh by exp2/rcp, log-prob
    from logstd directly), not the torch modules': the PPO update recomputes them with
    Agent.get_action_and_value on the stored obs and actions (notebook L340-380), so its first-epoch
    ratio exp(new - old) is 1 only up to that difference. Over a 32-step rollout (goals, the
    normaliser updating between steps as in training) the ratio stays within 1e-4 of 1 and the
    values within 1e-4 (DeviceRollout's docstring states the deviation)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from marlsoccer import SoccerBatch
    N, T = 1024, 32
    torch.manual_seed(0)
    agent = Agent().cuda()
    with torch.no_grad():
        agent.actor_logstd.copy_(torch.tensor([[-0.5, 0.0, 0.3]]))
    rms = RunningMeanStd((66,), device="cuda")
    rms.mean.copy_(torch.from_numpy(FX["run5_mean"]))
    rms.var.copy_(torch.from_numpy(FX["run5_var"]))
    b = SoccerBatch(N)
    b.reset(seed=12)
    ro = DeviceRollout(b, agent, rms, T, seed=3, update_normalizer=False)
    assert ro.policy == "fused"
    out = ro.collect()
    with torch.no_grad():
        x = rms.normalize(out["obs"].reshape(-1, 66))
        _, newlogprob, _, newvalue = agent.get_action_and_value(x, out["actions"].reshape(-1, 3))
    ratio = torch.exp(newlogprob - out["logprobs"].reshape(-1))
    assert float((ratio - 1.0).abs().max()) <= 1e-4
    assert float((newvalue.reshape(-1) - out["values"].reshape(-1)).abs().max()) <= 1e-4
    b.close()
