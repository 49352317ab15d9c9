"""GPU (HIP kernel through the C-ABI) vs the oracle — the parity tests proper.

Bars:
  - vs the fp32 oracle (the kernel's arithmetic contract): bit-exact for every output and
    the full exported state, over trajectories that cross goals, soft resets, episode ends
    and auto-resets. (The north-star 1e-5 fp32 tolerance is implied by equality.)
  - vs the golden fixtures captured from the reference glue (identical input states):
    spawn positions exact after fp32 rounding, PCG64 stream exact, observations within
    1e-5, rewards within 1e-5 (+ fp32 relative rounding on synthetic teleports).
"""
import numpy as np
import pytest

import golden_io as gio
import oracle as orc
import sim_helpers as sh

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ms():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    import marlsoccer
    return marlsoccer


def cfg_dict(**over):
    from marlsoccer.config import load_config
    c = load_config()
    for k, v in over.items():
        sect = "simulation" if k == "max_steps" else ("physics" if k in c["physics"] else "rewards")
        c[sect][k] = v
    return c


def oracle_cfg(ms_cfg):
    o = orc.MsConfig()
    for name, _ in ms_cfg._fields_:
        setattr(o, name, getattr(ms_cfg, name))
    return o


def assert_state_equal(gpu_st, orc_st, where=""):
    for f in ("steps", "score_blue", "score_red", "mode", "hist_empty", "n_arb", "has_uint32", "uinteger",
              "pcg_state_hi", "pcg_state_lo", "pcg_inc_hi", "pcg_inc_lo"):
        np.testing.assert_array_equal(gpu_st[f], orc_st[f], err_msg=f"{where} {f}")
    for f in ("px", "py", "vx", "vy", "angle", "w", "vbx", "vby", "wb"):
        np.testing.assert_array_equal(gpu_st["body"][f], orc_st["body"][f], err_msg=f"{where} body.{f}")
    np.testing.assert_array_equal(gpu_st["snap"], orc_st["snap"], err_msg=f"{where} snap")
    for i in range(len(gpu_st)):
        k = int(orc_st["n_arb"][i])
        for f in ("pair", "count", "idle", "hash", "jn", "jt"):
            np.testing.assert_array_equal(gpu_st["arb"][f][i, :k], orc_st["arb"][f][i, :k],
                                          err_msg=f"{where} env {i} arb.{f}")


def run_pair(ms, n, steps, seed=19, mode_opts=None, chase=True, check_state_every=50, lanes=None, **over):
    config = cfg_dict(**over)
    gpu = ms.SoccerBatch(n, config=config, autoreset=True)
    if lanes is not None:  # 0: the per-lane kernel, 8: the lane-group kernel (the default below 8,192 envs)
        gpu.set_lane_group(lanes)
        assert gpu.lane_group == lanes
    ocfg = oracle_cfg(ms.to_ms_config(config, True))
    ref = orc.OracleBatch(n, "f32", ocfg)
    mode = ms.spawn_mode(mode_opts)
    pcg = np.stack([orc.pcg_from_seed(seed + i) for i in range(n)])
    go = gpu.reset(seed=seed, options=mode_opts).cpu().numpy()
    ro = ref.reset(pcg, mode)
    np.testing.assert_array_equal(go, ro)
    rng = np.random.default_rng(seed)
    chaser = np.arange(n) % 4
    counts = {"goals": 0, "dones": 0}
    for t in range(steps):
        if chase:
            st = ref.export_state()
            pos = np.stack([st["body"]["px"], st["body"]["py"]], -1)
            act = sh.chase_actions(pos, st["body"]["angle"][:, :4], rng, chaser)
        else:
            act = sh.hash_actions(n, t)
        out = gpu.step(torch.from_numpy(act).to(gpu.device))
        obs, rew, trunc, goal, score, bad = ref.step(act)
        assert bad == 0
        g_obs = out.obs.cpu().numpy()
        np.testing.assert_array_equal(out.goal.cpu().numpy(), goal, err_msg=f"goal t={t}")
        np.testing.assert_array_equal(out.score.cpu().numpy(), score, err_msg=f"score t={t}")
        np.testing.assert_array_equal(out.trunc.cpu().numpy().astype(bool), trunc, err_msg=f"trunc t={t}")
        assert not out.term.cpu().numpy().any()
        np.testing.assert_array_equal(out.rew.cpu().numpy(), rew.astype(np.float32), err_msg=f"rew t={t}")
        np.testing.assert_array_equal(g_obs, obs, err_msg=f"obs t={t}")
        counts["goals"] += int((goal != 0).sum())
        counts["dones"] += int(trunc[:, 0].sum())
        if check_state_every and (t % check_state_every == check_state_every - 1 or t == steps - 1):
            assert_state_equal(gpu.export_state(), ref.export_state(), f"t={t}")
    assert gpu.stats()["arbiter_overflow"] == 0 and ref.overflow() == 0
    gpu.close()
    return counts


def test_reset_modes_bitexact(ms):
    for opts in (None, {"use_full_random_positions": True}, {"use_fixed_positions": True}):
        n = 300
        gpu = ms.SoccerBatch(n)
        ref = orc.OracleBatch(n, "f32")
        pcg = np.stack([orc.pcg_from_seed(7 + i) for i in range(n)])
        go = gpu.reset(seed=7, options=opts).cpu().numpy()
        ro = ref.reset(pcg, ms.spawn_mode(opts))
        np.testing.assert_array_equal(go, ro)
        assert_state_equal(gpu.export_state(), ref.export_state(), str(opts))
        gpu.close()


LANES = [0, 8, 2]
LANE_IDS = ["per-lane", "lane-group", "lane-pair"]


@pytest.mark.parametrize("lanes", LANES, ids=LANE_IDS)
def test_trajectory_chase_bitexact(ms, lanes):
    c = run_pair(ms, 128, 1100, seed=19, lanes=lanes)
    assert c["goals"] > 10 and c["dones"] == 128, c


def test_trajectory_random_bitexact(ms):
    run_pair(ms, 256, 400, seed=3, chase=False, check_state_every=100)


@pytest.mark.parametrize("lanes", LANES, ids=LANE_IDS)
def test_short_episodes_full_random_bitexact(ms, lanes):
    c = run_pair(ms, 96, 500, seed=5, mode_opts={"use_full_random_positions": True}, max_steps=70,
                 score_difference_multiplier=5.0, goal_conceded_penalty=1.0, lanes=lanes)
    assert c["dones"] >= 96 * 7 and c["goals"] > 0, c


@pytest.mark.parametrize("lanes", LANES, ids=LANE_IDS)
def test_nondefault_physics_generic_kernel_bitexact(ms, lanes):
    """A config with other physics (speed cap, masses, damping, torque) runs the generic step
    kernel (parameters from the kernel arguments), bit for bit against the oracle."""
    over = dict(max_velocity=150, agent_mass=12, ball_mass=2, agent_friction=0.95, ball_friction=0.9,
                action_torque_max=800.0, max_steps=150)
    from marlsoccer import _native as N
    from marlsoccer.config import to_ms_config
    assert not N.config_specialised(to_ms_config(cfg_dict(**over), True))
    c = run_pair(ms, 96, 400, seed=23, lanes=lanes, **over)
    assert c["dones"] >= 96 * 2, c


def test_fixed_spawn_no_truncation_bitexact(ms):
    run_pair(ms, 64, 600, seed=11, mode_opts={"use_fixed_positions": True}, max_steps=0)


# ---- golden fixtures (reference glue) through the GPU path --------------------------------

def test_gpu_spawn_matches_reference_fixture(ms):
    fx = gio.load("spawn.npz")
    n = len(fx["seed"])
    gpu = ms.SoccerBatch(n)
    for mode in (0, 1, 2):
        sel = fx["mode"] == mode
        pcg = np.zeros((n, 4), np.uint64)
        pcg[:] = fx["pcg0"]
        mask = torch.from_numpy(sel.astype(np.uint8))
        gpu.reset(seed=pcg, options=[None, {"use_full_random_positions": True}, {"use_fixed_positions": True}][mode],
                  mask=mask)
    st = gpu.export_state()
    pos = np.stack([st["body"]["px"], st["body"]["py"]], -1)
    np.testing.assert_array_equal(pos, fx["pos"][:, 0].astype(np.float32))
    rng = np.stack([st["pcg_state_hi"], st["pcg_state_lo"], st["pcg_inc_hi"], st["pcg_inc_lo"],
                    st["has_uint32"].astype(np.uint64), st["uinteger"].astype(np.uint64)], -1)
    np.testing.assert_array_equal(rng, fx["rng"][:, 0])
    np.testing.assert_array_equal(st["body"]["angle"][:, :4], fx["angle"][:, 0].astype(np.float32))
    gpu.close()


def test_gpu_observations_match_reference_fixture(ms):
    fx = gio.load("obs.npz")
    n = len(fx["frames"])
    st = np.zeros((n,), orc.ENV_STATE_DTYPE)
    st["body"]["px"] = fx["pos"][..., 0]
    st["body"]["py"] = fx["pos"][..., 1]
    st["body"]["vx"] = fx["vel"][..., 0]
    st["body"]["vy"] = fx["vel"][..., 1]
    st["body"]["angle"][:, :4] = fx["angle"]
    st["body"]["w"][:, :4] = fx["w"]
    gpu = ms.SoccerBatch(n)
    gpu.import_state(st)
    got = gpu.observe().cpu().numpy()
    np.testing.assert_allclose(got, fx["frames"], rtol=0, atol=1e-5)
    ref = orc.OracleBatch(n, "f32")
    ref.import_state(st)
    np.testing.assert_array_equal(got, ref.observe())
    gpu.close()


@pytest.mark.parametrize("variant", ["default", "conceded"])
def test_gpu_rewards_match_reference_fixture(ms, variant):
    fx = gio.load("rewards.npz")
    n = len(fx["goal"])
    over = {} if variant == "default" else {"goal_conceded_penalty": 1.5, "ball_proximity_multiplier": 0.0}
    gpu = ms.SoccerBatch(n, config=cfg_dict(**over))
    got = gpu.debug_rewards(fx["prev"], fx["cur"], fx["goal"], np.zeros(n, np.uint8),
                            np.zeros((n, 2), np.int32)).cpu().numpy()
    np.testing.assert_allclose(got, fx[f"rew_{variant}"], rtol=1e-6, atol=1e-5)
    gpu.close()


def test_gpu_terminal_override(ms):
    n = 4
    gpu = ms.SoccerBatch(n, config=cfg_dict(score_difference_multiplier=5.0))
    pos = np.random.default_rng(0).uniform(20, 500, (n, 5, 2)).astype(np.float32)
    score = np.array([[0, 0], [2, 1], [0, 3], [4, 4]], np.int32)
    got = gpu.debug_rewards(pos, pos, np.array([0, 1, 2, 0], np.int8), np.ones(n, np.uint8), score).cpu().numpy()
    np.testing.assert_array_equal(got[:, 0], 5.0 * (score[:, 0] - score[:, 1]))
    gpu.close()


# ---- edge cases --------------------------------------------------------------------------

@pytest.mark.parametrize("lanes", LANES, ids=LANE_IDS)
def test_nonfinite_actions_skip_env_and_count(ms, lanes):
    n = 64
    gpu = ms.SoccerBatch(n)
    gpu.set_lane_group(lanes)
    gpu.reset(seed=1)
    before = gpu.export_state()
    act = torch.zeros((n, 4, 3), device=gpu.device)
    act[5, 2, 1] = float("nan")
    act[9, 0, 0] = float("inf")
    gpu.step(act)
    st = gpu.export_state()
    s = gpu.stats()
    assert s["nonfinite_envs"] == 2 and s["first_nonfinite_env"] == 5
    np.testing.assert_array_equal(st[[5, 9]]["body"]["px"], before[[5, 9]]["body"]["px"])
    assert (st["steps"][[5, 9]] == 0).all() and (np.delete(st["steps"], [5, 9]) == 1).all()
    rew = gpu.rew.cpu().numpy()
    assert np.isnan(rew[[5, 9], :2]).all() and np.isfinite(np.delete(rew, [5, 9], axis=0)).all()
    # the skipped envs' other outputs are defined (ABI 5): NaN obs, no episode end, no goal, score kept
    obs = gpu.obs.cpu().numpy()
    assert np.isnan(obs[[5, 9]]).all() and np.isfinite(np.delete(obs, [5, 9], axis=0)).all()
    assert (gpu.term.cpu().numpy()[[5, 9]] == 0).all() and (gpu.trunc.cpu().numpy()[[5, 9]] == 0).all()
    assert (gpu.goal.cpu().numpy()[[5, 9]] == 0).all() and (gpu.score.cpu().numpy()[[5, 9]] == 0).all()
    # the device path raises the reference's ValueError (soccer_env.py:116-117) when asked
    with pytest.raises(ValueError, match=r"Action contains non-finite values for agent 'agent_2'"):
        gpu.raise_if_nonfinite(act)
    gpu.raise_if_nonfinite()  # the count was cleared
    with pytest.raises(ValueError, match=r"non-finite values for agent 'agent_2'.*env 5"):
        gpu.step(act, check=True)
    gpu.step(torch.zeros_like(act), check=True)
    gpu.close()


def test_rollout_raises_on_nonfinite_policy_output(ms):
    from marlsoccer.rollout import Agent, DeviceRollout, RunningMeanStd
    n = 64
    gpu = ms.SoccerBatch(n)
    gpu.reset(seed=3)
    agent = Agent().to(gpu.device)
    with torch.no_grad():
        agent.actor_mean[-1].bias.fill_(float("nan"))
    ro = DeviceRollout(gpu, agent, RunningMeanStd(device=gpu.device), num_steps=4, deterministic=True)
    with pytest.raises(ValueError, match="non-finite"):
        ro.collect()
    gpu.close()


def test_side_stream_ordering(ms):
    """A batch bound to its own stream, driven from torch's default stream with freshly made
    action tensors: results equal a batch on the default stream (SoccerBatch orders the two
    streams and keeps temporaries alive for the kernel)."""
    n = 2048
    side = torch.cuda.Stream()
    a = ms.SoccerBatch(n, stream=side)
    b = ms.SoccerBatch(n)
    a.reset(seed=4)
    b.reset(seed=4)
    for t in range(40):
        act = torch.from_numpy(sh.hash_actions(n, t)).to(b.device) * 1.0  # a temporary per step
        oa = a.step(act).obs.clone()
        ob = b.step(act).obs.clone()
        del act
        torch.cuda.current_stream().synchronize()
        assert torch.equal(oa, ob), t
    a.close()
    b.close()


def test_single_env_and_ragged_sizes(ms):
    for n in (1, 31, 33, 63, 65, 1000):
        for lanes in LANES:
            c = run_pair(ms, n, 30, seed=n, chase=False, check_state_every=30, lanes=lanes)
            assert c["dones"] == 0


@pytest.mark.parametrize("lanes", LANES, ids=LANE_IDS)
def test_actions_out_of_range_are_clipped(ms, lanes):
    n = 32
    gpu = ms.SoccerBatch(n)
    gpu.set_lane_group(lanes)
    ref = orc.OracleBatch(n, "f32")
    gpu.reset(seed=2)
    ref.reset(np.stack([orc.pcg_from_seed(2 + i) for i in range(n)]), 0)
    for t in range(50):
        act = (sh.hash_actions(n, t) * 7.5).astype(np.float32)
        out = gpu.step(torch.from_numpy(act).to(gpu.device))
        obs = ref.step(act)[0]
        np.testing.assert_array_equal(out.obs.cpu().numpy(), obs)
    gpu.close()


# ---- full-size properties (BASELINE configs) ------------------------------------------------

@pytest.mark.parametrize("n,max_steps,steps,env0", [
    pytest.param(4096, 1000, 1020, 0, id="configs1-4096envs-whole-episode"),
    pytest.param(65536, 1000, 1020, 0, id="configs2-65536envs-whole-episode"),
    pytest.param(8192, 1000, 120, 3 * 8192, id="configs3-rank3-shard-8192envs-120steps"),
    pytest.param(32768, 512, 560, 5 * 32768, id="configs4-rank5-shard-32768envs-maxsteps512-whole-episode"),
])
def test_config_sizes_hash_actions_subsample(ms, n, max_steps, steps, env0):
    """The BASELINE configs' per-GPU batch sizes, with deterministic hash actions (a function of
    the global env index and the step; configs 1-2 over a whole 1,000-step episode plus its
    auto-reset, config 3's rank-3 shard (65,536 envs / 8 GPUs = 8,192, global envs
    24,576..32,767) for 120 steps, config 4's rank-5 shard (262,144 / 8 = 32,768, max_steps=512)
    over a whole episode plus its auto-reset). A shard is seeded and driven by its global env
    indices (seed 19 + g), as bench.py and marlsoccer.distributed do. At every step the rewards,
    truncation flags, goal flags and scores of a 64-env subsample match the fp32 oracle bit for bit,
    and every 20th step their obs; at the end the subsample's state equals the oracle's, the whole
    batch's is finite and inside the field, no arbiter overflowed. (Device-Philox uniform actions as in the bench:
    test_config5_whole_batch_one_gpu_subsample.)"""
    gpu = ms.SoccerBatch(n, config=cfg_dict(max_steps=max_steps))
    gpu.reset(seed=19 + env0)
    sub = np.linspace(0, n - 1, 64).astype(np.int64)
    sub_d = torch.from_numpy(sub).to(gpu.device)
    ref = orc.OracleBatch(64, "f32", oracle_cfg(gpu._cfg))
    ref.reset(np.stack([orc.pcg_from_seed(19 + env0 + int(i)) for i in sub]), 0)
    dones = 0
    for t in range(steps):
        act = sh.hash_actions(n, t, env0=env0)
        out = gpu.step(torch.from_numpy(act).to(gpu.device))
        robs, rrew, rtrunc, rgoal, rscore = ref.step(act[sub])[:5]
        dones += int(rtrunc[:, 0].sum())
        np.testing.assert_array_equal(out.rew[sub_d].cpu().numpy(), rrew.astype(np.float32), err_msg=f"rew t={t}")
        np.testing.assert_array_equal(out.trunc[sub_d].cpu().numpy().astype(bool), rtrunc, err_msg=f"trunc t={t}")
        np.testing.assert_array_equal(out.goal[sub_d].cpu().numpy(), rgoal, err_msg=f"goal t={t}")
        np.testing.assert_array_equal(out.score[sub_d].cpu().numpy(), rscore, err_msg=f"score t={t}")
        if t % 20 == 19 or t == max_steps - 1:
            np.testing.assert_array_equal(out.obs[sub_d].cpu().numpy(), robs, err_msg=f"t={t}")
    assert dones == 64 * (steps // max_steps)
    st = gpu.export_state()
    r = ref.export_state()
    for f in ("px", "py", "vx", "vy", "angle", "w"):
        np.testing.assert_array_equal(st["body"][f][sub], r["body"][f], err_msg=f"body.{f}")
    np.testing.assert_array_equal(st["steps"][sub], r["steps"])
    assert np.isfinite(st["body"]["px"]).all() and np.isfinite(st["body"]["vx"]).all()
    assert (st["body"]["px"] > -50).all() and (st["body"]["px"] < 850).all()
    assert (st["body"]["py"] > -50).all() and (st["body"]["py"] < 650).all()
    assert gpu.stats()["arbiter_overflow"] == 0
    gpu.close()


def test_config5_whole_batch_one_gpu_subsample(ms):
    """BASELINE config 5's whole batch on one GPU: 262,144 envs, max_steps=512, a whole episode
    plus its auto-reset (560 steps). Actions are uniform(-1, 1) from the device Philox (as in the
    bench); the 64-env subsample's rows are copied to the host and stepped through the fp32
    oracle, whose rewards, flags and scores (every step), obs (every 20th step) and final state
    must match the GPU's bit for bit."""
    n, max_steps, steps = 262144, 512, 560
    gpu = ms.SoccerBatch(n, config=cfg_dict(max_steps=max_steps))
    gpu.reset(seed=19)
    sub = np.linspace(0, n - 1, 64).astype(np.int64)
    sub_d = torch.from_numpy(sub).to(gpu.device)
    ref = orc.OracleBatch(64, "f32", oracle_cfg(gpu._cfg))
    ref.reset(np.stack([orc.pcg_from_seed(19 + int(i)) for i in sub]), 0)
    gen = torch.Generator(device=gpu.device)
    gen.manual_seed(1234)
    dones = 0
    for t in range(steps):
        act = torch.rand((n, 4, 3), generator=gen, device=gpu.device) * 2.0 - 1.0
        out = gpu.step(act)
        robs, rrew, rtrunc, rgoal, rscore = ref.step(act[sub_d].cpu().numpy())[:5]
        dones += int(rtrunc[:, 0].sum())
        np.testing.assert_array_equal(out.rew[sub_d].cpu().numpy(), rrew.astype(np.float32), err_msg=f"rew t={t}")
        np.testing.assert_array_equal(out.trunc[sub_d].cpu().numpy().astype(bool), rtrunc, err_msg=f"trunc t={t}")
        np.testing.assert_array_equal(out.goal[sub_d].cpu().numpy(), rgoal, err_msg=f"goal t={t}")
        np.testing.assert_array_equal(out.score[sub_d].cpu().numpy(), rscore, err_msg=f"score t={t}")
        if t % 20 == 19 or t == max_steps - 1:
            np.testing.assert_array_equal(out.obs[sub_d].cpu().numpy(), robs, err_msg=f"obs t={t}")
    assert dones == 64  # every subsampled env crossed its episode end and auto-reset
    g = gpu.export_state()
    r = ref.export_state()
    for f in ("px", "py", "vx", "vy", "angle", "w"):
        np.testing.assert_array_equal(g["body"][f][sub], r["body"][f], err_msg=f"body.{f}")
    np.testing.assert_array_equal(g["steps"][sub], r["steps"])
    assert gpu.stats()["arbiter_overflow"] == 0
    gpu.close()


@pytest.mark.parametrize("lanes,solve", [(0, 0), (8, 0), (16, 0), (8, 2), (16, 2), (2, 0)],
                         ids=["lanes0", "lanes8", "lanes16", "lanes8-rounds", "lanes16-rounds", "lanes2"])
def test_corner_pileups_spill_path_bitexact(ms, lanes, solve):
    """All four agents and the ball wedged into the corners and pushed into them: more contacts
    per env than the kernel's 8 register slots: contacts 9-11 are staged in LDS for the solver and
    12+ stay in the global spill buffer (SP) — the rare paths of real play, held here for 80 steps
    (up to 20 contacts per env) — bit for bit against the oracle. lanes 8/16: the lane-group
    kernel (contacts in LDS, the solve's first 8 in registers, pair tests over the group);
    solve 2: the contact solve in dependency-level rounds (two contacts per lane beyond 8 per env)
    wherever a wave's envs have at most 16 contacts."""
    n = 64
    gpu = ms.SoccerBatch(n)  # default physics: the specialised kernel
    assert gpu.specialised
    gpu.set_lane_group(lanes)
    gpu.set_group_solve(solve)
    assert gpu.lane_group == lanes and gpu.group_solve == solve
    gpu.reset(seed=5)
    st = gpu.export_state()
    rng = np.random.default_rng(0)
    corners = [(10.0, 10.0, 1.0, 1.0), (790.0, 10.0, -1.0, 1.0), (10.0, 590.0, 1.0, -1.0), (790.0, 590.0, -1.0, -1.0)]
    offs = [(17.0, 17.0), (47.0, 17.0), (17.0, 47.0), (47.0, 47.0)]
    sign = np.zeros((n, 2), np.float32)
    for i in range(n):
        cx, cy, sx, sy = corners[i % 4]
        sign[i] = (sx, sy)
        for a, (ox, oy) in enumerate(offs):
            j = rng.uniform(-1.5, 1.5, 2)
            st["body"]["px"][i, a] = cx + sx * (ox + j[0])
            st["body"]["py"][i, a] = cy + sy * (oy + j[1])
            st["body"]["angle"][i, a] = rng.uniform(-0.05, 0.05)
        st["body"]["px"][i, 4] = cx + sx * 74.0
        st["body"]["py"][i, 4] = cy + sy * rng.uniform(13.0, 20.0)
    for f in ("vx", "vy", "w", "vbx", "vby", "wb"):
        st["body"][f] = 0.0
    st["n_arb"] = 0
    st["hist_empty"] = 1
    gpu.import_state(st)
    ref = orc.OracleBatch(n, "f32")
    ref.import_state(st)
    most = 0
    for t in range(80):
        act = np.zeros((n, 4, 3), np.float32)
        act[:, :, 0] = -sign[:, None, 0]  # agents face +x (angle ~ 0): push into the corner
        act[:, :, 1] = -sign[:, None, 1]
        act[:, :, 2] = sh.hash_actions(n, t)[:, :, 2] * 0.2
        out = gpu.step(torch.from_numpy(act).to(gpu.device))
        obs, rew, trunc, goal, score, bad = ref.step(act)
        np.testing.assert_array_equal(out.obs.cpu().numpy(), obs, err_msg=f"obs t={t}")
        np.testing.assert_array_equal(out.rew.cpu().numpy(), rew.astype(np.float32), err_msg=f"rew t={t}")
        g = gpu.export_state()
        touching = (g["arb"]["idle"] == 0) & (np.arange(ms_max_arbiters())[None, :] < g["n_arb"][:, None])
        most = max(most, int((g["arb"]["count"] * touching).sum(1).max()))
        if t % 20 == 19:
            assert_state_equal(g, ref.export_state(), f"t={t}")
    assert most > 11, most  # both the LDS-staged (9-11) and the global (12+) spill paths ran
    assert gpu.stats()["arbiter_overflow"] == 0 and ref.overflow() == 0
    gpu.close()


def ms_max_arbiters():
    from marlsoccer import _native as N
    return N.MAX_ARBITERS


def test_long_horizon_subsample_bitexact(ms):
    """3,000 steps of 4,096 envs (three whole episodes, their synchronised auto-resets, goals and
    respawns): a 64-env subsample bit for bit against the fp32 oracle every 250 steps — obs,
    rewards, flags, scores — and the complete state (bodies, history, contact cache, RNG) at
    the end: no drift over long horizons."""
    n, steps = 4096, 3000
    gpu = ms.SoccerBatch(n)
    gpu.reset(seed=19)
    sub = np.arange(0, n, 64)
    ref = orc.OracleBatch(len(sub), "f32")
    ref.reset(np.stack([orc.pcg_from_seed(19 + int(i)) for i in sub]), 0)
    goals = 0
    for t in range(steps):
        act = sh.hash_actions(n, t)
        out = gpu.step(torch.from_numpy(act).to(gpu.device))
        obs, rew, trunc, goal, score, bad = ref.step(act[sub])
        assert bad == 0
        goals += int((goal != 0).sum())
        if t % 250 == 249:
            np.testing.assert_array_equal(out.obs.cpu().numpy()[sub], obs, err_msg=f"obs t={t}")
            np.testing.assert_array_equal(out.rew.cpu().numpy()[sub], rew.astype(np.float32), err_msg=f"rew t={t}")
            np.testing.assert_array_equal(out.goal.cpu().numpy()[sub], goal, err_msg=f"goal t={t}")
            np.testing.assert_array_equal(out.score.cpu().numpy()[sub], score, err_msg=f"score t={t}")
            np.testing.assert_array_equal(out.trunc.cpu().numpy()[sub].astype(bool), trunc, err_msg=f"trunc t={t}")
    assert_state_equal(gpu.export_state()[sub], ref.export_state(), "end")
    assert gpu.stats()["arbiter_overflow"] == 0
    gpu.close()


@pytest.mark.parametrize("lanes", LANES, ids=LANE_IDS)
def test_obs_fallback_for_operands_outside_fast_domain_bitexact(ms, lanes):
    """Frames whose operands fall outside the reduced-range division's domain (velocities and
    spins below 2^-100, in the t-2 snapshot, the step-start state and the new state) take the
    IEEE path for those lanes only; lanes of the same waves inside the domain keep the fast
    path. Obs, rewards and state bit for bit against the fp32 oracle."""
    n = 128
    gpu = ms.SoccerBatch(n)
    assert gpu.specialised
    gpu.set_lane_group(lanes)
    gpu.reset(seed=11)
    for _ in range(3):  # leave the refilled stacks: the next steps emit t-2, t-1, t
        gpu.step(torch.zeros((n, 4, 3), device=gpu.device))
    st = gpu.export_state()
    odd = np.arange(n) % 2 == 1
    for f in ("vx", "vy", "w"):
        st["body"][f][:, :4] = 0.0
    st["body"]["vx"][odd, 1] = 1e-32     # below 2^-100: outside the fast domain
    st["body"]["w"][odd, 2] = -3e-33
    st["body"]["vy"][np.arange(n) % 4 == 2, 0] = 2e-38
    st["snap"][odd, 0, 10 + 3] = 5e-34   # snapshot t-2: vx of agent 3
    st["snap"][~odd, 0, 22 + 0] = 0.0
    b = st["body"]  # snapshot t-1 is the step-start body state
    st["snap"][:, 1] = np.concatenate([b["px"], b["py"], b["vx"][:, :4], b["vy"][:, :4], b["angle"][:, :4],
                                       b["w"][:, :4]], axis=1)
    assert int(st["hist_empty"].max()) == 0
    gpu.import_state(st)
    ref = orc.OracleBatch(n, "f32")
    ref.import_state(st)
    for t in range(6):
        act = np.zeros((n, 4, 3), np.float32)
        act[::3, 0, 0] = 0.5  # some envs move, so lanes of one wave differ
        out = gpu.step(torch.from_numpy(act).to(gpu.device))
        obs, rew, trunc, goal, score, bad = ref.step(act)
        np.testing.assert_array_equal(out.obs.cpu().numpy(), obs, err_msg=f"obs t={t}")
        np.testing.assert_array_equal(out.rew.cpu().numpy(), rew.astype(np.float32), err_msg=f"rew t={t}")
    assert_state_equal(gpu.export_state(), ref.export_state(), "end")
    gpu.close()


@pytest.mark.parametrize("n,lanes,over,solve", [
    pytest.param(1000, 8, {}, 0, id="1000envs-8lanes"),
    pytest.param(1000, 8, {}, 1, id="1000envs-8lanes-serial"),
    pytest.param(1000, 8, {}, 2, id="1000envs-8lanes-rounds"),
    pytest.param(333, 16, {}, 0, id="333envs-16lanes"),
    pytest.param(333, 16, {}, 2, id="333envs-16lanes-rounds"),
    pytest.param(96, 8, dict(max_velocity=150, agent_mass=12, ball_mass=2, agent_friction=0.95,
                             action_torque_max=800.0, goal_conceded_penalty=1.0), 0, id="96envs-8lanes-generic"),
    pytest.param(96, 8, dict(max_velocity=150, agent_mass=12, ball_mass=2, agent_friction=0.95,
                             action_torque_max=800.0, goal_conceded_penalty=1.0), 2, id="96envs-8lanes-generic-rounds"),
    pytest.param(1000, 2, {}, 0, id="1000envs-2lanes"),
    pytest.param(333, 2, {}, 0, id="333envs-2lanes"),
    pytest.param(96, 2, dict(max_velocity=150, agent_mass=12, ball_mass=2, agent_friction=0.95,
                             action_torque_max=800.0, goal_conceded_penalty=1.0), 0, id="96envs-2lanes-generic"),
])
def test_lane_group_kernel_bitexact(ms, n, lanes, over, solve):
    """ms_step's lane-group kernel (ms_set_lane_group: G lanes per env, the default for batches
    of at most the device's lanes / 8 envs) against the one-lane-per-env kernel and the fp32
    oracle on every env: chase actions (goals, soft resets), episode ends and auto-resets
    (max_steps 60), ragged last waves (1,000 and 333 envs). Obs, rewards, goals, scores and flags
    at every step; the whole state (bodies, history, arbiter cache, RNG) and the cache tallies at
    the end. The generic-parameter case runs the kernel instantiation without constant folding.
    solve (ms_set_group_solve) runs the contact solve's automatic choice, the serial halves only
    or the dependency-level rounds wherever they apply."""
    steps = 150
    cfg = cfg_dict(max_steps=60, **over)
    a = ms.SoccerBatch(n, config=cfg)
    b = ms.SoccerBatch(n, config=cfg)
    a.set_lane_group(0)
    b.set_lane_group(lanes)
    b.set_group_solve(solve)
    assert a.lane_group == 0 and b.lane_group == lanes and b.group_solve == solve
    assert a.specialised == (not over)
    ref = orc.OracleBatch(n, "f32", oracle_cfg(a._cfg))
    pcg = np.stack([orc.pcg_from_seed(29 + i) for i in range(n)])
    a.reset(seed=29)
    b.reset(seed=29)
    ref.reset(pcg, 0)
    rng = np.random.default_rng(29)
    chaser = np.arange(n) % 4
    goals = 0
    for t in range(steps):
        st = ref.export_state()
        pos = np.stack([st["body"]["px"], st["body"]["py"]], -1)
        act = sh.chase_actions(pos, st["body"]["angle"][:, :4], rng, chaser)
        at = torch.from_numpy(act).to(a.device)
        oa = a.step(at)
        ob = b.step(at)
        obs, rew, trunc, goal, score, bad = ref.step(act)
        assert bad == 0
        goals += int((goal != 0).sum())
        np.testing.assert_array_equal(ob.obs.cpu().numpy(), obs, err_msg=f"obs t={t}")
        np.testing.assert_array_equal(ob.rew.cpu().numpy(), rew.astype(np.float32), err_msg=f"rew t={t}")
        np.testing.assert_array_equal(ob.goal.cpu().numpy(), goal, err_msg=f"goal t={t}")
        np.testing.assert_array_equal(ob.score.cpu().numpy(), score, err_msg=f"score t={t}")
        np.testing.assert_array_equal(ob.trunc.cpu().numpy().astype(bool), trunc, err_msg=f"trunc t={t}")
        np.testing.assert_array_equal(oa.obs.cpu().numpy(), obs, err_msg=f"per-lane obs t={t}")
    assert goals > 0 or n < 300, goals
    assert_state_equal(b.export_state(), ref.export_state(), "lane-group end")
    assert_state_equal(a.export_state(), ref.export_state(), "per-lane end")
    sa, sb = a.stats(), b.stats()
    assert sb["env_steps"] == sa["env_steps"] == n * steps
    assert sb["cache_entries_read"] == sa["cache_entries_read"]
    assert sb["cache_entries_written"] == sa["cache_entries_written"]
    assert sb["arbiter_overflow"] == 0 and ref.overflow() == 0
    a.close()
    b.close()


@pytest.mark.parametrize("n,max_steps,steps", [
    pytest.param(32768, 512, 530, id="configs4-shard-32768envs-maxsteps512"),
    pytest.param(65536, 1000, 150, id="configs2-65536envs"),
])
def test_lane_pair_full_size_equals_per_lane(ms, n, max_steps, steps):
    """The lane-pair kernel (two lanes per env) against the one-lane-per-env kernel on every env of
    a full-size batch (BASELINE configs[4]'s per-GPU shard across its auto-reset, configs[2]'s
    65,536 envs): obs, rewards, flags, goals and scores compared on the device at every step, the
    whole exported state at the end, and a 32-env subsample against the fp32 oracle."""
    cfg = cfg_dict(max_steps=max_steps)
    a = ms.SoccerBatch(n, config=cfg)
    b = ms.SoccerBatch(n, config=cfg)
    a.set_lane_group(0)
    b.set_lane_group(2)
    assert b.step_kernel == "ms_step_pair_kernel" and a.step_kernel == "ms_step_kernel"
    a.reset(seed=19)
    b.reset(seed=19)
    sub = np.linspace(0, n - 1, 32).astype(np.int64)
    ref = orc.OracleBatch(len(sub), "f32", oracle_cfg(a._cfg))
    ref.reset(np.stack([orc.pcg_from_seed(19 + int(i)) for i in sub]), 0)
    gen = torch.Generator(device=a.device)
    gen.manual_seed(77)
    for t in range(steps):
        act = torch.rand((n, 4, 3), generator=gen, device=a.device) * 2.0 - 1.0
        oa = a.step(act)
        ob = b.step(act)
        for f in ("obs", "rew", "trunc", "goal", "score", "term"):
            assert torch.equal(getattr(oa, f), getattr(ob, f)), f"{f} t={t}"
        robs = ref.step(act[torch.from_numpy(sub).to(a.device)].cpu().numpy())[0]
        if t % 25 == 24:
            np.testing.assert_array_equal(ob.obs.cpu().numpy()[sub], robs, err_msg=f"oracle obs t={t}")
    assert_state_equal(b.export_state(), a.export_state(), "end")
    sa, sb = a.stats(), b.stats()
    assert sb["env_steps"] == sa["env_steps"] == n * steps
    assert sb["cache_entries_read"] == sa["cache_entries_read"]
    assert sb["cache_entries_written"] == sa["cache_entries_written"]
    assert sb["arbiter_overflow"] == 0
    a.close()
    b.close()


def test_kernel_switching_between_steps_bitexact(ms):
    """The step kernels leave one state format, so a batch may change kernels between steps: lane
    pairs, lane groups (8, 16), one lane per env, and the K-step launch, in an irregular order, with
    chase actions, goals and auto-resets (max_steps 40). The lane-pair kernel carries its fast-path
    range decisions of the t-1 / t-2 snapshots in the history pad (MS_PAIR_RANGE_CACHE); every other
    kernel stores +0 there, so after a switch the pair kernel takes the IEEE frame path until its own
    decisions are in place. Obs and rewards at every step and the whole state at the end against the
    fp32 oracle."""
    n = 320
    cfg = cfg_dict(max_steps=40)
    gpu = ms.SoccerBatch(n, config=cfg)
    ref = orc.OracleBatch(n, "f32", oracle_cfg(gpu._cfg))
    pcg = np.stack([orc.pcg_from_seed(41 + i) for i in range(n)])
    gpu.reset(seed=41)
    ref.reset(pcg, 0)
    rng = np.random.default_rng(41)
    chaser = np.arange(n) % 4
    plan = [2, 2, 2, 8, 2, 2, 0, 2, 2, 2, "n3", 2, 2, 16, 2, 8, 8, 2, 2, 2, "n2", 0, 2, 2, 2] * 4
    t = 0
    for what in plan:
        if isinstance(what, str):  # a K-step launch (lane pairs)
            K = int(what[1:])
            gpu.set_lane_group(2)
            acts, want = [], []
            for _ in range(K):
                st = ref.export_state()
                pos = np.stack([st["body"]["px"], st["body"]["py"]], -1)
                act = sh.chase_actions(pos, st["body"]["angle"][:, :4], rng, chaser)
                obs, rew, trunc, goal, score, bad = ref.step(act)
                assert bad == 0
                acts.append(act)
                want.append((obs, rew))
            out = gpu.step_n(torch.from_numpy(np.stack(acts)).to(gpu.device))
            for k, (obs, rew) in enumerate(want):
                np.testing.assert_array_equal(out.obs[k].cpu().numpy(), obs, err_msg=f"step_n obs t={t + k}")
                np.testing.assert_array_equal(out.rew[k].cpu().numpy(), rew.astype(np.float32),
                                              err_msg=f"step_n rew t={t + k}")
            t += K
            continue
        gpu.set_lane_group(what)
        st = ref.export_state()
        pos = np.stack([st["body"]["px"], st["body"]["py"]], -1)
        act = sh.chase_actions(pos, st["body"]["angle"][:, :4], rng, chaser)
        o = gpu.step(torch.from_numpy(act).to(gpu.device))
        obs, rew, trunc, goal, score, bad = ref.step(act)
        assert bad == 0
        np.testing.assert_array_equal(o.obs.cpu().numpy(), obs, err_msg=f"obs t={t} lanes={what}")
        np.testing.assert_array_equal(o.rew.cpu().numpy(), rew.astype(np.float32), err_msg=f"rew t={t} lanes={what}")
        t += 1
    assert_state_equal(gpu.export_state(), ref.export_state(), "end")
    gpu.close()
