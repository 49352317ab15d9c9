"""Frame-ring observations (ms_step_ring / ms_reset_ring, FrameRingBatch) on the GPU.

The ring is an alternative output layout of the same step: its window of three frames must
equal, bit for bit, the contiguous (N, 4, 66) observation (itself bit-exact against the
oracle in test_gpu_parity.py) at every step — across window advances, wraps to the ring's
start, goals, episode ends with auto-reset, masked resets and the generic-parameter kernel —
and the env state after the run must be identical. One run is also checked against the
oracle directly.
"""
import ctypes as C

import numpy as np
import pytest

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


def run_ring_vs_contiguous(ms, n, ring, steps, seed=7, mask_reset_at=None, autoreset=True, lanes=None, **over):
    config = cfg_dict(**over)
    a = ms.SoccerBatch(n, config=config, autoreset=autoreset)
    b = ms.FrameRingBatch(n, ring=ring, config=config, autoreset=autoreset)
    if lanes is not None:  # 2: ms_step_ring on the lane-pair launch (ms_step_pair_ring_kernel)
        a.set_lane_group(lanes)
        b.set_lane_group(lanes)
        assert a.lane_group == lanes and b.lane_group == lanes
    oa = a.reset(seed=seed).clone()
    ob = b.reset(seed=seed)
    assert ob.shape == (n, 4, 66) and b.window_index() == 0
    torch.testing.assert_close(ob, oa, rtol=0, atol=0)
    wraps = dones = 0
    for t in range(steps):
        act = torch.from_numpy(sh.hash_actions(n, t)).to(a.device)
        if mask_reset_at is not None and t == mask_reset_at:
            m = torch.zeros(n, dtype=torch.uint8, device=a.device)
            m[::3] = 1
            oa = a.reset(seed=seed + 1000, mask=m).clone()
            ob = b.reset(seed=seed + 1000, mask=m)
            torch.testing.assert_close(ob, oa, rtol=0, atol=0, msg=f"masked reset t={t}")
        if not autoreset and t % 17 == 16:
            a.reset(options={"use_full_random_positions": True})
            b.reset(options={"use_full_random_positions": True})
        pos_before = b.window_index()
        ra = a.step(act)
        rb = b.step(act)
        wraps += int(b.window_index() == 0 and pos_before != 0)
        for k in range(6):
            torch.testing.assert_close(rb[k], ra[k], rtol=0, atol=0, msg=f"output {k} t={t} pos={b.window_index()}")
        dones += int(ra.trunc[:, 0].sum())
    ea, eb = a.export_state(), b.export_state()
    assert ea.tobytes() == eb.tobytes()
    a.close()
    b.close()
    return wraps, dones


@pytest.mark.parametrize("lanes", [None, 2], ids=["default-launch", "lane-pair"])
@pytest.mark.parametrize("ring", [4, 6, 32])
def test_ring_matches_contiguous_with_autoresets(ms, ring, lanes):
    wraps, dones = run_ring_vs_contiguous(ms, 1000, ring, 90, max_steps=20, lanes=lanes)
    assert wraps >= 2 and dones > 0


@pytest.mark.parametrize("lanes", [None, 2], ids=["default-launch", "lane-pair"])
def test_ring_matches_contiguous_masked_reset_and_manual_reset(ms, lanes):
    run_ring_vs_contiguous(ms, 333, 8, 60, mask_reset_at=23, autoreset=False, lanes=lanes)


@pytest.mark.parametrize("lanes", [None, 2], ids=["default-launch", "lane-pair"])
def test_ring_matches_contiguous_staggered_episode_clocks(ms, lanes):
    # a masked reset with auto-reset on: the masked envs' episodes end 7 steps after the others', so
    # on steps where the window does not wrap a wave holds refilling and shifting envs at once (the
    # lane-pair ring kernel's three-frame path must then keep the shifting envs' frame t-2)
    wraps, dones = run_ring_vs_contiguous(ms, 1000, 32, 70, mask_reset_at=7, max_steps=20, lanes=lanes)
    assert dones > 0


@pytest.mark.parametrize("lanes", [None, 2], ids=["default-launch", "lane-pair"])
def test_ring_generic_kernel_matches_contiguous(ms, lanes):
    # non-default physics: the generic kernels (runtime parameters)
    run_ring_vs_contiguous(ms, 257, 6, 40, max_steps=15, ball_mass=1.5, lanes=lanes)


def test_ring_reward_config_lane_pair_matches_contiguous(ms):
    # reward multipliers only: the lane-pair ring kernel with the default physics compiled in (PM 2)
    run_ring_vs_contiguous(ms, 300, 8, 60, max_steps=25, score_difference_multiplier=5.0, goal_conceded_penalty=1.0,
                           lanes=2)


def test_ring_full_size_window_matches_contiguous(ms):
    # 65,536 envs (the bench batch): the ring's windows equal the contiguous obs over a wrap
    n, ring = 65536, 8
    a = ms.SoccerBatch(n)
    b = ms.FrameRingBatch(n, ring=ring)
    a.reset(seed=19)
    b.reset(seed=19)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    for t in range(2 * ring):
        act = torch.rand((n, 4, 3), device="cuda", generator=g) * 2 - 1
        ra, rb = a.step(act), b.step(act)
        assert torch.equal(rb.obs, ra.obs), f"t={t}"
        assert torch.equal(rb.rew, ra.rew)
    a.close()
    b.close()


@pytest.mark.parametrize("lanes", [None, 2], ids=["default-launch", "lane-pair"])
def test_ring_window_vs_oracle(ms, lanes):
    n, ring, seed = 64, 6, 19
    gpu = ms.FrameRingBatch(n, ring=ring, config=cfg_dict(max_steps=30))
    if lanes is not None:
        gpu.set_lane_group(lanes)
    ocfg = orc.MsConfig()
    mc = ms.to_ms_config(cfg_dict(max_steps=30), True)
    for name, _ in mc._fields_:
        setattr(ocfg, name, getattr(mc, name))
    ref = orc.OracleBatch(n, "f32", ocfg)
    pcg = np.stack([orc.pcg_from_seed(seed + i) for i in range(n)])
    np.testing.assert_array_equal(gpu.reset(seed=seed).cpu().numpy(), ref.reset(pcg, 0))
    for t in range(70):
        act = sh.hash_actions(n, t)
        out = gpu.step(torch.from_numpy(act).to(gpu.device))
        obs, rew, trunc, goal, score, bad = ref.step(act)
        np.testing.assert_array_equal(out.obs.cpu().numpy(), obs, err_msg=f"obs t={t}")
        np.testing.assert_array_equal(out.rew.cpu().numpy(), rew.astype(np.float32), err_msg=f"rew t={t}")
    gpu.close()


def test_ring_argument_errors(ms):
    from marlsoccer import _native as N
    with pytest.raises(ValueError):
        ms.FrameRingBatch(8, ring=5)
    b = ms.FrameRingBatch(8, ring=6)
    b.reset(seed=1)
    L = N.lib()
    act = torch.zeros((8, 4, 3), device=b.device)
    fr = C.c_void_p(b.frames.data_ptr())
    for R, pos, wrap in ((6, 4, 0), (6, -1, 0), (7, 0, 1), (2, 0, 1), (6, 0, 2)):
        rc = L.ms_step_ring(b._h, C.c_void_p(act.data_ptr()), fr, R, pos, wrap, None, None, None, None, None)
        assert rc == N.MS_ERR_INVALID_ARGUMENT, (R, pos, wrap)
    misaligned = C.c_void_p(b.frames.data_ptr() + 8)
    assert L.ms_step_ring(b._h, C.c_void_p(act.data_ptr()), misaligned, 6, 0, 1, None, None, None, None,
                          None) == N.MS_ERR_INVALID_ARGUMENT
    assert L.ms_reset_ring(b._h, None, None, 0, fr, 6, 4) == N.MS_ERR_INVALID_ARGUMENT
    with pytest.raises(NotImplementedError):
        b.step_into(act, None)
    b.close()
