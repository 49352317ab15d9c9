"""The north-star precision bound on the GPU: the HIP kernel (fp32) against the f64 oracle
(the reference's precision) on identical states — precision_common.py has the method and the
bars — and SURVEY §8(c)'s T3 invariant (a goal-free episode's return telescopes) over a full
1,000-step episode of 4,096 envs."""
import numpy as np
import pytest

import golden_io as gio
import oracle as orc
import precision_common as pc

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ms():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    import marlsoccer
    return marlsoccer


def gpu_one_step(ms, name, states, actions):
    gpu = ms.SoccerBatch(len(states), config=pc.config_json_for(name), autoreset=True)
    gpu.import_state(states)
    out = gpu.step(torch.from_numpy(actions).to(gpu.device))
    res = (gpu.export_state(), out.obs.cpu().numpy(), out.rew.cpu().numpy(),
           {"goal": out.goal.cpu().numpy(), "trunc": out.trunc.cpu().numpy().astype(bool),
            "score": out.score.cpu().numpy()})
    assert gpu.stats()["arbiter_overflow"] == 0
    gpu.close()
    return res


@pytest.mark.parametrize("name", gio.TRAJ_NAMES)
def test_gpu_one_step_within_bound_of_f64(ms, name):
    """Every state of the golden trajectory, imported into the GPU env (one env per state) and
    into the f64 oracle, stepped once with the fixture's action: the kernel's fp32 step is
    within the north-star bound of the reference precision, flags and scores bit-exact."""
    states, actions, cfg = pc.fixture_states(name)
    s32, o32, r32, f32 = gpu_one_step(ms, name, states, actions)
    s64, o64, r64, f64 = pc.oracle_one_step(states, actions, cfg, "f64")
    pc.flags_equal(f32, f64, name)
    pc.check_one_step(pc.step_errors(s32, s64, o32, o64, r32, r64), pc.conditioning(name), name)


def test_gpu_horizons_from_identical_states(ms):
    """1, 5, 30 and 120 steps of the GPU env and the f64 oracle from identical states at three
    points of every golden trajectory: positions, angles, rewards and position-derived
    observations within 1e-5 for pc.HORIZON_BARS steps."""
    for name in gio.TRAJ_NAMES:
        fx = gio.load(f"traj_{name}.npz")
        states, _, cfg = pc.fixture_states(name)
        n = fx["obs"].shape[1]
        for t0 in (0, 100, 250):
            st0 = states[t0 * n:(t0 + 1) * n]
            gpu = ms.SoccerBatch(n, config=pc.config_json_for(name), autoreset=True)
            gpu.import_state(st0)
            ref = orc.OracleBatch(n, "f64", cfg)
            ref.import_state(st0)

            def run_gpu(k):
                out = gpu.step(torch.from_numpy(np.ascontiguousarray(fx["actions"][t0 + k])).to(gpu.device))
                return gpu.export_state(), out.obs.cpu().numpy(), out.rew.cpu().numpy()

            def run_ref(k):
                obs, rew = ref.step(fx["actions"][t0 + k])[:2]
                return ref.export_state(), obs, rew

            h = pc.horizon(run_gpu, run_ref, 120)
            gpu.close()
            for q, at_least in pc.HORIZON_BARS.items():
                assert h[q] > at_least, (name, t0, q, h)


def test_gpu_telescoping_return_full_episode(ms):
    """SURVEY §8(c) T3 on the GPU: 4,096 envs, one whole 1,000-step episode of uniform(-1, 1)
    actions; for every env without a goal the sum of its fp32 rewards equals the telescoped
    distance improvement of its first and last states minus 999 alive penalties
    (game.py:324-375; the terminal step's reward is score_difference_multiplier * 0 = 0,
    game.py:425-433), within the north-star 1e-5 (the fp32 oracle, the kernel's contract, is
    within 4e-7 on 256 envs: the rewards' difference-of-squares form telescopes almost
    exactly)."""
    n, T = 4096, 1000
    gpu = ms.SoccerBatch(n)
    gpu.reset(seed=19)
    st0 = gpu.export_state()
    gen = torch.Generator(device=gpu.device)
    gen.manual_seed(77)
    total = torch.zeros(n, dtype=torch.float64, device=gpu.device)
    goals = torch.zeros(n, dtype=torch.bool, device=gpu.device)
    st_last = None
    for t in range(T):
        if t == T - 1:
            st_last = gpu.export_state()
        out = gpu.step(torch.rand((n, 4, 3), generator=gen, device=gpu.device) * 2.0 - 1.0)
        total += out.rew[:, 0].double()
        goals |= out.goal != 0
    assert bool(out.trunc.all())
    keep = ~goals.cpu().numpy()
    assert keep.sum() > n // 2
    want = pc.telescoped_return(st0, st_last, T)
    got = total.cpu().numpy()
    np.testing.assert_allclose(got[keep], want[keep], rtol=0, atol=1e-5)
    # envs with a goal do not telescope (the soft reset teleports the bodies): sanity only
    assert np.isfinite(got).all()
    gpu.close()
