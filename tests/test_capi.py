"""C-ABI checks that need no GPU: the library loads, exports every entry point declared in
include/marl_soccer.h, and its host-side numpy-RNG seeding matches numpy itself."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "marl_soccer.h")).read()
    return sorted(set(re.findall(r"^(?:const\s+)?(?:int|void|int64_t|char)\s*\*?\s*(ms_\w+)\s*\(", text, re.M)))


def test_header_declares_expected_api():
    syms = declared_symbols()
    for s in ("ms_create", "ms_reset", "ms_step", "ms_destroy", "ms_last_error", "ms_observe",
              "ms_export_state", "ms_import_state", "ms_seed_pcg64"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from marlsoccer import _native as N
    if not os.path.exists(N.LIB_PATH):
        import build_native
        build_native.build()
    import ctypes
    lib = ctypes.CDLL(N.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(N.EXPORTED) <= set(declared_symbols())


def test_abi_version_and_config_defaults():
    from marlsoccer import _native as N
    assert N.lib().ms_abi_version() == 5
    c = N.default_config()
    assert c.max_velocity == 200 and c.agent_mass == 10 and c.ball_mass == 1
    assert c.action_force_max == 150000.0 and c.action_torque_max == 1000.0 and c.max_steps == 1000
    assert c.autoreset == 1


def test_default_config_selects_specialised_step_kernel():
    """ms_create launches the constant-folded step kernel for parameters equal, bit for bit, to the
    reference's defaults (max_steps/autoreset excepted), the default-physics kernel for configs
    that change reward multipliers only, and the generic kernel for anything else."""
    from marlsoccer import _native as N
    from marlsoccer.config import load_config, to_ms_config
    assert N.config_specialised(N.default_config())
    cfg = load_config()
    assert N.config_specialised(to_ms_config(cfg, True))
    assert N.config_specialised(to_ms_config(cfg, False))
    cfg["simulation"]["max_steps"] = 70
    assert N.config_specialised(to_ms_config(cfg, True))
    assert N.config_specialised(N.default_config()) == 1
    # reward multipliers only: the default physics stays compile-time (mode 2); any physics value: generic
    for sect, key, val, mode in (("rewards", "score_difference_multiplier", 5.0, 2),
                                 ("rewards", "goal_conceded_penalty", 1.0, 2),
                                 ("rewards", "ball_proximity_multiplier", 0.003, 2),
                                 ("physics", "ball_mass", 2.0, 0), ("physics", "max_velocity", 150.0, 0),
                                 ("physics", "action_torque_max", 800.0, 0)):
        c = load_config()
        c[sect][key] = val
        assert N.config_specialised(to_ms_config(c, True)) == mode, key


@pytest.mark.parametrize("seed", [0, 1, 19, 123456, 2 ** 32 - 1, 2 ** 32, 2 ** 40 + 7, 2 ** 64 - 1, 2 ** 70 + 3])
def test_seed_sequence_matches_numpy(seed):
    from marlsoccer import _native as N
    got = N.pcg_state_for_seed(seed)
    st = np.random.default_rng(seed).bit_generator.state["state"]
    assert (int(got[0]) << 64 | int(got[1])) == st["state"]
    assert (int(got[2]) << 64 | int(got[3])) == st["inc"]


def test_seed_range_matches_vec_env_seeding():
    """SyncMultiAgentVecEnv.reset seeds env i with seed + i (marl_vecenv.py:23)."""
    from marlsoccer import _native as N
    out = N.pcg_states_for_range(19, 50)
    for i in range(50):
        st = np.random.default_rng(19 + i).bit_generator.state["state"]
        assert (int(out[i, 0]) << 64 | int(out[i, 1])) == st["state"]


def test_entropy_seed_is_fresh():
    from marlsoccer import _native as N
    a, b = N.pcg_state_for_seed(None), N.pcg_state_for_seed(None)
    assert not np.array_equal(a, b)


def test_create_without_device_fails_loudly():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    from marlsoccer import SoccerBatch
    with pytest.raises(RuntimeError):
        SoccerBatch(4)


def test_state_record_layout_matches_oracle():
    import oracle as orc
    from marlsoccer import _native as N
    assert N.ENV_STATE_DTYPE == orc.ENV_STATE_DTYPE
    assert N.ENV_STATE_DTYPE.itemsize == 1216
