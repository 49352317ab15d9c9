"""The north-star precision bound: the fp32 path against the reference's double precision.

See precision_common.py for the method and the bars. CPU tests here run the fp32 oracle (the
GPU kernel's arithmetic contract, bit-exact with it: test_gpu_parity.py) against the f64
oracle (reproduces the reference fixtures: test_oracle_golden.py); the GPU tests run the HIP
kernel itself against the f64 oracle. The mutant tests show the bars have teeth: a wrong
fused form in the fp32 contract breaks them.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

import golden_io as gio
import oracle as orc
import precision_common as pc


def _one_step_errors(name, precision="f32", lib=None):
    states, actions, cfg = pc.fixture_states(name)
    s32, o32, r32, f32 = pc.oracle_one_step(states, actions, cfg, precision, lib)
    s64, o64, r64, f64 = pc.oracle_one_step(states, actions, cfg, "f64")
    return pc.step_errors(s32, s64, o32, o64, r32, r64), f32, f64


@pytest.mark.parametrize("name", gio.TRAJ_NAMES)
def test_one_step_fp32_within_bound_of_f64(name):
    errs, f32, f64 = _one_step_errors(name)
    pc.flags_equal(f32, f64, name)
    pc.check_one_step(errs, pc.conditioning(name), name)


def test_horizons_from_identical_states():
    """Up to 120 steps from identical states at three points of every trajectory: positions,
    angles and rewards stay within 1e-5 of the f64 run for pc.HORIZON_BARS steps from every
    start (the horizons at which each quantity first leaves the bound are tabulated in
    DESIGN.md §4)."""
    for name in gio.TRAJ_NAMES:
        fx = gio.load(f"traj_{name}.npz")
        states, _, cfg = pc.fixture_states(name)
        T, n = fx["obs"].shape[:2]
        for t0 in (0, 100, 250):
            st0 = states[t0 * n:(t0 + 1) * n]
            runs = {}
            for prec in ("f32", "f64"):
                b = orc.OracleBatch(n, prec, cfg)
                b.import_state(st0)
                runs[prec] = b

            def make(prec):
                def run(k):
                    obs, rew = runs[prec].step(fx["actions"][t0 + k])[:2]
                    return runs[prec].export_state(), obs, rew
                return run

            h = pc.horizon(make("f32"), make("f64"), 120)
            for q, at_least in pc.HORIZON_BARS.items():
                assert h[q] > at_least, (name, t0, q, h)


MUTANTS = {
    # the impulse rotation's outer add with the wrong sign inside the fused form (cpvrotate)
    "vrotate_sign": ("static inline vec vrotate(vec a, vec b) { return v2(SMADD(a.x, b.x, -(a.y * b.y)),",
                     "static inline vec vrotate(vec a, vec b) { return v2(SMADD(a.x, b.x, +(a.y * b.y)),"),
    # the velocity update fused with its operands swapped: v * m^-1 + j instead of j * m^-1 + v
    "vmadd_operands": ("static inline vec vmadd(vec a, real s, vec c) { return v2(SMADD(a.x, s, c.x), SMADD(a.y, s, c.y)); }",
                       "static inline vec vmadd(vec a, real s, vec c) { return v2(SMADD(c.x, s, a.x), SMADD(c.y, s, a.y)); }"),
}


@pytest.fixture(scope="module")
def mutant_dir(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    return tmp_path_factory.mktemp("mutants")


@pytest.mark.parametrize("mutant", sorted(MUTANTS))
def test_mutated_fp32_contract_breaks_the_bound(mutant, mutant_dir):
    """A deliberately wrong fused form in the fp32 contract must fail the one-step bound."""
    src = open(os.path.join(orc.HERE, "soccer_oracle.c")).read()
    old, new = MUTANTS[mutant]
    assert src.count(old) == 1, mutant
    d = mutant_dir / mutant
    (d / "oracle").mkdir(parents=True)
    (d / "include").symlink_to(os.path.join(orc.ROOT, "include"))
    (d / "oracle" / "soccer_oracle.c").write_text(src.replace(old, new))
    so = d / "oracle" / "liborc_mutant.so"
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-std=gnu11", "-ffp-contract=off", "-fno-fast-math", "-DORC_F32",
                    "-pthread", "-o", str(so), str(d / "oracle" / "soccer_oracle.c"), "-lm"], check=True)
    lib = orc.load_path(str(so))
    caught = []
    for name in gio.TRAJ_NAMES:
        errs, f32, f64 = _one_step_errors(name, lib=lib)
        try:
            pc.flags_equal(f32, f64, name)
            pc.check_one_step(errs, pc.conditioning(name), name)
        except AssertionError as e:
            caught.append(str(e).splitlines()[0])
    assert caught, f"mutant {mutant} passed every bar"


def test_telescoping_return_f64():
    """SURVEY §8(c) T3 on the reference-precision oracle: a goal-free episode's return is the
    telescoped distance improvement minus the alive penalty (game.py:324-375, 425-433)."""
    n, T = 16, 1000
    b = orc.OracleBatch(n, "f64")
    b.reset(np.stack([orc.pcg_from_seed(100 + i) for i in range(n)]), 0)
    st0 = b.export_state()
    rng = np.random.default_rng(7)
    total = np.zeros(n)
    goals = np.zeros(n, bool)
    for t in range(T):
        if t == T - 1:
            st_last = b.export_state()
        obs, rew, trunc, goal, score, bad = b.step(rng.uniform(-1, 1, (n, 4, 3)).astype(np.float32))
        total += rew[:, 0]
        goals |= goal != 0
    assert trunc.all()
    keep = ~goals
    assert keep.sum() >= n // 2
    want = pc.telescoped_return(st0, st_last, T)
    # exported positions are fp32-rounded (3e-5 px at 400 px): 0.1 * 3e-5 * 4 terms
    np.testing.assert_allclose(total[keep], want[keep], rtol=0, atol=2e-5)
