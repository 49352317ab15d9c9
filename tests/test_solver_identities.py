"""Float identities the contact solve's restatements rely on (CPU, numpy float32).

The GPU kernels compute two parts of cpArbiterApplyImpulse (Chipmunk's contact solve, restated by
the fp32 oracle `oracle/soccer_oracle.c` `orc_space_solve`, soccer_oracle.c:790-815) in forms that
differ from the oracle's text, and the GPU parity tests prove them bit-exact on trajectories. These
tests pin the float reasoning behind each form on edge values (signed zeros, ties with the bounds,
denormals), so a regression in the argument shows up without a GPU:

1. `fclamp_sym(f, M)` (ms_device.h) = fclamp(f, -M, M) with fmaxr/fminr's select semantics, as
   `M > 0 ? med3(f, -M, M) : M`.
2. The lane-group kernel's velocity half forms the normal impulse as ((-bounce) - vrn) * nMass
   instead of -(bounce + vrn) * nMass: the two differ at most in the sign of an exact zero, and
   the accumulation fmaxr(jnOld + jn, 0) with jnOld >= +0 (never -0) gives the same bits.
3. Its bias half applies vrotate(n, (d, +0)) instead of vmult(n, d): component by component
   equal but for the sign of an exact zero; bias velocities start at +0 and are never -0, so the
   velocity update fma(J, m, v) gives the same bits.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def bits(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


def fmaxr(a, b):  # cpfmax: (a > b) ? a : b
    return np.where(a > b, a, b).astype(np.float32)


def fminr(a, b):  # cpfmin: (a < b) ? a : b
    return np.where(a < b, a, b).astype(np.float32)


def fclamp(f, lo, hi):
    return fminr(fmaxr(f, lo), hi)


def med3(a, b, c):
    """Median of three non-NaN floats whose median value is attained by one operand; returns that
    operand's bits (v_med3_f32 on distinct bounds -M < M)."""
    lo, hi = np.minimum(b, c), np.maximum(b, c)
    return np.where(a < lo, lo, np.where(a > hi, hi, a)).astype(np.float32)


def fclamp_sym(f, M):
    return np.where(M > 0, med3(f, -M, M), M).astype(np.float32)


def edge_values(rng, n):
    base = np.array([0.0, -0.0, 1.0, -1.0, 0.5, -0.5, 1e-40, -1e-40, 3.4e38, -3.4e38, 1e-7, -1e-7,
                     0.25, -0.25, 7.0, -7.0], np.float32)
    rnd = (rng.standard_normal(n) * rng.choice([1e-3, 1.0, 1e3], n)).astype(np.float32)
    return np.concatenate([base, rnd])


def test_fclamp_sym_equals_fclamp_bitwise():
    rng = np.random.default_rng(0)
    f = edge_values(rng, 4000)
    M = np.concatenate([edge_values(rng, 4000), f[:64]])  # includes M == +-f (ties with a bound)
    F, MM = np.meshgrid(f, M)
    F, MM = F.ravel(), MM.ravel()
    ref = fclamp(F, (-MM).astype(np.float32), MM)
    got = fclamp_sym(F, MM)
    assert np.array_equal(bits(ref), bits(got))


def test_velocity_half_normal_impulse_form():
    rng = np.random.default_rng(1)
    b = edge_values(rng, 600)
    v = np.concatenate([edge_values(rng, 600)[:300], -b[:300]])  # exact cancellations bounce + vrn = 0
    B, V = np.meshgrid(b, v)
    B, V = B.ravel(), V.ravel()
    nm = np.abs(edge_values(rng, B.size - 32))[: B.size].astype(np.float32)
    nm = np.resize(nm, B.size)
    old = np.abs(np.resize(edge_values(rng, 100), B.size)).astype(np.float32)  # jnOld >= +0, never -0
    old = np.where(old == 0, f32(0.0), old).astype(np.float32)
    with np.errstate(over="ignore", invalid="ignore"):
        j_ref = (-(B + V)).astype(np.float32) * nm
        j_alt = ((-B) - V).astype(np.float32) * nm
        acc_ref = fmaxr((old + j_ref).astype(np.float32), f32(0.0))
        acc_alt = fmaxr((old + j_alt).astype(np.float32), f32(0.0))
    ok = np.isfinite(j_ref) & np.isfinite(acc_ref)
    # the two impulses differ at most in the sign of zero ...
    diff = bits(j_ref) != bits(j_alt)
    assert np.all((j_ref[diff & ok] == 0) & (j_alt[diff & ok] == 0))
    # ... and the accumulated impulse is identical
    assert np.array_equal(bits(acc_ref[ok]), bits(acc_alt[ok]))


def test_bias_half_impulse_form():
    rng = np.random.default_rng(2)
    ang = rng.uniform(-np.pi, np.pi, 2000)
    n = np.stack([np.cos(ang), np.sin(ang)], 1).astype(np.float32)
    n = np.concatenate([n, np.array([[1, 0], [0, 1], [-1, 0], [0, -1], [-0.6, -0.8], [0.6, -0.8]], np.float32)])
    for d in (f32(0.0), f32(1e-40), f32(-1e-40), f32(2.5), f32(-3.0e-3)):
        mult = (n * d).astype(np.float32)
        # vrotate(n, (d, +0)): (fma(n.x, d, -(n.y * 0)), fma(n.x, 0, n.y * d)); the products are
        # exact or round once, the added term is a signed zero, so the f64 evaluation is exact
        rx = (n[:, 0].astype(np.float64) * d + (-(n[:, 1] * f32(0.0))).astype(np.float64)).astype(np.float32)
        ry = (n[:, 0].astype(np.float64) * 0.0 + (n[:, 1] * d).astype(np.float64)).astype(np.float32)
        rot = np.stack([rx, ry], 1)
        diff = bits(mult) != bits(rot)
        assert np.all((mult[diff] == 0) & (rot[diff] == 0)), "differ only in the sign of a zero"
        # bias velocity update fma(J, m, v) with v never -0: the same bits either way
        for m in (f32(0.0), f32(0.25), f32(1.5)):
            for v in (f32(0.0), f32(0.75), f32(-2.0)):
                a = (mult.astype(np.float64) * m + np.float64(v)).astype(np.float32)
                b = (rot.astype(np.float64) * m + np.float64(v)).astype(np.float32)
                zero_prod = (mult * m == 0) | (rot * m == 0)
                # wherever the two products differ they are zeros, and zero + v is exact
                assert np.array_equal(bits(a[zero_prod]), bits(b[zero_prod]))
                assert np.array_equal(bits(a[~zero_prod]), bits(b[~zero_prod]))
