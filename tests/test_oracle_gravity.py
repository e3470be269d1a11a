"""Pin the gravity oracle (oracle/gravity_ref.c) — CPU only.

The reference holds no golden vectors for direct summation, so the
restatement is pinned by (a) analytic known answers, (b) the reference's
own invariants, (c) agreement between its two summation branches
(direct.rs N<512 symmetric loop vs N>=512 per-target loop) and (d) the
softening-kernel formulas of kernel.rs.
"""
import numpy as np
import pytest

from oracle import gravity as og
from pynbodyext.synthetic import plummer

R2_TINY = np.finfo(np.float64).tiny


def test_two_body_known_answer():
    pos = np.array([[0.0, 0.0, 0.0], [3.0, 4.0, 0.0]])
    mass = np.array([2.0, 5.0])
    pot = og.direct_potentials(pos, mass)
    acc = og.direct_accelerations(pos, mass)
    assert pot[0] == pytest.approx(-5.0 / 5.0, rel=1e-15)
    assert pot[1] == pytest.approx(-2.0 / 5.0, rel=1e-15)
    np.testing.assert_allclose(acc[0], 5.0 * np.array([3, 4, 0]) / 125.0, rtol=1e-15)
    np.testing.assert_allclose(acc[1], -2.0 * np.array([3, 4, 0]) / 125.0, rtol=1e-15)


def test_momentum_conservation_and_branches_agree():
    # N=511 uses the symmetric i<j loop, N=512 the per-target loop.
    for n in (511, 512):
        pos, mass = plummer(n, seed=7)
        acc = og.direct_accelerations(pos, mass)
        f = (mass[:, None] * acc).sum(axis=0)
        scale = np.abs(mass[:, None] * acc).sum()
        assert np.all(np.abs(f) < 1e-12 * scale)
    pos, mass = plummer(511, seed=9)
    pot_sym = og.direct_potentials(pos, mass)
    acc_sym = og.direct_accelerations(pos, mass)
    pot_pt, acc_pt = og.direct_subset(pos, mass, np.arange(511))
    np.testing.assert_allclose(pot_sym, pot_pt, rtol=1e-13)
    np.testing.assert_allclose(acc_sym, acc_pt, rtol=1e-10, atol=1e-13 * np.abs(acc_pt).max())


def test_subset_is_bitwise_the_full_per_target_loop():
    pos, mass = plummer(1500, seed=3)
    pot = og.direct_potentials(pos, mass)
    acc = og.direct_accelerations(pos, mass)
    idx = np.array([0, 17, 999, 1499])
    ps, as_ = og.direct_subset(pos, mass, idx)
    assert np.array_equal(ps, pot[idx])
    assert np.array_equal(as_, acc[idx])


def test_at_points_matches_self_form_away_from_particles():
    pos, mass = plummer(700, seed=5)
    tgt = np.array([[0.1, 0.2, 0.3], [5.0, -1.0, 2.0]])
    p1 = og.direct_potentials_at_points(pos, tgt, mass)
    # brute force numpy in the same summation order
    d = pos[None, :, :] - tgt[:, None, :]
    r = np.sqrt((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2])
    np.testing.assert_allclose(p1, -(mass / r).sum(axis=1), rtol=1e-13)


def test_coincident_target_reference_semantics():
    # at-points has no self-skip: r2 = 0 -> 1/sqrt(tiny) potential, 0*inf = NaN force
    pos = np.array([[0.0, 0.0, 0.0], [1.0, 0.0, 0.0]])
    pot = og.direct_potentials_at_points(pos, pos[:1], np.ones(2))
    acc = og.direct_accelerations_at_points(pos, pos[:1], np.ones(2))
    assert pot[0] == pytest.approx(-1.0 / np.sqrt(R2_TINY) - 1.0, rel=1e-15)
    assert np.isnan(acc[0, 0])


def test_kernel_formulas():
    # Plummer
    assert og.kernel_potential(0, 2.0, 1.5) == pytest.approx(-1.0 / 2.5, rel=1e-15)
    assert og.kernel_accel_factor(0, 2.0, 1.5) == pytest.approx(1.0 / 2.5 ** 3, rel=1e-15)
    assert og.kernel_potential(0, 0.0, 1.0) == 0.0
    # spline: Newtonian outside h, continuous at u = 0.5 and u = 1
    h = 0.7
    assert og.kernel_potential(1, 2.0, h) == pytest.approx(-0.5, rel=1e-15)
    assert og.kernel_accel_factor(1, 2.0, h) == pytest.approx(1 / 8.0, rel=1e-15)
    for u in (0.5, 1.0):
        lo = og.kernel_potential(1, (u - 1e-9) * h, h)
        hi = og.kernel_potential(1, (u + 1e-9) * h, h)
        assert lo == pytest.approx(hi, rel=1e-7)
        glo = og.kernel_accel_factor(1, (u - 1e-9) * h, h)
        ghi = og.kernel_accel_factor(1, (u + 1e-9) * h, h)
        assert glo == pytest.approx(ghi, rel=1e-6)
    # W2(0) = -14/5 per unit h
    assert og.kernel_potential(1, 1e-300, 2.0) == pytest.approx(-14.0 / 5.0 / 2.0, rel=1e-12)
    # h <= 0 falls back to Newtonian
    assert og.kernel_potential(1, 2.0, 0.0) == -0.5
    # multipole softening guard (kernel.rs:20-37)
    assert og.multipole_soft_ok(0, 2.9, 1.0) and not og.multipole_soft_ok(0, 2.8, 1.0)
    assert og.multipole_soft_ok(1, 1.01, 1.0) and not og.multipole_soft_ok(1, 1.0, 1.0)
    assert og.multipole_soft_ok(0, 0.0, 0.0)


def test_softened_direct_uses_max_softening():
    pos = np.array([[0.0, 0.0, 0.0], [1.0, 0.0, 0.0]])
    h = np.array([0.5, 2.0])
    pot = og.direct_potentials(pos, np.ones(2), softenings=h, kernel=0)
    assert pot[0] == pytest.approx(-1.0 / np.sqrt(1.0 + 4.0), rel=1e-14)
    # at points: only the source softening counts, max(h_j, 0)
    pot_t = og.direct_potentials_at_points(pos, np.array([[0.0, 3.0, 0.0]]), np.ones(2),
                                           softenings=np.array([np.nan, -1.0]), kernel=0)
    expect = -1.0 / 3.0 - 1.0 / np.sqrt(10.0)
    assert pot_t[0] == pytest.approx(expect, rel=1e-14)


def test_plummer_sphere_potential_statistics():
    # mean potential energy of a Plummer sphere: W = -3 pi G M^2 / (32 a)
    pos, mass = plummer(4000, seed=11)
    pot = og.direct_potentials(pos, mass)
    w = 0.5 * np.sum(mass * pot)
    assert w == pytest.approx(-3 * np.pi / 32, rel=0.05)


def test_empty_inputs():
    z = np.zeros((0, 3))
    assert og.direct_potentials(z).shape == (0,)
    assert og.direct_accelerations_at_points(z, np.ones((2, 3))).tolist() == [[0, 0, 0]] * 2
