"""Snapshot-level gravity helpers on the GPU: ``calculate_potential`` /
``calculate_acceleration`` (reference gravity/pyn_gravity.py:31-216).

Each result must equal the raw ``Gravity`` solve (itself checked against
the oracle in test_gpu_direct.py / test_gpu_tree.py) times the unit factor
G * mass_unit / pos_unit (** 2 for accelerations) converted to km**2 s**-2 /
km s**-2, computed here by hand from the constants the package uses:

    G = 6.6743e-11 m^3 kg^-1 s^-2 (CODATA 2018), Msol = 1.98847e30 kg (IAU
    2015 nominal), kpc = 3.0856775814913673e19 m (IAU 2012 au x 648000/pi x 1e3).

pynbody is absent here and on the GPU box, so agreement with pynbody's own
unit table is parity unpinned.
"""
import numpy as np
import pytest

from pynbodyext import _native as nat
from pynbodyext.gravity import Gravity, KernelKind
from pynbodyext.gravity.pyn_gravity import calculate_acceleration, calculate_potential
from pynbodyext.simcore import SimArray, SimSnap, units
from pynbodyext.synthetic import plummer

pytestmark = pytest.mark.gpu

G_SI, MSOL, KPC = 6.6743e-11, 1.98847e30, 3.0856775814913673e19
POT_FACTOR = G_SI * MSOL / KPC / 1e6          # (km/s)^2 per (G Msol / kpc)
ACC_FACTOR = G_SI * MSOL / KPC ** 2 / 1e3     # km s^-2 per (G Msol / kpc^2)


@pytest.fixture(scope="module")
def sim():
    pos, mass = plummer(20_000, seed=12)
    return SimSnap({"pos": pos * 10.0, "mass": mass * 1e10},
                   families={"dm": slice(0, 12_000), "star": slice(12_000, 20_000)},
                   units_map={"pos": "kpc", "mass": "Msol"})


def _raw(sim, **kw):
    return Gravity(np.asarray(sim["pos"]), np.asarray(sim["mass"]), **kw)


def test_unit_factors():
    assert POT_FACTOR == pytest.approx(4.301047e-6, rel=1e-6)
    assert ACC_FACTOR == pytest.approx(1.393875e-22, rel=1e-6)


@pytest.mark.parametrize("method", ["direct", "tree"])
def test_potential_units_and_values(gpu, sim, method):
    pot = calculate_potential(sim, method=method)
    assert isinstance(pot, SimArray)
    assert pot.sim is sim
    assert pot.units.ratio(units.Unit("km**2 s**-2")) == pytest.approx(1.0, rel=1e-15)
    g = _raw(sim)
    raw = g.direct_potentials() if method == "direct" else g.tree_potentials(theta=0.7)
    np.testing.assert_allclose(np.asarray(pot), raw * POT_FACTOR, rtol=1e-13)
    assert np.all(np.asarray(pot) < 0)


@pytest.mark.parametrize("method", ["direct", "tree"])
def test_acceleration_units_and_values(gpu, sim, method):
    acc = calculate_acceleration(sim, method=method)
    assert acc.shape == (len(sim), 3)
    assert acc.units.ratio(units.Unit("km s**-2")) == pytest.approx(1.0, rel=1e-15)
    g = _raw(sim)
    raw = g.direct_accelerations() if method == "direct" else g.tree_accelerations(theta=0.7)
    np.testing.assert_allclose(np.asarray(acc), raw * ACC_FACTOR, rtol=1e-13)


def test_softening_simarray_in_other_units(gpu, sim):
    """A SimArray softening is converted to sim['pos'] units (pc -> kpc)."""
    soft_pc = SimArray(np.full(len(sim), 50.0), "pc")
    pot = calculate_potential(sim, softening=soft_pc, method="direct", kernel=KernelKind.Plummer)
    raw = _raw(sim, softening=np.full(len(sim), 0.05),
               kernel=KernelKind.Plummer).direct_potentials()
    np.testing.assert_allclose(np.asarray(pot), raw * POT_FACTOR, rtol=1e-12)
    # scalar softening, spline kernel, tree
    acc = calculate_acceleration(sim, softening=0.02, method="tree", kernel=KernelKind.Spline,
                                 theta=0.6)
    raw = _raw(sim, softening=0.02, kernel=KernelKind.Spline).tree_accelerations(theta=0.6)
    np.testing.assert_allclose(np.asarray(acc), raw * ACC_FACTOR, rtol=1e-13)


def test_softening_without_kernel_is_rejected(gpu, sim):
    with pytest.raises(ValueError, match="softenings require an explicit kernel"):
        calculate_potential(sim, softening=0.01, method="direct")


@pytest.mark.parametrize("method", ["direct", "tree"])
def test_simarray_targets_in_other_units(gpu, sim, method):
    """SimArray target positions are converted to sim['pos'] units."""
    pts_kpc = np.random.default_rng(3).normal(scale=5.0, size=(700, 3))
    pts_pc = SimArray(pts_kpc * 1000.0, "pc")
    pot = calculate_potential(sim, positions=pts_pc, method=method, theta=0.6)
    acc = calculate_acceleration(sim, positions=pts_pc, method=method, theta=0.6)
    conv = np.asarray(pts_pc.in_units("kpc"))
    np.testing.assert_allclose(conv, pts_kpc, rtol=1e-15)
    g = _raw(sim)
    if method == "direct":
        rp, ra = g.direct_potentials(conv), g.direct_accelerations(conv)
    else:
        rp, ra = g.tree_potentials(conv, theta=0.6), g.tree_accelerations(conv, theta=0.6)
    np.testing.assert_allclose(np.asarray(pot), rp * POT_FACTOR, rtol=1e-13)
    np.testing.assert_allclose(np.asarray(acc), ra * ACC_FACTOR, rtol=1e-13)


def test_tree_kwargs_quirk_uses_default_tree(gpu, sim):
    """pyn_gravity.py:96-97: leaf_capacity / multipole_order configure the
    helper, but tree_potentials asks get_tree() for the defaults (8, 3), so a
    non-default request yields the default tree's values."""
    pot = calculate_potential(sim, method="tree", leaf_capacity=32, multipole_order=1)
    raw = _raw(sim).tree_potentials(theta=0.7)
    np.testing.assert_allclose(np.asarray(pot), raw * POT_FACTOR, rtol=1e-13)


def test_unknown_method(gpu, sim):
    with pytest.raises(ValueError, match="Unknown method"):
        calculate_potential(sim, method="fmm")
    with pytest.raises(ValueError, match="Unknown method"):
        calculate_acceleration(sim, method="pm")
