"""Host-side argument handling of the gravity boundary (CPU only).

Messages and exception types follow crates/pynbodyext-rust/src/gravity.rs
and pynbodyext/gravity/base.py; all of these raise before any device call.
"""
import numpy as np
import pytest

from pynbodyext import _engine
from pynbodyext.gravity.base import Gravity, KernelKind, TreeOptions

POS = np.random.default_rng(0).random((6, 3))


def test_masses_length():
    with pytest.raises(ValueError, match="^masses must be length N$"):
        _engine.direct_potentials_py(POS, np.ones(5))


def test_softenings_length():
    with pytest.raises(ValueError, match="^softenings must be length N$"):
        _engine.direct_accelerations_py(POS, None, 0, np.ones(2), 0)


def test_softenings_need_kernel():
    with pytest.raises(ValueError, match="softenings require an explicit kernel"):
        _engine.direct_potentials_py(POS, None, 0, np.ones(6), None)


def test_bad_kernel_code():
    with pytest.raises(ValueError, match=r"kernel must be 0 \(Plummer\) or 1 \(CubicSplineW2\)"):
        _engine.direct_potentials_py(POS, None, 0, None, 2)


def test_positions_shape_and_dtype():
    with pytest.raises(ValueError, match=r"positions must be \(N,3\) float64 array"):
        _engine.direct_potentials_py(np.zeros((2, 2)))
    with pytest.raises(TypeError):
        _engine.direct_potentials_py(np.zeros((2, 3), dtype=np.float32))
    with pytest.raises(ValueError, match=r"^targets must be"):
        _engine.direct_potentials_at_points_py(POS, np.zeros((2, 4))[:, :2])
    # contiguous fast path only checks len % 3 (gravity.rs:38-50)
    assert _engine.extract_vec3(np.zeros((2, 6)), "positions").shape == (4, 3)


def test_negative_threads():
    with pytest.raises(OverflowError):
        _engine.direct_potentials_py(POS, threads=-1)


def test_gravity_init_validation():
    with pytest.raises(ValueError, match=r"positions must be a float64 array of shape \(N, 3\)"):
        Gravity(np.zeros((3, 2)), np.ones(3))
    with pytest.raises(ValueError, match=r"masses must be a float64 array of shape \(N,\)"):
        Gravity(POS, np.ones(5))
    with pytest.raises(ValueError, match=r"softening must be a float64 array of shape \(N,\)"):
        Gravity(POS, np.ones(6), softening=np.ones(3))
    g = Gravity(POS.astype(np.float32), np.ones(6, dtype=np.int64), softening=0.1)
    assert g.pos.dtype == np.float64 and g.mass.dtype == np.float64
    assert g.softening.shape == (6,) and np.all(g.softening == 0.1)
    assert g.tree_options == TreeOptions(8, 3, KernelKind.No)


def test_kernelkind_values():
    assert KernelKind(None) is KernelKind.No
    assert KernelKind(0) is KernelKind.Plummer
    assert KernelKind(1) is KernelKind.Spline


def test_direct_targets_assert():
    g = Gravity(POS, np.ones(6))
    with pytest.raises(AssertionError):
        g.direct_potentials(positions=np.zeros((3, 2)))
