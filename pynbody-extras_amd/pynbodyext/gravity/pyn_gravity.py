"""Snapshot-level gravity helpers (reference pynbodyext/gravity/pyn_gravity.py).

``calculate_potential`` / ``calculate_acceleration`` take a snapshot with
``pos`` and ``mass``, run :class:`Gravity` (direct or tree, on the GPU) and
return SimArrays in km**2 s**-2 / km s**-2, i.e. the raw result times
G * mass_units / pos_units (pyn_gravity.py:121-123, 214-216).

Reference quirk kept on purpose: ``leaf_capacity`` / ``multipole_order``
kwargs configure the Gravity helper, but the tree solve asks ``get_tree``
for the defaults (8, 3) (pyn_gravity.py:96-97,116-117), so non-default
values build a default tree.
"""
from __future__ import annotations

from typing import Any, Literal

import numpy as np

from .._pyn import SimArray, units
from .base import Gravity, KernelKind

__all__ = ["calculate_potential", "calculate_acceleration"]


def _coerce_softening(sim, softening):
    if softening is None:
        return None
    if isinstance(softening, SimArray):
        arr = np.asarray(softening.in_units(sim["pos"].units), dtype=np.float64)
        return float(arr) if arr.ndim == 0 else arr
    if isinstance(softening, (float, int)):
        return float(softening)
    return np.asarray(softening, dtype=np.float64)


def _helper(sim, softening, kernel, kwargs) -> Gravity:
    return Gravity(
        sim["pos"],
        sim["mass"],
        softening=_coerce_softening(sim, softening),
        kernel=kernel,
        leaf_capacity=kwargs.get("leaf_capacity", 8),
        multipole_order=kwargs.get("multipole_order", 3),
    )


def _targets(sim, positions):
    if isinstance(positions, SimArray):
        return positions.in_units(sim["pos"].units)
    return positions


def calculate_potential(sim, positions=None, softening=None,
                        method: Literal["direct", "tree"] = "tree", threads: int = 0, *,
                        kernel: KernelKind = KernelKind.No, **kwargs: Any):
    """Gravitational potential of ``sim`` (at its particles or ``positions``)."""
    grav = _helper(sim, softening, kernel, kwargs)
    positions = _targets(sim, positions)
    if method == "direct":
        pot = grav.direct_potentials(positions, threads)
    elif method == "tree":
        pot = grav.tree_potentials(positions, kwargs.get("theta", 0.7), threads)
    else:
        raise ValueError(f"Unknown method: {method}")
    res = SimArray(pot, units.G * sim["mass"].units / sim["pos"].units)
    res.sim = sim
    return res.in_units("km**2 s**-2")


def calculate_acceleration(sim, positions=None, softening=None,
                           method: Literal["direct", "tree"] = "tree", threads: int = 0, *,
                           kernel: KernelKind = KernelKind.No, **kwargs: Any):
    """Gravitational acceleration of ``sim`` (at its particles or ``positions``)."""
    grav = _helper(sim, softening, kernel, kwargs)
    positions = _targets(sim, positions)
    if method == "direct":
        acc = grav.direct_accelerations(positions, threads)
    elif method == "tree":
        acc = grav.tree_accelerations(positions, kwargs.get("theta", 0.7), threads)
    else:
        raise ValueError(f"Unknown method: {method}")
    res = SimArray(acc, units.G * sim["mass"].units / sim["pos"].units ** 2)
    res.sim = sim
    return res.in_units("km s**-2")
