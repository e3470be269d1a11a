"""Gravity front end: direct summation and Barnes-Hut tree on MI355X.

Public surface, validation and defaults follow the reference's
pynbodyext/gravity/base.py (KernelKind :71-79, TreeOptions :82-100,
Gravity :132-454); every solve is delegated to the native engine
(``pynbodyext._engine``, the drop-in for the PyO3 module ``_rust``), whose
kernels run on the GPU.

Softening: None (Newtonian), a scalar (broadcast to all particles with
``np.full``, as base.py:192-193 does, so the engine always receives a
per-particle array) or an (N,) array.  The kernel is a :class:`KernelKind`;
``KernelKind.No`` combined with a softening array is rejected by the engine
with the reference's ValueError.
"""
from __future__ import annotations

from dataclasses import dataclass
from enum import Enum

import numpy as np

from pynbodyext import _engine
from pynbodyext.log import logger

__all__ = ["Gravity", "KernelKind", "TreeOptions"]


class KernelKind(Enum):
    """Softening kernel: ``No`` (Newtonian), ``Plummer`` or ``Spline`` (W2).

    The values are the engine's kernel codes (None, 0, 1).
    """

    No = None
    Plummer = 0
    Spline = 1


@dataclass(eq=True, frozen=True)
class TreeOptions:
    """Octree construction options (leaf size, multipole order, kernel)."""

    leaf_capacity: int = 8
    multipole_order: int = 3
    kernel: KernelKind = KernelKind.No


def _build_tree(positions, masses, softening, options: TreeOptions):
    return _engine.Octree(
        positions,
        masses,
        options.leaf_capacity,
        options.multipole_order,
        softening,
        options.kernel.value,
    )


def _targets(positions) -> np.ndarray:
    pts = np.asarray(positions, dtype=np.float64)
    assert pts.ndim == 2 and pts.shape[1] == 3, "positions must be of shape (N, 3)"
    return pts


class Gravity:
    """Direct-sum and tree gravity for one fixed particle set.

    Parameters
    ----------
    positions : (N, 3) array
    masses : (N,) array
    softening : None, float, or (N,) array
    kernel : KernelKind
        Default kernel for every method (overridable per call).
    leaf_capacity, multipole_order : int
        Options of the lazily built, cached octree (:pyattr:`tree`).
    """

    def __init__(self, positions, masses, softening=None, kernel=KernelKind.No,
                 leaf_capacity: int = 8, multipole_order: int = 3) -> None:
        pos = np.asarray(positions)
        mass = np.asarray(masses)
        if pos.ndim != 2 or pos.shape[1] != 3:
            raise ValueError("positions must be a float64 array of shape (N, 3)")
        n = pos.shape[0]
        if mass.shape != (n,):
            raise ValueError("masses must be a float64 array of shape (N,)")
        if softening is None:
            soft = None
        elif np.isscalar(softening):
            soft = np.full((n,), float(softening), dtype=np.float64)
        else:
            soft = np.asarray(softening, dtype=np.float64)
            if soft.shape != (n,):
                raise ValueError("softening must be a float64 array of shape (N,)")
        self.pos = pos.astype(np.float64)
        self.mass = mass.astype(np.float64)
        self.softening = soft
        self.tree_options = TreeOptions(leaf_capacity, multipole_order, kernel=KernelKind(kernel))
        self._tree = None

    # -- tree management (base.py:213-238) --------------------------------
    def get_tree(self, leaf_capacity: int = 8, multipole_order: int = 3,
                 kernel=KernelKind.No):
        """The cached tree when the options match the instance's, else a new one."""
        opts = TreeOptions(leaf_capacity, multipole_order, kernel=KernelKind(kernel))
        if opts == self.tree_options:
            return self.tree
        logger.debug("Building new Octree with leaf_capacity=%d, multipole_order=%d",
                     leaf_capacity, multipole_order)
        return _build_tree(self.pos, self.mass, self.softening, opts)

    @property
    def tree(self):
        """Octree for the instance's TreeOptions (built on first access)."""
        if self._tree is None:
            self._tree = _build_tree(self.pos, self.mass, self.softening, self.tree_options)
        return self._tree

    def _kernel(self, kernel) -> KernelKind:
        return self.tree_options.kernel if kernel is None else KernelKind(kernel)

    # -- direct summation (base.py:240-332) --------------------------------
    def direct_potentials(self, positions=None, threads: int = 0, kernel=None) -> np.ndarray:
        """Potentials by direct summation, at the particles or at ``positions``."""
        k = self._kernel(kernel)
        if positions is None:
            return _engine.direct_potentials_py(self.pos, self.mass, threads, self.softening,
                                                k.value)
        return _engine.direct_potentials_at_points_py(self.pos, _targets(positions), self.mass,
                                                      threads, self.softening, k.value)

    def direct_accelerations(self, positions=None, threads: int = 0, kernel=None) -> np.ndarray:
        """Accelerations by direct summation, at the particles or at ``positions``."""
        k = self._kernel(kernel)
        if positions is None:
            return _engine.direct_accelerations_py(self.pos, self.mass, threads,
                                                   self.softening, k.value)
        return _engine.direct_accelerations_at_points_py(self.pos, _targets(positions),
                                                         self.mass, threads, self.softening,
                                                         k.value)

    # -- Barnes-Hut tree (base.py:336-454) ----------------------------------
    def tree_potentials(self, positions=None, theta: float = 0.7, threads: int = 0,
                        leaf_capacity: int = 8, multipole_order: int = 3,
                        kernel=None) -> np.ndarray:
        """Potentials from the Barnes-Hut tree (opening angle ``theta``)."""
        tree = self.get_tree(leaf_capacity=leaf_capacity, multipole_order=multipole_order,
                             kernel=self._kernel(kernel))
        if positions is None:
            return tree.compute_potentials(theta, threads)
        return tree.potentials_at_points(_targets(positions), theta, threads)

    def tree_accelerations(self, positions=None, theta: float = 0.7, threads: int = 0,
                           leaf_capacity: int = 8, multipole_order: int = 3,
                           kernel=None) -> np.ndarray:
        """Accelerations from the Barnes-Hut tree (opening angle ``theta``)."""
        tree = self.get_tree(leaf_capacity=leaf_capacity, multipole_order=multipole_order,
                             kernel=self._kernel(kernel))
        if positions is None:
            return tree.compute_accelerations(theta, threads)
        return tree.accelerations_at_points(_targets(positions), theta, threads)
