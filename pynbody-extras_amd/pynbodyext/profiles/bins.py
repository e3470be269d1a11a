"""1-D binning of particle data, computed on the GPU.

:class:`BinsSet` keeps the reference's interface (pynbodyext/profiles/
bins.py:68-790): the ``bins_by`` / ``bins_type`` / ``bins_area`` registries
and decorators, construction arguments, materialised attributes (``x``,
``bin_edges``, ``rbins``, ``dr``, ``binind``, ``npart_bins``,
``binsize``), ``__call__`` as a factory, ``spawn_with_same_edges``.

What runs where:
  * the binned quantity ``x`` is uploaded to HBM once per materialisation
    (or produced there by a fused selection, see profiles/base.py);
  * ``lin`` / ``log`` edges: np.linspace / np.logspace of the device
    min / max (same numpy calls as the reference, so the same bits);
  * ``equaln`` edges: exact order statistics from a device radix sort;
  * particle -> bin assignment, counts and the per-bin index lists
    (``binind``): device kernels; ``binind`` is a lazy sequence of views
    into the device-built CSR, downloaded on first access.
Custom registered algorithms / areas / extractors are user callables and
run wherever the user's code runs.
"""
from __future__ import annotations

from collections.abc import Callable, Sequence
from typing import Any

import numpy as np

from .._pyn import SimArray
from ..simcore import PendingField
from ._device import DeviceBins

__all__ = ["BinsSet", "BinIndexLists"]


class BinIndexLists(Sequence):
    """``binind`` as a sequence of per-bin ascending index arrays.

    Backed by the CSR built on the device; the CSR is downloaded the first
    time an element is accessed (``len`` does not need it).
    """

    def __init__(self, device: DeviceBins, nbins: int):
        self._device = device
        self._nbins = int(nbins)
        self._lists = None

    def _materialise(self):
        if self._lists is None:
            perm, offs = self._device.csr()
            self._lists = [perm[offs[i]:offs[i + 1]] for i in range(self._nbins)]
        return self._lists

    @property
    def csr(self):
        return self._device.csr()

    def __len__(self):
        return self._nbins

    def __getitem__(self, i):
        return self._materialise()[i]

    def __iter__(self):
        return iter(self._materialise())

    def __repr__(self):
        return f"BinIndexLists(nbins={self._nbins}, n_valid={self._device.n_valid})"


class BinsSet:
    """Pluggable 1-D binning helper (see module docstring)."""

    _bins_by_registry: dict[str, Callable] = {}
    _bins_area_registry: dict[str, Callable] = {}
    _bins_algorithm_registry: dict[str, Callable] = {}

    def __init__(self, bins_by, bins_area, bins_type, nbins, bin_min: float | None = None,
                 bin_max: float | None = None, **kwargs: Any) -> None:
        self._bins_by = bins_by
        self._bins_area = bins_area
        self._bins_type = bins_type
        self._nbins = nbins
        self._bin_min = bin_min
        self._bin_max = bin_max
        self._kwargs = kwargs
        self._x = None  # x, or a PendingField (device-held, read on first use)
        self.bin_edges = None
        self.rbins = None
        self.dr = None
        self.binind = None
        self.npart_bins = None
        self.binsize = None
        self._device: DeviceBins | None = None
        self._device_x = None

    @property
    def x(self):
        v = self._x
        if isinstance(v, PendingField):
            pend, v = v, v.resolve()
            self._x = v
            if self._device_x is pend:
                self._device_x = v  # (the device copy is of these values)
        return v

    @x.setter
    def x(self, value):
        self._x = value

    # ---- read-only configuration -------------------------------------------------
    @property
    def bins_by(self):
        return self._bins_by

    @property
    def bins_area(self):
        return self._bins_area

    @property
    def bins_type(self):
        return self._bins_type

    @property
    def bin_min(self):
        return self._bin_min

    @property
    def bin_max(self):
        return self._bin_max

    @property
    def nbins(self) -> int:
        nb = self._nbins
        if isinstance(nb, (int, np.integer)):
            return int(nb)
        if isinstance(nb, np.ndarray):
            return len(nb) - 1
        raise TypeError(f"Invalid _nbins type: {type(nb)}")

    def is_defined(self) -> bool:
        return all(a is not None for a in (self.bin_edges, self.rbins, self.dr, self._x,
                                           self.binind, self.npart_bins, self.binsize))

    # ---- device state ------------------------------------------------------------
    def _device_for(self, x) -> DeviceBins:
        """The device copy of x (uploaded once per distinct x object)."""
        if self._device is None or self._device_x is not x:
            self._device = DeviceBins.from_x(np.asarray(x, dtype=np.float64))
            self._device_x = x
        return self._device

    def _adopt_device(self, device: DeviceBins, x) -> None:
        self._device = device
        self._device_x = x

    # ---- stages (bins.py:195-395) -------------------------------------------------
    def _resolve_x(self, sim):
        if callable(self._bins_by):
            return self._bins_by(sim)
        if isinstance(self._bins_by, str):
            fn = self._bins_by_registry.get(self._bins_by)
            return fn(sim) if fn is not None else sim[self._bins_by]
        raise ValueError(f"Invalid bins_by: {self._bins_by}, required callable or registry keys: "
                         f"{list(self._bins_by_registry)}")

    @staticmethod
    def _coerce_edges_units(edges, x):
        if isinstance(x, PendingField) and not isinstance(edges, SimArray):
            out = SimArray(edges)
            out.units = x.units
            out.sim = x.sim
            return out
        if isinstance(x, SimArray) and not isinstance(edges, SimArray):
            out = SimArray(edges)
            out.units = x.units
            out.sim = x.sim
            return out
        return edges

    def _build_edges(self, x):
        if not isinstance(self._nbins, (int, np.integer)):
            arr = np.asarray(self._nbins)
            if arr.ndim != 1 or arr.shape[0] < 2:
                raise ValueError("Explicit bin_edges must be a 1D array of length >= 2")
            return self._coerce_edges_units(arr, x)
        if callable(self._bins_type):  # (a user's algorithm reads the values)
            xv = x.resolve() if isinstance(x, PendingField) else x
            return self._coerce_edges_units(self._bins_type(self, xv), x)
        if isinstance(self._bins_type, str):
            return self._coerce_edges_units(self._bins_algorithm_registry[self._bins_type](self, x), x)
        raise ValueError(f"Invalid bins_type: {self._bins_type}, required callable or registry keys: "
                         f"{list(self._bins_algorithm_registry)}")

    def _calc_area_or_volume(self, bin_edges):
        if callable(self._bins_area):
            return self._bins_area(self, bin_edges)
        if isinstance(self._bins_area, str):
            return self._bins_area_registry[self._bins_area](self, bin_edges)
        raise ValueError(f"Invalid bins_area: {self._bins_area}, required callable or registry keys: "
                         f"{list(self._bins_area_registry)}")

    @staticmethod
    def _calc_binmid(bin_edges):
        return 0.5 * (bin_edges[:-1] + bin_edges[1:])

    def _assign_particles(self, x, bin_edges):
        """(binind, npart_bins) for the given x and edges, on the device.

        Same result as the reference's digitize / bincount / stable argsort
        (bins.py:346-395): bin = searchsorted(edges, x, 'left') - 1, x equal
        to the first edge -> bin 0, then equal to the last -> last bin,
        out-of-range and NaN values dropped, ascending indices per bin.
        """
        edges = np.asarray(bin_edges, dtype=np.float64)
        nb = len(edges) - 1
        if nb <= 0:
            return [], np.array([], dtype=int)
        if nb > 1 and np.any(edges[1:] < edges[:-1]):
            if np.all(edges[1:] <= edges[:-1]):
                raise NotImplementedError("descending bin edges are not supported")
            raise ValueError("bins must be monotonically increasing or decreasing")
        dev = self._device_for(x)
        counts = dev.assign(edges)
        if not counts.any():
            return [np.empty(0, dtype=int) for _ in range(nb)], np.zeros(nb, dtype=int)
        return BinIndexLists(dev, nb), counts

    # ---- materialisation -----------------------------------------------------------
    def _config_copy(self, nbins=None) -> "BinsSet":
        return BinsSet(bins_by=self._bins_by, bins_area=self._bins_area, bins_type=self._bins_type,
                       nbins=self._nbins if nbins is None else nbins, bin_min=self._bin_min,
                       bin_max=self._bin_max, **self._kwargs)

    def _materialise(self, x) -> None:
        self._x = x
        self.bin_edges = self._build_edges(x)
        if self.bin_edges.ndim != 1 or self.bin_edges.shape[0] < 2:
            self.bin_edges = np.asarray([0.0, 1.0])
        self.rbins = self._calc_binmid(self.bin_edges)
        self.dr = np.gradient(self.rbins)
        self.binind, self.npart_bins = self._assign_particles(x, self.bin_edges)
        self.binsize = self._calc_area_or_volume(self.bin_edges)

    def __call__(self, sim, inplace: bool = False) -> "BinsSet":
        target = self if inplace else self._config_copy()
        target._materialise(target._resolve_x(sim))
        return target

    def materialise_on_device(self, x, device: DeviceBins) -> "BinsSet":
        """Materialise from x already resident on the device (fused path;
        x may be a PendingField: then the host reads it only when asked,
        bins.x or the view's field)."""
        target = self._config_copy()
        target._adopt_device(device, x)
        target._materialise(x)
        return target

    def spawn_with_same_edges(self, sim) -> "BinsSet":
        if not self.is_defined():
            raise ValueError("Cannot spawn with same edges: parent BinsSet is not materialized. "
                             "Call the instance with a simulation first.")
        child = self._config_copy(nbins=self.bin_edges)
        child.x = child._resolve_x(sim)
        child.bin_edges = self.bin_edges
        child.rbins = self.rbins
        child.dr = self.dr
        child.binind, child.npart_bins = child._assign_particles(child.x, child.bin_edges)
        child.binsize = self.binsize
        return child

    @classmethod
    def available_options(cls) -> dict:
        return {"bins_by": list(cls._bins_by_registry), "bins_area": list(cls._bins_area_registry),
                "bins_type": list(cls._bins_algorithm_registry)}

    def __repr__(self) -> str:
        cfg = (f"bins_by={self._bins_by}, bins_area={self._bins_area}, bins_type={self._bins_type}, "
               f"nbins={self.nbins if self.is_defined() else self._nbins}, "
               f"bin_min={self._bin_min}, bin_max={self._bin_max}")
        if self.is_defined():
            return f"BinsSet(materialized: {cfg}, x len={len(self._x)}, "
        return f"BinsSet(config: {cfg})"

    # ---- registries ------------------------------------------------------------------
    @classmethod
    def _register(cls, registry: dict, fn, name):
        def deco(f):
            registry[name or f.__name__] = f
            return f
        return deco if fn is None else deco(fn)

    @classmethod
    def bins_by_register(cls, fn=None, name: str | None = None):
        return cls._register(cls._bins_by_registry, fn, name)

    @classmethod
    def bins_area_register(cls, fn=None, name: str | None = None):
        return cls._register(cls._bins_area_registry, fn, name)

    @classmethod
    def bins_algorithm_register(cls, fn=None, name: str | None = None):
        return cls._register(cls._bins_algorithm_registry, fn, name)


# ---------------------------------------------------------------- edge algorithms
def _domain(self: BinsSet, x):
    lo, hi = self._bin_min, self._bin_max
    if lo is None or hi is None:
        mn, mx = self._device_for(x).minmax()
        lo = mn if lo is None else lo
        hi = mx if hi is None else hi
    return lo, hi


@BinsSet.bins_algorithm_register(name="lin")
def linear_bins_algorithm(self: BinsSet, x):
    """nbins+1 linearly spaced edges over [bin_min or min(x), bin_max or max(x)]."""
    lo, hi = _domain(self, x)
    return np.linspace(lo, hi, self.nbins + 1)


@BinsSet.bins_algorithm_register(name="log")
def logarithmic_bins_algorithm(self: BinsSet, x):
    """nbins+1 logarithmically spaced edges; needs a positive lower bound."""
    lo, hi = _domain(self, x)
    if lo <= 0:
        raise ValueError("Logarithmic bins require xmin to be non-negative")
    return np.logspace(np.log10(lo), np.log10(hi), self.nbins + 1)


@BinsSet.bins_algorithm_register(name="equaln")
def equal_number_bins_algorithm(self: BinsSet, x):
    """Edges at the order statistics s[int(i*n/nbins)] of x (clipped to
    [bin_min, bin_max]), first and last value as outer edges."""
    return self._device_for(x).edges_equaln(self.nbins, self._bin_min, self._bin_max)


# ---------------------------------------------------------------- areas
@BinsSet.bins_area_register(name="length")
def length_area(self: BinsSet, bin_edges):
    return bin_edges[1:] - bin_edges[:-1]


@BinsSet.bins_area_register(name="annulus")
def annulus_area(self: BinsSet, bin_edges):
    return np.pi * (bin_edges[1:] ** 2 - bin_edges[:-1] ** 2)


@BinsSet.bins_area_register(name="spherical_shell")
def spherical_shell_area(self: BinsSet, bin_edges):
    return 4 / 3 * np.pi * (bin_edges[1:] ** 3 - bin_edges[:-1] ** 3)


@BinsSet.bins_area_register(name="cylindrical_shell")
def cylindrical_shell_area(self: BinsSet, bin_edges):
    z = self._kwargs.get("z", None)
    if z is None:
        raise ValueError("Parameter 'z' must be provided for cylindrical_shell area calculation")
    return np.pi * (bin_edges[1:] ** 2 - bin_edges[:-1] ** 2) * z
