"""Profile builders (calculators) — reference pynbodyext/profiles/base.py.

``RadialProfileBuilder(ndim, weight, bins_type, nbins, bin_min, bin_max,
bins_set, **kwargs)`` is a calculator: ``builder(sim)`` or
``builder.filter(Sphere(r) & FamilyFilter("dm"))(sim)`` returns a
:class:`RadialProfile` (base.py:75-140).

Fused device path (MI355X): when the builder runs behind a filter scope
that the device understands (a Sphere and/or family ranges, see
pynbodyext/filters), the mask, r (or rxy), the order-preserving
compaction, the edges and the bin assignment all run in one GPU pipeline
on the unfiltered snapshot's arrays; the masked sub-snapshot is then built
from the kept indices.  Results are identical to filtering first (the
device mask and r are bit-exact with numpy's).
"""
from __future__ import annotations

from typing import Any

import numpy as np

from ..calculate import CalculatorBase
from ..simcore import PendingField, SimSnap, SubSnap
from ._device import DeviceBins
from .bins import BinsSet
from .profile import ProfileBase
from .spatial_profile import RadialProfile

__all__ = ["ProfileBuilderBase", "RadialProfileBuilder"]


def _native_float(a) -> np.ndarray:
    """float32 stays float32; anything else is taken as float64."""
    a = np.asarray(a)
    return a if a.dtype in (np.float32, np.float64) else a.astype(np.float64)


class ProfileBuilderBase(CalculatorBase):
    """Calculator building a profile from the active snapshot."""

    def execute(self, ctx, input):
        sim = input.active_sim
        with ctx.phase(self, "build profile"):
            params = self.resolve_dynamic_params(ctx, input)
            return self._build_runtime(sim, params, ctx, input)

    def _build_runtime(self, sim, params, ctx, input):
        return self.build_profile(sim, params)

    def build_profile(self, sim, params: dict[str, Any]) -> ProfileBase:
        raise NotImplementedError("Subclasses must implement build_profile()")

    def __repr__(self) -> str:
        return f"ProfBuilder {self.__class__.__name__}()"


class RadialProfileBuilder(ProfileBuilderBase):
    """Radial profile builder (3-D shells by r, or 2-D annuli by rxy)."""

    dynamic_param_specs = {"bin_min": None, "bin_max": None}

    def __init__(self, ndim=3, weight=None, bins_type="lin", nbins=100, bin_min=None,
                 bin_max=None, bins_set: BinsSet | None = None, **kwargs: Any):
        super().__init__()
        if ndim not in (2, 3):
            raise ValueError("ndim must be either 2 or 3")
        self.ndim = ndim
        self.weight = weight
        self.bins_type = bins_type
        self.nbins = nbins
        self.bin_min = bin_min
        self.bin_max = bin_max
        self.bins_set = bins_set
        self.kwargs = kwargs

    def instance_signature(self):
        return (type(self).__name__, self.ndim, self.weight, self.bins_type, id(self.nbins),
                self.bins_set)

    def build_profile(self, sim, params):
        return RadialProfile(sim, ndim=self.ndim, weight=self.weight, bins_type=self.bins_type,
                             nbins=self.nbins, bin_min=params["bin_min"], bin_max=params["bin_max"],
                             bins_set=self.bins_set, **self.kwargs)

    # ---- fused device path -------------------------------------------------------
    def execute_fused(self, ctx, input, filt):
        if self.bins_set is not None:
            return NotImplemented
        # dynamic parameters that depend on the filtered snapshot keep the
        # two-step semantics
        for name in self.dynamic_param_specs:
            v = getattr(self, name)
            if callable(v) or isinstance(v, CalculatorBase):
                return NotImplemented
        source = input.source_sim
        spec = filt.device_spec(source)
        if spec is None or "pos" not in getattr(source, "keys", lambda: [])():
            return NotImplemented
        params = self.resolve_dynamic_params(ctx, input)
        with ctx.phase(self, "device select"):
            # float32 snapshots go to the device as float32 (no host copy):
            # r / rxy are then float32 values, exactly pynbody's derived array
            pos = _native_float(source["pos"])
            mass = _native_float(source["mass"]) if "mass" in source.keys() else None
            dev = DeviceBins.select(pos, mass, sphere=spec.get("sphere"),
                                    families=spec.get("families"), ndim=self.ndim)
            # the kept masses: read from the device (the same values: a copy,
            # through pinned chunks) instead of a host gather of the
            # sub-snapshot's column
            wdev = mass is not None and mass.dtype == np.float64 and isinstance(source, SimSnap)
            idx = dev.selection(idx=True, x=False, w=False)[0]
        # (the selection keeps index order: the view's indices increase)
        sub = SubSnap(source, idx, increasing=True) if isinstance(source, SimSnap) else source[idx]
        key = "r" if self.ndim == 3 else "rxy"
        if isinstance(sub, SubSnap):
            # r / rxy (the same values, in the positions' precision) and the
            # kept masses stay on the device until the host reads them (sub[key],
            # bins.x, sub["mass"], a host-side statistic): device sums never do
            def fetch_x(dev=dev, dt=pos.dtype):
                x = dev.selection(idx=False, x=True, w=False)[1]
                return x.astype(dt) if dt != x.dtype else x

            sub._pending[key] = fetch_x
            if wdev:
                sub._pending["mass"] = lambda dev=dev: dev.selection(idx=False, x=False, w=True)[2]
            xs = PendingField(sub, key)
        else:
            xs = sub[key]
        bins_area = "spherical_shell" if self.ndim == 3 else "annulus"
        with ctx.phase(self, "device bins"):
            template = BinsSet(bins_by=key, bins_area=bins_area, bins_type=self.bins_type,
                               nbins=self.nbins, bin_min=params["bin_min"],
                               bin_max=params["bin_max"], **self.kwargs)
            bins = template.materialise_on_device(xs, dev)
        prof = RadialProfile(sub, ndim=self.ndim, weight=self.weight, bins_type=self.bins_type,
                             nbins=self.nbins, bin_min=params["bin_min"],
                             bin_max=params["bin_max"], bins_set=bins, **self.kwargs)
        if self.weight == "mass" and mass is not None:
            prof._device_weight_name = "mass"
        return prof
