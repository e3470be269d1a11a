"""Particle selection filters on the radial-profile path.

``Sphere`` and ``FamilyFilter`` keep the reference's constructor signatures
(pynbodyext/filters/filt.py:42-86: ``Sphere(radius, cen=(0, 0, 0))``,
``FamilyFilter(family)``) and mask semantics of pynbody.filt.  Besides the
host mask they describe themselves to the device (``device_spec``) so a
radial profile behind ``Sphere & FamilyFilter`` is selected, measured and
binned in one GPU pipeline (csrc/profile.hip, select).

The other reference filters (Cuboid, Disc, BandPass, ...) are not on the
hot path and are not provided.
"""
from __future__ import annotations

import numpy as np

from .._pyn import get_family
from ..calculate import AndFilter, FilterBase, NotFilter, OrFilter, resolve_value_in_units

__all__ = ["FilterBase", "Sphere", "FamilyFilter", "AndFilter", "OrFilter", "NotFilter"]


class Sphere(FilterBase):
    """Particles with ((x-cx)^2 + (y-cy)^2) + (z-cz)^2 < radius^2."""

    dynamic_param_specs = {"radius": "pos", "cen": "pos"}

    def __init__(self, radius, cen=(0, 0, 0)):
        self.radius = radius
        self.cen = cen

    def _resolved(self, sim):
        r = self.radius(sim) if callable(self.radius) else self.radius
        c = self.cen(sim) if callable(self.cen) else self.cen
        r = resolve_value_in_units(r, sim, "pos")
        c = np.asarray(c, dtype=np.float64).reshape(3)
        return c, float(r)

    def build_mask(self, sim, params=None):
        cen, radius = self._resolved(sim)
        p = np.asarray(sim["pos"])
        dx = p[:, 0] - cen[0]
        dy = p[:, 1] - cen[1]
        dz = p[:, 2] - cen[2]
        return ((dx * dx + dy * dy) + dz * dz) < radius * radius

    def device_spec(self, sim):
        cen, radius = self._resolved(sim)
        return {"sphere": (cen, radius)}

    def volume(self, sim=None):
        _, radius = self._resolved(sim) if sim is not None else (None, float(self.radius))
        return 4.0 / 3.0 * np.pi * radius ** 3

    def __repr__(self):
        return f"Sphere(radius={self.radius!r}, cen={self.cen!r})"


class FamilyFilter(FilterBase):
    """Particles of one family (dm, gas, star, ...)."""

    def __init__(self, family):
        if isinstance(family, str):
            family = get_family(family, False)
        self.family = family

    def build_mask(self, sim, params=None):
        mask = np.zeros(len(sim), dtype=bool)
        fam = get_family(self.family(sim) if callable(self.family) and not hasattr(self.family, "name")
                         else self.family)
        slices = getattr(sim, "_family_slices", {})
        sl = slices.get(fam)
        if sl is not None:
            mask[sl] = True
        return mask

    def device_spec(self, sim):
        slices = getattr(sim, "_family_slices", None)
        if slices is None or callable(self.family) and not hasattr(self.family, "name"):
            return None
        sl = slices.get(get_family(self.family))
        if sl is None:
            return {"families": []}
        return {"families": [(int(sl.start), int(sl.stop))]}

    def __repr__(self):
        return f"FamilyFilter({getattr(self.family, 'name', self.family)!r})"
