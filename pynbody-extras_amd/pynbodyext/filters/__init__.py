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

from .._pyn import filt, get_family
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


def _family_slice(sim, fam):
    """The family's contiguous index range in ``sim`` through pynbody's own
    snapshot interface (``SimSnap._get_family_slice``, as the reference's
    chunk.py:186,232 uses it), or None when the members do not form one
    range (e.g. an index-list sub-snapshot) or ``sim`` has no families."""
    get = getattr(sim, "_get_family_slice", None)
    if get is None:
        return None
    sl = get(fam)
    if not isinstance(sl, slice) or sl.step not in (None, 1):
        return None
    start, stop, _ = sl.indices(len(sim))
    return slice(start, max(start, stop))


class FamilyFilter(FilterBase):
    """Particles of one family (dm, gas, star, ...).  The mask is pynbody's
    own ``filt.FamilyFilter(family)(sim)`` (reference filt.py:84-86 delegates
    to it); the device selection takes the family's index range."""

    def __init__(self, family):
        if isinstance(family, str):
            family = get_family(family, False)
        self.family = family

    def _family(self, sim):
        fam = self.family
        if callable(fam) and not hasattr(fam, "name"):
            fam = fam(sim)
        return get_family(fam, False) if isinstance(fam, str) else fam

    def build_mask(self, sim, params=None):
        return np.asarray(filt.FamilyFilter(self._family(sim))(sim), dtype=bool)

    def device_spec(self, sim):
        if callable(self.family) and not hasattr(self.family, "name"):
            return None
        sl = _family_slice(sim, self._family(sim))
        if sl is None:
            return None
        return {"families": [(sl.start, sl.stop)] if sl.stop > sl.start else []}

    def __repr__(self):
        return f"FamilyFilter({getattr(self.family, 'name', self.family)!r})"
