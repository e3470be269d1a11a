"""Radial profiles (reference pynbodyext/profiles/spatial_profile.py).

``RadialProfile(sim, ndim=3|2, ...)`` bins by ``r`` over spherical shells
or by ``rxy`` over annuli; profile properties ``density`` (Σm / shell
volume), ``mass_enc`` (cumulative Σm, NaN after an empty bin like
numpy's cumsum) and the anisotropy ``beta``.
"""
from __future__ import annotations

from .profile import Profile

__all__ = ["SpatialProfile", "RadialProfile"]


class SpatialProfile(Profile):
    pass


class RadialProfile(SpatialProfile):
    def __init__(self, sim, *, ndim=3, weight=None, bins_type="lin", nbins=100, bin_min=None,
                 bin_max=None, bins_set=None, **kwargs):
        if ndim == 2:
            bins_by, bins_area = "rxy", "annulus"
        elif ndim == 3:
            bins_by, bins_area = "r", "spherical_shell"
        else:
            raise ValueError("ndim must be 2 or 3")
        super().__init__(sim, weight=weight, bins_by=bins_by, bins_area=bins_area,
                         bins_type=bins_type, nbins=nbins, bin_min=bin_min, bin_max=bin_max,
                         bins_set=bins_set, **kwargs)


@SpatialProfile.profile_property
def density(pro):
    return pro["mass"]["sum"] / pro["binsize"]


@SpatialProfile.profile_property
def mass_enc(pro):
    return pro["mass"]["sum"].cumsum()


@SpatialProfile.profile_property
def beta(pro):
    """Velocity anisotropy 1 - (<v_phi^2> + <v_theta^2>) / (2 <v_r^2>)."""
    from ..log import logger

    if pro.bins.bins_by not in ("r",):
        logger.warning("Beta parameter is useful for spherical systems. Consider using "
                       "RadialProfile with ndim=3")
    return 1 - (pro["vphi"]["rms"] ** 2 + pro["vtheta"]["rms"] ** 2) / (2 * pro["vr"]["rms"] ** 2)
