"""Per-bin profile arrays and their statistics.

:class:`ProfileArray` and the :class:`StatisticBase` plug-in registry keep
the reference's interface (pynbodyext/profiles/proarray.py:119-860): string
indexing computes a statistic (``pa["median"]``, ``pa["p84"]``,
``pa["abs_mean"]``), results are cached on the owning profile, an empty bin
gives NaN for every statistic (including ``sum``).

Evaluation: statistics that are functions of per-bin sums — ``mean``,
``sum``, ``sum_w``, ``rms``, ``disp`` and their ``abs_`` forms — are
computed from one device reduction (Σw, Σf·w, Σf²·w, Σf, Σf², Σ|f|·w,
Σ|f| per bin, csrc/profile.hip moments) using the reference's formulas.
Order statistics (``pXX``, ``median``, ``abs_pXX``) are computed on the
device too (segmented radix sort by bin and value, the reference's
sequential weight cumsum and np.interp per bin, pbx_profile_percentiles);
user-registered statistics run the reference's per-bin loop over the
device-built bin index lists.
"""
from __future__ import annotations

import re
import warnings
from typing import Union

import numpy as np

from .._pyn import IndexedSimArray, SimArray
from ..simcore import PendingField, is_pending
from ._device import SRC_HOST, SRC_NONE, SRC_W, SRC_X

__all__ = ["ProfileArray", "StatisticBase", "Mean", "Sum", "Sum_w", "Percentile", "RMS", "Median",
           "Abs", "Dispersion"]


class _StatAccessor:
    def __init__(self, owner: "ProfileArray"):
        if not owner._check_base_for_stats():
            raise RuntimeError("Cannot compute statistics on this ProfileArray")
        self._owner = owner

    def __getitem__(self, key: str) -> "ProfileArray":
        owner = self._owner
        profile, name = owner._profile, owner._name
        if profile.is_cached(name, key):
            return profile.get_cached(name, key)
        out, mode = owner._compute(profile, name, compute_mode=key)
        res = ProfileArray(profile, name=name, array=out, mode=mode)
        profile.cache(res)
        return res

    def _ipython_key_completions_(self):
        return self._owner.keys()


class ProfileArray(SimArray):
    """A 1-D per-bin array bound to a profile and a per-particle source field."""

    _registry: list[type["StatisticBase"]] = []

    def __new__(cls, profile, *, name: str, array=None, mode: str | None = None):
        if not isinstance(name, str):
            raise ValueError("name must be a string")
        src = name if array is None else array
        if array is not None:
            arr = array
        elif is_pending(profile.sim, name):  # (device-held: its length, no host copy)
            arr = PendingField(profile.sim, name)
        else:
            arr = profile.sim[name]
        if not isinstance(arr, (np.ndarray, SimArray, IndexedSimArray, PendingField)):
            raise ValueError("array must be a numpy ndarray or SimArray, got " + str(type(arr)))
        n_particles, n_bins = len(profile.sim), profile.nbins
        if len(arr) == n_particles:
            base, mode = cls._compute(profile, src, compute_mode=mode if mode is not None else "mean")
            obj = np.asarray(base).view(cls)
            obj.units, obj.sim = getattr(base, "units", None), getattr(base, "sim", None)
            obj._source = "per_particle"
        elif len(arr) == n_bins:
            obj = np.asarray(arr).view(cls)
            if isinstance(arr, SimArray):
                obj.units, obj.sim = arr.units, arr.sim
            obj._source = "per_bin" if mode is None else "per_particle"
        else:
            raise ValueError(f"array length {len(arr)} not compatible: expected number of particles "
                             f"({n_particles}) or number of bins ({n_bins})")
        obj._arr = arr
        obj._name = name
        obj._mode = mode
        obj._profile = profile
        obj._is_view = False
        return obj

    def __init__(self, profile, *, name: str, array=None, mode: str | None = None):
        pass

    def __array_finalize__(self, obj):
        super().__array_finalize__(obj)
        if obj is None:
            return
        self._profile = getattr(obj, "_profile", None)
        self._name = getattr(obj, "_name", "None")
        self._source = getattr(obj, "_source", "per_bin")
        self._arr = getattr(obj, "_arr", None)
        self._mode = getattr(obj, "_mode", None)
        self._is_view = True

    # ---- statistics -------------------------------------------------------------
    @classmethod
    def get_statistic(cls, key: str) -> Union["StatisticBase", None]:
        for stat in cls._registry:
            res = stat.valid(key)
            if res is not None:
                return res
        return None

    @classmethod
    def _compute(cls, profile, arr, compute_mode: str):
        """Per-bin statistic of a per-particle field (name or array)."""
        calc = cls.get_statistic(compute_mode)
        if calc is None:
            raise ValueError(f"Statistic '{compute_mode}' not found")
        name = arr if isinstance(arr, str) else None
        # a device-held field of the view (fused selection) is not read onto
        # the host when the device sums it (arr_pp None until a path needs it)
        pending = name is not None and is_pending(profile.sim, name)
        arr_pp = None if pending else (profile.sim[arr] if isinstance(arr, str) else arr)
        weighted = profile._weighted
        fast = calc.from_moments if hasattr(calc, "from_moments") else None
        dev = getattr(profile.bins, "_device", None) if fast is not None else None
        pct = _percentile_of(calc)
        pdev = getattr(profile.bins, "_device", None) if pct is not None else None
        if dev is not None and dev.nbins == profile.nbins:
            cols = _columns_of(fast, profile.nbins, weighted)
            vals = fast(_moments_for(profile, dev, name, arr_pp, cols),
                        np.asarray(profile.npart_bins), weighted)
        elif pdev is not None and pdev.nbins == profile.nbins:
            fsrc, wsrc = _sources_for(profile, pdev, name, arr_pp)
            vals = pdev.percentiles([pct[0] / 100], fsrc, wsrc, absval=pct[1])[:, 0]
        else:
            if arr_pp is None:
                arr_pp = profile.sim[arr]
            weights = profile._weight
            vals = np.zeros(profile.nbins)
            for i, ind in enumerate(profile.binind):
                if len(ind) == 0:
                    vals[i] = np.nan
                    continue
                vals[i] = calc(arr_pp[ind], None if weights is None else weights[ind])
        res = np.asarray(vals, dtype=np.float64).view(SimArray)
        if arr_pp is None:  # (what sim[arr] would carry)
            res.units = profile.sim._unit_of(arr)
            res.sim = profile.sim
        elif isinstance(arr_pp, (SimArray, IndexedSimArray)):
            res.units = arr_pp.units
            res.sim = arr_pp.sim
        return res, calc.key

    @property
    def stat(self) -> _StatAccessor:
        return _StatAccessor(self)

    def _check_base_for_stats(self) -> bool:
        if self._profile is None or self._source == "per_bin":
            warnings.warn("Statistics are only available on the base ProfileData.", stacklevel=2)
            return False
        return True

    @property
    def profile(self):
        return self._profile

    @profile.setter
    def profile(self, value):
        self._profile = value

    def __getitem__(self, item):
        if isinstance(item, str):
            return self.stat[item]
        return super().__getitem__(item)

    def keys(self) -> list[str]:
        if not self._check_base_for_stats():
            return []
        return [s.example_name for s in ProfileArray._registry if s.example_name is not None]

    def units_latex(self) -> str:
        u = getattr(self, "units", None)
        if u is None or (u.is_dimensionless() and u.ratio(type(u)()) == 1):
            return ""
        la = u.latex()
        return f" [${la}$]" if la is not None else ""

    def _ipython_key_completions_(self):
        return self.keys()

    def __repr__(self):
        x = np.ndarray.__repr__(np.asarray(self))
        flag = f", '{self._source}::{self._name}"
        if self._mode is not None:
            flag += f"::{self._mode}"
        if self._is_view:
            flag += "::View"
        return x[:-1] + flag + "')"


class _ColumnProbe:
    """Stands in for the (nbins, 7) moments in one dry run of a statistic's
    ``from_moments`` to learn which columns it reads."""

    def __init__(self, nb):
        self.nb, self.cols = nb, 0

    def __getitem__(self, key):
        self.cols |= 1 << int(key[1])
        return np.ones(self.nb)


def _columns_of(fast, nb, weighted) -> int:
    probe = _ColumnProbe(nb)
    with np.errstate(all="ignore"):
        fast(probe, np.ones(nb), weighted)
    return probe.cols


def _percentile_of(calc):
    """(percent, absval) when ``calc`` is an order statistic the device
    computes (pXX, median, abs_pXX, abs_median), else None."""
    absval = False
    if isinstance(calc, Abs):
        calc, absval = calc._substat, True
    if isinstance(calc, Percentile):
        return calc.percentile, absval
    if isinstance(calc, Median):
        return 50, absval
    return None


def _sources_for(profile, dev, name, arr_pp):
    """Device source selectors (or host arrays) of a field and the weights
    (arr_pp None: the field is device-held and not on the host yet)."""
    bins = profile.bins
    if name is not None and isinstance(bins.bins_by, str) and name == bins.bins_by:
        fsrc = SRC_X
    elif name is not None and dev.has_selection and name == getattr(profile, "_device_weight_name", None):
        fsrc = SRC_W
    else:
        fsrc = np.asarray(profile.sim[name] if arr_pp is None else arr_pp, dtype=np.float64)
    if not profile._weighted:
        wsrc = SRC_NONE
    elif getattr(profile, "_device_weight_name", None) is not None and dev.has_selection:
        wsrc = SRC_W
    else:
        wsrc = np.asarray(profile._weight, dtype=np.float64)
    return fsrc, wsrc


def _moments_for(profile, dev, name, arr_pp, cols=(1 << 7) - 1) -> np.ndarray:
    """(nbins, 7) device sums of a field, reusing device-resident arrays;
    only the columns in ``cols`` are accumulated."""
    fsrc, wsrc = _sources_for(profile, dev, name, arr_pp)
    return dev.moments(fsrc, wsrc, cols)


# ---------------------------------------------------------------- plug-ins
class StatisticBase:
    """Base of per-bin statistics; subclasses self-register."""

    example_name: str | None = None

    def __init_subclass__(cls) -> None:
        if getattr(cls, "example_name", None) is None:
            warnings.warn(f"StatisticBase subclass {cls.__name__} missing example_name attribute, "
                          "would be good to add one for clarity.", DeprecationWarning, stacklevel=2)
        ProfileArray._registry.append(cls)

    def __init__(self, key: str):
        self.key = key

    def __call__(self, arr, weight):
        raise NotImplementedError

    @classmethod
    def valid(cls, key: str):
        return cls(key) if key == cls.__name__ else None


def _nan_empty(vals, counts):
    vals = np.asarray(vals, dtype=np.float64)
    vals[np.asarray(counts) == 0] = np.nan
    return vals


# column indices of the device moments
W, FW, F2W, F, F2, AW, A = range(7)


class Mean(StatisticBase):
    """(Σ x w) / Σ w, or the plain mean."""

    example_name = "mean"

    def __call__(self, arr, weight):
        return (arr * weight).sum() / weight.sum() if weight is not None else arr.mean()

    def from_moments(self, m, counts, weighted, col=F, wcol=FW):
        with np.errstate(divide="ignore", invalid="ignore"):
            v = m[:, wcol] / m[:, W] if weighted else m[:, col] / counts
        return _nan_empty(v, counts)

    @classmethod
    def valid(cls, key):
        return cls("mean") if key.lower() == "mean" else None


class Sum(StatisticBase):
    """Σ x (never weighted)."""

    example_name = "sum"

    def __call__(self, arr, weight):
        return arr.sum()

    def from_moments(self, m, counts, weighted, col=F, wcol=FW):
        return _nan_empty(m[:, col].copy(), counts)

    @classmethod
    def valid(cls, key):
        return cls("sum") if key.lower() == "sum" else None


class Sum_w(StatisticBase):  # noqa: N801 - reference name
    """Σ x w (plain sum when unweighted)."""

    example_name = "sum_w"

    def __call__(self, arr, weight):
        return (arr * weight).sum() if weight is not None else arr.sum()

    def from_moments(self, m, counts, weighted, col=F, wcol=FW):
        return _nan_empty((m[:, wcol] if weighted else m[:, col]).copy(), counts)

    @classmethod
    def valid(cls, key):
        return cls("sum_w") if key.lower() == "sum_w" else None


class Percentile(StatisticBase):
    """Weighted / unweighted percentile ``pXX`` (interpolated cumulative weight)."""

    example_name = "p16"

    def __init__(self, key: str, percentile: int):
        super().__init__(key)
        self.percentile = percentile

    def __call__(self, arr, weight):
        if len(arr) == 0:
            return np.nan
        idx = np.argsort(arr)
        s = arr[idx]
        if weight is None:
            cdf = np.linspace(0, 1, len(s))
        else:
            cdf = weight[idx].cumsum()
            cdf -= cdf[0]
            cdf /= cdf[-1]
        return np.interp(self.percentile / 100, cdf, s)

    @classmethod
    def valid(cls, key):
        k = key.lower()
        m = re.match(r"^p(\d{1,3})$", k)
        if m and 0 <= int(m.group(1)) <= 100:
            return cls(k, int(m.group(1)))
        return None

    @classmethod
    def name(cls):
        return "p**"


class RMS(StatisticBase):
    """sqrt(Σ x² w / Σ w), or sqrt(mean(x²))."""

    example_name = "rms"

    def __call__(self, arr, weight):
        if len(arr) == 0:
            return np.nan
        if weight is not None:
            return np.sqrt((arr ** 2 * weight).sum() / weight.sum())
        return np.sqrt((arr ** 2).mean())

    def from_moments(self, m, counts, weighted, col=F, wcol=FW):
        with np.errstate(divide="ignore", invalid="ignore"):
            v = np.sqrt(m[:, F2W] / m[:, W]) if weighted else np.sqrt(m[:, F2] / counts)
        return _nan_empty(v, counts)

    @classmethod
    def valid(cls, key):
        return cls("rms") if key.lower() == "rms" else None


class Median(StatisticBase):
    """Median per bin (``p50``)."""

    example_name = "median"

    def __call__(self, arr, weight):
        return Percentile(self.key, 50)(arr, weight)

    @classmethod
    def valid(cls, key):
        return cls("median") if key.lower() in ("med", "median") else None


class Abs(StatisticBase):
    """Any statistic of |x|: ``abs`` (= ``abs_mean``), ``abs_p16``, ``abs_sum``, ..."""

    example_name = "abs"

    def __init__(self, key: str, substat: StatisticBase):
        super().__init__(key)
        self._substat = substat
        if hasattr(substat, "from_moments"):
            self.from_moments = self._from_moments

    def __call__(self, arr, weight):
        return self._substat(np.abs(arr), weight)

    def _from_moments(self, m, counts, weighted):
        return self._substat.from_moments(m, counts, weighted, col=A, wcol=AW)

    @classmethod
    def valid(cls, key):
        k = key.lower()
        if k in ("abs", "abs_"):
            sub = "mean"
        elif k.startswith("abs_"):
            sub = k[4:]
        else:
            return None
        s = ProfileArray.get_statistic(sub)
        if s is None:
            return None
        return cls("abs_" + s.key, s)


class Dispersion(StatisticBase):
    """sqrt(E[x²] - E[x]²) with the reference's -1e-12 clamp."""

    example_name = "disp"

    def __call__(self, arr, weight):
        if len(arr) == 0:
            return np.nan
        if weight is not None:
            ws = float(np.asarray(weight.sum()))
            if ws == 0:
                return np.nan
            sq = float(np.asarray((arr ** 2 * weight).sum() / ws))
            mn = float(np.asarray((arr * weight).sum() / ws)) ** 2
        else:
            sq = float(np.asarray((arr ** 2).mean()))
            mn = float(np.asarray(arr.mean())) ** 2
        d = sq - mn
        if -1e-12 < d < 0:
            d = 0.0
        return float(np.sqrt(d)) if d >= 0 else np.nan

    def from_moments(self, m, counts, weighted, col=F, wcol=FW):
        with np.errstate(divide="ignore", invalid="ignore"):
            if weighted:
                ws = m[:, W]
                sq = m[:, F2W] / ws
                mn = (m[:, wcol] / ws) ** 2
            else:
                sq = m[:, F2] / counts
                mn = (m[:, col] / counts) ** 2
            d = sq - mn
            d = np.where((d < 0) & (d > -1e-12), 0.0, d)
            v = np.where(d >= 0, np.sqrt(np.where(d >= 0, d, 0.0)), np.nan)
            if weighted:
                v = np.where(ws == 0, np.nan, v)
        return _nan_empty(v, counts)

    @classmethod
    def valid(cls, key):
        return cls("disp") if key.lower() in ("dispersion", "disp") else None
