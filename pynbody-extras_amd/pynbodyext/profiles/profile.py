"""Profile objects: bins + weights + cached per-bin arrays.

Interface of the reference's pynbodyext/profiles/profile.py (ProfileBase
:102-522, Profile :528-606, SubProfile :612-630): string keys give
:class:`ProfileArray` s (``prof["mass"]``, ``prof["mass"]["sum"]``, the
``"mass_p16"`` shorthand), registered profile properties (``density``,
``mass_enc``, ...), per-bin properties (``rbins``, ``dr``, ``binsize``,
``npart_bins``), filter / family indexing returning sub-profiles that reuse
the parent's edges, and ``particles_at_bin``.
"""
from __future__ import annotations

import warnings
from collections import defaultdict
from collections.abc import Sequence
from typing import Any

import numpy as np

from .._pyn import SimSnap
from ..simcore import PendingField, is_pending
from .bins import BinsSet
from .proarray import ProfileArray

__all__ = ["Profile", "SubProfile", "ProfileBase"]

_PARENT_KEYS = ("rbins", "dr", "binsize")
_BIN_PROPERTY_KEYS = ("rbins", "dr", "binsize", "npart_bins")


class _ParticlesAtBin:
    def __init__(self, profile: "ProfileBase"):
        self._p = profile

    def __getitem__(self, sel):
        p = self._p
        if isinstance(sel, slice):
            parts = [p.binind[i] for i in range(*sel.indices(p.nbins))]
        elif isinstance(sel, np.ndarray) and sel.dtype == bool:
            if sel.size != p.nbins:
                raise ValueError("Boolean array length must match number of bins.")
            parts = [p.binind[i] for i in range(p.nbins) if sel[i]]
        elif isinstance(sel, Sequence):
            parts = [p.binind[i] for i in sel]
        else:
            return p.sim[np.sort(p.binind[sel])]
        idx = np.concatenate(parts) if parts else np.array([], dtype=int)
        return p.sim[np.sort(idx)]


class ProfileBase:
    """Shared mechanics of root and sub profiles."""

    _profile_property_registry: defaultdict = defaultdict(dict)

    def __init__(self, sim, bins_set: BinsSet, weight=None, parent: "Profile | None" = None):
        self.sim = sim
        self._bins = bins_set if bins_set.is_defined() else bins_set(sim)
        self._parent = parent
        # the weights, or a PendingField (device-held, read on first use)
        self._weight_v = weight
        if weight is not None:
            assert len(weight) == len(sim), "Weight array length must match simulation length."
        self._data_cache: dict[str, ProfileArray] = {}
        self._stats_cache: defaultdict[str, dict[str, ProfileArray]] = defaultdict(dict)
        # name of the per-particle field whose values the device holds as the
        # selection weights (fused path), if any
        self._device_weight_name: str | None = None

    @property
    def _weight(self):
        w = self._weight_v
        if isinstance(w, PendingField):
            w = self._weight_v = w.resolve()
        return w

    @property
    def _weighted(self) -> bool:
        return self._weight_v is not None

    # ---- caching -------------------------------------------------------------
    def cache(self, pro_arr: ProfileArray) -> None:
        if pro_arr._name is None or pro_arr._mode is None:
            return
        self._stats_cache.setdefault(pro_arr._name, {})[pro_arr._mode] = pro_arr

    def is_cached(self, key: str, item: str) -> bool:
        return key in self._stats_cache and item in self._stats_cache[key]

    def get_cached(self, key: str, item: str) -> ProfileArray:
        return self._stats_cache[key][item]

    # ---- bins -----------------------------------------------------------------
    @property
    def bins(self) -> BinsSet:
        return self._bins

    @property
    def nbins(self) -> int:
        return self._bins.nbins

    @property
    def binind(self):
        return self._bins.binind or []

    @property
    def rbins(self):
        return self._bins.rbins

    @property
    def bin_edges(self):
        return self._bins.bin_edges

    @property
    def binsize(self):
        return self._bins.binsize

    @property
    def dr(self):
        return self._bins.dr

    @property
    def npart_bins(self):
        return self._bins.npart_bins

    @property
    def particles_at_bin(self) -> _ParticlesAtBin:
        return _ParticlesAtBin(self)

    def families(self):
        return self.sim.families()

    # ---- keys -----------------------------------------------------------------
    def keys(self) -> list[str]:
        data = list(self._data_cache) + list(self._stats_cache)
        return sorted(set(data).union(_BIN_PROPERTY_KEYS))

    def property_keys(self) -> list[str]:
        reg = self.parent.__class__._profile_property_registry
        keys: set[str] = set()
        for c in self.parent.__class__.mro():
            keys |= set(reg.get(c, {}))
        return sorted(keys)

    def all_keys(self) -> list[str]:
        return sorted(set(self.keys()) | set(self.property_keys()))

    def _ipython_key_completions_(self):
        return self.all_keys()

    @property
    def parent(self) -> "Profile":
        root = self
        while root._parent is not None:
            root = root._parent
        return root

    @property
    def num_cached_arr(self) -> int:
        return len(self._data_cache) + sum(len(v) for v in self._stats_cache.values())

    # ---- sub profiles ---------------------------------------------------------
    def _spawn(self, subset) -> "SubProfile":
        child_bins = self._bins.spawn_with_same_edges(subset)
        w = self._weight[subset.get_index_list(self.sim)] if self._weight is not None else None
        return SubProfile(subset, bins_set=child_bins, weight=w, parent=self.parent)

    # ---- field resolution -----------------------------------------------------
    def _get_property_func(self, key: str):
        reg = self.parent.__class__._profile_property_registry
        for c in self.parent.__class__.mro():
            bucket = reg.get(c)
            if bucket and key in bucket:
                return bucket[key]
        return None

    def _resolve_field(self, key: str) -> ProfileArray:
        if key in self._data_cache:
            return self._data_cache[key]
        if key in self._stats_cache and "mean" in self._stats_cache[key]:
            return self._stats_cache[key]["mean"]
        func = self._get_property_func(key)
        if key in _BIN_PROPERTY_KEYS or func is not None:
            arr = None
            if key in _BIN_PROPERTY_KEYS:
                arr = getattr(self, key)
            if func is not None:
                arr = func(self)
            base = ProfileArray(self, name=key, array=arr, mode=None)
            self._data_cache[key] = base
            return base
        base = ProfileArray(self, name=key, mode="mean")
        self._stats_cache[key][base._mode] = base
        return base

    def get_subprofile(self, subset) -> "SubProfile":
        warnings.warn("get_subprofile is deprecated; use __getitem__ with a filter instead",
                      DeprecationWarning, stacklevel=2)
        return self._spawn(subset)

    def __getitem__(self, key):
        if isinstance(key, str):
            try:
                return self._resolve_field(key)
            except KeyError as orig:
                if "_" not in key:
                    raise orig
                for pos in reversed([i for i, ch in enumerate(key) if ch == "_"]):
                    field, stat = key[:pos], key[pos + 1:]
                    if not field or not stat or ProfileArray.get_statistic(stat) is None:
                        continue
                    try:
                        base = self._resolve_field(field)
                    except KeyError:
                        continue
                    return base[stat]
                raise orig
        subset = self.sim[key]
        if isinstance(subset, SimSnap):
            return self.get_subprofile(subset)
        raise ValueError(f"ProfileBase.__getitem__: key type {type(key)} is not supported for "
                         f"indexing. Key: {key!r}")

    def __getattr__(self, name: str):
        if name.startswith("_"):
            raise AttributeError(name)
        try:
            sub = getattr(self.sim, name)
        except AttributeError as e:
            raise AttributeError(name) from e
        if isinstance(sub, SimSnap):
            return self.get_subprofile(sub)
        raise AttributeError(name)

    def plot(self, y: str, x: str = "rbins", ax=None, set_label: bool = True, y_name=None,
             x_name=None, **kwargs: Any):
        import matplotlib.pyplot as plt

        xdata, ydata = self[x], self[y]
        if ax is None:
            _, ax = plt.subplots()
        line = ax.plot(xdata, ydata, **kwargs)
        if set_label:
            ax.set_xlabel((x if x_name is None else x_name) + xdata.units_latex())
            ax.set_ylabel((y if y_name is None else y_name) + ydata.units_latex())
        return line

    def __repr__(self) -> str:
        fams = [f.name for f in self.families()]
        kind = "root" if self._parent is None else "sub"
        return (f"<{type(self).__name__} type={kind} nbins={self.nbins} families={fams} "
                f"ncached={self.num_cached_arr}>")

    @classmethod
    def profile_property(cls, fn=None, name: str | None = None):
        def deco(f):
            cls._profile_property_registry[cls][name or f.__name__] = f
            return f
        return deco if fn is None else deco(fn)


class Profile(ProfileBase):
    """Root profile of a snapshot; builds its bins on construction."""

    def __init__(self, sim, *, weight=None, bins_by="r", bins_area="spherical_shell",
                 bins_type="lin", nbins=100, bin_min=None, bin_max=None, bins_set=None,
                 **kwargs: Any):
        bset = bins_set if bins_set is not None else BinsSet(
            bins_by=bins_by, bins_area=bins_area, bins_type=bins_type, nbins=nbins,
            bin_min=bin_min, bin_max=bin_max, **kwargs)
        if weight is None:
            w = None
        elif isinstance(weight, str):
            w = PendingField(sim, weight) if is_pending(sim, weight) else sim[weight]
        elif callable(weight):
            w = weight(sim)
        else:
            w = weight
        super().__init__(sim, bset, weight=w, parent=None)
        self._subs_cache: dict = {}

    def get_subprofile(self, subset) -> "SubProfile":
        if subset in self._subs_cache:
            return self._subs_cache[subset]
        sub = self._spawn(subset)
        self._subs_cache[subset] = sub
        return sub

    @property
    def nsubs(self) -> int:
        return len(self._subs_cache)

    @property
    def total_cached_arr(self) -> int:
        return self.num_cached_arr + sum(s.num_cached_arr for s in self._subs_cache.values())

    def __repr__(self) -> str:
        fams = [f.name for f in self.families()]
        kind = "root" if self._parent is None else "sub"
        return (f"<{type(self).__name__} type={kind} nbins={self.nbins} families={fams} "
                f"nsubs={len(self._subs_cache)} ncache={self.total_cached_arr}>")


class SubProfile(ProfileBase):
    """Subset of a root profile: same edges, its own assignment."""

    def get_subprofile(self, subset) -> "SubProfile":
        return self.parent.get_subprofile(subset)

    def _resolve_field(self, key: str) -> ProfileArray:
        if key in _PARENT_KEYS:
            return self.parent._resolve_field(key)
        return super()._resolve_field(key)
