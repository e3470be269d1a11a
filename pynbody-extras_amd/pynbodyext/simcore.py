"""Minimal pynbody-compatible snapshot layer.

pynbody is not installed in this image (nor on the GPU boxes), so the hot
path needs a stand-in for the few pieces of pynbody its callers touch:

* ``SimArray`` — ndarray subclass carrying ``units`` and ``sim``,
  ``in_units``;
* ``units`` — a small dimensional unit system (length, mass, time, G) with
  string parsing such as ``"km**2 s**-2"``;
* ``SimSnap`` / ``SubSnap`` — named arrays, contiguous family slices,
  boolean / index / slice sub-snapshots, ``get_index_list``;
* derived fields ``r = sqrt((x*x + y*y) + z*z)`` and ``rxy``
  (pynbody/derived.py evaluates ``(pos**2).sum(axis=1) ** 0.5``, which
  numpy computes as exactly this expression followed by a correctly rounded
  sqrt);
* ``filt`` — Sphere / FamilyFilter / And / Or / Not masks.

When the real pynbody is importable, :mod:`pynbodyext._pyn` uses it instead.
"""
from __future__ import annotations

import re
from fractions import Fraction

import numpy as np

# --------------------------------------------------------------------------
# units
# --------------------------------------------------------------------------
_SI = {
    # name: (scale in SI, (L, M, T))
    "m": (1.0, (1, 0, 0)),
    "cm": (1e-2, (1, 0, 0)),
    "km": (1e3, (1, 0, 0)),
    "au": (1.495978707e11, (1, 0, 0)),
    "pc": (3.0856775814913673e16, (1, 0, 0)),
    "kpc": (3.0856775814913673e19, (1, 0, 0)),
    "Mpc": (3.0856775814913673e22, (1, 0, 0)),
    "kg": (1.0, (0, 1, 0)),
    "g": (1e-3, (0, 1, 0)),
    "Msol": (1.98847e30, (0, 1, 0)),
    "s": (1.0, (0, 0, 1)),
    "yr": (3.15576e7, (0, 0, 1)),
    "Myr": (3.15576e13, (0, 0, 1)),
    "Gyr": (3.15576e16, (0, 0, 1)),
    "G": (6.6743e-11, (3, -1, -2)),
}


class UnitsException(ValueError):
    pass


class Unit:
    """scale x m^L kg^M s^T with rational exponents."""

    __slots__ = ("scale", "dims")

    def __init__(self, scale: float = 1.0, dims=(0, 0, 0)):
        self.scale = float(scale)
        self.dims = tuple(Fraction(d) for d in dims)

    def __mul__(self, o):
        o = as_unit(o)
        return Unit(self.scale * o.scale, tuple(a + b for a, b in zip(self.dims, o.dims)))

    __rmul__ = __mul__

    def __truediv__(self, o):
        o = as_unit(o)
        return Unit(self.scale / o.scale, tuple(a - b for a, b in zip(self.dims, o.dims)))

    def __rtruediv__(self, o):
        return as_unit(o) / self

    def __pow__(self, p):
        if isinstance(p, tuple):
            p = Fraction(p[0], p[1])
        p = Fraction(p)
        return Unit(self.scale ** float(p), tuple(d * p for d in self.dims))

    def __eq__(self, o):
        try:
            o = as_unit(o)
        except Exception:
            return False
        return self.dims == o.dims and np.isclose(self.scale, o.scale, rtol=1e-14, atol=0)

    def __hash__(self):
        return hash((round(self.scale, 12), self.dims))

    def ratio(self, other) -> float:
        other = as_unit(other)
        if self.dims != other.dims:
            raise UnitsException(f"incompatible units {self} and {other}")
        return self.scale / other.scale

    def is_dimensionless(self) -> bool:
        return all(d == 0 for d in self.dims)

    def latex(self):
        return str(self)

    def __repr__(self):
        parts = []
        for sym, d in zip(("m", "kg", "s"), self.dims):
            if d == 1:
                parts.append(sym)
            elif d != 0:
                parts.append(f"{sym}**{d}")
        body = " ".join(parts)
        if self.scale != 1.0:
            body = f"{self.scale:.6g} {body}".strip()
        return body or "1"


NoUnit = Unit()
_TOKEN = re.compile(r"^([A-Za-z]+)(?:\*\*\(?(-?\d+(?:/\d+)?)\)?)?$")


def parse_unit(text: str) -> Unit:
    u = Unit()
    for tok in text.replace("^", "**").split():
        try:
            u = u * float(tok)
            continue
        except ValueError:
            pass
        m = _TOKEN.match(tok)
        if not m or m.group(1) not in _SI:
            raise UnitsException(f"unknown unit token {tok!r} in {text!r}")
        scale, dims = _SI[m.group(1)]
        p = Fraction(m.group(2)) if m.group(2) else Fraction(1)
        u = u * (Unit(scale, dims) ** p)
    return u


def as_unit(x) -> Unit:
    if isinstance(x, Unit):
        return x
    if isinstance(x, str):
        return parse_unit(x)
    if isinstance(x, (int, float, np.floating, np.integer)):
        return Unit(float(x))
    if x is None:
        return NoUnit
    raise UnitsException(f"cannot interpret {x!r} as a unit")


_UnitCls = Unit


class _UnitsNamespace:
    Unit = staticmethod(as_unit)
    UnitBase = _UnitCls
    NoUnit = NoUnit
    UnitsException = UnitsException
    G = _UnitCls(*_SI["G"])
    kpc = _UnitCls(*_SI["kpc"])
    km = _UnitCls(*_SI["km"])
    s = _UnitCls(*_SI["s"])
    Msol = _UnitCls(*_SI["Msol"])


units = _UnitsNamespace()


# --------------------------------------------------------------------------
# arrays
# --------------------------------------------------------------------------
class SimArray(np.ndarray):
    """ndarray with ``units`` and ``sim`` attributes."""

    def __new__(cls, data, units=None, sim=None, dtype=None):
        obj = np.asarray(data, dtype=dtype).view(cls)
        obj.units = as_unit(units) if units is not None else NoUnit
        obj.sim = sim
        return obj

    def __array_finalize__(self, obj):
        self.units = getattr(obj, "units", NoUnit)
        self.sim = getattr(obj, "sim", None)

    def in_units(self, new_unit, **kw) -> "SimArray":
        target = as_unit(new_unit)
        out = (np.asarray(self) * self.units.ratio(target)).view(SimArray)
        out.units = target
        out.sim = self.sim
        return out

    def convert_units(self, new_unit) -> None:
        target = as_unit(new_unit)
        self *= self.units.ratio(target)
        self.units = target


IndexedSimArray = SimArray


# --------------------------------------------------------------------------
# families
# --------------------------------------------------------------------------
class Family:
    _registry: dict[str, "Family"] = {}

    def __new__(cls, name: str):
        if name in cls._registry:
            return cls._registry[name]
        obj = super().__new__(cls)
        obj.name = name
        cls._registry[name] = obj
        return obj

    def __repr__(self):
        return f"<Family {self.name}>"

    def __reduce__(self):
        return (Family, (self.name,))


for _n in ("dm", "star", "gas", "bh"):
    Family(_n)


def get_family(name, create: bool = False) -> Family:
    if isinstance(name, Family):
        return name
    if name in Family._registry or create:
        return Family(name)
    raise ValueError(f"{name!r} is not a family")


# --------------------------------------------------------------------------
# snapshots
# --------------------------------------------------------------------------
class SimSnap:
    """A particle snapshot: named per-particle arrays + contiguous families."""

    def __init__(self, arrays: dict, families: dict | None = None, units_map: dict | None = None):
        self._arrays: dict[str, np.ndarray] = {}
        n = None
        for k, v in arrays.items():
            v = np.asarray(v)
            n = len(v) if n is None else n
            if len(v) != n:
                raise ValueError(f"array {k!r} has length {len(v)}, expected {n}")
            self._arrays[k] = v
        self._n = n or 0
        units_map = units_map or {}
        self._units = {k: as_unit(u) for k, u in units_map.items()}
        # family name -> slice of the particle index range
        self._family_slice: dict[Family, slice] = {}
        for name, sl in (families or {}).items():
            self._family_slice[get_family(name, True)] = sl
        self._derived: dict[str, np.ndarray] = {}

    # ---- basic protocol ----------------------------------------------------
    def __len__(self) -> int:
        return self._n

    def families(self) -> list[Family]:
        return [f for f, sl in self._family_slice.items() if sl.stop > sl.start]

    def family_slice(self, fam) -> slice:
        return self._family_slice[get_family(fam)]

    def _get_family_slice(self, fam) -> slice:
        """pynbody's SimSnap._get_family_slice: the family's index range, or
        an empty slice when the snapshot has no such particles."""
        return self._family_slice.get(get_family(fam), slice(0, 0))

    def keys(self):
        return list(self._arrays)

    def _array(self, key: str) -> np.ndarray:
        if key in self._arrays:
            return self._arrays[key]
        if key in self._derived:
            return self._derived[key]
        if key in ("x", "y", "z"):
            return self._array("pos")[:, "xyz".index(key)]
        if key in ("vx", "vy", "vz"):
            return self._array("vel")[:, "xyz".index(key[1])]
        if key == "r":
            p = self._array("pos")
            x, y, z = p[:, 0], p[:, 1], p[:, 2]
            val = np.sqrt((x * x + y * y) + z * z)
        elif key == "rxy":
            p = self._array("pos")
            x, y = p[:, 0], p[:, 1]
            val = np.sqrt(x * x + y * y)
        else:
            raise KeyError(key)
        self._derived[key] = val
        return val

    def _unit_of(self, key: str):
        if key in self._units:
            return self._units[key]
        if key in ("r", "rxy", "x", "y", "z") and "pos" in self._units:
            return self._units["pos"]
        if key in ("vx", "vy", "vz") and "vel" in self._units:
            return self._units["vel"]
        return NoUnit

    def __setitem__(self, key: str, value):
        value = np.asarray(value)
        if len(value) != self._n:
            raise ValueError("array length mismatch")
        self._arrays[key] = value
        if isinstance(value, SimArray) and value.units is not NoUnit:
            self._units[key] = value.units
        self._derived.pop(key, None)
        self.__dict__.get("_pending", {}).pop(key, None)

    def __getitem__(self, key):
        if isinstance(key, str):
            a = self._array(key).view(SimArray)
            a.units = self._unit_of(key)
            a.sim = self
            return a
        if isinstance(key, Family):
            return SubSnap(self, np.arange(self._n)[self._family_slice.get(key, slice(0, 0))])
        if isinstance(key, slice):
            return SubSnap(self, np.arange(self._n)[key])
        if callable(key) and hasattr(key, "__call__") and not isinstance(key, np.ndarray):
            return SubSnap(self, np.nonzero(np.asarray(key(self)))[0])
        idx = np.asarray(key)
        if idx.dtype == bool:
            if idx.shape != (self._n,):
                raise IndexError("boolean mask length mismatch")
            return SubSnap(self, np.nonzero(idx)[0])
        return SubSnap(self, idx.astype(np.int64))

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        fams = self.__dict__.get("_family_slice", {})
        for f in fams:
            if f.name == name:
                return self[f]
        raise AttributeError(name)

    def get_index_list(self, relative_to: "SimSnap") -> np.ndarray:
        if relative_to is self:
            return np.arange(self._n)
        raise ValueError("snapshot is not a subsnap of relative_to")

    @property
    def ancestor(self) -> "SimSnap":
        return self

    def __repr__(self):
        return f"<SimSnap n={self._n} families={[f.name for f in self.families()]}>"


class SubSnap(SimSnap):
    """Index-list view of a parent snapshot (pynbody IndexedSubSnap)."""

    def __init__(self, base: SimSnap, index: np.ndarray, increasing: bool | None = None):
        self._base = base
        self._index = np.asarray(index, dtype=np.int64)
        self._n = len(self._index)
        self._derived = {}
        # fields a device holds for this view, read on first access
        # (key -> fetch(): the array); see PendingField
        self._pending = {}
        root = base.ancestor
        # family slices of the view: families of the root restricted to index
        self._family_slice = {}
        self._root_index = base._root_index[self._index] if isinstance(base, SubSnap) else self._index
        # strictly increasing root indices (checked once; a caller that knows
        # it — the device selection's compacted indices — says so)
        if increasing is None or isinstance(base, SubSnap):
            ri = self._root_index
            increasing = bool(len(ri) < 2 or np.all(ri[1:] > ri[:-1]))
        self._increasing = increasing
        if increasing:
            for f, sl in root._family_slice.items():
                lo = np.searchsorted(self._root_index, sl.start, side="left")
                hi = np.searchsorted(self._root_index, sl.stop, side="left")
                self._family_slice[f] = slice(int(lo), int(hi))
        self._arrays = {}
        self._units = {}

    def _get_family_slice(self, fam):
        """Index range of the family in this view; for a view whose root
        indices are not increasing (families need not be contiguous) the
        positions of its members as an index array."""
        fam = get_family(fam)
        if fam in self._family_slice or self._increasing:
            return self._family_slice.get(fam, slice(0, 0))
        sl = self.ancestor._get_family_slice(fam)
        return np.nonzero((self._root_index >= sl.start) & (self._root_index < sl.stop))[0]

    @property
    def ancestor(self) -> SimSnap:
        return self._base.ancestor

    def keys(self):
        return self._base.keys()

    def _array(self, key: str) -> np.ndarray:
        if key in self._arrays:
            return self._arrays[key]
        if key in self._derived:
            return self._derived[key]
        fetch = self._pending.pop(key, None)
        val = fetch() if fetch is not None else self._base._array(key)[self._index]
        self._derived[key] = val
        return val

    def is_pending(self, key: str) -> bool:
        """The field is held by a device and not read onto the host yet."""
        return key in self._pending and key not in self._arrays and key not in self._derived

    def _unit_of(self, key: str):
        return self._base._unit_of(key)

    def get_index_list(self, relative_to: SimSnap) -> np.ndarray:
        if relative_to is self._base:
            return self._index
        if relative_to is self:
            return np.arange(self._n)
        if isinstance(self._base, SubSnap):
            return self._base.get_index_list(relative_to)[self._index]
        if relative_to is self.ancestor:
            return self._root_index
        raise ValueError("snapshot is not a subsnap of relative_to")

    def __repr__(self):
        return f"<SubSnap n={self._n} of {self._base!r}>"


IndexedSubSnap = SubSnap


class PendingField:
    """A view's field that a device holds and the host has not read yet
    (SubSnap._pending): its length and units without the copy; resolve()
    reads it (sim[key], the same values)."""

    __slots__ = ("sim", "key")

    def __init__(self, sim: SubSnap, key: str):
        self.sim, self.key = sim, key

    def __len__(self) -> int:
        return len(self.sim)

    @property
    def units(self):
        return self.sim._unit_of(self.key)

    def resolve(self) -> SimArray:
        return self.sim[self.key]


def is_pending(sim, key) -> bool:
    """``key`` of ``sim`` is a device-held field not read onto the host yet."""
    f = getattr(sim, "is_pending", None)
    return isinstance(key, str) and f is not None and f(key)


def new_snapshot(pos, mass, families: dict | None = None, units_map: dict | None = None,
                 **arrays) -> SimSnap:
    """Build a snapshot from (N,3) positions, (N,) masses and extra arrays."""
    arrs = {"pos": np.asarray(pos, dtype=np.float64), "mass": np.asarray(mass, dtype=np.float64)}
    arrs.update(arrays)
    return SimSnap(arrs, families=families, units_map=units_map)


# --------------------------------------------------------------------------
# filters returning boolean masks (pynbody.filt semantics)
# --------------------------------------------------------------------------
class Filter:
    def __call__(self, sim) -> np.ndarray:
        raise NotImplementedError

    def __and__(self, other):
        return And(self, other)

    def __or__(self, other):
        return Or(self, other)

    def __invert__(self):
        return Not(self)


class And(Filter):
    def __init__(self, a, b):
        self.f1, self.f2 = a, b

    def __call__(self, sim):
        return self.f1(sim) & self.f2(sim)


class Or(Filter):
    def __init__(self, a, b):
        self.f1, self.f2 = a, b

    def __call__(self, sim):
        return self.f1(sim) | self.f2(sim)


class Not(Filter):
    def __init__(self, a):
        self.f = a

    def __call__(self, sim):
        return ~self.f(sim)


class Sphere(Filter):
    """((x-cx)^2 + (y-cy)^2) + (z-cz)^2 < radius^2 (strict, no periodic wrap)."""

    def __init__(self, radius, cen=(0, 0, 0)):
        self.radius = float(radius)
        self.cen = np.asarray(cen, dtype=np.float64).reshape(3)

    def __call__(self, sim):
        p = np.asarray(sim["pos"])
        dx = p[:, 0] - self.cen[0]
        dy = p[:, 1] - self.cen[1]
        dz = p[:, 2] - self.cen[2]
        return ((dx * dx + dy * dy) + dz * dz) < self.radius * self.radius


class FamilyFilter(Filter):
    def __init__(self, family):
        self.family = get_family(family)

    def __call__(self, sim):
        mask = np.zeros(len(sim), dtype=bool)
        mask[sim._get_family_slice(self.family)] = True
        return mask


class filt:  # namespace mirroring pynbody.filt
    Filter = Filter
    And = And
    Or = Or
    Not = Not
    Sphere = Sphere
    FamilyFilter = FamilyFilter
