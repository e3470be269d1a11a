"""Calculator layer: the call surface that drives the radial-profile path.

The reference's calculator DAG framework (pynbodyext/core/calculate/, ~7.6k
lines: engine, caching, tracing, pipelines) is out of scope (SURVEY.md §2
row 15); this module keeps the part of its API the hot path is reached
through, with the same names and semantics:

* ``CalculatorBase.__call__(sim, options=None, **overrides)`` -> value,
  ``run(...)`` -> :class:`Result`, ``filter(f)`` / ``with_filter(f)``
  (core/calculate/base.py:559-704),
* ``BoundCalculator``: evaluates its filter scope, then the wrapped
  calculator on ``source_sim[mask]`` (base.py:874-1008,
  context.py:610-646),
* ``FilterBase`` with ``&``, ``|``, ``~`` composition (filters.py:124-313),
* ``RunOptions`` / ``ExecutionContext.phase`` / dynamic parameters
  (context.py:503-533, base.py:422).

MI355X addition: a calculator may implement ``execute_fused(ctx, input,
filt)``; a bound calculator offers it its filter first, so a radial profile
behind a Sphere / FamilyFilter scope runs mask + r + binning as one device
pipeline instead of materialising the masked snapshot on the host.
"""
from __future__ import annotations

import copy
import time
from contextlib import contextmanager
from dataclasses import dataclass, field
from typing import Any

import numpy as np

__all__ = ["RunOptions", "Result", "NodeInput", "ExecutionContext", "CalculatorBase",
           "BoundCalculator", "FilterBase", "AndFilter", "OrFilter", "NotFilter",
           "resolve_value_in_units"]


@dataclass
class RunOptions:
    cache: bool = True
    progress: Any = False
    perf_time: bool = False
    perf_memory: bool = False
    backend: str = "mi355x"
    default_record_policy: Any = None
    errors: str = "raise"
    cache_small_value_bytes: int = 0


@dataclass
class Result:
    value: Any
    perf: dict = field(default_factory=dict)

    def perf_summary(self) -> str:
        return ", ".join(f"{k}={v * 1e3:.2f} ms" for k, v in self.perf.items())


class NodeInput:
    """Snapshot view of one evaluation: the source snapshot and its selection."""

    def __init__(self, source_sim, mask=None, filt=None):
        self.source_sim = source_sim
        self.mask = mask
        self.filter = filt
        self._active = None

    @property
    def active_sim(self):
        if self.mask is None:
            return self.source_sim
        if self._active is None:
            self._active = self.source_sim[np.asarray(self.mask, dtype=bool)]
        return self._active

    def with_selection(self, mask, filt=None) -> "NodeInput":
        if self.mask is not None:
            full = np.zeros(len(self.source_sim), dtype=bool)
            full[np.nonzero(self.mask)[0][np.asarray(mask, dtype=bool)]] = True
            mask = full
        return NodeInput(self.source_sim, mask, filt)


class ExecutionContext:
    def __init__(self, options: RunOptions):
        self.options = options
        self.perf: dict[str, float] = {}

    @contextmanager
    def phase(self, node, name: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if self.options.perf_time:
                key = f"{type(node).__name__}.{name}"
                self.perf[key] = self.perf.get(key, 0.0) + time.perf_counter() - t0

    def raw_value(self, node: "CalculatorBase", input: NodeInput):
        return node.execute(self, input)

    def public_value(self, node: "CalculatorBase", input: NodeInput):
        return node.public_value(node.execute(self, input))


def resolve_value_in_units(value, sim, field_name: str | None):
    """Numbers pass through; unit strings / unit objects convert to the
    units of ``sim[field_name]``."""
    if value is None or isinstance(value, (int, float, np.floating, np.integer)):
        return value
    from ._pyn import units as _units

    if isinstance(value, str) or isinstance(value, getattr(_units, "UnitBase", ())):
        target = sim[field_name].units if field_name else None
        u = _units.Unit(value) if isinstance(value, str) else value
        return float(u.ratio(target)) if target is not None else float(u.ratio(_units.NoUnit))
    return value


class CalculatorBase:
    """Base of every calculator node (reference core/calculate/base.py:209)."""

    dynamic_param_specs: dict[str, str | None] = {}
    default_options = RunOptions()

    # -- evaluation ------------------------------------------------------------
    def execute(self, ctx: ExecutionContext, input: NodeInput):
        raise NotImplementedError

    def public_value(self, value):
        return value

    def run(self, sim, options: RunOptions | None = None, **overrides) -> Result:
        opts = copy.copy(options) if options is not None else copy.copy(self.default_options)
        for k, v in overrides.items():
            if v is not None:
                if not hasattr(opts, k):
                    raise TypeError(f"unknown run option {k!r}")
                setattr(opts, k, v)
        ctx = ExecutionContext(opts)
        value = self.public_value(ctx.raw_value(self, NodeInput(sim)))
        return Result(value, ctx.perf)

    def __call__(self, sim, options: RunOptions | None = None, *, cache=None, progress=None,
                 perf_time=None, perf_memory=None, backend=None, default_record_policy=None,
                 errors=None, cache_small_value_bytes=None):
        return self.run(sim, options, cache=cache, progress=progress, perf_time=perf_time,
                        perf_memory=perf_memory, backend=backend,
                        default_record_policy=default_record_policy, errors=errors,
                        cache_small_value_bytes=cache_small_value_bytes).value

    def value(self, sim, options: RunOptions | None = None, **overrides):
        return self.run(sim, options, **overrides).value

    # -- scoping -----------------------------------------------------------------
    def with_filter(self, filt: "FilterBase") -> "BoundCalculator":
        return BoundCalculator(self, filt)

    def filter(self, filt: "FilterBase") -> "BoundCalculator":
        return self.with_filter(filt)

    # -- dynamic parameters ------------------------------------------------------
    def resolve_dynamic_params(self, ctx: ExecutionContext, input: NodeInput) -> dict:
        out = {}
        sim = input.active_sim
        for name, field_name in self.dynamic_param_specs.items():
            v = getattr(self, name, None)
            if isinstance(v, CalculatorBase):
                v = ctx.public_value(v, input)
            elif callable(v):
                v = v(sim)
            out[name] = resolve_value_in_units(v, sim, field_name or "pos")
        return out

    def instance_signature(self):
        return (type(self).__name__, id(self))


class BoundCalculator(CalculatorBase):
    """A calculator evaluated on the subset selected by a filter scope."""

    def __init__(self, base: CalculatorBase, filt: "FilterBase"):
        self.base = base
        self.pre_filter = filt

    def with_filter(self, filt: "FilterBase") -> "BoundCalculator":
        return BoundCalculator(self.base, self.pre_filter & filt)

    def public_value(self, value):
        return self.base.public_value(value)

    def execute(self, ctx: ExecutionContext, input: NodeInput):
        fused = getattr(self.base, "execute_fused", None)
        if fused is not None and input.mask is None:
            with ctx.phase(self, "fused"):
                res = fused(ctx, input, self.pre_filter)
            if res is not NotImplemented:
                return res
        with ctx.phase(self, "filter"):
            mask = ctx.raw_value(self.pre_filter, input)
            work = input.with_selection(mask, self.pre_filter)
        with ctx.phase(self, "calculate"):
            return ctx.raw_value(self.base, work)


class FilterBase(CalculatorBase):
    """Calculator producing a boolean mask over the active snapshot."""

    def build_mask(self, sim, params: dict) -> np.ndarray:
        raise NotImplementedError

    def execute(self, ctx: ExecutionContext, input: NodeInput) -> np.ndarray:
        sim = input.active_sim
        params = self.resolve_dynamic_params(ctx, input)
        return np.asarray(self.build_mask(sim, params), dtype=bool)

    def __call__(self, sim, *args, **kwargs):
        return self.value(sim)

    def device_spec(self, sim):
        """Device-fusable description ({"sphere": (cen, r), "families": [...]})
        or None when this filter cannot be fused."""
        return None

    def __and__(self, other: "FilterBase") -> "AndFilter":
        return AndFilter(self, other)

    def __or__(self, other: "FilterBase") -> "OrFilter":
        return OrFilter(self, other)

    def __invert__(self) -> "NotFilter":
        return NotFilter(self)


class AndFilter(FilterBase):
    def __init__(self, a: FilterBase, b: FilterBase):
        self.f1, self.f2 = a, b

    def execute(self, ctx, input):
        return ctx.raw_value(self.f1, input) & ctx.raw_value(self.f2, input)

    def device_spec(self, sim):
        s1, s2 = self.f1.device_spec(sim), self.f2.device_spec(sim)
        if s1 is None or s2 is None:
            return None
        if "sphere" in s1 and "sphere" in s2:
            return None
        out = {}
        sph = s1.get("sphere") or s2.get("sphere")
        if sph is not None:
            out["sphere"] = sph
        f1, f2 = s1.get("families"), s2.get("families")
        if f1 is not None and f2 is not None:
            out["families"] = _intersect_ranges(f1, f2)
        elif f1 is not None or f2 is not None:
            out["families"] = f1 if f1 is not None else f2
        return out


class OrFilter(FilterBase):
    def __init__(self, a: FilterBase, b: FilterBase):
        self.f1, self.f2 = a, b

    def execute(self, ctx, input):
        return ctx.raw_value(self.f1, input) | ctx.raw_value(self.f2, input)

    def device_spec(self, sim):
        s1, s2 = self.f1.device_spec(sim), self.f2.device_spec(sim)
        # a union is fusable only between pure family selections
        if s1 is None or s2 is None or set(s1) != {"families"} or set(s2) != {"families"}:
            return None
        return {"families": sorted(s1["families"] + s2["families"])}


class NotFilter(FilterBase):
    def __init__(self, a: FilterBase):
        self.f = a

    def execute(self, ctx, input):
        return ~ctx.raw_value(self.f, input)


def _intersect_ranges(a, b):
    out = []
    for lo1, hi1 in a:
        for lo2, hi2 in b:
            lo, hi = max(lo1, lo2), min(hi1, hi2)
            if hi > lo:
                out.append((lo, hi))
    return out
