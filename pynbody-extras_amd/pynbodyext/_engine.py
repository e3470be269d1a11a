"""Python surface of the native gravity engine.

Same names, signatures, argument checks and error messages as the
reference's PyO3 module ``pynbodyext._rust``
(crates/pynbodyext-rust/src/lib.rs:10-27, gravity.rs:33-709), computed by
the HIP kernels of libpbx.so instead of rayon threads.  ``threads`` is
accepted for signature compatibility; on the GPU it has no effect.

Argument handling restated from gravity.rs:
  * positions / targets / points: 2-D float64 arrays (PyO3's typed
    extraction -> TypeError otherwise); a C-contiguous array only has to
    hold a multiple of 3 values (gravity.rs:38-50), a strided one must be
    (N, 3) (gravity.rs:52-58) -> ValueError "{name} must be (N,3) float64
    array".
  * masses / softenings: contiguous 1-D float64 of length N
    ("masses must be length N", "softenings must be length N").
  * softenings without a kernel -> ValueError (gravity.rs:480-484).
  * kernel: None, 0 (Plummer) or 1 (CubicSplineW2) (gravity.rs:67-75).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as nat


def _require_f64(arr, ndim: int, argname: str) -> np.ndarray:
    if not isinstance(arr, np.ndarray) or arr.dtype != np.float64 or arr.ndim != ndim:
        got = type(arr).__name__
        if isinstance(arr, np.ndarray):
            got = f"ndarray(dtype={arr.dtype}, ndim={arr.ndim})"
        raise TypeError(
            f"argument '{argname}': {got} cannot be converted to "
            f"'PyArray<f64, Dim<[usize; {ndim}]>>'")
    return arr


def extract_vec3(arr, name: str, argname: str | None = None) -> np.ndarray:
    """(N,3) float64 C-contiguous copy/view, gravity.rs:33-65."""
    a = _require_f64(arr, 2, argname or name)
    if a.flags.c_contiguous:
        if a.size % 3 != 0:
            raise ValueError(f"{name} must be (N,3) float64 array")
        return a.reshape(-1, 3)
    if a.shape[1] != 3:
        raise ValueError(f"{name} must be (N,3) float64 array")
    return np.ascontiguousarray(a)


def _extract_vec1(arr, n: int, what: str, argname: str) -> np.ndarray | None:
    if arr is None:
        return None
    a = _require_f64(arr, 1, argname)
    if not a.flags.c_contiguous:
        raise TypeError(f"argument '{argname}': The given array is not contiguous")
    if a.shape[0] != n:
        raise ValueError(f"{what} must be length N")
    return a


def _kernel_code(kernel) -> int:
    if kernel is None:
        return nat.KERNEL_NONE
    if isinstance(kernel, bool) or not isinstance(kernel, (int, np.integer)):
        raise TypeError(f"argument 'kernel': '{type(kernel).__name__}' object cannot be "
                        "interpreted as an integer")
    k = int(kernel)
    if k < 0 or k > 255:
        raise OverflowError("can't convert to u8")
    if k not in (0, 1):
        raise ValueError("kernel must be 0 (Plummer) or 1 (CubicSplineW2)")
    return k


def _threads(threads) -> int:
    t = int(threads)
    if t < 0:
        raise OverflowError("can't convert negative int to unsigned")
    return t


def _common(positions, masses, softenings, kernel, threads):
    _threads(threads)
    pos = extract_vec3(positions, "positions")
    n = pos.shape[0]
    m = _extract_vec1(masses, n, "masses", "masses")
    h = _extract_vec1(softenings, n, "softenings", "softenings")
    return pos, n, m, h


def _kernel_checks(kernel, h):
    if kernel is None and h is not None:
        raise ValueError(
            "softenings require an explicit kernel; pass kernel=0/1 (or omit softenings)")
    return _kernel_code(kernel)


def direct_accelerations_py(positions, masses=None, threads=0, softenings=None, kernel=None):
    """Direct-sum accelerations at the particles (gravity.rs:448-512)."""
    pos, n, m, h = _common(positions, masses, softenings, kernel, threads)
    k = _kernel_checks(kernel, h)
    out = np.zeros((n, 3), dtype=np.float64)
    if n:
        nat.call("pbx_direct_accelerations", nat.dptr(pos), n, nat.dptr(m), nat.dptr(h), k,
                 nat.dptr(out))
    return out


def direct_potentials_py(positions, masses=None, threads=0, softenings=None, kernel=None):
    """Direct-sum potentials at the particles (gravity.rs:585-644)."""
    pos, n, m, h = _common(positions, masses, softenings, kernel, threads)
    k = _kernel_checks(kernel, h)
    out = np.zeros(n, dtype=np.float64)
    if n:
        nat.call("pbx_direct_potentials", nat.dptr(pos), n, nat.dptr(m), nat.dptr(h), k,
                 nat.dptr(out))
    return out


def direct_accelerations_at_points_py(positions, targets, masses=None, threads=0,
                                      softenings=None, kernel=None):
    """Direct-sum accelerations at arbitrary points (gravity.rs:514-583)."""
    pos, n, m, h = _common(positions, masses, softenings, kernel, threads)
    tgt = extract_vec3(targets, "targets")
    k = _kernel_checks(kernel, h)
    mt = tgt.shape[0]
    out = np.zeros((mt, 3), dtype=np.float64)
    if mt:
        nat.call("pbx_direct_accelerations_at_points", nat.dptr(pos), n, nat.dptr(tgt), mt,
                 nat.dptr(m), nat.dptr(h), k, nat.dptr(out))
    return out


def direct_potentials_at_points_py(positions, targets, masses=None, threads=0,
                                   softenings=None, kernel=None):
    """Direct-sum potentials at arbitrary points (gravity.rs:646-709)."""
    pos, n, m, h = _common(positions, masses, softenings, kernel, threads)
    tgt = extract_vec3(targets, "targets")
    k = _kernel_checks(kernel, h)
    mt = tgt.shape[0]
    out = np.zeros(mt, dtype=np.float64)
    if mt:
        nat.call("pbx_direct_potentials_at_points", nat.dptr(pos), n, nat.dptr(tgt), mt,
                 nat.dptr(m), nat.dptr(h), k, nat.dptr(out))
    return out


def _usize(v, argname: str) -> int:
    if isinstance(v, bool) or not isinstance(v, (int, np.integer)):
        raise TypeError(f"argument '{argname}': '{type(v).__name__}' object cannot be "
                        "interpreted as an integer")
    v = int(v)
    if v < 0:
        raise OverflowError("can't convert negative int to unsigned")
    return v


def _u8(v, argname: str) -> int:
    v = _usize(v, argname)
    if v > 255:
        raise OverflowError("can't convert to u8")
    return v


def _kernel_opt(kernel) -> int:
    """parse_kernel_opt (gravity.rs:77-82): None -> Plummer."""
    if kernel is None:
        return nat.KERNEL_PLUMMER
    return _kernel_code(kernel)


class Octree:
    """Barnes–Hut octree with the PyO3 class surface of the reference
    (crates/pynbodyext-rust/src/gravity.rs:114-445); the tree and every walk
    live on the GPU (include/pbx.h ``pbx_octree_*``).

    ``Octree(positions, masses=None, leaf_capacity=32, multipole_order=0,
    softenings=None, kernel=None)`` copies its inputs, builds the octree, and
    builds the mass payload only when masses are given (gravity.rs:210-220).
    """

    def __init__(self, positions, masses=None, leaf_capacity=32, multipole_order=0,
                 softenings=None, kernel=None):
        leaf_capacity = _usize(leaf_capacity, "leaf_capacity")
        multipole_order = _u8(multipole_order, "multipole_order")
        if kernel is not None:
            _u8(kernel, "kernel")
        self._h = None
        pos = extract_vec3(positions, "positions")
        n = pos.shape[0]
        m = _extract_vec1(masses, n, "masses", "masses")
        h = _extract_vec1(softenings, n, "softenings", "softenings")
        if kernel is None and h is not None:
            raise ValueError(
                "softenings require an explicit kernel; pass kernel=0/1 (or omit softenings)")
        k = _kernel_opt(kernel)
        handle = ctypes.c_void_p()
        nat.call("pbx_octree_create", nat.vptr(pos), n, nat.vptr(m), nat.vptr(h),
                 leaf_capacity, multipole_order, k, 0, ctypes.byref(handle))
        self._h = handle
        self._n = n

    @classmethod
    def _from_device(cls, d_pos, n, d_mass=None, leaf_capacity=8, multipole_order=3,
                     d_soft=None, kernel=0) -> "Octree":
        """Build from HBM-resident arrays (device pointers; bench / multi-GPU)."""
        self = cls.__new__(cls)
        self._h = None
        handle = ctypes.c_void_p()
        nat.call("pbx_octree_create", d_pos, int(n), d_mass, d_soft, int(leaf_capacity),
                 int(multipole_order), int(kernel), 1, ctypes.byref(handle))
        self._h = handle
        self._n = int(n)
        return self

    def _rebuild_device(self, d_pos, n, d_mass=None, d_soft=None) -> None:
        """Rebuild on new HBM-resident particles, reusing this tree's buffers."""
        nat.call("pbx_octree_rebuild", self._h, d_pos, int(n), d_mass, d_soft, 1)
        self._n = int(n)

    def __del__(self):  # pragma: no cover - GC timing
        self.close()

    def close(self) -> None:
        h = getattr(self, "_h", None)
        if h is not None and h.value and nat._lib is not None:
            try:
                nat.call("pbx_octree_destroy", h)
            except Exception:
                pass
        self._h = None

    # -- mutation (gravity.rs:228-265) ------------------------------------
    def build_mass(self, masses=None):
        m = _extract_vec1(masses, self._n, "masses", "masses")
        nat.call("pbx_octree_build_mass", self._h, nat.vptr(m), 0)

    def set_softenings(self, softenings=None):
        h = _extract_vec1(softenings, self._n, "softenings", "softenings")
        nat.call("pbx_octree_set_softenings", self._h, nat.vptr(h), 0)

    def set_kernel(self, kernel=None):
        if kernel is not None:
            _u8(kernel, "kernel")
        nat.call("pbx_octree_set_kernel", self._h, _kernel_opt(kernel))

    # -- queries (gravity.rs:267-445) --------------------------------------
    def compute_accelerations(self, theta, threads=0):
        _threads(threads)
        out = np.zeros((self._n, 3), dtype=np.float64)
        nat.call("pbx_octree_compute", self._h, float(theta), nat.WANT_ACC, None,
                 nat.vptr(out), 0)
        return out

    def compute_potentials(self, theta, threads=0):
        _threads(threads)
        out = np.zeros(self._n, dtype=np.float64)
        nat.call("pbx_octree_compute", self._h, float(theta), nat.WANT_POT, nat.vptr(out),
                 None, 0)
        return out

    def _at_points(self, points, theta, threads, want, method):
        _threads(threads)
        if not self.info()["has_mass_payload"]:
            raise ValueError(f"mass payload not built; call build_mass() before {method}")
        pts = extract_vec3(points, "points")
        m = pts.shape[0]
        pot = np.zeros(m, dtype=np.float64) if want == nat.WANT_POT else None
        acc = np.zeros((m, 3), dtype=np.float64) if want == nat.WANT_ACC else None
        nat.call("pbx_octree_at_points", self._h, nat.vptr(pts), m, float(theta), want,
                 nat.vptr(pot), nat.vptr(acc), 0)
        return pot if want == nat.WANT_POT else acc

    def accelerations_at_points(self, points, theta, threads=0):
        return self._at_points(points, theta, threads, nat.WANT_ACC, "accelerations_at_points")

    def potentials_at_points(self, points, theta, threads=0):
        return self._at_points(points, theta, threads, nat.WANT_POT, "potentials_at_points")

    # -- device-resident form (bench) --------------------------------------
    def _compute_device(self, theta, want, d_pot=None, d_acc=None):
        nat.call("pbx_octree_compute", self._h, float(theta), int(want), d_pot, d_acc, 1)

    def _compute_range_device(self, theta, want, first, count, compact, d_pot=None, d_acc=None,
                              d_cost=None):
        """Walk the leaf-order targets [first, first+count) (multi-GPU shard)."""
        nat.call("pbx_octree_compute_range", self._h, float(theta), int(want), int(first),
                 int(count), int(compact), d_pot, d_acc, d_cost)

    def _leaf_particles_device(self, first, count, d_pos=None, d_mass=None, d_idx=None):
        nat.call("pbx_octree_leaf_particles", self._h, int(first), int(count), d_pos, d_mass,
                 d_idx)

    def _radial_moments_device(self, first, count, d_f, edges):
        """(counts (nbins,) int64, moments (nbins, 7)) of the 3-D radial
        profile of a leaf-order field over the targets [first, first + count)
        (pbx_octree_radial_moments: the pbx_profile_moments columns with the
        mass as weight)."""
        edges = np.ascontiguousarray(edges, dtype=np.float64)
        nb = len(edges) - 1
        counts = np.zeros(nb, dtype=np.int64)
        mom = np.zeros((nb, 7))
        nat.call("pbx_octree_radial_moments", self._h, int(first), int(count), d_f,
                 nat.dptr(edges), nb, counts.ctypes.data_as(nat._i64p), nat.dptr(mom))
        return counts, mom

    def _radial_moments_into(self, first: int, count: int, d_f, edges, d_out) -> None:
        """_radial_moments_device into device memory (no sync): d_out holds
        nbins int64 counts, then nbins x 7 doubles."""
        edges = np.ascontiguousarray(edges, dtype=np.float64)
        nat.call("pbx_octree_radial_moments_device", self._h, int(first), int(count), d_f,
                 nat.dptr(edges), len(edges) - 1, d_out)

    def _cost_to_orig_device(self, d_cost_leaf, d_cost_orig) -> None:
        """Per-target costs in this build's leaf order -> original order."""
        nat.call("pbx_octree_cost_to_orig", self._h, d_cost_leaf, d_cost_orig)


    def _set_walk_counters(self, enabled: bool = True) -> None:
        """Walk statistics (info()'s interaction / step counts) on or off for
        later fast-mode order-3 walks (pbx_octree_set_walk_counters)."""
        nat.call("pbx_octree_set_walk_counters", self._h, int(bool(enabled)))

    def _set_cost_kind(self, kind: int) -> None:
        """compute_range's d_cost: 0 interactions per target, 1 the wave's work."""
        nat.call("pbx_octree_set_cost_kind", self._h, int(kind))

    def _balance_device(self, d_cost_orig, world: int) -> list[tuple[int, int]]:
        """[(first, count)] per rank: contiguous leaf-order ranges of equal
        summed cost (costs in original order, e.g. from the previous step)."""
        cuts = np.zeros(int(world) + 1, dtype=np.int64)
        nat.call("pbx_octree_balance", self._h, d_cost_orig, int(world),
                 cuts.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
        return [(int(cuts[r]), int(cuts[r + 1] - cuts[r])) for r in range(int(world))]

    # -- introspection -----------------------------------------------------
    def info(self) -> dict:
        out = np.zeros(13, dtype=np.int64)
        nat.call("pbx_octree_info", self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
        keys = ("n", "nodes", "levels", "has_mass_payload", "has_hmax", "node_interactions",
                "leaf_pairs", "path_words", "wave_steps", "active_lane_steps", "leaf_wave_steps",
                "leaf_active_lanes", "descend_wave_steps")
        return {k: int(v) for k, v in zip(keys, out)}

    def export(self) -> dict:
        """Node arrays (device breadth-first numbering) for parity tests."""
        inf = self.info()
        nn, n = inf["nodes"], inf["n"]
        i64 = ctypes.POINTER(ctypes.c_int64)
        d = dict(center=np.zeros((nn, 4)), com=np.zeros((nn, 4)) if inf["has_mass_payload"] else None,
                 hmax=np.zeros(nn) if inf["has_hmax"] else None,
                 links=np.zeros((nn, 3), dtype=np.int64), leaf=np.zeros((nn, 2), dtype=np.int64),
                 perm=np.zeros(n, dtype=np.int64))
        nat.call("pbx_octree_export", self._h, nat.dptr(d["center"]), nat.dptr(d["com"]),
                 nat.dptr(d["hmax"]), d["links"].ctypes.data_as(i64),
                 d["leaf"].ctypes.data_as(i64), d["perm"].ctypes.data_as(i64), None)
        return d

    def export_moments(self, ncoef: int) -> np.ndarray:
        nn = self.info()["nodes"]
        out = np.zeros((nn, ncoef))
        nat.call("pbx_octree_export", self._h, None, None, None, None, None, None, nat.dptr(out))
        return out


__all__ = [
    "Octree",
    "direct_accelerations_py",
    "direct_potentials_py",
    "direct_accelerations_at_points_py",
    "direct_potentials_at_points_py",
]
