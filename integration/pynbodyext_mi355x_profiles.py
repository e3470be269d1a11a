"""MI355X backend for an UNMODIFIED pynbodyext.profiles — the profile half of
the drop-in boundary.

A maintainer copies this one file into the reference tree (e.g. as
``pynbodyext/profiles/_mi355x.py``) and calls ``install()`` once; nothing
else in the reference changes.  It needs only numpy, ctypes and
``libpbx.so`` (path: ``install(lib_path)`` or ``$PBX_LIBRARY``), and patches
the three numpy seams of the reference's profile path:

* ``BinsSet._assign_particles``  (profiles/bins.py:346-395): bin assignment
  (``digitize(right=True) - 1`` + the two extrema fix-ups), counts and the
  stable per-bin index lists on the GPU (pbx_profile_set_x / _assign / _csr);
* the ``"equaln"`` entry of ``BinsSet._bins_algorithm_registry``
  (bins.py:720-746): the equal-number edges as order statistics by the
  device radix select (pbx_profile_edges_equaln), same degenerate and
  empty-input behaviour;
* ``ProfileArray._compute`` (profiles/proarray.py:272-334): the per-bin loop
  of Mean / Sum / Sum_w / RMS / Dispersion / Abs_* from one device reduction
  of the bin members (pbx_profile_moments_cols), Percentile / Median /
  Abs_pXX by the device per-bin order statistics (pbx_profile_percentiles);
  any other statistic, or a profile whose bins were not made here, runs the
  original method.

Numerics: edges, counts and index lists are bit-identical to numpy's; the
per-bin sums differ from numpy's pairwise summation by rounding only
(tests/test_gpu_integration.py checks 1e-12).  There is no CPU fallback
inside the patched methods: without a gfx950 GPU every call raises
RuntimeError, like the rest of libpbx.

Uninstall with ``uninstall()`` (restores the three originals).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, byref, c_double, c_int, c_int64, c_uint32, c_void_p

import numpy as np

__all__ = ["install", "uninstall", "DeviceBinsHandle"]

# pbx_profile_moments source selectors (include/pbx.h)
_SRC_NONE, _SRC_X, _SRC_W, _SRC_HOST = -1, 0, 1, 2
# moment columns: Σw, Σf·w, Σf²·w, Σf, Σf², Σ|f|·w, Σ|f|
_W, _FW, _F2W, _F, _F2, _AFW, _AF = range(7)

_dp = POINTER(c_double)
_i64p = POINTER(c_int64)
_SIGS = {
    "pbx_last_error": (ctypes.c_char_p, []),
    "pbx_profile_create": (c_int, [POINTER(c_void_p)]),
    "pbx_profile_destroy": (c_int, [c_void_p]),
    "pbx_profile_set_x": (c_int, [c_void_p, _dp, c_int64]),
    "pbx_profile_edges_equaln": (c_int, [c_void_p, c_int64, c_int, c_double, c_int, c_double, _dp,
                                         _i64p]),
    "pbx_profile_assign": (c_int, [c_void_p, _dp, c_int64, _i64p, _i64p]),
    "pbx_profile_csr": (c_int, [c_void_p, _i64p, _i64p]),
    "pbx_profile_binned_equaln": (c_int, [c_void_p, c_int64, c_int, c_double, c_int, c_double,
                                          c_int, c_int, c_void_p, c_void_p, c_void_p, _dp, _i64p,
                                          _i64p, _i64p, _dp]),
    "pbx_profile_moments_cols": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_uint32,
                                         _dp]),
    "pbx_profile_percentiles": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int,
                                        c_void_p, c_void_p]),
}
_lib = None


def _load(path: str | None = None):
    global _lib
    if _lib is None:
        path = path or os.environ.get("PBX_LIBRARY")
        if not path:
            raise ImportError("libpbx.so: pass install(lib_path) or set PBX_LIBRARY")
        lib = ctypes.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _lib = lib
    return _lib


def _call(name, *args):
    st = getattr(_lib, name)(*args)
    if st == 0:
        return
    msg = (_lib.pbx_last_error() or b"").decode("utf-8", "replace")
    if st == 1:  # PBX_ERR_VALUE: the reference's ValueError / IndexError messages
        if msg.startswith("index 0 is out of bounds"):
            raise IndexError(msg)
        raise ValueError(msg)
    raise RuntimeError(msg or f"libpbx error {st}")


class DeviceBinsHandle:
    """One binned quantity x in HBM (a pbx_profile handle) and what the
    device derived from it: edges, assignment, CSR.

    x is uploaded by ``upload`` once per BinsSet materialisation (the
    equaln seam, or the assignment seam when no equaln call preceded it):
    a BinsSet re-materialised in place over the same, mutated array object
    sees the array's current values, as the reference's numpy code does."""

    # the fused one-round-trip pass (pbx_profile_binned_equaln) takes nbins <= 1024
    FUSED_MAX_BINS = 1024

    def __init__(self, x):
        h = c_void_p()
        _call("pbx_profile_create", byref(h))
        self._h = h
        self.x_ref = None
        self.n = 0
        self.nbins = None
        self.n_valid = 0
        self.pending = None  # (edges, counts) of a fused equaln pass not yet consumed
        self.upload(x)

    def upload(self, x):
        a = np.ascontiguousarray(np.asarray(x), dtype=np.float64).reshape(-1)
        _call("pbx_profile_set_x", self._h, a.ctypes.data_as(_dp), a.shape[0])
        self.x_ref = x
        self.n = a.shape[0]
        self.nbins = None
        self.n_valid = 0
        self.pending = None

    def equaln_fused(self, nbins, bin_min, bin_max) -> np.ndarray:
        """equaln edges, their assignment, counts and the device CSR in one
        host round trip (pbx_profile_binned_equaln); the counts wait in
        ``pending`` for the assignment seam that follows (bins.py:386-387)."""
        nb = int(nbins)
        edges = np.empty(nb + 1)
        counts = np.zeros(nb, dtype=np.int64)
        ne, nv = c_int64(0), c_int64(0)
        _call("pbx_profile_binned_equaln", self._h, nb, int(bin_min is not None),
              float(bin_min) if bin_min is not None else 0.0, int(bin_max is not None),
              float(bin_max) if bin_max is not None else 0.0, 1, 0, None, None, None,
              edges.ctypes.data_as(_dp), byref(ne), counts.ctypes.data_as(_i64p), byref(nv), None)
        edges = edges[: ne.value].copy()
        counts = counts[: ne.value - 1].copy()
        self.nbins, self.n_valid = counts.shape[0], nv.value
        self.pending = (edges, counts)
        return edges

    def take_pending(self, edges):
        """The counts of the fused pass whose edges are exactly ``edges``
        (then the device assignment and CSR are already those of edges), or
        None.  Consumed either way."""
        p, self.pending = self.pending, None
        if p is None:
            return None
        e = np.asarray(edges, dtype=np.float64).reshape(-1)
        if e.shape != p[0].shape or not np.array_equal(e.view(np.uint64), p[0].view(np.uint64)):
            return None
        return p[1]

    def edges_equaln(self, nbins, bin_min, bin_max) -> np.ndarray:
        out = np.empty(int(nbins) + 1)
        ne = c_int64(0)
        _call("pbx_profile_edges_equaln", self._h, int(nbins), int(bin_min is not None),
              float(bin_min) if bin_min is not None else 0.0, int(bin_max is not None),
              float(bin_max) if bin_max is not None else 0.0, out.ctypes.data_as(_dp), byref(ne))
        return out[: ne.value].copy()

    def assign(self, edges) -> np.ndarray:
        e = np.ascontiguousarray(np.asarray(edges), dtype=np.float64).reshape(-1)
        counts = np.zeros(max(e.shape[0] - 1, 0), dtype=np.int64)
        nv = c_int64(0)
        _call("pbx_profile_assign", self._h, e.ctypes.data_as(_dp), e.shape[0],
              counts.ctypes.data_as(_i64p), byref(nv))
        self.nbins, self.n_valid = counts.shape[0], nv.value
        return counts

    def csr(self):
        perm = np.empty(self.n_valid, dtype=np.int64)
        offs = np.empty(self.nbins + 1, dtype=np.int64)
        _call("pbx_profile_csr", self._h, perm.ctypes.data_as(_i64p), offs.ctypes.data_as(_i64p))
        return perm, offs

    def moments(self, f, w, cols: int) -> np.ndarray:
        """(nbins, 7) sums over each bin's members of host arrays f / w
        (per element of x; w None = unweighted)."""
        fa = np.ascontiguousarray(f, dtype=np.float64)
        wa = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
        out = np.zeros((self.nbins, 7))
        _call("pbx_profile_moments_cols", self._h, _SRC_HOST, fa.ctypes.data_as(c_void_p),
              _SRC_NONE if wa is None else _SRC_HOST,
              None if wa is None else wa.ctypes.data_as(c_void_p), int(cols) & 0x7F,
              out.ctypes.data_as(_dp))
        return out

    def percentile(self, p: float, f, w, absval: bool) -> np.ndarray:
        fa = np.ascontiguousarray(f, dtype=np.float64)
        wa = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
        q = np.array([p / 100.0])
        out = np.zeros((self.nbins, 1))
        _call("pbx_profile_percentiles", self._h, _SRC_HOST, fa.ctypes.data_as(c_void_p),
              _SRC_NONE if wa is None else _SRC_HOST,
              None if wa is None else wa.ctypes.data_as(c_void_p), int(bool(absval)), 1,
              q.ctypes.data_as(c_void_p), out.ctypes.data_as(c_void_p))
        return out[:, 0]

    def close(self):
        if self._h is not None and self._h.value and _lib is not None:
            try:
                _call("pbx_profile_destroy", self._h)
            except Exception:
                pass
        self._h = None

    __del__ = close


def _handle_for(binsset, x) -> DeviceBinsHandle:
    """The BinsSet's device handle, with x uploaded for this materialisation."""
    h = binsset.__dict__.get("_pbx_handle")
    if h is None:
        h = DeviceBinsHandle(x)
        binsset.__dict__["_pbx_handle"] = h
    else:
        h.upload(x)
    return h


# ----------------------------------------------------------------- the seams
def _assign_particles(self, x, bin_edges):
    """bins.py:346-395 on the device: (binind list, npart_bins)."""
    arr_edges = np.asarray(bin_edges, dtype=np.float64)
    nbins = len(arr_edges) - 1
    if nbins <= 0:
        return [], np.array([], dtype=int)
    h = self.__dict__.get("_pbx_handle")
    counts = None
    if h is not None and h.x_ref is x:
        # the equaln seam of this same materialisation already assigned and
        # built the CSR with exactly these edges (one host round trip)
        counts = h.take_pending(arr_edges)
    if counts is None:
        h = _handle_for(self, x)
        counts = h.assign(arr_edges)
    if not counts.any():
        return [np.empty(0, dtype=int) for _ in range(nbins)], np.zeros(nbins, dtype=int)
    perm, offs = h.csr()
    perm = perm.astype(np.intp, copy=False)
    return [perm[offs[i]:offs[i + 1]] for i in range(nbins)], counts.astype(int)


def _equal_number_bins_algorithm(self, x):
    """bins.py:720-746 on the device (the same edges, bit for bit), fused
    with the assignment and CSR the next seam of the same materialisation
    asks for (bins.py:386-387)."""
    h = _handle_for(self, x)
    nb = int(self.nbins)
    if 1 <= nb <= DeviceBinsHandle.FUSED_MAX_BINS:
        return h.equaln_fused(nb, self._bin_min, self._bin_max)
    return h.edges_equaln(nb, self._bin_min, self._bin_max)


def _stat_plan(calc):
    """(kind, absval, percent) of a reference statistic the device computes,
    or None.  kind: mean / sum / sum_w / rms / disp / pct."""
    absval = False
    if type(calc).__name__ == "Abs":
        calc, absval = calc._substat, True
    name = type(calc).__name__
    if name == "Percentile":
        return "pct", absval, float(calc.percentile)
    if name == "Median":
        return "pct", absval, 50.0
    kind = {"Mean": "mean", "Sum": "sum", "Sum_w": "sum_w", "RMS": "rms",
            "Dispersion": "disp"}.get(name)
    return None if kind is None else (kind, absval, None)


def _from_moments(kind, absval, m, counts, weighted):
    """The reference statistics (proarray.py:632-860) from per-bin sums."""
    f, fw = (_AF, _AFW) if absval else (_F, _FW)
    with np.errstate(divide="ignore", invalid="ignore"):
        if kind == "mean":
            v = m[:, fw] / m[:, _W] if weighted else m[:, f] / counts
        elif kind == "sum":
            v = m[:, f].copy()
        elif kind == "sum_w":
            v = (m[:, fw] if weighted else m[:, f]).copy()
        elif kind == "rms":
            v = np.sqrt(m[:, _F2W] / m[:, _W]) if weighted else np.sqrt(m[:, _F2] / counts)
        else:  # disp: sqrt(E[f^2] - E[f]^2), the reference's clamp of tiny negatives
            if weighted:
                ws = m[:, _W]
                d = m[:, _F2W] / ws - (m[:, fw] / ws) ** 2
            else:
                d = m[:, _F2] / counts - (m[:, f] / counts) ** 2
            d = np.where((d < 0) & (d > -1e-12), 0.0, d)
            v = np.where(d >= 0, np.sqrt(np.where(d >= 0, d, 0.0)), np.nan)
            if weighted:
                v = np.where(ws == 0, np.nan, v)
    v = np.asarray(v, dtype=np.float64)
    v[np.asarray(counts) == 0] = np.nan
    return v


_COLS = {"mean": (1 << _W) | (1 << _FW) | (1 << _F), "sum": 1 << _F,
         "sum_w": (1 << _FW) | (1 << _F), "rms": (1 << _W) | (1 << _F2W) | (1 << _F2),
         "disp": (1 << _W) | (1 << _FW) | (1 << _F2W) | (1 << _F) | (1 << _F2)}
_ABS_COLS = {1 << _F: 1 << _AF, 1 << _FW: 1 << _AFW}


def _make_compute(orig, simarray_types):
    SimArray, IndexedSimArray = simarray_types

    def _compute(cls, profile, arr, compute_mode):
        """proarray.py:272-334 with the per-bin loop on the device."""
        calculator = cls.get_statistic(compute_mode)
        if calculator is None:
            raise ValueError(f"Statistic '{compute_mode}' not found")
        plan = _stat_plan(calculator)
        h = profile.bins.__dict__.get("_pbx_handle")
        if plan is None or h is None or h.nbins != profile.nbins:
            return orig.__func__(cls, profile, arr, compute_mode)
        arr_pp = profile.sim[arr] if isinstance(arr, str) else arr
        weights = profile._weight
        if hasattr(arr_pp, "compute") and not isinstance(arr_pp, np.ndarray):  # dask
            arr_pp = arr_pp.compute()
        if weights is not None and hasattr(weights, "compute") and not isinstance(weights, np.ndarray):
            weights = weights.compute()
        f = np.asarray(arr_pp, dtype=np.float64)
        w = None if weights is None else np.asarray(weights, dtype=np.float64)
        kind, absval, pct = plan
        if kind == "pct":
            vals = h.percentile(pct, f, w, absval)
        else:
            cols = _COLS[kind]
            if absval:
                for a, b in _ABS_COLS.items():
                    if cols & a:
                        cols |= b
            m = h.moments(f, w, cols)
            vals = _from_moments(kind, absval, m, np.asarray(profile.npart_bins), w is not None)
        res_val = np.asarray(vals, dtype=np.float64).view(SimArray)
        if isinstance(arr_pp, (SimArray, IndexedSimArray)):
            res_val.units = arr_pp.units
            res_val.sim = arr_pp.sim
        return res_val, calculator.key

    return _compute


_saved = {}


def install(lib_path: str | None = None, bins_module=None, proarray_module=None) -> None:
    """Patch pynbodyext.profiles (or the given bins / proarray modules) to
    run its binning and per-bin statistics on the MI355X."""
    _load(lib_path)
    if bins_module is None:
        from pynbodyext.profiles import bins as bins_module
    if proarray_module is None:
        from pynbodyext.profiles import proarray as proarray_module
    BinsSet = bins_module.BinsSet
    ProfileArray = proarray_module.ProfileArray
    if _saved:
        return
    _saved["assign"] = (BinsSet, BinsSet.__dict__["_assign_particles"])
    _saved["equaln"] = (BinsSet, BinsSet._bins_algorithm_registry.get("equaln"))
    _saved["compute"] = (ProfileArray, ProfileArray.__dict__["_compute"])
    BinsSet._assign_particles = _assign_particles
    BinsSet._bins_algorithm_registry["equaln"] = _equal_number_bins_algorithm
    sim_types = (proarray_module.SimArray, getattr(proarray_module, "IndexedSimArray",
                                                   proarray_module.SimArray))
    ProfileArray._compute = classmethod(_make_compute(_saved["compute"][1], sim_types))


def uninstall() -> None:
    if not _saved:
        return
    BinsSet, assign = _saved.pop("assign")
    BinsSet._assign_particles = assign
    BinsSet, eq = _saved.pop("equaln")
    if eq is not None:
        BinsSet._bins_algorithm_registry["equaln"] = eq
    ProfileArray, comp = _saved.pop("compute")
    ProfileArray._compute = comp
