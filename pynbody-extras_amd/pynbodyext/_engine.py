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


__all__ = [
    "direct_accelerations_py",
    "direct_potentials_py",
    "direct_accelerations_at_points_py",
    "direct_potentials_at_points_py",
]
