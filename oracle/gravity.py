"""ctypes binding of oracle/build/liboracle.so (ORACLE: test infrastructure).

Function-for-function restatement of crates/gravity/src/direct.rs and
kernel.rs; see gravity_ref.c for the citations and the parity status.
"""
from __future__ import annotations

import ctypes
import subprocess
from ctypes import POINTER, c_double, c_int, c_int64
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_SO = _HERE / "build" / "liboracle.so"
_lib = None
_dp = POINTER(c_double)


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not _SO.exists():
            build()
        L = ctypes.CDLL(str(_SO))
        for name in ("pbxref_direct_accelerations", "pbxref_direct_potentials"):
            getattr(L, name).argtypes = [_dp, c_int64, _dp, _dp]
        for name in ("pbxref_direct_accelerations_at_points", "pbxref_direct_potentials_at_points"):
            getattr(L, name).argtypes = [_dp, c_int64, _dp, _dp, c_int64, _dp]
        for name in ("pbxref_direct_potentials_kernel", "pbxref_direct_accelerations_kernel"):
            getattr(L, name).argtypes = [_dp, c_int64, _dp, _dp, c_int, _dp]
        for name in ("pbxref_direct_potentials_kernel_at_points",
                     "pbxref_direct_accelerations_kernel_at_points"):
            getattr(L, name).argtypes = [_dp, c_int64, _dp, _dp, _dp, c_int64, c_int, _dp]
        L.pbxref_kernel_potential.argtypes = [c_int, c_double, c_double]
        L.pbxref_kernel_potential.restype = c_double
        L.pbxref_kernel_accel_factor.argtypes = [c_int, c_double, c_double]
        L.pbxref_kernel_accel_factor.restype = c_double
        L.pbxref_multipole_soft_ok.argtypes = [c_int, c_double, c_double]
        L.pbxref_direct_subset.argtypes = [_dp, c_int64, _dp, POINTER(c_int64), c_int64, _dp, _dp]
        L.pbxref_num_threads.restype = c_int
        L.pbxref_set_num_threads.argtypes = [c_int]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(_dp)


def _c(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float64)


def direct_potentials(pos, mass=None, softenings=None, kernel=None):
    """Restates _rust.direct_potentials_py dispatch (gravity.rs:625-641)."""
    pos, mass, h = _c(pos), _c(mass), _c(softenings)
    n = pos.shape[0]
    out = np.zeros(n)
    if kernel is None:
        lib().pbxref_direct_potentials(_p(pos), n, _p(mass), _p(out))
    else:
        lib().pbxref_direct_potentials_kernel(_p(pos), n, _p(mass), _p(h), int(kernel), _p(out))
    return out


def direct_accelerations(pos, mass=None, softenings=None, kernel=None):
    pos, mass, h = _c(pos), _c(mass), _c(softenings)
    n = pos.shape[0]
    out = np.zeros((n, 3))
    if kernel is None:
        lib().pbxref_direct_accelerations(_p(pos), n, _p(mass), _p(out))
    else:
        lib().pbxref_direct_accelerations_kernel(_p(pos), n, _p(mass), _p(h), int(kernel), _p(out))
    return out


def direct_potentials_at_points(pos, targets, mass=None, softenings=None, kernel=None):
    pos, tgt, mass, h = _c(pos), _c(targets), _c(mass), _c(softenings)
    n, m = pos.shape[0], tgt.shape[0]
    out = np.zeros(m)
    if kernel is None:
        lib().pbxref_direct_potentials_at_points(_p(pos), n, _p(mass), _p(tgt), m, _p(out))
    else:
        lib().pbxref_direct_potentials_kernel_at_points(_p(pos), n, _p(mass), _p(h), _p(tgt), m,
                                                        int(kernel), _p(out))
    return out


def direct_accelerations_at_points(pos, targets, mass=None, softenings=None, kernel=None):
    pos, tgt, mass, h = _c(pos), _c(targets), _c(mass), _c(softenings)
    n, m = pos.shape[0], tgt.shape[0]
    out = np.zeros((m, 3))
    if kernel is None:
        lib().pbxref_direct_accelerations_at_points(_p(pos), n, _p(mass), _p(tgt), m, _p(out))
    else:
        lib().pbxref_direct_accelerations_kernel_at_points(_p(pos), n, _p(mass), _p(h), _p(tgt), m,
                                                           int(kernel), _p(out))
    return out


def direct_subset(pos, mass, idx):
    """(pot, acc) of the all-particles Newtonian form for target indices idx."""
    pos, mass = _c(pos), _c(mass)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    k = idx.shape[0]
    pot = np.zeros(k)
    acc = np.zeros((k, 3))
    lib().pbxref_direct_subset(_p(pos), pos.shape[0], _p(mass),
                               idx.ctypes.data_as(POINTER(c_int64)), k, _p(pot), _p(acc))
    return pot, acc


def kernel_potential(kind, r, h):
    return lib().pbxref_kernel_potential(int(kind), float(r), float(h))


def kernel_accel_factor(kind, r, h):
    return lib().pbxref_kernel_accel_factor(int(kind), float(r), float(h))


def multipole_soft_ok(kind, r, h):
    return bool(lib().pbxref_multipole_soft_ok(int(kind), float(r), float(h)))


def num_threads() -> int:
    return lib().pbxref_num_threads()


def set_num_threads(n: int) -> None:
    lib().pbxref_set_num_threads(int(n))
