"""ctypes binding of the tree restatement in oracle/tree_ref.c (ORACLE: test
infrastructure only; see tree_ref.c for the tree.rs / multipole.rs citations
and the parity status).

``RefOctree`` mirrors the PyO3 ``Octree`` class (crates/pynbodyext-rust/src/
gravity.rs:114-445) closely enough for the parity tests to call both the same
way, plus ``export()`` for geometry / payload comparisons.
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, c_double, c_int, c_int64, c_void_p

import numpy as np

from . import gravity as _g

_dp = POINTER(c_double)
_ip = POINTER(c_int64)
NMOM = 56
_ready = False


def lib():
    global _ready
    L = _g.lib()
    if not _ready:
        L.pbxref_tree_new.restype = c_void_p
        L.pbxref_tree_new.argtypes = [_dp, c_int64, _dp, _dp, c_int64, c_int, c_int]
        L.pbxref_tree_free.argtypes = [c_void_p]
        L.pbxref_tree_build_mass.argtypes = [c_void_p, _dp]
        L.pbxref_tree_build_mass_payload.argtypes = [c_void_p]
        L.pbxref_tree_set_softenings.argtypes = [c_void_p, _dp]
        L.pbxref_tree_set_kernel.argtypes = [c_void_p, c_int]
        L.pbxref_tree_has_bh.argtypes = [c_void_p]
        L.pbxref_tree_has_hmax.argtypes = [c_void_p]
        L.pbxref_tree_has_moments.argtypes = [c_void_p]
        L.pbxref_tree_num_nodes.argtypes = [c_void_p]
        L.pbxref_tree_num_nodes.restype = c_int64
        L.pbxref_tree_compute.argtypes = [c_void_p, c_double, c_int, _dp, _dp]
        L.pbxref_tree_compute_subset.argtypes = [c_void_p, c_double, c_int, _ip, c_int64, _dp,
                                                 _dp, _ip, _ip]
        L.pbxref_tree_at_points.argtypes = [c_void_p, _dp, c_int64, c_double, c_int, _dp, _dp]
        L.pbxref_tree_export.argtypes = [c_void_p, _dp, _dp, _dp, _ip, _ip, _ip, _ip, _dp, _dp,
                                         _dp, _dp, _ip]
        L.pbxref_multipole_from_points.argtypes = [_dp, _dp, _ip, c_int64, _dp, c_int, _dp]
        L.pbxref_translate_multipole.argtypes = [_dp, _dp, c_int, _dp]
        L.pbxref_potential_derivatives.argtypes = [c_double, c_double, c_double, c_double, c_int,
                                                   _dp]
        L.pbxref_gravity_potential_multipole.argtypes = [_dp, _dp, c_int]
        L.pbxref_gravity_potential_multipole.restype = c_double
        L.pbxref_gravity_accel_multipole.argtypes = [_dp, _dp, c_int, _dp]
        _ready = True
    return L


def _p(a):
    return None if a is None else a.ctypes.data_as(_dp)


def _i(a):
    return None if a is None else a.ctypes.data_as(_ip)


def _c(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float64)


# --- multipole primitives (multipole.rs) ----------------------------------
def multipole_from_points(pos, mass, center, order, idx=None):
    pos = _c(pos).reshape(-1, 3)
    mass = _c(mass)
    idx = np.arange(pos.shape[0], dtype=np.int64) if idx is None else \
        np.ascontiguousarray(idx, dtype=np.int64)
    out = np.zeros(NMOM)
    lib().pbxref_multipole_from_points(_p(pos), _p(mass), _i(idx), idx.shape[0],
                                       _p(_c(center)), int(order), _p(out))
    return out


def translate_multipole(m, shift, order):
    out = np.zeros(NMOM)
    lib().pbxref_translate_multipole(_p(_c(m)), _p(_c(shift)), int(order), _p(out))
    return out


def potential_derivatives(dx, dy, dz, eps2, order):
    out = np.zeros(NMOM)
    lib().pbxref_potential_derivatives(float(dx), float(dy), float(dz), float(eps2), int(order),
                                       _p(out))
    return out


def gravity_potential_multipole(m, d, order):
    return lib().pbxref_gravity_potential_multipole(_p(_c(m)), _p(_c(d)), int(order))


def gravity_accel_multipole(m, d, order):
    out = np.zeros(3)
    lib().pbxref_gravity_accel_multipole(_p(_c(m)), _p(_c(d)), int(order), _p(out))
    return out


# --- octree ---------------------------------------------------------------
class RefOctree:
    """Octree::from_owned (+ build_mass_payload when masses are given, like
    the PyO3 constructor gravity.rs:198-220).  ``tree3d=True`` restates
    Tree3D::build (tree.rs:1394-1413): Plummer, no softening, payload always.
    kernel None means Plummer (gravity.rs:77-82)."""

    def __init__(self, positions, masses=None, leaf_capacity=32, multipole_order=0,
                 softenings=None, kernel=None, tree3d=False):
        self.pos = _c(positions).reshape(-1, 3)
        self.n = self.pos.shape[0]
        m, h = _c(masses), _c(softenings)
        self._h = lib().pbxref_tree_new(_p(self.pos), self.n, _p(m), _p(h), int(leaf_capacity),
                                        int(multipole_order), 0 if kernel is None else int(kernel))
        if tree3d or masses is not None:
            lib().pbxref_tree_build_mass_payload(self._h)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().pbxref_tree_free(self._h)
            self._h = None

    @property
    def num_nodes(self) -> int:
        return lib().pbxref_tree_num_nodes(self._h)

    def build_mass(self, masses=None):
        lib().pbxref_tree_build_mass(self._h, _p(_c(masses)))

    def set_softenings(self, softenings=None):
        lib().pbxref_tree_set_softenings(self._h, _p(_c(softenings)))

    def set_kernel(self, kernel=None):
        lib().pbxref_tree_set_kernel(self._h, 0 if kernel is None else int(kernel))

    def _need_bh(self, what):
        if not lib().pbxref_tree_has_bh(self._h):
            raise ValueError(f"mass payload not built; call build_mass() before {what}")

    def compute_potentials(self, theta, threads=0):
        self._need_bh("compute_potentials")
        out = np.zeros(self.n)
        lib().pbxref_tree_compute(self._h, float(theta), 1, _p(out), None)
        return out

    def compute_accelerations(self, theta, threads=0):
        self._need_bh("compute_accelerations")
        out = np.zeros((self.n, 3))
        lib().pbxref_tree_compute(self._h, float(theta), 2, None, _p(out))
        return out

    def compute_subset(self, idx, theta, want=3):
        """(pot, acc, accepted-node count, leaf-particle count) for targets idx."""
        self._need_bh("compute_subset")
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        k = idx.shape[0]
        pot, acc = np.zeros(k), np.zeros((k, 3))
        nn, npp = np.zeros(k, dtype=np.int64), np.zeros(k, dtype=np.int64)
        lib().pbxref_tree_compute_subset(self._h, float(theta), int(want), _i(idx), k, _p(pot),
                                         _p(acc), _i(nn), _i(npp))
        return pot, acc, nn, npp

    def potentials_at_points(self, points, theta, threads=0):
        self._need_bh("potentials_at_points")
        pts = _c(points).reshape(-1, 3)
        out = np.zeros(pts.shape[0])
        lib().pbxref_tree_at_points(self._h, _p(pts), pts.shape[0], float(theta), 1, _p(out), None)
        return out

    def accelerations_at_points(self, points, theta, threads=0):
        self._need_bh("accelerations_at_points")
        pts = _c(points).reshape(-1, 3)
        out = np.zeros((pts.shape[0], 3))
        lib().pbxref_tree_at_points(self._h, _p(pts), pts.shape[0], float(theta), 2, None, _p(out))
        return out

    def export(self) -> dict:
        nn = self.num_nodes
        L = lib()
        d = dict(center=np.zeros((nn, 3)), half=np.zeros(nn), size2=np.zeros(nn),
                 first=np.zeros(nn, dtype=np.int64), next=np.zeros(nn, dtype=np.int64),
                 leaf_off=np.zeros(nn, dtype=np.int64), leaf_len=np.zeros(nn, dtype=np.int64),
                 com=np.zeros((nn, 3)), mass=np.zeros(nn), hmax=np.zeros(nn),
                 mom=np.zeros((nn, NMOM)), perm=np.zeros(self.n, dtype=np.int64))
        L.pbxref_tree_export(self._h, _p(d["center"]), _p(d["half"]), _p(d["size2"]),
                             _i(d["first"]), _i(d["next"]), _i(d["leaf_off"]), _i(d["leaf_len"]),
                             _p(d["com"]), _p(d["mass"]), _p(d["hmax"]), _p(d["mom"]),
                             _i(d["perm"]))
        if not L.pbxref_tree_has_hmax(self._h):
            d["hmax"] = None
        if not L.pbxref_tree_has_moments(self._h):
            d["mom"] = None
        return d
