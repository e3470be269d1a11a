"""ctypes binding of libpbx.so, the gfx950 HIP engine (C ABI: include/pbx.h).

This is the only place Python touches native code.  There is deliberately no
CPU fallback: if the shared library is missing, or a call finds no MI355X
(gfx950) device, the call raises.  Status codes map to exceptions the way
the reference's PyO3 layer maps Rust errors (crates/pynbodyext-rust/src/
gravity.rs: ValueError for argument errors).

ctypes releases the GIL around every foreign call, like the reference's
``py.allow_threads`` (gravity.rs:103-111).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_size_t, c_uint32,
                    c_uint64, c_void_p)
from pathlib import Path

import numpy as np

PBX_OK = 0
PBX_ERR_VALUE = 1
PBX_ERR_RUNTIME = 2
PBX_ERR_NODEV = 3

KERNEL_NONE = -1
KERNEL_PLUMMER = 0
KERNEL_SPLINE = 1

WANT_POT = 1
WANT_ACC = 2

_LIB_NAME = "libpbx.so"
_lib: ctypes.CDLL | None = None

_dp = POINTER(c_double)
_i64p = POINTER(c_int64)

# pbx_host_collective_fn (include/pbx.h, pbx_comm_init_host)
HOST_COLLECTIVE_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_int, c_void_p, c_int64, c_int, c_int,
                                      _i64p, _i64p)
COLL_ALLREDUCE = 0
COLL_ALLGATHERV = 1


class NativeLibraryMissing(ImportError):
    """libpbx.so has not been built (run ``__graft_entry__.build()``)."""


def lib_path() -> Path:
    """The library this process loads: $PBX_AB_LIBRARY (a same-box A/B build,
    bound leniently), else $PBX_LIBRARY (strict, like the built product),
    else the in-tree product build."""
    override = os.environ.get("PBX_AB_LIBRARY") or os.environ.get("PBX_LIBRARY")
    if override:
        return Path(override)
    return Path(__file__).resolve().parent / "lib" / _LIB_NAME


# name -> (restype, argtypes); every symbol include/pbx.h declares
_SIGNATURES: dict[str, tuple] = {
    "pbx_last_error": (c_char_p, []),
    "pbx_version": (c_int, []),
    "pbx_device_count": (c_int, [POINTER(c_int)]),
    "pbx_set_device": (c_int, [c_int]),
    "pbx_get_device": (c_int, [POINTER(c_int)]),
    "pbx_set_precise": (c_int, [c_int]),
    "pbx_get_precise": (c_int, [POINTER(c_int)]),
    "pbx_device_synchronize": (c_int, []),
    "pbx_device_name": (c_int, [c_char_p, c_int]),
    "pbx_malloc": (c_int, [POINTER(c_void_p), c_size_t]),
    "pbx_free": (c_int, [c_void_p]),
    "pbx_memcpy_htod": (c_int, [c_void_p, c_void_p, c_size_t]),
    "pbx_measure_h2d": (c_int, [c_int64, POINTER(c_double), POINTER(c_double)]),
    "pbx_device_pool_stats": (c_int, [POINTER(c_int64)]),
    "pbx_device_pool_trim": (c_int, []),
    "pbx_memcpy_dtoh": (c_int, [c_void_p, c_void_p, c_size_t]),
    "pbx_memcpy_dtod": (c_int, [c_void_p, c_void_p, c_size_t]),
    "pbx_memset": (c_int, [c_void_p, c_int, c_size_t]),
    "pbx_stream": (c_int, [POINTER(c_void_p)]),
    "pbx_event_create": (c_int, [POINTER(c_void_p)]),
    "pbx_event_destroy": (c_int, [c_void_p]),
    "pbx_event_record": (c_int, [c_void_p]),
    "pbx_event_elapsed_ms": (c_int, [c_void_p, c_void_p, POINTER(c_float)]),
    "pbx_stream_synchronize": (c_int, []),
    "pbx_direct_accelerations": (c_int, [_dp, c_int64, _dp, _dp, c_int, _dp]),
    "pbx_direct_potentials": (c_int, [_dp, c_int64, _dp, _dp, c_int, _dp]),
    "pbx_direct_accelerations_at_points": (c_int, [_dp, c_int64, _dp, c_int64, _dp, _dp, c_int, _dp]),
    "pbx_direct_potentials_at_points": (c_int, [_dp, c_int64, _dp, c_int64, _dp, _dp, c_int, _dp]),
    "pbx_pack_sources": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "pbx_direct_dev": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64,
                               c_int64, c_int, c_int, c_void_p, c_void_p]),
    "pbx_direct_sym_plan": (c_int, [c_int64, _i64p, _i64p, _i64p]),
    "pbx_direct_sym_accumulate": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int, c_void_p]),
    "pbx_direct_sym_finish": (c_int, [c_void_p, c_int64, c_int64, c_int, c_void_p, c_void_p]),
    "pbx_octree_create": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int, c_int,
                                  c_int, POINTER(c_void_p)]),
    "pbx_octree_destroy": (c_int, [c_void_p]),
    "pbx_octree_rebuild": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int]),
    "pbx_octree_build_mass": (c_int, [c_void_p, c_void_p, c_int]),
    "pbx_octree_set_softenings": (c_int, [c_void_p, c_void_p, c_int]),
    "pbx_octree_set_kernel": (c_int, [c_void_p, c_int]),
    "pbx_octree_compute": (c_int, [c_void_p, c_double, c_int, c_void_p, c_void_p, c_int]),
    "pbx_octree_at_points": (c_int, [c_void_p, c_void_p, c_int64, c_double, c_int, c_void_p,
                                     c_void_p, c_int]),
    "pbx_octree_compute_range": (c_int, [c_void_p, c_double, c_int, c_int64, c_int64, c_int,
                                         c_void_p, c_void_p, c_void_p]),
    "pbx_octree_leaf_particles": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p,
                                          c_void_p]),
    "pbx_octree_radial_moments": (c_int, [c_void_p, c_int64, c_int64, c_void_p, _dp, c_int64,
                                          _i64p, _dp]),
    "pbx_octree_radial_moments_device": (c_int, [c_void_p, c_int64, c_int64, c_void_p, _dp,
                                                 c_int64, c_void_p]),
    "pbx_octree_cost_to_orig": (c_int, [c_void_p, c_void_p, c_void_p]),
    "pbx_octree_balance": (c_int, [c_void_p, c_void_p, c_int, _i64p]),
    "pbx_octree_set_cost_kind": (c_int, [c_void_p, c_int]),
    "pbx_octree_set_walk_counters": (c_int, [c_void_p, c_int]),
    "pbx_octree_info": (c_int, [c_void_p, _i64p]),
    "pbx_octree_export": (c_int, [c_void_p, _dp, _dp, _dp, _i64p, _i64p, _i64p, _dp]),
    "pbx_profile_create": (c_int, [POINTER(c_void_p)]),
    "pbx_profile_destroy": (c_int, [c_void_p]),
    "pbx_profile_set_x": (c_int, [c_void_p, _dp, c_int64]),
    "pbx_profile_select": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, _dp, _i64p,
                                   c_int, c_int, _i64p]),
    "pbx_profile_select_typed": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int64,
                                         c_int, c_int, c_void_p, c_void_p, c_int, c_int,
                                         POINTER(c_int64)]),
    "pbx_profile_get_selection": (c_int, [c_void_p, _i64p, _dp, _dp]),
    "pbx_profile_minmax": (c_int, [c_void_p, _dp, _dp]),
    "pbx_profile_edges_equaln": (c_int, [c_void_p, c_int64, c_int, c_double, c_int, c_double, _dp,
                                         _i64p]),
    "pbx_profile_assign": (c_int, [c_void_p, _dp, c_int64, _i64p, _i64p]),
    "pbx_profile_csr": (c_int, [c_void_p, _i64p, _i64p]),
    "pbx_profile_moments": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, _dp]),
    "pbx_profile_moments_cols": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_uint32,
                                         _dp]),
    "pbx_profile_percentiles": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int,
                                        c_void_p, c_void_p]),
    "pbx_profile_radial_equaln": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int,
                                          c_void_p, c_void_p, c_int, c_int, c_int64, c_int,
                                          c_double, c_int, c_double, c_int, c_int, c_void_p,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_void_p]),
    "pbx_profile_radial_equaln_comm": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                               c_int, c_int, c_void_p, c_void_p, c_int, c_int,
                                               c_int64, c_int, c_double, c_int, c_double, c_int,
                                               c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                               c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                               c_void_p]),
    "pbx_profile_binned_equaln": (c_int, [c_void_p, c_int64, c_int, c_double, c_int, c_double,
                                          c_int, c_int, POINTER(c_int), POINTER(c_int),
                                          POINTER(c_uint32), _dp, POINTER(c_int64), _i64p,
                                          POINTER(c_int64), _dp]),
    "pbx_comm_unique_id_size": (c_int, []),
    "pbx_comm_unique_id": (c_int, [c_char_p, c_int]),
    "pbx_comm_init": (c_int, [POINTER(c_void_p), c_int, c_int, c_char_p]),
    "pbx_comm_destroy": (c_int, [c_void_p]),
    "pbx_comm_allgatherv": (c_int, [c_void_p, c_void_p, _i64p, _i64p]),
    "pbx_comm_allreduce_f64": (c_int, [c_void_p, c_void_p, c_void_p, c_int64]),
    "pbx_comm_allreduce_i64": (c_int, [c_void_p, c_void_p, c_void_p, c_int64]),
    "pbx_comm_allreduce": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int]),
    "pbx_comm_allreduce_host": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int]),
    "pbx_profile_path_stats": (c_int, [c_void_p, _i64p]),
    "pbx_profile_mono_stats": (c_int, [c_void_p, _i64p]),
    "pbx_profile_level0_stats": (c_int, [c_void_p, _i64p]),
    "pbx_profile_spec_stats": (c_int, [c_void_p, _i64p]),
    "pbx_profile_set_level0_hint": (c_int, [c_void_p, c_int]),
    "pbx_profile_set_source_stable": (c_int, [c_void_p, c_int]),
    "pbx_profile_key_range": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
    "pbx_profile_msel_begin": (c_int, [c_void_p, c_int64, c_int, c_double, c_int, c_double,
                                       c_uint64, c_uint64, POINTER(c_int)]),
    "pbx_profile_msel_hist": (c_int, [c_void_p, c_int, POINTER(c_void_p), POINTER(c_int64)]),
    "pbx_profile_msel_resolve": (c_int, [c_void_p, c_int]),
    "pbx_profile_msel_edges": (c_int, [c_void_p, _dp, POINTER(c_int64)]),
    "pbx_comm_barrier": (c_int, [c_void_p]),
    "pbx_comm_max_f64": (c_int, [c_void_p, c_double, POINTER(c_double)]),
    "pbx_comm_init_host": (c_int, [POINTER(c_void_p), c_int, c_int, HOST_COLLECTIVE_FN, c_void_p]),
}


def load() -> ctypes.CDLL:
    """Load libpbx.so once; raise NativeLibraryMissing if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not path.exists():
        raise NativeLibraryMissing(
            f"{path} not found: the HIP engine is not built "
            "(python -c 'import __graft_entry__ as g; g.build()')")
    lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
    # an A/B build named by PBX_AB_LIBRARY may predate a symbol: bind what it
    # has (calling a missing one raises AttributeError); any other library —
    # the product build, or one named by PBX_LIBRARY — must export every
    # declared symbol (tests/test_abi.py)
    lenient = bool(os.environ.get("PBX_AB_LIBRARY"))
    for name, (res, args) in _SIGNATURES.items():
        if lenient and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols() -> list[str]:
    return sorted(_SIGNATURES)


def last_error() -> str:
    msg = load().pbx_last_error()
    return msg.decode("utf-8", "replace") if msg else ""


def check(status: int) -> None:
    if status == PBX_OK:
        return
    msg = last_error()
    if status == PBX_ERR_VALUE:
        raise ValueError(msg)
    raise RuntimeError(msg or f"libpbx error {status}")


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args))


_raw_lib = None
_CArg = type(ctypes.byref(ctypes.c_int()))


class Prepared:
    """A native call whose arguments do not change between calls, converted
    to ctypes objects once: a repeated 26-argument call otherwise spends
    ~4 us per call in ctypes' per-argument conversions (measured on the
    1M-particle profile step, whose whole host share is ~30 us)."""

    __slots__ = ("fn", "args")

    def __init__(self, name: str, *args):
        global _raw_lib
        lib = load()
        if _raw_lib is None:  # a second handle: its functions carry no argtypes
            _raw_lib = ctypes.CDLL(lib._name, mode=ctypes.RTLD_GLOBAL)
        self.fn = getattr(_raw_lib, name)
        self.fn.restype = c_int
        conv = []
        for t, v in zip(_SIGNATURES[name][1], args, strict=True):
            if isinstance(v, (ctypes._SimpleCData, ctypes._Pointer, ctypes.Array, _CArg)):
                conv.append(v)
            elif v is None:
                conv.append(t())
            else:
                conv.append(t(v))
        self.args = tuple(conv)

    def __call__(self) -> None:
        check(self.fn(*self.args))


def dptr(a: np.ndarray | None):
    """double* of a C-contiguous float64 array (or NULL)."""
    if a is None:
        return None
    return a.ctypes.data_as(_dp)


def vptr(a: np.ndarray | None):
    """void* of a C-contiguous array (or NULL)."""
    if a is None:
        return None
    return a.ctypes.data_as(c_void_p)


def device_count() -> int:
    n = c_int(0)
    call("pbx_device_count", ctypes.byref(n))
    return n.value


def set_device(dev: int) -> None:
    call("pbx_set_device", int(dev))


def device_name() -> str:
    buf = ctypes.create_string_buffer(256)
    call("pbx_device_name", buf, 256)
    return buf.value.decode()


def set_precise(on: bool) -> None:
    """Direct-sum precision (include/pbx.h pbx_set_precise): True refines
    every 1/sqrt with a Newton step (~1e-16); False (default) lets the
    all-particles symmetric kernel use v_rsq_f64 as is (~1e-7 of the
    reference, inside the 1e-5 contract)."""
    call("pbx_set_precise", 1 if on else 0)


def get_precise() -> bool:
    v = ctypes.c_int()
    call("pbx_get_precise", ctypes.byref(v))
    return bool(v.value)


class precise_mode:
    """``with precise_mode(True): ...`` — set the precision, restore after."""

    def __init__(self, on: bool = True):
        self.on = on

    def __enter__(self):
        self.prev = get_precise()
        set_precise(self.on)
        return self

    def __exit__(self, *exc):
        set_precise(self.prev)
        return False


def synchronize() -> None:
    call("pbx_device_synchronize")


class DeviceArray:
    """An HBM allocation owned by Python (freed on ``free()`` / GC).

    Used by the device-resident API (bench, multi-GPU sharding); the
    host-array gravity / profile entry points manage their own workspace.
    """

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = c_void_p()
        call("pbx_malloc", ctypes.byref(p), c_size_t(max(self.nbytes, 16)))
        self.ptr = p

    @classmethod
    def from_host(cls, a: np.ndarray) -> "DeviceArray":
        a = np.ascontiguousarray(a)
        d = cls(a.nbytes)
        d.upload(a)
        return d

    def upload(self, a: np.ndarray) -> None:
        a = np.ascontiguousarray(a)
        if a.nbytes > self.nbytes:
            raise ValueError("host array larger than device allocation")
        call("pbx_memcpy_htod", self.ptr, a.ctypes.data_as(c_void_p), c_size_t(a.nbytes))

    def download(self, out: np.ndarray) -> np.ndarray:
        if not out.flags.c_contiguous or out.nbytes > self.nbytes:
            raise ValueError("bad host output buffer")
        call("pbx_memcpy_dtoh", out.ctypes.data_as(c_void_p), self.ptr, c_size_t(out.nbytes))
        return out

    def offset(self, nbytes: int) -> c_void_p:
        return c_void_p(self.ptr.value + int(nbytes))

    def free(self) -> None:
        if self.ptr is not None and self.ptr.value:
            lib = _lib
            if lib is not None:
                lib.pbx_free(self.ptr)
        self.ptr = c_void_p()

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.free()
        except Exception:
            pass


class Event:
    """A HIP event on the library stream (kernel timing on the right stream)."""

    def __init__(self):
        p = c_void_p()
        call("pbx_event_create", ctypes.byref(p))
        self.ptr = p

    def record(self) -> None:
        call("pbx_event_record", self.ptr)

    def elapsed_ms(self, later: "Event") -> float:
        ms = c_float(0.0)
        call("pbx_event_elapsed_ms", self.ptr, later.ptr, ctypes.byref(ms))
        return float(ms.value)

    def __del__(self):  # pragma: no cover
        try:
            if _lib is not None and self.ptr.value:
                _lib.pbx_event_destroy(self.ptr)
        except Exception:
            pass
