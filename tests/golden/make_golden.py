#!/usr/bin/env python3
"""Generate the profile golden fixtures from the REFERENCE's own code.

Run here only (needs /root/reference; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It loads /root/reference/pynbodyext/profiles/bins.py and proarray.py by file
path.  pynbody is not installed in this image, so the import-time names
those modules reference (pynbody.array.SimArray / IndexedSimArray,
pynbody.snapshot.SimSnap, the pynbodyext.util._type aliases and
pynbodyext.chunk.is_dask_array) are provided as minimal stand-ins.  None of
the code paths recorded here calls into pynbody: the edge algorithms
(bins.py:689-746), BinsSet._assign_particles (bins.py:346-395) and
ProfileArray._compute with the registered statistics (proarray.py:272-334,
632-860) operate on plain numpy arrays; SimArray is only used as a view
type.  Nothing from the reference is copied into the repository: only input
arrays (or their seeds) and the reference's outputs are written, as .npz
files next to this script, together with the numpy version used.
"""
from __future__ import annotations

import hashlib
import importlib.util
import sys
import types
import typing
from pathlib import Path
from types import SimpleNamespace

import numpy as np

REF = Path("/root/reference/pynbodyext/profiles")
OUT = Path(__file__).resolve().parent


# ---------------------------------------------------------------- stand-ins
def _install_import_stubs():
    class SimArray(np.ndarray):
        def __array_finalize__(self, obj):
            self.units = getattr(obj, "units", None)
            self.sim = getattr(obj, "sim", None)

    pyn = types.ModuleType("pynbody")
    arr = types.ModuleType("pynbody.array")
    arr.SimArray = SimArray
    arr.IndexedSimArray = SimArray
    snap = types.ModuleType("pynbody.snapshot")
    snap.SimSnap = type("SimSnap", (), {})
    pyn.array, pyn.snapshot = arr, snap
    sys.modules.update({"pynbody": pyn, "pynbody.array": arr, "pynbody.snapshot": snap})

    ext = types.ModuleType("pynbodyext")
    ext.__path__ = []
    util = types.ModuleType("pynbodyext.util")
    util.__path__ = []
    typ = types.ModuleType("pynbodyext.util._type")
    for name in ("BinByFunc", "BinsAlgorithmFunc", "BinsAreaFunc", "RegistBinAlgorithmString",
                 "RegistBinAreaString", "RegistBinByString", "SimNpArray"):
        setattr(typ, name, typing.Any)
    chunk = types.ModuleType("pynbodyext.chunk")
    chunk.is_dask_array = lambda o: False
    prof = types.ModuleType("pynbodyext.profiles")
    prof.__path__ = []
    sys.modules.update({"pynbodyext": ext, "pynbodyext.util": util, "pynbodyext.util._type": typ,
                        "pynbodyext.chunk": chunk, "pynbodyext.profiles": prof})
    return SimArray


def _load(name: str, file: Path):
    spec = importlib.util.spec_from_file_location(name, file)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    _install_import_stubs()
    bins = _load("pynbodyext.profiles.bins", REF / "bins.py")
    proarray = _load("pynbodyext.profiles.proarray", REF / "proarray.py")
    return bins, proarray


# ---------------------------------------------------------------- inputs
def plummer_r(n: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    x = rng.random(n)
    r = (x ** (-2.0 / 3.0) - 1.0) ** -0.5
    return np.minimum(r, 50.0)


def dataset(n: int, seed: int):
    x = plummer_r(n, seed)
    rng = np.random.default_rng(seed + 1)
    w = rng.uniform(0.5, 1.5, n)
    f = rng.normal(size=n)
    return x, w, f


STATS = ["mean", "sum", "sum_w", "rms", "disp", "p16", "p50", "median", "abs_mean", "abs_sum",
         "abs_p84"]


def binind_checksums(binind):
    s1 = np.array([int(b.sum()) for b in binind], dtype=np.int64)
    s2 = np.array([int((b.astype(np.int64) ** 2).sum()) for b in binind], dtype=np.int64)
    first = np.array([int(b[0]) if len(b) else -1 for b in binind], dtype=np.int64)
    last = np.array([int(b[-1]) if len(b) else -1 for b in binind], dtype=np.int64)
    return s1, s2, first, last


def run_case(bins_mod, pa_mod, out, tag, x, w, f, bins_type, nb, bin_min=None, bin_max=None,
             store_perm=True, stats=False):
    BinsSet = bins_mod.BinsSet
    bs = BinsSet(bins_by="r", bins_area="spherical_shell", bins_type=bins_type, nbins=nb,
                 bin_min=bin_min, bin_max=bin_max)
    edges = np.asarray(BinsSet._bins_algorithm_registry[bins_type](bs, x), dtype=np.float64)
    binind, counts = bs._assign_particles(x, edges)
    out[f"{tag}/edges"] = edges
    out[f"{tag}/counts"] = np.asarray(counts, dtype=np.int64)
    if store_perm:
        out[f"{tag}/perm"] = (np.concatenate(binind) if len(binind) else np.zeros(0)).astype(np.int64)
    s1, s2, first, last = binind_checksums(binind)
    out[f"{tag}/idx_sum"], out[f"{tag}/idx_sq"] = s1, s2
    out[f"{tag}/idx_first"], out[f"{tag}/idx_last"] = first, last
    if stats:
        nbins = len(edges) - 1
        for wname, weights in (("w", w), ("none", None)):
            prof = SimpleNamespace(nbins=nbins, _weight=weights, binind=binind)
            for key in STATS:
                vals, canon = pa_mod.ProfileArray._compute(prof, f, key)
                out[f"{tag}/stat/{wname}/{key}"] = np.asarray(vals, dtype=np.float64)
                out[f"{tag}/statkey/{key}"] = np.array(canon)


def edge_cases(bins_mod):
    """Hand-made assignment / edge-algorithm corner cases (Appendix B)."""
    BinsSet = bins_mod.BinsSet
    out = {}
    cases = {
        # values exactly on edges, below/above range, NaN, duplicates
        "on_edges": (np.array([0.0, 0.5, 1.0, 1.5, 2.0, 2.0, -0.1, 2.1, np.nan, 1.0, 0.25]),
                     np.array([0.0, 0.5, 1.0, 1.5, 2.0])),
        "dup_edges": (np.array([0.0, 1.0, 1.0, 1.5, 2.0, 0.5, 3.0]),
                      np.array([0.0, 1.0, 1.0, 2.0])),
        "all_dropped": (np.array([5.0, 6.0, np.nan]), np.array([0.0, 1.0, 2.0])),
        "single_bin": (np.array([1.0, 1.0, 1.0, 0.0]), np.array([1.0, 1.0])),
        "empty_x": (np.zeros(0), np.array([0.0, 1.0, 2.0])),
        "neg_values": (np.array([-3.0, -2.0, -1.5, -1.0, 0.0, 1.0]),
                       np.array([-3.0, -1.0, 0.0, 1.0])),
    }
    for name, (x, edges) in cases.items():
        binind, counts = BinsSet._assign_particles(None, x, edges)
        out[f"{name}/x"] = x
        out[f"{name}/edges"] = edges
        out[f"{name}/counts"] = np.asarray(counts, dtype=np.int64)
        out[f"{name}/nbin_lists"] = np.array(len(binind))
        out[f"{name}/perm"] = (np.concatenate(binind) if len(binind) else np.zeros(0)).astype(np.int64)
        out[f"{name}/offsets"] = np.concatenate([[0], np.cumsum([len(b) for b in binind])]).astype(np.int64)
    # equaln corner cases
    eq = {
        "eq_degenerate": (np.array([3.0]), 4, None, None),
        "eq_clip": (np.linspace(0.0, 10.0, 101), 5, 2.0, 7.5),
        "eq_dups": (np.array([1.0] * 10 + [2.0] * 10 + [3.0] * 5), 4, None, None),
        "eq_with_nan": (np.array([3.0, 1.0, np.nan, 2.0, 5.0, 4.0]), 3, None, None),
        "eq_clip_nan": (np.array([3.0, 1.0, np.nan, 2.0, 5.0, 4.0]), 3, 0.0, 10.0),
    }
    for name, (x, nb, lo, hi) in eq.items():
        bs = BinsSet(bins_by="r", bins_area="length", bins_type="equaln", nbins=nb, bin_min=lo,
                     bin_max=hi)
        edges = BinsSet._bins_algorithm_registry["equaln"](bs, x)
        out[f"{name}/x"] = x
        out[f"{name}/nb"] = np.array(nb)
        out[f"{name}/bin_min"] = np.array(np.nan if lo is None else lo)
        out[f"{name}/bin_max"] = np.array(np.nan if hi is None else hi)
        out[f"{name}/edges"] = np.asarray(edges, dtype=np.float64)
    # log domain error message
    bs = BinsSet(bins_by="r", bins_area="length", bins_type="log", nbins=4)
    try:
        BinsSet._bins_algorithm_registry["log"](bs, np.array([0.0, 1.0]))
    except ValueError as e:
        out["log_error/message"] = np.array(str(e))
    return out


def main():
    bins_mod, pa_mod = load_reference()
    meta = {"numpy_version": np.array(np.__version__)}
    for n, seed, full in ((1000, 2001, True), (10000, 2002, True), (100000, 2003, False)):
        x, w, f = dataset(n, seed)
        out = dict(meta)
        out["seed"] = np.array(seed)
        out["x_sha256"] = np.array(hashlib.sha256(x.tobytes()).hexdigest())
        if full:
            out["x"], out["w"], out["f"] = x, w, f
        for bins_type in ("lin", "log", "equaln"):
            for nb in (8, 128, 256):
                tag = f"{bins_type}_{nb}"
                run_case(bins_mod, pa_mod, out, tag, x, w, f, bins_type, nb,
                         store_perm=full and (n <= 1000 or nb == 128),
                         stats=(nb == 128))
        run_case(bins_mod, pa_mod, out, "equaln_100_clip", x, w, f, "equaln", 100,
                 bin_min=0.05, bin_max=20.0, store_perm=full)
        run_case(bins_mod, pa_mod, out, "lin_64_range", x, w, f, "lin", 64, bin_min=0.1,
                 bin_max=5.0, store_perm=full, stats=True)
        run_case(bins_mod, pa_mod, out, "log_256_range", x, w, f, "log", 256, bin_min=0.01,
                 bin_max=50.0, store_perm=full)
        np.savez_compressed(OUT / f"profile_n{n}.npz", **out)
        print(f"wrote profile_n{n}.npz ({len(out)} arrays)")
    np.savez_compressed(OUT / "profile_edge_cases.npz", **meta, **edge_cases(bins_mod))
    print("wrote profile_edge_cases.npz")


if __name__ == "__main__":
    main()
