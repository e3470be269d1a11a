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


def spatial_cases(bins_mod, pa_mod):
    """RadialProfile's two spatial forms (spatial_profile.py:30-35):
    * ann_*: ndim=2 — bins_by "rxy", bins_area "annulus" (bins.py:759-765)
      on a thin disk; rxy = sqrt(x*x + y*y) (pynbody's derived rxy, which
      pynbody is absent to confirm: parity with pynbody unpinned);
    * f32_*: a float32 snapshot behind Sphere & FamilyFilter, ndim=3 equaln
      128 weight mass — numpy's dtype rules: the Sphere distance against the
      float64 centre is float64, r of the float32 positions is float32, and
      the reference's binning / statistics then run on float32 arrays.
    Only inputs and the reference's outputs are stored."""
    BinsSet = bins_mod.BinsSet
    out = {}
    rng = np.random.default_rng(2101)
    n = 20000
    pos = np.column_stack([rng.normal(scale=3.0, size=n), rng.normal(scale=3.0, size=n),
                           rng.normal(scale=0.3, size=n)])
    mass = rng.uniform(0.5, 1.5, n)
    out["ann/pos"], out["ann/mass"] = pos, mass
    rxy = np.sqrt(pos[:, 0] * pos[:, 0] + pos[:, 1] * pos[:, 1])
    for tag, bt, nb, lo, hi in (("lin_64", "lin", 64, None, None),
                                ("log_64", "log", 64, 0.05, 15.0),
                                ("equaln_100", "equaln", 100, None, None)):
        bs = BinsSet(bins_by="rxy", bins_area="annulus", bins_type=bt, nbins=nb, bin_min=lo,
                     bin_max=hi)
        edges = np.asarray(BinsSet._bins_algorithm_registry[bt](bs, rxy), dtype=np.float64)
        binind, counts = bs._assign_particles(rxy, edges)
        area = BinsSet._bins_area_registry["annulus"](bs, edges)
        prof = SimpleNamespace(nbins=len(edges) - 1, _weight=mass, binind=binind)
        msum, _ = pa_mod.ProfileArray._compute(prof, mass, "sum")
        out[f"ann/{tag}/edges"] = edges
        out[f"ann/{tag}/counts"] = np.asarray(counts, dtype=np.int64)
        out[f"ann/{tag}/perm"] = np.concatenate(binind).astype(np.int64)
        out[f"ann/{tag}/area"] = np.asarray(area, dtype=np.float64)
        out[f"ann/{tag}/mass_sum"] = np.asarray(msum, dtype=np.float64)
    # float32 snapshot
    x = rng.random(n)
    r = np.minimum((x ** (-2.0 / 3.0) - 1.0) ** -0.5, 50.0)
    ct, ph = rng.uniform(-1.0, 1.0, n), rng.uniform(0.0, 2 * np.pi, n)
    st = np.sqrt(1.0 - ct * ct)
    pos32 = np.column_stack([r * st * np.cos(ph), r * st * np.sin(ph), r * ct]).astype(np.float32)
    mass32 = rng.uniform(0.5, 1.5, n).astype(np.float32)
    cen, radius, fam = np.array([0.5, -0.25, 0.125]), 10.0, (0, 12000)
    dx, dy, dz = (pos32[:, 0] - cen[0], pos32[:, 1] - cen[1], pos32[:, 2] - cen[2])
    mask = ((dx * dx + dy * dy) + dz * dz) < radius * radius
    mask[fam[1]:] = False
    kept = np.nonzero(mask)[0]
    p = pos32[kept]
    r32 = np.sqrt((p[:, 0] * p[:, 0] + p[:, 1] * p[:, 1]) + p[:, 2] * p[:, 2])
    assert r32.dtype == np.float32 and dx.dtype == np.float64
    m32 = mass32[kept]
    bs = BinsSet(bins_by="r", bins_area="spherical_shell", bins_type="equaln", nbins=128)
    edges = BinsSet._bins_algorithm_registry["equaln"](bs, r32)
    binind, counts = bs._assign_particles(r32, edges)
    prof = SimpleNamespace(nbins=len(edges) - 1, _weight=m32, binind=binind)
    msum, _ = pa_mod.ProfileArray._compute(prof, m32, "sum")
    rmean, _ = pa_mod.ProfileArray._compute(prof, r32, "mean")
    out.update({"f32/pos": pos32, "f32/mass": mass32, "f32/cen": cen,
                "f32/radius": np.array(radius), "f32/fam": np.array(fam, dtype=np.int64),
                "f32/kept": kept.astype(np.int64), "f32/r": r32,
                "f32/edges": np.asarray(edges), "f32/counts": np.asarray(counts, dtype=np.int64),
                "f32/perm": np.concatenate(binind).astype(np.int64),
                "f32/mass_sum": np.asarray(msum), "f32/r_mean": np.asarray(rmean)})
    return out


def main():
    bins_mod, pa_mod = load_reference()
    np.savez_compressed(OUT / "profile_spatial.npz", numpy_version=np.array(np.__version__),
                        **spatial_cases(bins_mod, pa_mod))
    print("wrote profile_spatial.npz")
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
