"""The profile drop-in (integration/pynbodyext_mi355x_profiles.py) installed
onto the REFERENCE's own classes: /root/reference/pynbodyext/profiles/bins.py
and proarray.py, loaded by tests/golden/make_golden.py's stub harness (the
import-time names of the absent pynbody stubbed, as when the fixtures were
made).  Runs on the CPU of this container only and skips where the reference
tree is absent (the GPU box).

libpbx cannot run without a GPU, so its profile entry points are stood in for
by ``FakePbx``: the same C signatures called through the module's own ctypes
plumbing (pointers, byref outputs, status codes and pbx_last_error), computed
by oracle/profile_ref.py.  What this pins is the SEAM, not the kernels (those
are pinned by tests/test_gpu_integration.py and test_gpu_profile.py):

* install() replaces exactly BinsSet._assign_particles (bins.py:346-395), the
  "equaln" registry entry (bins.py:634-685, :720-746) and the classmethod
  ProfileArray._compute (proarray.py:272-334) of the reference's classes;
* BinsSet(...)(sim) and ProfileArray._compute give the unpatched reference
  methods' results (edges, counts, binind lists bit-exact; statistics to
  rounding), through the fused equaln pass + CSR read-back;
* a BinsSet re-materialised in place over the same, mutated x sees the new
  values (x uploaded once per materialisation);
* uninstall() restores the original objects.
"""
from __future__ import annotations

import ctypes
import importlib.util
import sys
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import pytest

from oracle import profile_ref as pr

ROOT = Path(__file__).resolve().parent.parent
REF = Path("/root/reference/pynbodyext/profiles")
pytestmark = pytest.mark.skipif(not (REF / "bins.py").exists(),
                                reason="needs the reference tree (/root/reference)")


def _load_file(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture
def reference():
    """(bins, proarray) of the reference, with sys.modules restored after."""
    saved = dict(sys.modules)
    try:
        golden = _load_file("_pbx_make_golden", ROOT / "tests" / "golden" / "make_golden.py")
        bins_mod, pa_mod = golden.load_reference()
        yield bins_mod, pa_mod
    finally:
        for k in list(sys.modules):
            if k not in saved:
                del sys.modules[k]
        sys.modules.update(saved)


# ------------------------------------------------------------ libpbx stand-in
def _arr(ptr, n, dtype=np.float64):
    if n == 0:
        return np.zeros(0, dtype)
    ct = ctypes.c_double if dtype == np.float64 else ctypes.c_int64
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), shape=(n,))


class FakePbx:
    """pbx_profile_* with libpbx's C signatures and status codes, computed by
    the oracle (test infrastructure: no product code runs here)."""

    def __init__(self):
        self.h = {}
        self.err = b""
        self.calls = []

    def _run(self, name, fn):
        self.calls.append(name)
        try:
            fn()
            return 0
        except (ValueError, IndexError) as e:  # PBX_ERR_VALUE (IndexError: numpy's s[0] message)
            self.err = (f"index 0 is out of bounds for axis 0 with size 0" if isinstance(e, IndexError)
                        else str(e)).encode()
            return 1

    def pbx_last_error(self):
        return self.err

    def pbx_profile_create(self, ph):
        key = len(self.h) + 1
        self.h[key] = {}
        ph._obj.value = key
        return 0

    def pbx_profile_destroy(self, h):
        self.h.pop(h.value, None)
        return 0

    def pbx_profile_set_x(self, h, xp, n):
        def f():
            self.h[h.value] = {"x": _arr(xp, n).copy()}
        return self._run("set_x", f)

    def _equaln(self, P, nb, has_min, mn, has_max, mx):
        return pr.edges_equaln(P["x"], int(nb), mn if has_min else None, mx if has_max else None)

    def pbx_profile_edges_equaln(self, h, nb, has_min, mn, has_max, mx, out, ne):
        def f():
            e = self._equaln(self.h[h.value], nb, has_min, mn, has_max, mx)
            _arr(out, len(e))[:] = e
            ne._obj.value = len(e)
        return self._run("edges_equaln", f)

    def _assign(self, P, e):
        perm, offs, counts = pr.assign(P["x"], e)
        P.update(perm=perm, offs=offs, counts=counts, nb=len(e) - 1)
        return counts

    def pbx_profile_assign(self, h, ep, ne, cp, nv):
        def f():
            c = self._assign(self.h[h.value], _arr(ep, ne).copy())
            _arr(cp, len(c), np.int64)[:] = c
            nv._obj.value = int(c.sum())
        return self._run("assign", f)

    def pbx_profile_binned_equaln(self, h, nb, has_min, mn, has_max, mx, csr, n_stats, fs, ws, cols,
                                  ep, ne, cp, nv, mom):
        def f():
            assert csr == 1 and n_stats == 0
            P = self.h[h.value]
            if P["x"].size == 0:
                raise ValueError("Cannot create bins: input array is empty")
            e = self._equaln(P, nb, has_min, mn, has_max, mx)
            c = self._assign(P, e)
            _arr(ep, len(e))[:] = e
            _arr(cp, len(c), np.int64)[:] = c
            ne._obj.value = len(e)
            nv._obj.value = int(c.sum())
        return self._run("binned_equaln", f)

    def pbx_profile_csr(self, h, pp, op):
        def f():
            P = self.h[h.value]
            if pp:
                _arr(pp, len(P["perm"]), np.int64)[:] = P["perm"]
            if op:
                _arr(op, len(P["offs"]), np.int64)[:] = P["offs"]
        return self._run("csr", f)

    def pbx_profile_moments_cols(self, h, fsrc, fp, wsrc, wp, cols, out):
        def f():
            P = self.h[h.value]
            n = len(P["x"])
            fa = _arr(fp, n)
            wa = None if wp is None else _arr(wp, n)
            m = np.zeros((P["nb"], 7))
            for i in range(P["nb"]):
                ind = P["perm"][P["offs"][i]:P["offs"][i + 1]]
                a = fa[ind]
                w = np.ones(len(ind)) if wa is None else wa[ind]
                row = [w.sum(), (a * w).sum(), (a * a * w).sum(), a.sum(), (a * a).sum(),
                       (np.abs(a) * w).sum(), np.abs(a).sum()]
                if wa is None:
                    row[0] = row[1] = row[2] = row[5] = 0.0
                m[i] = [v if (cols >> k) & 1 else 0.0 for k, v in enumerate(row)]
            _arr(out, m.size)[:] = m.reshape(-1)
        return self._run("moments_cols", f)

    def pbx_profile_percentiles(self, h, fsrc, fp, wsrc, wp, absval, nq, qp, out):
        def f():
            P = self.h[h.value]
            n = len(P["x"])
            fa = _arr(fp, n)
            wa = None if wp is None else _arr(wp, n)
            q = float(_arr(qp, 1)[0])
            fn = pr.statistic(f"p{int(round(q * 100))}")[1]
            o = _arr(out, P["nb"])
            for i in range(P["nb"]):
                ind = P["perm"][P["offs"][i]:P["offs"][i + 1]]
                a = np.abs(fa[ind]) if absval else fa[ind]
                o[i] = np.nan if len(ind) == 0 else fn(a, None if wa is None else wa[ind])
        return self._run("percentiles", f)


def _integration():
    return _load_file("_pbx_integration_ref", ROOT / "integration" / "pynbodyext_mi355x_profiles.py")


def _sim(x, SimArray=None):
    # plain ndarrays: the stub SimArray is a bare ndarray subclass without
    # pynbody's constructor (bins.py:251-255 only wraps edges for SimArray x)
    return {"r": x}


def _seams(bins_mod, pa_mod):
    B, P = bins_mod.BinsSet, pa_mod.ProfileArray
    return (B.__dict__["_assign_particles"], B._bins_algorithm_registry["equaln"],
            P.__dict__["_compute"])


def _materialise(bins_mod, sim, **kw):
    return bins_mod.BinsSet(bins_by="r", bins_area="spherical_shell", **kw)(sim)


STATS = ["mean", "sum", "sum_w", "rms", "disp", "p16", "median", "abs_mean"]
CASES = [dict(bins_type="equaln", nbins=128), dict(bins_type="equaln", nbins=16, bin_min=0.3,
                                                   bin_max=4.0),
         dict(bins_type="lin", nbins=32), dict(bins_type="log", nbins=20, bin_min=0.05,
                                               bin_max=20.0)]


def _results(bins_mod, pa_mod, sim, w, f, kw):
    bs = _materialise(bins_mod, sim, **kw)
    prof = SimpleNamespace(nbins=len(bs.bin_edges) - 1, _weight=w, binind=bs.binind, bins=bs,
                           npart_bins=bs.npart_bins, sim=sim)
    stats = {k: np.asarray(pa_mod.ProfileArray._compute(prof, f, k)[0]) for k in STATS}
    return bs, stats


@pytest.mark.parametrize("kw", CASES, ids=lambda k: "-".join(str(v) for v in k.values()))
def test_install_on_reference_classes(reference, kw):
    bins_mod, pa_mod = reference
    SimArray = pa_mod.SimArray
    rng = np.random.default_rng(77)
    n = 20_000
    x = pr.radial_r(rng.normal(size=(n, 3)) * 2.0)
    w = rng.uniform(0.5, 1.5, n)
    f = rng.normal(size=n)
    sim = _sim(x, SimArray)
    before = _seams(bins_mod, pa_mod)
    ref_bs, ref_stats = _results(bins_mod, pa_mod, sim, w, f, kw)

    mod = _integration()
    fake = FakePbx()
    mod._lib = fake  # the module's _load() keeps an already bound library
    mod.install(bins_module=bins_mod, proarray_module=pa_mod)
    try:
        B, P = bins_mod.BinsSet, pa_mod.ProfileArray
        assert B.__dict__["_assign_particles"] is mod._assign_particles
        assert B._bins_algorithm_registry["equaln"] is mod._equal_number_bins_algorithm
        assert isinstance(P.__dict__["_compute"], classmethod)
        assert P.__dict__["_compute"] is not before[2]
        # the other registry entries are the reference's own
        assert B._bins_algorithm_registry["lin"] is not mod._equal_number_bins_algorithm
        bs, stats = _results(bins_mod, pa_mod, sim, w, f, kw)
        assert isinstance(bs.__dict__.get("_pbx_handle"), mod.DeviceBinsHandle)
    finally:
        mod.uninstall()
    assert _seams(bins_mod, pa_mod) == before

    if kw["bins_type"] == "equaln":  # one fused pass, the CSR read back, no separate assign
        assert "binned_equaln" in fake.calls and "assign" not in fake.calls
    else:
        assert "assign" in fake.calls and "binned_equaln" not in fake.calls
    assert "csr" in fake.calls and "moments_cols" in fake.calls and "percentiles" in fake.calls
    e0, e1 = np.asarray(ref_bs.bin_edges), np.asarray(bs.bin_edges)
    assert np.array_equal(e0.view(np.uint64), e1.view(np.uint64))
    assert np.array_equal(ref_bs.npart_bins, bs.npart_bins)
    assert len(ref_bs.binind) == len(bs.binind)
    for a, b in zip(ref_bs.binind, bs.binind):
        assert np.array_equal(a, b)
    for k in STATS:
        assert np.array_equal(np.isnan(ref_stats[k]), np.isnan(stats[k])), k
        ok = ~np.isnan(ref_stats[k])
        np.testing.assert_allclose(stats[k][ok], ref_stats[k][ok], rtol=1e-10, atol=1e-13,
                                   err_msg=k)

    # after uninstall the reference runs its own numpy code again
    bs2, _ = _results(bins_mod, pa_mod, sim, w, f, kw)
    assert "_pbx_handle" not in bs2.__dict__
    assert np.array_equal(np.asarray(bs2.bin_edges), e0)


def test_inplace_rematerialisation_sees_mutated_x(reference):
    """x mutated in place between two in-place materialisations
    of one BinsSet (same array object) — the device copy is refreshed."""
    bins_mod, pa_mod = reference
    rng = np.random.default_rng(5)
    x = rng.lognormal(size=5000)
    sim = _sim(x, pa_mod.SimArray)
    mod = _integration()
    mod._lib = FakePbx()
    mod.install(bins_module=bins_mod, proarray_module=pa_mod)
    try:
        for kw in (dict(bins_type="equaln", nbins=10), dict(bins_type="lin", nbins=10)):
            bs = bins_mod.BinsSet(bins_by="r", bins_area="length", **kw)
            bs(sim, inplace=True)
            sim["r"][:] = rng.lognormal(sigma=2.0, size=x.size)  # same object, new values
            bs(sim, inplace=True)
            want_e = pr.EDGE_ALGORITHMS[kw["bins_type"]](np.asarray(sim["r"]), 10)
            assert np.array_equal(np.asarray(bs.bin_edges), want_e)
            _, _, counts = pr.assign(np.asarray(sim["r"]), want_e)
            assert np.array_equal(bs.npart_bins, counts)
    finally:
        mod.uninstall()


def test_equaln_errors_and_degenerate_through_the_seam(reference):
    """bins.py:731-740 behaviour through the fused seam: empty input raises
    ValueError, an empty clip window IndexError, < 2 values two equal edges."""
    bins_mod, pa_mod = reference
    mod = _integration()
    mod._lib = FakePbx()
    mod.install(bins_module=bins_mod, proarray_module=pa_mod)
    try:
        SA = pa_mod.SimArray
        with pytest.raises(ValueError, match="input array is empty"):
            _materialise(bins_mod, _sim(np.zeros(0), SA), bins_type="equaln", nbins=4)
        with pytest.raises(IndexError):
            _materialise(bins_mod, _sim(np.arange(5.0), SA), bins_type="equaln", nbins=4,
                         bin_min=10.0)
        # (a whole materialisation of one bin fails inside the reference itself,
        # np.gradient of one midpoint: the two seams are called as __call__ does)
        x = np.array([1.0, 7.0, 9.0])
        bs = bins_mod.BinsSet(bins_by="r", bins_area="length", bins_type="equaln", nbins=4,
                              bin_min=8.0)
        edges = bins_mod.BinsSet._bins_algorithm_registry["equaln"](bs, x)
        assert np.array_equal(np.asarray(edges), [9.0, 9.0])
        binind, counts = bs._assign_particles(x, edges)
        assert np.array_equal(counts, [1])
        assert [list(b) for b in binind] == [[2]]
    finally:
        mod.uninstall()
