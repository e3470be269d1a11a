"""The two spatial forms of RadialProfile on the GPU against fixtures the
reference's own bins.py / proarray.py produced (tests/golden/make_golden.py,
spatial_cases; spatial_profile.py:30-35, bins.py:689-789):

* ndim=2: bins_by rxy, bins_area annulus, on a thin disk — edges, counts and
  binind bit-exact, areas bit-exact, per-bin mass sums to 1e-12;
* a float32 snapshot behind Sphere & FamilyFilter (ndim=3, equaln 128,
  weight mass): the positions go to the device as float32 (no host up-cast);
  the kept set, r (float32 values) and edges / counts / binind are
  bit-exact; sums are float64 on the device where the reference sums the
  float32 arrays in float32 (rtol 1e-6, float32 rounding).
rxy / r / the Sphere distance are numpy's expressions; pynbody itself is
absent, so agreement with pynbody's derived arrays is parity unpinned.
"""
from pathlib import Path

import numpy as np
import pytest

from pynbodyext.filters import FamilyFilter, Sphere
from pynbodyext.profiles import RadialProfileBuilder
from pynbodyext.profiles._device import SRC_NONE, SRC_W, SRC_X, DeviceBins
from pynbodyext.simcore import SimSnap

pytestmark = pytest.mark.gpu

FIX = np.load(Path(__file__).resolve().parent / "golden" / "profile_spatial.npz")
CASES_2D = [("lin_64", "lin", 64, None, None), ("log_64", "log", 64, 0.05, 15.0),
            ("equaln_100", "equaln", 100, None, None)]


def _disk():
    pos, mass = FIX["ann/pos"], FIX["ann/mass"]
    n = len(mass)
    return SimSnap({"pos": pos, "mass": mass}, families={"dm": slice(0, n)})


@pytest.mark.parametrize("tag,bt,nb,lo,hi", CASES_2D)
@pytest.mark.parametrize("fused", [False, True])
def test_annulus_profile_matches_reference(gpu, tag, bt, nb, lo, hi, fused):
    sim = _disk()
    b = RadialProfileBuilder(ndim=2, weight="mass", bins_type=bt, nbins=nb, bin_min=lo, bin_max=hi)
    if fused:  # device selection computes rxy (ndim=2) for the whole disk
        b = b.filter(Sphere(1e6) & FamilyFilter("dm"))
    prof = b(sim)
    assert np.array_equal(np.asarray(prof.bin_edges), FIX[f"ann/{tag}/edges"])
    assert np.array_equal(prof.npart_bins, FIX[f"ann/{tag}/counts"])
    perm, _ = prof.bins.binind.csr
    assert np.array_equal(perm, FIX[f"ann/{tag}/perm"])
    assert np.array_equal(np.asarray(prof.binsize), FIX[f"ann/{tag}/area"])
    np.testing.assert_allclose(np.asarray(prof["mass"]["sum"]), FIX[f"ann/{tag}/mass_sum"],
                               rtol=1e-12)
    np.testing.assert_allclose(np.asarray(prof["density"]),
                               FIX[f"ann/{tag}/mass_sum"] / FIX[f"ann/{tag}/area"], rtol=1e-12)


def _f32_snapshot():
    pos, mass = FIX["f32/pos"], FIX["f32/mass"]
    assert pos.dtype == np.float32 and mass.dtype == np.float32
    lo, hi = (int(v) for v in FIX["f32/fam"])
    n = len(mass)
    return SimSnap({"pos": pos, "mass": mass}, families={"dm": slice(lo, hi), "star": slice(hi, n)})


def test_float32_device_selection(gpu):
    """DeviceBins.select on float32 arrays: kept particles and r identical to
    numpy's float32 / float64-mask evaluation."""
    pos, mass = FIX["f32/pos"], FIX["f32/mass"]
    lo, hi = (int(v) for v in FIX["f32/fam"])
    d = DeviceBins.select(pos, mass, sphere=(FIX["f32/cen"], float(FIX["f32/radius"])),
                          families=[(lo, hi)], ndim=3)
    try:
        idx, x, w = d.selection(idx=True, x=True, w=True)
        assert np.array_equal(idx, FIX["f32/kept"])
        assert np.array_equal(x, FIX["f32/r"].astype(np.float64))
        assert np.array_equal(w, mass[idx].astype(np.float64))
        edges = d.edges_equaln(128)
        assert np.array_equal(edges, FIX["f32/edges"].astype(np.float64))
        assert np.array_equal(d.assign(edges), FIX["f32/counts"])
        perm, _ = d.csr()
        assert np.array_equal(perm, FIX["f32/perm"])
        msum = d.moments(SRC_W, SRC_NONE, 1 << 3)[:, 3]
        np.testing.assert_allclose(msum, FIX["f32/mass_sum"], rtol=1e-6)
        mom = d.moments(SRC_X, SRC_W, 0b11)
        np.testing.assert_allclose(mom[:, 1] / mom[:, 0], FIX["f32/r_mean"], rtol=1e-6)
    finally:
        d.close()


def test_float32_fused_builder(gpu):
    """RadialProfileBuilder on a float32 snapshot behind Sphere & FamilyFilter:
    sim['r'] of the profile is float32 (pynbody's derived array dtype)."""
    sim = _f32_snapshot()
    cen, radius = FIX["f32/cen"], float(FIX["f32/radius"])
    prof = RadialProfileBuilder(ndim=3, weight="mass", bins_type="equaln", nbins=128).filter(
        Sphere(radius, cen=tuple(cen)) & FamilyFilter("dm"))(sim)
    assert len(prof.sim) == len(FIX["f32/kept"])
    r = np.asarray(prof.sim["r"])
    assert r.dtype == np.float32 and np.array_equal(r, FIX["f32/r"])
    assert np.array_equal(np.asarray(prof.bin_edges, dtype=np.float64),
                          FIX["f32/edges"].astype(np.float64))
    assert np.array_equal(prof.npart_bins, FIX["f32/counts"])
    perm, _ = prof.bins.binind.csr
    assert np.array_equal(perm, FIX["f32/perm"])
    np.testing.assert_allclose(np.asarray(prof["mass"]["sum"]), FIX["f32/mass_sum"], rtol=1e-6)
