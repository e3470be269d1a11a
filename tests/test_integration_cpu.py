"""integration/pynbodyext_mi355x_profiles.py on CPU: the statistic plans
and the reference statistics rebuilt from per-bin sums (proarray.py:632-860)
against oracle/profile_ref.compute, and install() without a library."""
import importlib.util
from pathlib import Path

import numpy as np
import pytest

from oracle import profile_ref as pr
from pynbodyext.profiles.proarray import ProfileArray

ROOT = Path(__file__).resolve().parent.parent


def _mod():
    path = ROOT / "integration" / "pynbodyext_mi355x_profiles.py"
    spec = importlib.util.spec_from_file_location("pbx_profiles_cpu", path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _moments(f, w, perm, offs):
    nb = len(offs) - 1
    m = np.zeros((nb, 7))
    for i in range(nb):
        ind = perm[offs[i]:offs[i + 1]]
        a, ww = f[ind], (np.ones(len(ind)) if w is None else w[ind])
        m[i] = [ww.sum(), (a * ww).sum(), (a * a * ww).sum(), a.sum(), (a * a).sum(),
                (np.abs(a) * ww).sum(), np.abs(a).sum()]
    return m


@pytest.mark.parametrize("key", ["mean", "sum", "sum_w", "rms", "disp", "abs_mean", "abs_sum",
                                 "abs_sum_w", "abs_rms", "abs_disp"])
@pytest.mark.parametrize("weighted", [True, False])
def test_from_moments_matches_oracle_statistics(key, weighted):
    mod = _mod()
    rng = np.random.default_rng(4)
    x = rng.lognormal(size=20_000)
    f = rng.normal(size=x.size)
    w = rng.uniform(0.5, 1.5, x.size) if weighted else None
    edges = pr.edges_equaln(x, 32)
    edges = np.concatenate([edges, [edges[-1] * 2, edges[-1] * 3]])  # two empty bins
    perm, offs, counts = pr.assign(x, edges)
    calc = ProfileArray.get_statistic(key)
    kind, absval, pct = mod._stat_plan(calc)
    assert pct is None
    got = mod._from_moments(kind, absval, _moments(f, w, perm, offs), counts, weighted)
    want, _ = pr.compute(f, w, perm, offs, key)
    assert np.array_equal(np.isnan(got), np.isnan(want))
    ok = ~np.isnan(want)
    np.testing.assert_allclose(got[ok], want[ok], rtol=1e-10, atol=1e-12)


def test_percentile_plans():
    mod = _mod()
    assert mod._stat_plan(ProfileArray.get_statistic("p16")) == ("pct", False, 16.0)
    assert mod._stat_plan(ProfileArray.get_statistic("median")) == ("pct", False, 50.0)
    assert mod._stat_plan(ProfileArray.get_statistic("abs_p84")) == ("pct", True, 84.0)


def test_install_needs_a_library(monkeypatch):
    mod = _mod()
    monkeypatch.delenv("PBX_LIBRARY", raising=False)
    with pytest.raises(ImportError, match="libpbx.so"):
        mod.install()
    mod.uninstall()  # nothing installed: no-op
