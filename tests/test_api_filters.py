"""Host side of the config-3 selection filters (CPU): FamilyFilter reads
family ranges through pynbody's own snapshot interface
(``SimSnap._family_slice`` / ``_get_family_slice``, the attributes the
reference itself uses, chunk.py:186,232), Sphere's strict inequality, and
the device description of ``Sphere & FamilyFilter`` (filt.py:42-86)."""
import numpy as np

from pynbodyext._pyn import get_family
from pynbodyext.filters import FamilyFilter, Sphere
from pynbodyext.simcore import SimSnap


class PynbodyLikeSnap:
    """Exposes ONLY what a pynbody SimSnap offers for families: the
    ``_family_slice`` dict and ``_get_family_slice`` (no ``_family_slices``)."""

    def __init__(self, pos, fams):
        self._pos = pos
        self._family_slice = {get_family(k, True): v for k, v in fams.items()}

    def __len__(self):
        return len(self._pos)

    def _get_family_slice(self, fam):
        return self._family_slice.get(fam, slice(0, 0))

    def __getitem__(self, key):
        assert key == "pos"
        return self._pos


def test_family_filter_on_pynbody_interface():
    pos = np.random.default_rng(0).normal(size=(100, 3))
    sim = PynbodyLikeSnap(pos, {"dm": slice(0, 60), "gas": slice(60, 90), "star": slice(90, 100)})
    f = FamilyFilter("gas")
    mask = f.build_mask(sim)
    want = np.zeros(100, dtype=bool)
    want[60:90] = True
    assert np.array_equal(mask, want)
    assert f.device_spec(sim) == {"families": [(60, 90)]}
    # a family the snapshot does not hold: empty mask, empty device range list
    assert not FamilyFilter("bh").build_mask(sim).any()
    assert FamilyFilter("bh").device_spec(sim) == {"families": []}


def test_sphere_and_family_device_spec():
    pos = np.random.default_rng(1).normal(size=(100, 3))
    sim = PynbodyLikeSnap(pos, {"dm": slice(0, 60), "gas": slice(60, 100)})
    filt = Sphere(1.5) & FamilyFilter("dm")
    spec = filt.device_spec(sim)
    assert spec["families"] == [(0, 60)]
    cen, radius = spec["sphere"]
    assert radius == 1.5 and np.array_equal(cen, np.zeros(3))
    host = np.asarray(filt(sim))
    r2 = (pos[:, 0] ** 2 + pos[:, 1] ** 2) + pos[:, 2] ** 2
    want = (r2 < 1.5 ** 2) & (np.arange(100) < 60)
    assert np.array_equal(host, want)


def test_family_filter_index_subsnap():
    """Index-list sub-snapshots: increasing indices keep a family range;
    a shuffled view falls back to the host mask (no device range)."""
    n = 50
    sim = SimSnap({"pos": np.random.default_rng(2).normal(size=(n, 3)), "mass": np.ones(n)},
                  families={"dm": slice(0, 20), "star": slice(20, 50)})
    sub = sim[np.array([3, 7, 19, 20, 33, 49])]
    f = FamilyFilter("star")
    assert np.array_equal(f.build_mask(sub), [False, False, False, True, True, True])
    assert f.device_spec(sub) == {"families": [(3, 6)]}
    shuffled = sim[np.array([33, 3, 49, 7, 20])]
    assert np.array_equal(f.build_mask(shuffled), [True, False, True, False, True])
    assert f.device_spec(shuffled) is None


def test_subsnap_pending_fields():
    """A view's device-held field (SubSnap._pending, the fused builder's r /
    rxy and kept masses) is fetched once, on the first host read, and gives
    what the read returns; PendingField carries length and units without the
    copy; assigning the field drops the pending fetch."""
    from pynbodyext.simcore import PendingField, SubSnap, is_pending

    rng = np.random.default_rng(3)
    pos = rng.normal(size=(50, 3))
    sim = SimSnap({"pos": pos, "mass": rng.random(50)}, families={"dm": slice(0, 50)},
                  units_map={"pos": "kpc", "mass": "Msol"})
    idx = np.arange(0, 50, 3)
    sub = SubSnap(sim, idx, increasing=True)
    calls = []
    r_true = np.sqrt((pos[idx, 0] ** 2 + pos[idx, 1] ** 2) + pos[idx, 2] ** 2)
    sub._pending["r"] = lambda: calls.append("r") or r_true.copy()
    assert is_pending(sub, "r") and not is_pending(sub, "mass")
    pf = PendingField(sub, "r")
    assert len(pf) == len(idx) and str(pf.units) == str(sim["pos"].units) and not calls
    r = pf.resolve()
    assert calls == ["r"] and np.array_equal(np.asarray(r), r_true)
    assert str(r.units) == str(sim["pos"].units) and r.sim is sub
    assert np.array_equal(np.asarray(sub["r"]), r_true) and calls == ["r"]  # fetched once
    assert not is_pending(sub, "r")
    sub._pending["mass"] = lambda: calls.append("mass") or np.zeros(len(idx))
    sub["mass"] = np.ones(len(idx))  # an assignment wins over the pending fetch
    assert not is_pending(sub, "mass") and np.array_equal(np.asarray(sub["mass"]), np.ones(len(idx)))
    assert calls == ["r"]
