"""Pin the profile oracle (oracle/profile_ref.py) against the golden fixtures
produced by the reference's own bins.py / proarray.py (tests/golden/).

Edges, counts and bin membership are compared bit-for-bit; statistics too
(the restatement evaluates the same numpy expressions on the same arrays).
"""
import hashlib
from pathlib import Path

import numpy as np
import pytest

from oracle import profile_ref as pr

GOLD = Path(__file__).resolve().parent / "golden"


def plummer_r(n, seed):
    rng = np.random.default_rng(seed)
    x = rng.random(n)
    return np.minimum((x ** (-2.0 / 3.0) - 1.0) ** -0.5, 50.0)


def load_dataset(n):
    g = np.load(GOLD / f"profile_n{n}.npz")
    if "x" in g:
        x, w, f = g["x"], g["w"], g["f"]
    else:
        seed = int(g["seed"])
        x = plummer_r(n, seed)
        rng = np.random.default_rng(seed + 1)
        w = rng.uniform(0.5, 1.5, n)
        f = rng.normal(size=n)
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["x_sha256"])
    return g, x, w, f


CASES = [(bt, nb, None, None, f"{bt}_{nb}") for bt in ("lin", "log", "equaln") for nb in (8, 128, 256)]
CASES += [("equaln", 100, 0.05, 20.0, "equaln_100_clip"), ("lin", 64, 0.1, 5.0, "lin_64_range"),
          ("log", 256, 0.01, 50.0, "log_256_range")]


@pytest.mark.parametrize("n", [1000, 10000, 100000])
@pytest.mark.parametrize("bins_type,nb,lo,hi,tag", CASES)
def test_edges_and_assignment(n, bins_type, nb, lo, hi, tag):
    g, x, w, f = load_dataset(n)
    edges = pr.EDGE_ALGORITHMS[bins_type](x, nb, lo, hi)
    assert np.array_equal(edges, g[f"{tag}/edges"])
    perm, offsets, counts = pr.assign(x, edges)
    assert np.array_equal(counts, g[f"{tag}/counts"])
    if f"{tag}/perm" in g:
        assert np.array_equal(perm, g[f"{tag}/perm"])
    lists = pr.binind_lists(perm, offsets)
    assert np.array_equal([int(b.sum()) for b in lists], g[f"{tag}/idx_sum"])
    assert np.array_equal([int((b ** 2).sum()) for b in lists], g[f"{tag}/idx_sq"])
    assert np.array_equal([int(b[0]) if len(b) else -1 for b in lists], g[f"{tag}/idx_first"])
    assert np.array_equal([int(b[-1]) if len(b) else -1 for b in lists], g[f"{tag}/idx_last"])


STATS = ["mean", "sum", "sum_w", "rms", "disp", "p16", "p50", "median", "abs_mean", "abs_sum",
         "abs_p84"]


@pytest.mark.parametrize("n", [1000, 10000, 100000])
@pytest.mark.parametrize("tag,bins_type,nb,lo,hi", [("lin_128", "lin", 128, None, None),
                                                    ("log_128", "log", 128, None, None),
                                                    ("equaln_128", "equaln", 128, None, None),
                                                    ("lin_64_range", "lin", 64, 0.1, 5.0)])
def test_statistics(n, tag, bins_type, nb, lo, hi):
    import warnings

    g, x, w, f = load_dataset(n)
    edges = pr.EDGE_ALGORITHMS[bins_type](x, nb, lo, hi)
    perm, offsets, _ = pr.assign(x, edges)
    for wname, weights in (("w", w), ("none", None)):
        for key in STATS:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", RuntimeWarning)
                vals, canon = pr.compute(f, weights, perm, offsets, key)
            assert canon == str(g[f"{tag}/statkey/{key}"])
            assert np.array_equal(vals, g[f"{tag}/stat/{wname}/{key}"], equal_nan=True), (wname, key)


def test_edge_cases():
    g = np.load(GOLD / "profile_edge_cases.npz")
    for name in ("on_edges", "dup_edges", "all_dropped", "single_bin", "empty_x", "neg_values"):
        x, edges = g[f"{name}/x"], g[f"{name}/edges"]
        perm, offsets, counts = pr.assign(x, edges)
        assert np.array_equal(counts, g[f"{name}/counts"]), name
        assert np.array_equal(perm, g[f"{name}/perm"]), name
        assert np.array_equal(offsets, g[f"{name}/offsets"]), name
    for name in ("eq_degenerate", "eq_clip", "eq_dups", "eq_with_nan", "eq_clip_nan"):
        lo, hi = float(g[f"{name}/bin_min"]), float(g[f"{name}/bin_max"])
        edges = pr.edges_equaln(g[f"{name}/x"], int(g[f"{name}/nb"]),
                                None if np.isnan(lo) else lo, None if np.isnan(hi) else hi)
        assert np.array_equal(edges, g[f"{name}/edges"], equal_nan=True), name
    with pytest.raises(ValueError) as e:
        pr.edges_log(np.array([0.0, 1.0]), 4)
    assert str(e.value) == str(g["log_error/message"])


SPATIAL = np.load(GOLD / "profile_spatial.npz")


@pytest.mark.parametrize("tag,bt,nb,lo,hi", [("lin_64", "lin", 64, None, None),
                                             ("log_64", "log", 64, 0.05, 15.0),
                                             ("equaln_100", "equaln", 100, None, None)])
def test_oracle_annulus_fixture(tag, bt, nb, lo, hi):
    """ndim=2 (rxy, annulus areas, bins.py:759-765) against the reference."""
    pos, mass = SPATIAL["ann/pos"], SPATIAL["ann/mass"]
    rxy = np.sqrt(pos[:, 0] * pos[:, 0] + pos[:, 1] * pos[:, 1])
    edges = pr.EDGE_ALGORITHMS[bt](rxy, nb, lo, hi)
    assert np.array_equal(edges, SPATIAL[f"ann/{tag}/edges"])
    perm, offsets, counts = pr.assign(rxy, edges)
    assert np.array_equal(counts, SPATIAL[f"ann/{tag}/counts"])
    assert np.array_equal(perm, SPATIAL[f"ann/{tag}/perm"])
    assert np.array_equal(pr.area_annulus(edges), SPATIAL[f"ann/{tag}/area"])
    msum, _ = pr.compute(mass, mass, perm, offsets, "sum")
    assert np.array_equal(msum, SPATIAL[f"ann/{tag}/mass_sum"], equal_nan=True)


def test_oracle_float32_fixture():
    """A float32 snapshot: numpy's dtype rules (float64 Sphere distance,
    float32 r) and the reference's binning of the float32 r array."""
    pos, mass = SPATIAL["f32/pos"], SPATIAL["f32/mass"]
    lo, hi = (int(v) for v in SPATIAL["f32/fam"])
    mask = pr.sphere_mask(pos, float(SPATIAL["f32/radius"]), SPATIAL["f32/cen"])
    mask[hi:] = False
    mask[:lo] = False
    kept = np.nonzero(mask)[0]
    assert np.array_equal(kept, SPATIAL["f32/kept"])
    r = pr.radial_r(pos[kept])
    assert r.dtype == np.float32 and np.array_equal(r, SPATIAL["f32/r"])
    edges = pr.edges_equaln(r, 128)
    assert edges.dtype == np.float32 and np.array_equal(edges, SPATIAL["f32/edges"])
    perm, offsets, counts = pr.assign(r, edges)
    assert np.array_equal(counts, SPATIAL["f32/counts"])
    assert np.array_equal(perm, SPATIAL["f32/perm"])
    msum, _ = pr.compute(mass[kept], mass[kept], perm, offsets, "sum")
    assert np.array_equal(msum, SPATIAL["f32/mass_sum"], equal_nan=True)
