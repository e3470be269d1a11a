"""Pin the Barnes–Hut oracle (oracle/tree_ref.c) — CPU only.

The reference holds no golden vectors for the tree, so the restatement is
pinned by re-running the reference's own Rust integration tests on it
(crates/gravity/tests/gravity_tests.rs:57-202, single_node.rs:20-109,
translate_multipole.rs:5-113; same sizes, thresholds and tolerances, numpy
point sets in place of rand's StdRng) plus structural invariants of the
octree that tree.rs:628-864 implies.
"""
import numpy as np
import pytest

from oracle import gravity as og
from oracle import tree as ot


def gen_points(seed, n):
    """gravity_tests.rs:3-14: uniform in [-0.5, 0.5)^3."""
    return np.random.default_rng(seed).random((n, 3)) - 0.5


def gen_masses(seed, n):
    """gravity_tests.rs:16-20: 0.5 + U[0,1)."""
    return 0.5 + np.random.default_rng(seed).random(n)


def rms(a, b):
    d = np.asarray(a) - np.asarray(b)
    return np.sqrt((d * d).reshape(len(d), -1).sum(axis=1).mean())


# --- gravity_tests.rs -----------------------------------------------------
def test_accelerations_match_direct_small_n():
    n = 256
    pts, masses = gen_points(1, n), gen_masses(2, n)
    tree = ot.RefOctree(pts, masses, 32, 2, tree3d=True)
    acc_tree = tree.compute_accelerations(0.0)
    acc_direct = og.direct_accelerations(pts, masses)
    assert np.abs(acc_tree - acc_direct).max() < 1e-10


def test_potentials_match_direct_small_n():
    n = 256
    pts, masses = gen_points(3, n), gen_masses(4, n)
    tree = ot.RefOctree(pts, masses, 32, 2, tree3d=True)
    pot_tree = tree.compute_potentials(0.0)
    pot_direct = og.direct_potentials(pts, masses)
    assert np.abs(pot_tree - pot_direct).max() < 1e-10


def test_queries_match_direct_at_points():
    src, masses, queries = gen_points(11, 512), gen_masses(12, 512), gen_points(13, 128)
    tree = ot.RefOctree(src, masses, 32, 2, tree3d=True)
    acc_tree = tree.accelerations_at_points(queries, 0.0)
    pot_tree = tree.potentials_at_points(queries, 0.0)
    acc_d = og.direct_accelerations_at_points(src, queries, masses)
    pot_d = og.direct_potentials_at_points(src, queries, masses)
    assert np.abs(acc_tree - acc_d).max() < 1e-10
    assert np.abs(pot_tree - pot_d).max() < 1e-10


def test_error_decreases_with_multipole_order_accel():
    n, theta = 800, 0.7
    pts, masses = gen_points(21, n), gen_masses(22, n)
    acc_ref = og.direct_accelerations(pts, masses)
    errs = []
    for order in (0, 3, 4, 5):
        tree = ot.RefOctree(pts, masses, 64, order, tree3d=True)
        errs.append(rms(tree.compute_accelerations(theta), acc_ref))
    assert all(errs[i] <= errs[i - 1] for i in range(1, len(errs))), errs
    assert errs[-1] <= errs[0] * 0.8, errs


def test_error_decreases_with_multipole_order_potential():
    n, theta = 800, 0.7
    pts, masses = gen_points(31, n), gen_masses(32, n)
    pot_ref = og.direct_potentials(pts, masses)
    errs = []
    for order in (0, 2, 3, 4, 5):
        tree = ot.RefOctree(pts, masses, 64, order, tree3d=True)
        errs.append(rms(tree.compute_potentials(theta), pot_ref))
    assert all(errs[i] <= errs[i - 1] for i in range(1, len(errs))), errs


# --- single_node.rs -------------------------------------------------------
def test_single_node_multipole_vs_direct():
    rng = np.random.default_rng(5)
    n = 4000
    positions = rng.uniform(-0.1, 0.1, (n, 3))
    masses = rng.uniform(0.1, 1.0, n)
    com = (positions * masses[:, None]).sum(axis=0) / masses.sum()
    mom = ot.multipole_from_points(positions, masses, com, 5)
    errs = {o: [] for o in range(6)}
    for _ in range(400):
        while True:
            v = rng.uniform(-1.0, 1.0, 3)
            r2 = v @ v
            if 1e-6 < r2 <= 1.0:
                break
        v /= np.sqrt(v @ v)
        target = com + rng.uniform(20.0, 30.0) * v
        d = positions - target
        phi_direct = -(masses / np.sqrt((d * d).sum(axis=1))).sum()
        dx, dy, dz = com - target
        D = ot.potential_derivatives(dx, dy, dz, 0.0, 5)
        for o in range(6):
            phi = ot.gravity_potential_multipole(mom, D, o)
            errs[o].append(abs((phi - phi_direct) / phi_direct))
    for o in range(6):
        e = np.sort(errs[o])
        assert e[min(int(len(e) * 0.9), len(e) - 1)] < 1e-2
    # the expansion converges: each order at least as good (p90) as monopole
    assert np.percentile(errs[5], 90) < np.percentile(errs[0], 90)


# --- translate_multipole.rs ----------------------------------------------
def test_translate_vs_direct():
    rng = np.random.default_rng(17)
    n = 200
    positions = rng.random((n, 3))
    masses = rng.random(n)
    center_b = np.array([0.3, 0.4, 0.5])
    center_a = np.array([0.8, -0.2, 0.1])
    m_b = ot.multipole_from_points(positions, masses, center_b, 5)
    m_trans = ot.translate_multipole(m_b, center_a - center_b, 5)
    m_direct = ot.multipole_from_points(positions, masses, center_a, 5)
    assert np.abs(m_trans - m_direct).max() <= 1e-10


# --- known answers / structural invariants of tree.rs ---------------------
def test_multipole_known_answer_two_points():
    pos = np.array([[1.0, 0.0, 0.0], [-1.0, 0.0, 0.0]])
    m = ot.multipole_from_points(pos, np.array([1.0, 1.0]), np.zeros(3), 5)
    assert m[0] == 2.0                  # m000
    assert m[1] == 0.0                  # m100
    assert m[4] == 1.0                  # m200 = 1/2 * sum x^2
    assert m[20] == pytest.approx(2.0 / 24.0)  # m400


def test_derivatives_match_finite_difference():
    dx, dy, dz = 0.7, -1.3, 2.1
    D = ot.potential_derivatives(dx, dy, dz, 0.0, 5)
    f = lambda x, y, z: 1.0 / np.sqrt(x * x + y * y + z * z)
    h = 1e-5
    assert D[0] == pytest.approx(f(dx, dy, dz), rel=1e-14)
    assert D[1] == pytest.approx((f(dx + h, dy, dz) - f(dx - h, dy, dz)) / (2 * h), rel=1e-8)
    fx = lambda x, y, z: (f(x + h, y, z) - f(x - h, y, z)) / (2 * h)
    assert D[7] == pytest.approx((fx(dx, dy + h, dz) - fx(dx, dy - h, dz)) / (2 * h), rel=1e-5)


def _check_structure(tree, pos, leaf_capacity):
    e = tree.export()
    nn = tree.num_nodes
    first, nxt = e["first"], e["next"]
    leaf = e["leaf_off"] >= 0
    # every particle appears in exactly one leaf
    assert np.array_equal(np.sort(e["perm"]), np.arange(len(pos)))
    assert e["leaf_len"][leaf].sum() == len(pos)
    # leaf lists are ascending (Rust bucket push order, tree.rs:815-828)
    for k in np.flatnonzero(leaf):
        ids = e["perm"][e["leaf_off"][k]:e["leaf_off"][k] + e["leaf_len"][k]]
        assert np.all(np.diff(ids) > 0)
        assert len(ids) <= leaf_capacity or np.all(pos[ids] == pos[ids[0]])
        # contained in the node's cube
        c, hh = e["center"][k], e["half"][k]
        assert np.all(np.abs(pos[ids] - c) <= hh * (1 + 1e-12))
    # the threaded walk with theta=0 visits every node once, in DFS preorder
    seen, k = [], 0
    while k != -1:
        seen.append(k)
        k = first[k] if first[k] != -1 else nxt[k]
    assert sorted(seen) == list(range(nn))
    assert np.all(e["size2"] == (2 * e["half"]) ** 2)
    return e


@pytest.mark.parametrize("leaf", [1, 8, 32])
def test_octree_structure(leaf):
    pos = gen_points(41, 3000)
    tree = ot.RefOctree(pos, gen_masses(42, 3000), leaf, 3)
    e = _check_structure(tree, pos, leaf)
    # root: cubic bbox centred at the midpoint of min/max (tree.rs:628-654)
    assert np.array_equal(e["center"][0], (pos.min(0) + pos.max(0)) / 2.0)
    assert e["half"][0] == ((pos.max(0) - pos.min(0)) / 2.0).max()
    # BH payload: root mass = total mass
    assert e["mass"][0] == pytest.approx(gen_masses(42, 3000).sum(), rel=1e-14)


def test_octree_coincident_particles_terminate():
    # tree.rs recurses forever here; both oracle and product stop splitting.
    pos = np.zeros((40, 3))
    pos[20:] = 1.0
    tree = ot.RefOctree(pos, np.ones(40), 8, 3)
    _check_structure(tree, pos, 8)
    pot = tree.compute_potentials(0.5)
    # coincident pairs contribute -m/sqrt(R2_TINY) ~ -6.7e153, finite as in direct.rs
    assert np.all(np.isfinite(pot)) and np.all(pot < -1e150)


def test_payload_requires_build_mass():
    tree = ot.RefOctree(gen_points(1, 100))
    with pytest.raises(ValueError, match="build_mass"):
        tree.compute_potentials(0.5)
    tree.build_mass()
    pot = tree.compute_potentials(0.0)
    np.testing.assert_allclose(pot, og.direct_potentials(gen_points(1, 100)), rtol=1e-12)


@pytest.mark.parametrize("kernel", [0, 1])
def test_softened_tree_theta0_matches_direct_kernel(kernel):
    n = 600
    pos, m = gen_points(51, n), gen_masses(52, n)
    h = 0.01 + 0.05 * np.random.default_rng(53).random(n)
    tree = ot.RefOctree(pos, m, 16, 3, softenings=h, kernel=kernel)
    pot = tree.compute_potentials(0.0)
    acc = tree.compute_accelerations(0.0)
    np.testing.assert_allclose(pot, og.direct_potentials(pos, m, h, kernel), rtol=1e-11)
    np.testing.assert_allclose(acc, og.direct_accelerations(pos, m, h, kernel), rtol=1e-9,
                               atol=1e-10)


def test_subset_equals_full():
    n = 2000
    pos, m = gen_points(61, n), gen_masses(62, n)
    tree = ot.RefOctree(pos, m, 8, 3)
    pot = tree.compute_potentials(0.5)
    acc = tree.compute_accelerations(0.5)
    idx = np.array([0, 5, 1999, 777])
    p, a, nn, npp = tree.compute_subset(idx, 0.5)
    assert np.array_equal(p, pot[idx]) and np.array_equal(a, acc[idx])
    assert np.all(nn > 0) and np.all(npp > 0)
