"""GPU parity of the Barnes–Hut octree (csrc/tree.hip) against the oracle
restatement of tree.rs / multipole.rs (oracle/tree_ref.c).

What is checked, per case:
  * geometry: the device tree equals the reference tree node for node in
    DFS order — bit-exact centres/half sizes, identical leaf index lists
    (ascending), bit-exact BH payload (mass, COM) and h_max;
  * moments: multipole moments within 1e-12 of the oracle's (P2M/M2M are
    computed with different (binomial) formulas);
  * decisions: the accepted-node and leaf-pair totals of the walk equal the
    oracle's, i.e. every target made the reference's opening decisions;
  * values: per particle |dphi|/|phi| <= 1e-5 and ||da||/||a|| <= 1e-5 (the
    contract), plus a tight 1e-9 bound (decisions identical => only
    rounding differs).
"""
import numpy as np
import pytest

from oracle import gravity as og
from oracle import tree as ot
from pynbodyext import _engine
from pynbodyext.gravity import Gravity
from pynbodyext.synthetic import plummer

pytestmark = pytest.mark.gpu

TOL = 1e-5
TIGHT = 1e-9     # precise mode (Newton-refined 1/sqrt): the oracle to rounding
FAST = 2e-6      # default fast mode (raw v_rsq_f64, ~5e-8 per interaction)
NCOEF = {2: 10, 3: 20, 4: 35, 5: 56}


@pytest.fixture(autouse=True)
def _precise(request):
    """Decision/value parity tests run the precise walk; the tests marked
    ``fast`` run the default fast mode against the same oracle."""
    from pynbodyext import _native as nat

    with nat.precise_mode("fast" not in request.keywords):
        yield


def rel_pot(a, b):
    return float(np.max(np.abs(a - b) / np.abs(b))) if len(b) else 0.0


def rel_acc(a, b):
    if not len(b):
        return 0.0
    return float(np.max(np.linalg.norm(a - b, axis=1) / np.linalg.norm(b, axis=1)))


def preorder(first, nxt):
    out, k = [], 0
    while k != -1:
        out.append(k)
        k = first[k] if first[k] != -1 else nxt[k]
    return np.array(out, dtype=np.int64)


def check_structure(dev: _engine.Octree, ref: ot.RefOctree, order: int, masses=True):
    d, r = dev.export(), ref.export()
    do = preorder(d["links"][:, 0], d["links"][:, 1])
    ro = preorder(r["first"], r["next"])
    assert len(do) == len(ro) == dev.info()["nodes"] == ref.num_nodes
    assert np.array_equal(d["center"][do, :3], r["center"][ro])
    assert np.array_equal(d["center"][do, 3], r["half"][ro])
    dleaf = d["links"][do, 0] == -1
    rleaf = r["leaf_off"][ro] >= 0
    assert np.array_equal(dleaf, rleaf)
    for a, b in zip(do[dleaf], ro[rleaf]):
        s, c = d["leaf"][a]
        ids_d = d["perm"][s:s + c]
        ids_r = r["perm"][r["leaf_off"][b]:r["leaf_off"][b] + r["leaf_len"][b]]
        assert np.array_equal(ids_d, ids_r)
    if d["com"] is not None:
        assert np.array_equal(d["com"][do, 3], r["mass"][ro])
        assert np.array_equal(d["com"][do, :3], r["com"][ro])
    if r["hmax"] is not None:
        assert np.array_equal(d["hmax"][do], r["hmax"][ro])
    P = min(order, 5)
    if P >= 2 and d["com"] is not None:
        md = dev.export_moments(NCOEF[P])[do]
        mr = r["mom"][ro][:, :NCOEF[P]]
        # each moment is a sum of products of masses and |x|^k: scale by the
        # node's mass * size^k
        size = (2 * r["half"][ro])[:, None]
        deg = np.array([[0, 1, 1, 1, 2, 2, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3] + [4] * 15 +
                        [5] * 21][0][:NCOEF[P]])
        scale = np.abs(r["mass"][ro])[:, None] * size ** deg[None, :] + 1e-300
        assert np.max(np.abs(md - mr) / scale) < 1e-12


def check_walk(dev, ref, theta, n, tight=TIGHT):
    pot_d = dev.compute_potentials(theta)
    cnt_d = dev.info()
    acc_d = dev.compute_accelerations(theta)
    pot_r, acc_r, nn_r, np_r = ref.compute_subset(np.arange(n), theta)
    assert cnt_d["node_interactions"] == int(nn_r.sum())
    assert cnt_d["leaf_pairs"] == int(np_r.sum())
    rp, ra = rel_pot(pot_d, pot_r), rel_acc(acc_d, acc_r)
    assert rp < TOL and ra < TOL
    assert rp < tight and ra < tight, (rp, ra)


def uniform(n, seed):
    return np.random.default_rng(seed).random((n, 3)) - 0.5


@pytest.mark.parametrize("order", [0, 1, 2, 3, 4, 5])
def test_plummer_orders(gpu, order):
    pos, mass = plummer(20_000, seed=70 + order)
    dev = _engine.Octree(pos, mass, 8, order)
    ref = ot.RefOctree(pos, mass, 8, order)
    check_structure(dev, ref, order)
    check_walk(dev, ref, 0.5, len(pos))


def test_zero_mass_subtrees(gpu):
    """Empty nodes (mass 0) are skipped (tree.rs:1087-1090): a region of
    zero-mass particles (whole empty subtrees) and scattered zero masses —
    the oracle's structure, opening decisions and values."""
    pos, mass = plummer(20_000, seed=77)
    mass = mass.copy()
    mass[pos[:, 0] > 0.3] = 0.0
    mass[::7] = 0.0
    dev = _engine.Octree(pos, mass, 8, 3)
    ref = ot.RefOctree(pos, mass, 8, 3)
    check_structure(dev, ref, 3)
    check_walk(dev, ref, 0.5, len(pos))
    q = plummer(2000, seed=78)[0] * 1.2
    assert rel_pot(dev.potentials_at_points(q, 0.5), ref.potentials_at_points(q, 0.5)) < TIGHT


@pytest.mark.parametrize("leaf", [1, 3, 32, 100])
def test_leaf_capacities(gpu, leaf):
    pos = uniform(6000, leaf)
    mass = 0.5 + np.random.default_rng(leaf).random(6000)
    dev = _engine.Octree(pos, mass, leaf, 3)
    ref = ot.RefOctree(pos, mass, leaf, 3)
    check_structure(dev, ref, 3)
    check_walk(dev, ref, 0.7, len(pos))


def test_unit_masses_build_mass_later(gpu):
    pos = uniform(5000, 9)
    dev = _engine.Octree(pos, None, 16, 2)
    with pytest.raises(ValueError, match="call build_mass\\(\\) before compute_potentials"):
        dev.compute_potentials(0.5)
    with pytest.raises(ValueError, match="before accelerations_at_points"):
        dev.accelerations_at_points(pos[:3].copy(), 0.5)
    dev.build_mass()
    ref = ot.RefOctree(pos, None, 16, 2, tree3d=True)
    check_structure(dev, ref, 2)
    check_walk(dev, ref, 0.6, len(pos))
    # new masses through build_mass(masses)
    m2 = np.random.default_rng(3).random(5000)
    dev.build_mass(m2)
    ref.build_mass(m2)
    check_structure(dev, ref, 2)
    check_walk(dev, ref, 0.6, len(pos))


@pytest.mark.parametrize("kernel", [0, 1])
def test_softened(gpu, kernel):
    pos, mass = plummer(12_000, seed=11)
    h = 0.005 + 0.02 * np.random.default_rng(12).random(len(pos))
    dev = _engine.Octree(pos, mass, 8, 3, h, kernel)
    ref = ot.RefOctree(pos, mass, 8, 3, softenings=h, kernel=kernel)
    check_structure(dev, ref, 3)
    check_walk(dev, ref, 0.5, len(pos))
    # set_kernel keeps h_max, changes the kernel (tree.rs:784-786)
    dev.set_kernel(1 - kernel)
    ref.set_kernel(1 - kernel)
    check_walk(dev, ref, 0.5, len(pos))
    # set_softenings(None) keeps the build-time h_max guard (tree.rs:777-782)
    dev.set_softenings(None)
    ref.set_softenings(None)
    check_walk(dev, ref, 0.5, len(pos))
    # and new softenings without a rebuild
    h2 = 0.5 * h
    dev.set_softenings(h2)
    ref.set_softenings(h2)
    check_walk(dev, ref, 0.5, len(pos))


def test_at_points(gpu):
    pos, mass = plummer(15_000, seed=21)
    q = plummer(3000, seed=22)[0] * 1.3
    q[:10] = pos[:10]  # coincident with particles: no self skip at points
    dev = _engine.Octree(pos, mass, 8, 3)
    ref = ot.RefOctree(pos, mass, 8, 3)
    pd, pr = dev.potentials_at_points(q, 0.5), ref.potentials_at_points(q, 0.5)
    ad, ar = dev.accelerations_at_points(q, 0.5), ref.accelerations_at_points(q, 0.5)
    finite = np.arange(len(q)) >= 10
    assert rel_pot(pd[finite], pr[finite]) < TIGHT
    assert rel_acc(ad[finite], ar[finite]) < TIGHT
    # coincident: -m/sqrt(R2_TINY) ~ -6.7e153 m dominates the potential and the
    # force term is (m*0)*inf = NaN, in the reference (tree.rs:313-318) as here
    assert np.all(pd[:10] < -1e140) and np.allclose(pd[:10], pr[:10], rtol=1e-9)
    assert np.array_equal(np.isnan(ad[:10]), np.isnan(ar[:10]))


def test_theta0_equals_direct(gpu):
    pos, mass = plummer(3000, seed=31)
    dev = _engine.Octree(pos, mass, 8, 3)
    assert rel_pot(dev.compute_potentials(0.0), og.direct_potentials(pos, mass)) < 1e-12
    assert rel_acc(dev.compute_accelerations(0.0), og.direct_accelerations(pos, mass)) < 1e-12


@pytest.mark.parametrize("n", [0, 1, 2, 8, 9])
def test_small_n(gpu, n):
    pos = uniform(n, 40 + n)
    mass = np.ones(n)
    dev = _engine.Octree(pos, mass, 8, 3)
    pot = dev.compute_potentials(0.5)
    acc = dev.compute_accelerations(0.5)
    assert pot.shape == (n,) and acc.shape == (n, 3)
    if n >= 2:
        ref = ot.RefOctree(pos, mass, 8, 3)
        check_structure(dev, ref, 3)
        check_walk(dev, ref, 0.5, n)
    elif n == 1:
        assert pot.tolist() == [0.0] and acc.tolist() == [[0.0, 0.0, 0.0]]
    assert dev.potentials_at_points(np.zeros((2, 3)), 0.5).shape == (2,)


def test_coincident_cluster(gpu):
    # 30 particles on one point (> leaf capacity): the reference recurses
    # forever; oracle and device both stop splitting there.
    pos = uniform(2000, 50)
    pos[100:130] = pos[100]
    mass = np.ones(2000)
    dev = _engine.Octree(pos, mass, 8, 3)
    ref = ot.RefOctree(pos, mass, 8, 3)
    check_structure(dev, ref, 3)
    pd, pr = dev.compute_potentials(0.5), ref.compute_potentials(0.5)
    assert rel_pot(pd, pr) < TIGHT


def test_deep_tree_needs_more_path_words(gpu):
    # two clusters 1e-14 apart at O(1) coordinates: > 42 levels
    pos = uniform(400, 60)
    pos[:20] = 0.25 + 1e-15 * np.arange(20)[:, None]
    mass = np.ones(400)
    dev = _engine.Octree(pos, mass, 4, 3)
    ref = ot.RefOctree(pos, mass, 4, 3)
    assert dev.info()["path_words"] >= 3
    check_structure(dev, ref, 3)
    assert rel_pot(dev.compute_potentials(0.5), ref.compute_potentials(0.5)) < TIGHT


@pytest.mark.parametrize("case", ["two_scale", "dup_pairs", "cap64", "cap1", "lattice", "line"])
def test_structure_varied(gpu, case):
    """The parallel structure build from the sorted paths (bp_* kernels) —
    or its level-synchronous fallback — equals the reference tree node for
    node on inputs that stress the split rule: a deep nested cluster (two
    path words), duplicate pairs below the capacity, large and unit
    capacities, particles exactly on octant boundaries, a degenerate line."""
    rng = np.random.default_rng(91)
    leaf = 8
    if case == "two_scale":
        pos = uniform(30_000, 3)
        pos[:10_000] = 0.1 + 1e-7 * (rng.random((10_000, 3)) - 0.5)
    elif case == "dup_pairs":
        pos = np.repeat(uniform(3000, 4), 2, axis=0)
        rng.shuffle(pos)
    elif case == "cap64":
        pos, _ = plummer(20_000, seed=5)
        leaf = 64
    elif case == "cap1":
        pos = uniform(3000, 6)
        leaf = 1
    elif case == "lattice":
        g = np.arange(16) / 8.0 - 1.0
        pos = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3).copy()
    else:  # all on one axis
        pos = np.zeros((5000, 3))
        pos[:, 0] = rng.random(5000)
    mass = 0.5 + rng.random(len(pos))
    dev = _engine.Octree(pos, mass, leaf, 3)
    ref = ot.RefOctree(pos, mass, leaf, 3)
    check_structure(dev, ref, 3)
    if case == "dup_pairs":  # coincident pairs: 0 * inf accelerations (NaN) on both sides
        pd, pr_ = dev.compute_potentials(0.6), ref.compute_potentials(0.6)
        assert rel_pot(pd, pr_) < TIGHT
        ad, ar = dev.compute_accelerations(0.6), ref.compute_accelerations(0.6)
        assert np.array_equal(np.isnan(ad), np.isnan(ar))
        return
    # a 1e-7 cluster inside a unit box: its moments cancel (binomial M2M vs
    # the reference's recurrences differ by rounding), 1e-8 on accelerations
    check_walk(dev, ref, 0.6, len(pos), tight=1e-7 if case == "two_scale" else TIGHT)


def test_errors(gpu):
    pos = uniform(10, 1)
    with pytest.raises(ValueError, match="masses must be length N"):
        _engine.Octree(pos, np.ones(3))
    with pytest.raises(ValueError, match="softenings require an explicit kernel"):
        _engine.Octree(pos, np.ones(10), 8, 3, np.ones(10))
    with pytest.raises(ValueError, match="kernel must be 0"):
        _engine.Octree(pos, np.ones(10), 8, 3, None, 2)
    with pytest.raises(TypeError):
        _engine.Octree(pos.astype(np.float32))
    with pytest.raises(OverflowError):
        _engine.Octree(pos, None, 8, 300)
    t = _engine.Octree(pos, np.ones(10))
    with pytest.raises(ValueError, match="points must be \\(N,3\\) float64 array"):
        t.potentials_at_points(np.zeros(4).reshape(2, 2), 0.5)


def test_gravity_front_end(gpu):
    pos, mass = plummer(8000, seed=81)
    g = Gravity(pos, mass)
    pot = g.tree_potentials(theta=0.5)
    acc = g.tree_accelerations(theta=0.5)
    ref = ot.RefOctree(pos, mass, 8, 3)  # TreeOptions defaults (base.py:82-100)
    assert rel_pot(pot, ref.compute_potentials(0.5)) < TIGHT
    assert rel_acc(acc, ref.compute_accelerations(0.5)) < TIGHT


def test_1m_subset(gpu):
    """1M Plummer, theta 0.5, leaf 8, order 3: full structure + 8192 targets."""
    pos, mass = plummer(1_000_000, seed=1002)
    dev = _engine.Octree(pos, mass, 8, 3)
    ref = ot.RefOctree(pos, mass, 8, 3)
    check_structure(dev, ref, 3)
    pot = dev.compute_potentials(0.5)
    acc = dev.compute_accelerations(0.5)
    idx = np.random.default_rng(0).choice(len(pos), 8192, replace=False)
    idx = np.concatenate([idx, np.argsort((pos * pos).sum(1))[:64]])
    pr, ar, _, _ = ref.compute_subset(idx, 0.5)
    assert rel_pot(pot[idx], pr) < TIGHT and rel_acc(acc[idx], ar) < TIGHT


def test_range_walk_shards_equal_full(gpu):
    """Multi-GPU shard path on one GPU: 3 cost-balanced leaf-order ranges
    (compact outputs) reassemble the full compute_*; costs add up to the
    interaction counters; profile partials add up to the full profile."""
    from pynbodyext import _native as nat
    from pynbodyext.parallel import balanced_ranges
    from pynbodyext.profiles._device import SRC_W, DeviceBins

    n = 30_000
    pos, mass = plummer(n, seed=97)
    dev = _engine.Octree(pos, mass, 8, 3)
    pot_full = dev.compute_potentials(0.5)
    acc_full = dev.compute_accelerations(0.5)
    totals = dev.info()
    d_pot, d_acc = nat.DeviceArray(8 * n), nat.DeviceArray(24 * n)
    d_cost, d_idx = nat.DeviceArray(4 * n), nat.DeviceArray(8 * n)
    dev._compute_range_device(0.5, nat.WANT_POT, 0, n, 1, d_pot.ptr, None, d_cost.ptr)
    cost = np.empty(n, dtype=np.int32)
    d_cost.download(cost)
    assert int(cost.astype(np.int64).sum()) == totals["node_interactions"] + totals["leaf_pairs"]
    order = np.empty(n, dtype=np.int64)
    dev._leaf_particles_device(0, n, None, None, d_idx.ptr)
    d_idx.download(order)
    assert np.array_equal(np.sort(order), np.arange(n))
    edges = np.logspace(np.log10(0.01), np.log10(50.0), 65)
    full = DeviceBins.select(pos, mass, ndim=3)
    full.assign(edges)
    mom_full = full.moments(pot_full, SRC_W)
    mom_sum = np.zeros_like(mom_full)
    mom_fused = np.zeros_like(mom_full)
    d_spos, d_smass = nat.DeviceArray(24 * n), nat.DeviceArray(8 * n)
    for first, count in balanced_ranges(cost, 3):
        dev._compute_range_device(0.5, nat.WANT_POT | nat.WANT_ACC, first, count, 1, d_pot.ptr,
                                  d_acc.ptr, None)
        p = np.empty(count)
        a = np.empty((count, 3))
        d_pot.download(p)
        d_acc.download(a)
        ids = order[first:first + count]
        assert np.array_equal(p, pot_full[ids]) and np.array_equal(a, acc_full[ids])
        dev._leaf_particles_device(first, count, d_spos.ptr, d_smass.ptr, None)
        part = DeviceBins.select(d_spos.ptr, d_smass.ptr, ndim=3, on_device=True, n=count)
        counts_part = part.assign(edges)
        mom_part = part.moments(d_pot, SRC_W)
        mom_sum += mom_part
        # the fused pass over the tree's records (pbx_octree_radial_moments)
        # = select + assign + moments of the same leaf-order range
        c_f, m_f = dev._radial_moments_device(first, count, d_pot.ptr, edges)
        assert np.array_equal(c_f, counts_part)
        np.testing.assert_allclose(m_f, mom_part, rtol=1e-12, atol=1e-300)
        mom_fused += m_f
    np.testing.assert_array_equal(mom_sum[:, 0] > 0, mom_full[:, 0] > 0)
    np.testing.assert_allclose(mom_sum, mom_full, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(mom_fused, mom_full, rtol=1e-12, atol=1e-300)
    with pytest.raises(ValueError, match="increasing"):
        dev._radial_moments_device(0, n, d_pot.ptr, edges[::-1])
    with pytest.raises(ValueError, match="outside"):
        dev._compute_range_device(0.5, nat.WANT_POT, n - 5, 10, 1, d_pot.ptr, None, None)


def test_range_walk_wave_costs(gpu):
    """ShardedTree's cost kind 1 writes every target its wave's work (node
    steps + 4-record leaf rounds, equal over the 64 targets of a wave,
    summing to at least the wave-step counters); outputs do not change."""
    from pynbodyext import _native as nat

    n = 64 * 4688
    pos, mass = plummer(n, seed=101)
    dev = _engine.Octree(pos, mass, 8, 3)
    want = nat.WANT_POT | nat.WANT_ACC
    d_pot, d_acc = nat.DeviceArray(8 * n), nat.DeviceArray(24 * n)
    d_cost = nat.DeviceArray(4 * n)

    def walk(first, count, cost=None):
        dev._compute_range_device(0.5, want, first, count, 1, d_pot.ptr, d_acc.ptr, cost)
        p, a = np.empty(count), np.empty((count, 3))
        d_pot.download(p)
        d_acc.download(a)
        return p, a

    p0, a0 = walk(0, n)
    with pytest.raises(ValueError, match="cost kind"):
        dev._set_cost_kind(2)
    dev._set_cost_kind(1)
    p1, a1 = walk(0, n, d_cost.ptr)
    assert np.array_equal(p1, p0) and np.array_equal(a1, a0)
    info = dev.info()
    cost = d_cost.download(np.empty(n, dtype=np.int32)).reshape(-1, 64)
    assert (cost == cost[:, :1]).all()  # one value per wave
    wave = cost[:, 0].astype(np.int64)
    assert wave.min() > 0
    assert info["wave_steps"] + info["leaf_wave_steps"] <= wave.sum()
    for a in (d_pot, d_acc, d_cost):
        a.free()


@pytest.mark.parametrize("nbins", [963, 964, 1024])
def test_radial_moments_max_bins(gpu, nbins):
    """pbx_octree_radial_moments at the largest bin counts: up to 963 bins the
    edges sit in LDS next to the accumulators, above that (the LDS a
    workgroup may allocate is 64 KB) they are read from global memory; both
    equal select + assign + moments of the same range, up to RM_MAXB."""
    from pynbodyext import _native as nat
    from pynbodyext.profiles._device import SRC_W, DeviceBins

    n = 200_000
    pos, mass = plummer(n, seed=98)
    dev = _engine.Octree(pos, mass, 8, 3)
    d_pot, d_spos, d_smass = nat.DeviceArray(8 * n), nat.DeviceArray(24 * n), nat.DeviceArray(8 * n)
    try:
        dev._compute_range_device(0.5, nat.WANT_POT, 0, n, 1, d_pot.ptr, None, None)
        edges = np.logspace(np.log10(0.005), np.log10(60.0), nbins + 1)
        c_f, m_f = dev._radial_moments_device(0, n, d_pot.ptr, edges)
        dev._leaf_particles_device(0, n, d_spos.ptr, d_smass.ptr, None)
        part = DeviceBins.select(d_spos.ptr, d_smass.ptr, ndim=3, on_device=True, n=n)
        try:
            assert np.array_equal(c_f, part.assign(edges))
            np.testing.assert_allclose(m_f, part.moments(d_pot, SRC_W), rtol=1e-12, atol=1e-300)
        finally:
            part.close()
        assert (c_f > 0).sum() > nbins // 2
    finally:
        for a in (d_pot, d_spos, d_smass):
            a.free()
        dev.close()


def test_rebuild_reuses_handle(gpu):
    from pynbodyext import _native as nat

    pos1, m1 = plummer(5000, seed=3)
    pos2, m2 = plummer(7000, seed=4)
    t = _engine.Octree(pos1, m1, 8, 3)
    d_pos, d_m = nat.DeviceArray.from_host(pos2), nat.DeviceArray.from_host(m2)
    t._rebuild_device(d_pos.ptr, len(pos2), d_m.ptr)
    ref = ot.RefOctree(pos2, m2, 8, 3)
    check_structure(t, ref, 3)
    check_walk(t, ref, 0.5, len(pos2))


@pytest.mark.fast
@pytest.mark.parametrize("order", [0, 1, 3, 5])
def test_fast_mode_walk(gpu, order):
    """Default (fast) mode: v_rsq_f64 unrefined in node and leaf interactions;
    same decisions and interaction counts, values within 2e-6 of the oracle
    (contract 1e-5)."""
    pos, mass = plummer(20_000, seed=401 + order)
    dev = _engine.Octree(pos, mass, leaf_capacity=8, multipole_order=order)
    ref = ot.RefOctree(pos, mass, 8, order)
    pot_d = dev.compute_potentials(0.5)
    cnt_d = dev.info()
    acc_d = dev.compute_accelerations(0.5)
    pot_r, acc_r, nn_r, np_r = ref.compute_subset(np.arange(len(pos)), 0.5)
    assert cnt_d["node_interactions"] == int(nn_r.sum())
    assert cnt_d["leaf_pairs"] == int(np_r.sum())
    rp, ra = rel_pot(pot_d, pot_r), rel_acc(acc_d, acc_r)
    assert rp < FAST and ra < FAST, (rp, ra)


@pytest.mark.fast
def test_fast_mode_softened_at_points(gpu):
    pos, mass = plummer(6000, seed=77)
    h = np.full(len(pos), 0.02)
    dev = _engine.Octree(pos, mass, leaf_capacity=8, multipole_order=3, softenings=h, kernel=0)
    ref = ot.RefOctree(pos, mass, 8, 3, softenings=h, kernel=0)
    assert rel_pot(dev.compute_potentials(0.5), ref.compute_potentials(0.5)) < FAST
    pts = np.random.default_rng(3).normal(size=(500, 3))
    assert rel_acc(dev.accelerations_at_points(pts, 0.5), ref.accelerations_at_points(pts, 0.5)) < FAST


@pytest.mark.fast
def test_walk_counters_off(gpu):
    """pbx_octree_set_walk_counters(0): the fast order-3 walk without its
    statistics — every target bit-identical, info() counts zero, a walk with
    them back on counts again (full walk and a range walk at 8 waves per
    SIMD)."""
    from pynbodyext import _native as nat

    n = 64 * 3000
    pos, mass = plummer(n, seed=151)
    dev = _engine.Octree(pos, mass, 8, 3)
    want = nat.WANT_POT | nat.WANT_ACC
    d_pot, d_acc = nat.DeviceArray(8 * n), nat.DeviceArray(24 * n)

    def walk(first, count):
        dev._compute_range_device(0.5, want, first, count, 1, d_pot.ptr, d_acc.ptr, None)
        p, a = np.empty(count), np.empty((count, 3))
        d_pot.download(p)
        d_acc.download(a)
        return p, a, dev.info()

    for first, count in ((0, n), (64 * 100, 64 * 1000 + 3)):
        p0, a0, i0 = walk(first, count)
        assert i0["node_interactions"] > 0 and i0["leaf_pairs"] > 0
        dev._set_walk_counters(False)
        p1, a1, i1 = walk(first, count)
        dev._set_walk_counters(True)
        assert np.array_equal(p1, p0) and np.array_equal(a1, a0)
        assert i1["node_interactions"] == 0 and i1["leaf_pairs"] == 0 and i1["wave_steps"] == 0
        _, _, i2 = walk(first, count)
        assert i2["node_interactions"] == i0["node_interactions"]
    d_pot.free()
    d_acc.free()


@pytest.mark.fast
def test_fast_mode_theta_changes(gpu):
    """The fast unsoftened walk's opening sizes are size2 / theta^2 written
    into the walk records once per theta (open_scale): a handle walked at
    alternating thetas, and again after a rebuild on other particles, gives
    the decisions of the oracle at each theta and values bit-identical to a
    fresh handle's."""
    from pynbodyext import _native as nat

    pos, mass = plummer(12_000, seed=613)
    pos2, mass2 = plummer(9_000, seed=614)
    dev = _engine.Octree(pos, mass, 8, 3)
    ref = ot.RefOctree(pos, mass, 8, 3)
    firsts = {}
    for theta in (0.5, 0.7, 0.5, 0.35, 0.7):
        pot = dev.compute_potentials(theta)
        cnt = dev.info()
        if theta not in firsts:
            _, _, nn_r, np_r = ref.compute_subset(np.arange(len(pos)), theta)
            assert cnt["node_interactions"] == int(nn_r.sum()), theta
            assert cnt["leaf_pairs"] == int(np_r.sum()), theta
            fresh = _engine.Octree(pos, mass, 8, 3).compute_potentials(theta)
            assert np.array_equal(pot, fresh), theta
            firsts[theta] = pot
        else:
            assert np.array_equal(pot, firsts[theta]), theta
    # a rebuild writes new records: their opening sizes are scaled again
    d_pos, d_m = nat.DeviceArray.from_host(pos2), nat.DeviceArray.from_host(mass2)
    dev._rebuild_device(d_pos.ptr, len(pos2), d_m.ptr)
    pot = dev.compute_potentials(0.7)
    assert np.array_equal(pot, _engine.Octree(pos2, mass2, 8, 3).compute_potentials(0.7))
    ref2 = ot.RefOctree(pos2, mass2, 8, 3)
    pot_r, _, nn_r, _ = ref2.compute_subset(np.arange(len(pos2)), 0.7)
    assert dev.info()["node_interactions"] == int(nn_r.sum())
    assert rel_pot(pot, pot_r) < FAST
    d_pos.free()
    d_m.free()
