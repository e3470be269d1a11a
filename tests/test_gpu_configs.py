"""GPU parity at BASELINE.json's full workload sizes, in the default (fast)
precision mode the bench runs:

* config 5 — 4M Plummer (seed 1003) Barnes–Hut, theta = 0.5, leaf 8, order 3,
  Newtonian, force + potential at every particle, then the 256-bin log
  radial profile (0.01 .. 50) of the mass-weighted potential, through
  ShardedTree (the bench's solver) at world 1:
    - the device tree equals the oracle tree (tree.rs:627-1067 restated)
      node for node: centres, half sizes, leaf lists, mass / COM exactly,
      order-3 moments to 1e-12 of mass * size^k;
    - 8192 random + 64 central targets: the per-target interaction count
      (accepted nodes + leaf pairs) equals the oracle's, i.e. the same
      opening decisions (tree.rs:1114-1131), and values within the 1e-5
      contract and a 2e-6 regression bound;
    - the profile: edges and counts bit-exact with the oracle restatement of
      bins.py (log edges :713-718, assign :346-395), per-bin mass sums and
      mass-weighted mean potential within 1e-12 of oracle/profile_ref.py on
      the same potentials (proarray.py:272-334, Mean :632-643);
* config 4 — 8M Plummer (seed 1004) direct sum, force + potential, through
  ShardedDirect on a world-1 RCCL communicator (symmetric kernel, RCCL
  all-reduce of the accumulator), checked on 2048 random + 64 central
  targets against the oracle restatement of direct.rs:115-313.
"""
import numpy as np
import pytest

from oracle import gravity as og
from oracle import profile_ref as pr
from oracle import tree as ot
from pynbodyext import _native as nat
from pynbodyext.synthetic import plummer

pytestmark = pytest.mark.gpu

TOL = 1e-5    # north_star contract
FAST = 2e-6   # regression bound of the fast (raw v_rsq_f64) walk


def _preorder(first, nxt):
    first = np.asarray(first)
    nxt = np.asarray(nxt)
    out = np.empty(len(first), dtype=np.int64)
    k, i = 0, 0
    while k != -1:
        out[i] = k
        i += 1
        f = first[k]
        k = f if f != -1 else nxt[k]
    return out[:i]


def _segments(starts, counts):
    """Concatenated index ranges [s, s + c) (vectorised)."""
    starts = np.asarray(starts, dtype=np.int64)
    counts = np.asarray(counts, dtype=np.int64)
    total = int(counts.sum())
    shift = np.repeat(starts - np.concatenate([[0], np.cumsum(counts)[:-1]]), counts)
    return shift + np.arange(total)


def _check_structure(dev, ref):
    d, r = dev.export(), ref.export()
    do = _preorder(d["links"][:, 0], d["links"][:, 1])
    ro = _preorder(r["first"], r["next"])
    assert len(do) == len(ro) == dev.info()["nodes"] == ref.num_nodes
    assert np.array_equal(d["center"][do, :3], r["center"][ro])
    assert np.array_equal(d["center"][do, 3], r["half"][ro])
    dleaf = d["links"][do, 0] == -1
    rleaf = r["leaf_off"][ro] >= 0
    assert np.array_equal(dleaf, rleaf)
    dl = d["leaf"][do[dleaf]]
    ids_d = d["perm"][_segments(dl[:, 0], dl[:, 1])]
    ids_r = r["perm"][_segments(r["leaf_off"][ro[rleaf]], r["leaf_len"][ro[rleaf]])]
    assert np.array_equal(ids_d, ids_r)
    assert np.array_equal(d["com"][do, 3], r["mass"][ro])
    assert np.array_equal(d["com"][do, :3], r["com"][ro])
    md = dev.export_moments(20)[do]
    mr = r["mom"][ro][:, :20]
    size = (2 * r["half"][ro])[:, None]
    deg = np.array([0, 1, 1, 1] + [2] * 6 + [3] * 10)
    scale = np.abs(r["mass"][ro])[:, None] * size ** deg[None, :] + 1e-300
    assert np.max(np.abs(md - mr) / scale) < 1e-12


def _central(pos, k):
    return np.argsort((pos ** 2).sum(1))[:k]


def test_config5_tree_4m_fast_with_potential_profile(gpu):
    from pynbodyext.parallel import ShardedTree
    from pynbodyext.profiles._device import DeviceBins

    n, theta = 4_000_000, 0.5
    pos, mass = plummer(n, seed=1003)
    d_pos, d_mass = nat.DeviceArray.from_host(pos), nat.DeviceArray.from_host(mass)
    edges = np.logspace(np.log10(0.01), np.log10(50.0), 257)
    prof = DeviceBins()
    solver = ShardedTree(None, n, d_pos, d_mass, 8, 3, theta)
    try:
        with nat.precise_mode(False):
            mom = solver.step(prof, edges)  # build, balance, walk, profile
            counts = prof.counts.copy()
            d_cost = nat.DeviceArray(4 * n)
            solver.tree._set_cost_kind(0)  # interaction counts (ShardedTree: wave work)
            solver.tree._compute_range_device(theta, nat.WANT_POT | nat.WANT_ACC, 0, n, 1,
                                              solver.d_pot.ptr, solver.d_acc.ptr, d_cost.ptr)
        info = solver.tree.info()
        d_idx = nat.DeviceArray(8 * n)
        solver.tree._leaf_particles_device(0, n, None, None, d_idx.ptr)
        order = d_idx.download(np.empty(n, dtype=np.int64))
        pot_l = solver.d_pot.download(np.empty(n))
        acc_l = solver.d_acc.download(np.empty((n, 3)))
        cost_l = d_cost.download(np.empty(n, dtype=np.int32))
        d_idx.free()
        d_cost.free()
        assert np.array_equal(np.sort(order), np.arange(n))
        pot = np.empty(n)
        acc = np.empty((n, 3))
        cost = np.empty(n, dtype=np.int64)
        pot[order], acc[order], cost[order] = pot_l, acc_l, cost_l
        assert int(cost.sum()) == info["node_interactions"] + info["leaf_pairs"]

        ref = ot.RefOctree(pos, mass, 8, 3)
        _check_structure(solver.tree, ref)

        rng = np.random.default_rng(5)
        idx = np.unique(np.concatenate([rng.choice(n, 8192, replace=False), _central(pos, 64)]))
        og.set_num_threads(16)
        pot_r, acc_r, nn_r, np_r = ref.compute_subset(idx, theta)
        assert np.array_equal(cost[idx], nn_r + np_r)          # same opening decisions
        rp = float(np.max(np.abs(pot[idx] - pot_r) / np.abs(pot_r)))
        ra = float(np.max(np.linalg.norm(acc[idx] - acc_r, axis=1) /
                          np.linalg.norm(acc_r, axis=1)))
        assert rp < TOL and ra < TOL
        assert rp < FAST and ra < FAST, (rp, ra)

        # the 256-bin log potential profile on the same potentials
        r = pr.radial_r(pos)
        assert np.array_equal(edges, pr.edges_log(r, 256, 0.01, 50.0))
        perm, offsets, counts_r = pr.assign(r, edges)
        assert np.array_equal(counts, counts_r)
        msum, _ = pr.compute(mass, mass, perm, offsets, "sum")
        phim, _ = pr.compute(pot, mass, perm, offsets, "mean")
        full = counts_r > 0
        assert np.array_equal(mom[:, 0] > 0, full)
        np.testing.assert_allclose(mom[full, 0], msum[full], rtol=1e-12, atol=0)
        np.testing.assert_allclose(mom[full, 1] / mom[full, 0], phim[full], rtol=1e-12, atol=0)
        assert np.all(phim[full] < 0)
    finally:
        solver.close()
        prof.close()
        d_pos.free()
        d_mass.free()


def test_config4_direct_8m_sharded_world1(gpu):
    from pynbodyext.parallel import Communicator, ShardedDirect

    n = 8_000_000
    pos, mass = plummer(n, seed=1004)
    comm = Communicator(1, 0, Communicator.unique_id())
    try:
        with nat.precise_mode(False):
            s = ShardedDirect(comm, n, pos, mass)
            assert s.symmetric
            s.step()
            nat.synchronize()
            pot, acc = s.results()
    finally:
        comm.destroy()
    rng = np.random.default_rng(6)
    idx = np.unique(np.concatenate([rng.choice(n, 2048, replace=False), _central(pos, 64)]))
    og.set_num_threads(16)
    pr_, ar_ = og.direct_subset(pos, mass, idx)
    rp = float(np.max(np.abs(pot[idx] - pr_) / np.abs(pr_)))
    ra = float(np.max(np.linalg.norm(acc[idx] - ar_, axis=1) / np.linalg.norm(ar_, axis=1)))
    assert rp < TOL and ra < TOL
    assert rp < 1e-6 and ra < 1e-6, (rp, ra)   # fast mode, measured <= 1e-7 at 1M
    assert np.all(np.isfinite(pot)) and np.all(pot < 0)


class _EmulatedComm:
    """Rank r of R emulated on one GPU: ShardedTree's collectives are done
    by the test between the ranks' calls (host sums / copies)."""

    def __init__(self, nranks, rank):
        self.nranks, self.rank = nranks, rank

    def allgatherv(self, *a):
        pass

    def allreduce_sum_f64(self, *a):
        pass

    def allreduce(self, *a):  # in place on the device: this rank's partials
        pass

    def allreduce_host(self, a, op=0):  # this rank's partials (the test sums them)
        return np.array(a, copy=True)


def test_sharded_tree_rccl_world1_matches_single(gpu):
    """ShardedTree through a 1-rank RCCL communicator: the profile's partial
    [counts | moments] all-reduced in place on the device, then read back
    once, equals the communicator-free solve, step after step."""
    from pynbodyext.parallel import Communicator, ShardedTree
    from pynbodyext.profiles._device import DeviceBins

    n, theta = 200_000, 0.5
    pos, mass = plummer(n, seed=23)
    d_pos, d_mass = nat.DeviceArray.from_host(pos), nat.DeviceArray.from_host(mass)
    edges = np.logspace(np.log10(0.01), np.log10(50.0), 129)
    comm = Communicator(1, 0, Communicator.unique_id())
    single = ShardedTree(None, n, d_pos, d_mass, 8, 3, theta)
    ranked = ShardedTree(comm, n, d_pos, d_mass, 8, 3, theta)
    b0, b1 = DeviceBins(), DeviceBins()
    try:
        mom0 = single.step(b0, edges)
        pot0 = single.d_pot.download(np.empty(n))
        for _ in range(2):
            mom1 = ranked.step(b1, edges)
            assert np.array_equal(b1.counts, b0.counts)
            assert np.array_equal(ranked.d_pot.download(np.empty(n)), pot0)
            np.testing.assert_allclose(mom1, mom0, rtol=1e-12, atol=1e-300)
    finally:
        for t in (single, ranked):
            t.close()
        for b in (b0, b1):
            b.close()
        comm.destroy()
        d_pos.free()
        d_mass.free()


def test_sharded_tree_emulated_ranks_match_single(gpu):
    """ShardedTree over 3 ranks emulated on one device (walk ranges, leaf
    particles, cost carry + device balance, profile partials) reassembles
    the single-rank solve and profile exactly / to rounding."""
    from pynbodyext.parallel import ShardedTree, balanced_ranges
    from pynbodyext.profiles._device import DeviceBins

    n, world, theta = 300_000, 3, 0.5
    pos, mass = plummer(n, seed=17)
    d_pos, d_mass = nat.DeviceArray.from_host(pos), nat.DeviceArray.from_host(mass)
    edges = np.logspace(np.log10(0.01), np.log10(50.0), 129)
    single = ShardedTree(None, n, d_pos, d_mass, 8, 3, theta)
    sp = DeviceBins()
    ranks = [ShardedTree(_EmulatedComm(world, r), n, d_pos, d_mass, 8, 3, theta)
             for r in range(world)]
    bins = [DeviceBins() for _ in range(world)]
    try:
        mom_full = single.step(sp, edges)
        pot_full = single.d_pot.download(np.empty(n))
        acc_full = single.d_acc.download(np.empty((n, 3)))
        for step in range(2):
            for t in ranks:
                t.build()
                t.balance()
            rng_list = ranks[0].ranges
            assert all(t.ranges == rng_list for t in ranks)
            assert sum(c for _, c in rng_list) == n and rng_list[0][0] == 0
            if step == 1:  # balanced on the costs carried from step 0
                assert rng_list == want
            if step == 0:
                assert rng_list == [(lo, hi - lo) for lo, hi in
                                    [(0, 100_000), (100_000, 200_000), (200_000, 300_000)]]
            mom = np.zeros_like(mom_full)
            pieces = []
            for t, b in zip(ranks, bins):
                first, count = t.walk(share=False)
                p = t.d_pot.download(np.empty(count))
                a = t.d_acc.download(np.empty((count, 3)))
                assert np.array_equal(p, pot_full[first:first + count])
                assert np.array_equal(a, acc_full[first:first + count])
                pieces.append(t.d_cost.download(np.empty(n, dtype=np.int32))[first:first + count])
                mom += t.profile(b, edges)
            np.testing.assert_array_equal(mom[:, 0] > 0, mom_full[:, 0] > 0)
            np.testing.assert_allclose(mom, mom_full, rtol=1e-12, atol=1e-300)
            # the all-gather of the costs, then every rank carries them
            cost = np.concatenate(pieces)
            for t in ranks:
                t.d_cost.upload(cost)
                t.share_costs()
            want = balanced_ranges(cost, world)
        # after a walk: the device balance = balanced_ranges on the carried costs
        for t in ranks:
            t.build()
            assert t.balance() == want
    finally:
        for t in ranks + [single]:
            t.close()
        for b in bins + [sp]:
            b.close()
        d_pos.free()
        d_mass.free()
