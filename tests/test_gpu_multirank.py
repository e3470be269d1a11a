"""World > 1 on ONE GPU: every multi-rank path of pynbodyext.parallel run
with 2-4 ranks as threads of this process, over the host-transport
communicator (parallel.HostCommunicator + ThreadLoopback, pbx_comm_init_host).

The ranks run exactly the code a multi-GPU job runs — the one-call
distributed profile pbx_profile_radial_equaln_comm with every collective
between its kernels (key-range max, kept count + look-back status, level-0
digit histogram, per-rank group counts, the zero-padded group-key segment
all-gathered by a sum, the packed counts and sums, the separate moment
passes, the degenerate one-bin branch), ShardedDirect (source all-gather-v,
symmetric triangle split + accumulator all-reduce), ShardedTree
(cost-balanced ranges, cost all-gather, profile all-reduce) and the staged
ShardedProfile — with RCCL replaced by a host sum in rank order.  Results
are checked against the oracle on the concatenation of all ranks' particles
(bins.py:346-395,720-746 for the profile; direct.rs / tree.rs for gravity)
and against the single-device call.
"""
import numpy as np
import pytest

from oracle import gravity as og
from oracle import profile_ref as pr
from pynbodyext import _native as nat
from pynbodyext.parallel import (HostCommunicator, ShardedDirect, ShardedProfile, ShardedTree,
                                 ThreadLoopback, all_shards)
from pynbodyext.profiles._device import SRC_NONE, SRC_W, SRC_X, DeviceBins
from pynbodyext.synthetic import plummer

pytestmark = pytest.mark.gpu

STATS = [(SRC_W, SRC_NONE, 1 << 3), (SRC_X, SRC_W, 0b11)]


def test_loopback_collectives(gpu):
    """The host-transport communicator: every pbx_comm_* call over 3 ranks."""
    import ctypes

    from pynbodyext.parallel import DT_F64, DT_U32, OP_MAX, OP_MIN

    world = 3

    def rank_fn(comm):
        r = comm.rank
        a = np.arange(10, dtype=np.float64) * (r + 1)
        d = nat.DeviceArray.from_host(a)
        comm.allreduce_sum_f64(d.ptr, d.ptr, 10)
        s = d.download(np.empty(10))
        u = nat.DeviceArray.from_host(np.full(4, 0xFFFFFFF0 + r, dtype=np.uint32))
        comm.allreduce(u.ptr, u.ptr, 4, DT_U32)              # wraps like RCCL's u32 sum
        us = u.download(np.empty(4, dtype=np.uint32))
        comm.allreduce(d.ptr, d.ptr, 10, DT_F64, OP_MIN)
        mn = d.download(np.empty(10))
        # uneven all-gather-v of bytes, rank 1 empty
        counts = [5, 0, 11]
        displs = [0, 5, 5]
        g = np.zeros(16, dtype=np.uint8)
        g[displs[r]:displs[r] + counts[r]] = 10 * (r + 1)
        dg = nat.DeviceArray.from_host(g)
        comm.allgatherv(dg.ptr, counts, displs)
        gg = dg.download(np.empty(16, dtype=np.uint8))
        h = comm.allreduce_host(np.array([r + 1, 7], dtype=np.int64))
        hm = comm.allreduce_host(np.array([float(r)]), OP_MAX)
        comm.barrier()
        mx = comm.max(float(r) + 0.5)
        for x in (d, u, dg):
            x.free()
        return s, us, mn, gg, h, hm, mx

    out = ThreadLoopback(world).run(rank_fn)
    base = np.arange(10, dtype=np.float64)
    for s, us, mn, gg, h, hm, mx in out:
        assert np.array_equal(s, base * 6)
        want = (sum(0xFFFFFFF0 + r for r in range(world))) & 0xFFFFFFFF
        assert np.all(us == want)
        assert np.array_equal(mn, base * 6)  # after the sum every rank holds the same
        assert np.array_equal(gg, np.array([10] * 5 + [30] * 11, dtype=np.uint8))
        assert np.array_equal(h, [6, 21]) and hm[0] == 2.0 and mx == 2.5
    del ctypes


def test_loopback_size_mismatch_fails_every_rank(gpu):
    """A collective whose size differs between ranks is an error on every
    rank (RCCL would hang), and no rank is left waiting."""

    def rank_fn(comm):
        d = nat.DeviceArray(8 * 4)
        nat.call("pbx_memset", d.ptr, 0, 32)
        comm.allreduce_sum_f64(d.ptr, d.ptr, 2 + comm.rank)

    with pytest.raises(RuntimeError, match="different sizes"):
        ThreadLoopback(2, timeout=30).run(rank_fn)


# ----------------------------------------------------------------- profile
def _families_local(fams, lo, hi):
    out = []
    for a, b in fams:
        a2, b2 = max(a, lo), min(b, hi)
        if b2 > a2:
            out.append((a2 - lo, b2 - lo))
    return out


def _case(case):
    """(pos, mass, cuts, kwargs) of a multi-rank profile case."""
    rng = np.random.default_rng(101)
    n = 300_000
    kw = dict(nbins=128, sphere=None, families=None, bin_min=None, bin_max=None, stats=STATS)
    cuts = [150_000]
    if case == "tiled":            # rank 0 >= 1024 selection tiles, rank 1 the lazy path
        n = 4_500_000
        cuts = [4_300_000]
    pos = rng.normal(scale=3.0, size=(n, 3))
    mass = rng.uniform(0.5, 1.5, n)
    if case == "uneven3":
        cuts = [1_000, 250_000]
    elif case == "empty_rank4":
        cuts = [100_000, 100_000, 180_000]     # rank 1 holds nothing
    elif case == "clip":
        kw.update(bin_min=0.5, bin_max=6.0)
        cuts = [40_000, 200_000]
    elif case == "nan":
        pos[::61] = np.nan
        cuts = [70_000, 71_000, 230_000]
    elif case == "family":
        kw.update(sphere=((0.0, 0.0, 0.0), 6.0), families=[(1_000, 120_000), (150_000, 290_000)])
        cuts = [60_000, 130_000, 200_000]      # rank 2: inside no family range at its start
    elif case == "single":
        kw.update(bin_min=1.0, bin_max=1.0)
        pos[200_000] = [1.0, 0.0, 0.0]
    elif case == "many_stats":
        kw.update(nbins=64, stats=[(SRC_W, SRC_NONE, 1 << 3), (SRC_X, SRC_W, 0b11),
                                   (SRC_X, SRC_NONE, 0x7f), (SRC_W, SRC_W, 0x7f),
                                   (SRC_X, SRC_W, 0x7f), (SRC_W, SRC_NONE, 0x18)])
    elif case == "wide":
        kw.update(nbins=300)
        cuts = [100_000, 200_000]
    return pos, mass, cuts, kw


def _run_profile(pos, mass, cuts, kw):
    """Every rank calls ShardedProfile.radial_equaln on its contiguous shard;
    returns per-rank (edges, counts, moments, local counts, n kept, perm, offs)."""
    bounds = list(zip([0] + cuts, cuts + [len(pos)]))
    world = len(bounds)

    def rank_fn(comm):
        lo, hi = bounds[comm.rank]
        k = dict(kw)
        if kw["families"] is not None:
            k["families"] = _families_local(kw["families"], lo, hi)
        dev = DeviceBins()
        try:
            sp = ShardedProfile(comm, dev, offset=lo)
            res = []
            for _ in range(2):  # the second call reuses the handle's buffers
                e, c, m = sp.radial_equaln(np.ascontiguousarray(pos[lo:hi]),
                                           np.ascontiguousarray(mass[lo:hi]), **k)
                perm, offs = dev.csr()
                res.append((e, c, m, dev.counts.copy(), dev.n, dev.n_valid, perm, offs))
            return res
        finally:
            dev.close()

    return ThreadLoopback(world).run(rank_fn)


def _global_csr(ranks):
    """The global binind of the concatenation from every rank's local CSR:
    bin b = the ranks' runs in rank order, indices shifted by the kept
    particles of the ranks before."""
    nb = len(ranks[0][7]) - 1
    before = np.cumsum([0] + [r[4] for r in ranks[:-1]])
    perm = []
    counts = np.zeros(nb, dtype=np.int64)
    for b in range(nb):
        for q, r in enumerate(ranks):
            p, o = r[6], r[7]
            perm.append(p[o[b]:o[b + 1]] + before[q])
            counts[b] += o[b + 1] - o[b]
    offs = np.concatenate([[0], np.cumsum(counts)])
    return np.concatenate(perm).astype(np.int64), offs


@pytest.mark.parametrize("case", ["halves", "uneven3", "empty_rank4", "clip", "nan", "family",
                                  "tiled", "single", "many_stats", "wide"])
def test_radial_equaln_comm_multirank(gpu, case):
    pos, mass, cuts, kw = _case(case)
    out = _run_profile(pos, mass, cuts, kw)
    # the single-device call on the concatenation, global family ranges
    one = DeviceBins()
    try:
        _, e1, c1, m1 = DeviceBins.radial_equaln(pos, mass, into=one, **kw)
        p1, o1 = one.csr()
        kept1, valid1 = one.n, one.n_valid
    finally:
        one.close()
    # the oracle on the concatenation
    mask = np.ones(len(pos), dtype=bool)
    if kw["sphere"] is not None:
        mask &= pr.sphere_mask(pos, kw["sphere"][1], kw["sphere"][0])
    if kw["families"] is not None:
        fm = np.zeros(len(pos), dtype=bool)
        for a, b in kw["families"]:
            fm[a:b] = True
        mask &= fm
    x = pr.radial_r(pos[mask])
    w = mass[mask]
    edges = pr.edges_equaln(x, kw["nbins"], kw["bin_min"], kw["bin_max"])
    perm, offs, counts = pr.assign(x, edges)
    assert np.array_equal(e1, edges, equal_nan=True) and np.array_equal(c1, counts)
    for call in range(2):
        ranks = [r[call] for r in out]
        assert sum(r[4] for r in ranks) == kept1 == len(x)
        assert sum(r[5] for r in ranks) == valid1
        for e, c, m, cl, *_ in ranks:
            assert np.array_equal(e, edges, equal_nan=True), case
            assert np.array_equal(c, counts), case
            for u, v in zip(m, m1):
                np.testing.assert_allclose(u, v, rtol=1e-12, atol=1e-300)
        loc = np.sum([r[3] for r in ranks], axis=0)
        assert np.array_equal(loc, counts)
        gp, go = _global_csr(ranks)
        assert np.array_equal(go, offs) and np.array_equal(gp, perm), case
    # per-bin Σm against the oracle's numpy sums
    msum, _ = pr.compute(w, w, perm, offs, "sum")
    got = out[0][1][2][0][:, 3]
    nz = counts > 0
    assert np.all(np.abs(got[nz] - msum[nz]) <= 1e-12 * np.abs(msum[nz]))


@pytest.mark.parametrize("case", ["nothing_kept", "empty_window"])
def test_radial_equaln_comm_multirank_errors(gpu, case):
    """Errors every rank reaches at the same point: all raise the
    single-device call's exception, none is left in a collective."""
    pos, mass, cuts, kw = _case("halves")
    if case == "nothing_kept":
        kw.update(sphere=((1e6, 0.0, 0.0), 1.0))
        exc = ValueError
    else:
        kw.update(bin_min=1e9, bin_max=2e9)
        exc = IndexError
    with pytest.raises(exc) as e2:
        DeviceBins.radial_equaln(pos, mass, **kw)
    with pytest.raises(exc) as e1:
        _run_profile(pos, mass, cuts, kw)
    assert str(e1.value) == str(e2.value)


def test_radial_equaln_comm_rank_without_kept_particles(gpu):
    """One rank keeps nothing (its shard lies outside the sphere) while the
    others do: the global profile is still the oracle's."""
    rng = np.random.default_rng(7)
    pos = rng.normal(scale=1.0, size=(200_000, 3))
    pos[100_000:150_000] += 1e3           # rank 1's shard: all outside the sphere
    mass = rng.uniform(0.5, 1.5, len(pos))
    kw = dict(nbins=128, sphere=((0.0, 0.0, 0.0), 5.0), families=None, bin_min=None,
              bin_max=None, stats=STATS)
    out = _run_profile(pos, mass, [100_000, 150_000], kw)
    x = pr.radial_r(pos[pr.sphere_mask(pos, 5.0)])
    edges = pr.edges_equaln(x, 128)
    perm, offs, counts = pr.assign(x, edges)
    ranks = [r[0] for r in out]
    assert ranks[1][4] == 0
    for e, c, *_ in ranks:
        assert np.array_equal(e, edges) and np.array_equal(c, counts)
    gp, go = _global_csr(ranks)
    assert np.array_equal(go, offs) and np.array_equal(gp, perm)


def test_staged_sharded_profile_multirank(gpu):
    """The staged distributed profile (ShardedProfile.edges_equaln -> assign
    -> moments -> csr, parallel.distributed_equaln over the loopback) on 3
    ranks with an empty one = the oracle on the concatenation."""
    rng = np.random.default_rng(9)
    x = rng.lognormal(0.0, 1.5, 200_000)
    x[::97] = 3.0  # ties across ranks
    w = rng.uniform(0.5, 1.5, len(x))
    bounds = [(0, 50_000), (50_000, 50_000), (50_000, len(x))]

    def rank_fn(comm):
        lo, hi = bounds[comm.rank]
        dev = DeviceBins.from_x(x[lo:hi])
        try:
            sp = ShardedProfile(comm, dev, offset=lo)
            e = sp.edges_equaln(128)
            c = sp.assign(e)
            m = sp.moments(w[lo:hi], SRC_NONE)  # column 3: Σ field = Σw
            p, o, start = sp.csr()
            return e, c, m, p, o, start, dev.counts.copy()
        finally:
            dev.close()

    out = ThreadLoopback(3).run(rank_fn)
    edges = pr.edges_equaln(x, 128)
    perm, offs, counts = pr.assign(x, edges)
    for e, c, m, p, o, start, _ in out:
        assert np.array_equal(e, edges) and np.array_equal(c, counts) and np.array_equal(o, offs)
    # rank runs placed at their start offsets = the global binind
    g = np.empty(len(perm), dtype=np.int64)
    for e, c, m, p, o, start, loc in out:
        lo_o = np.concatenate([[0], np.cumsum(loc)])
        for b in range(128):
            g[start[b]:start[b] + loc[b]] = p[lo_o[b]:lo_o[b + 1]]
    assert np.array_equal(g, perm)
    msum, _ = pr.compute(w, w, perm, offs, "sum")
    np.testing.assert_allclose(out[0][2][:, 3], msum, rtol=1e-12)


# ----------------------------------------------------------------- gravity
@pytest.mark.parametrize("n,world,symmetric", [(2501, 3, False), (20_000, 3, True),
                                               (9_000, 4, True)])
def test_sharded_direct_multirank(gpu, n, world, symmetric):
    """ShardedDirect over 3-4 ranks: source all-gather-v (uneven shards) and,
    symmetric, the weight-split unit triangle + accumulator all-reduce."""
    pos, mass = plummer(n, seed=13)
    shards = all_shards(n, world)

    def rank_fn(comm):
        lo, hi = shards[comm.rank]
        s = ShardedDirect(comm, n, pos[lo:hi], mass[lo:hi], symmetric=symmetric)
        s.step()
        nat.synchronize()
        return s.results()

    out = ThreadLoopback(world).run(rank_fn)
    pot = np.concatenate([o[0] for o in out])
    acc = np.concatenate([o[1] for o in out])
    pr_, ar = og.direct_potentials(pos, mass), og.direct_accelerations(pos, mass)
    lim = 1e-6 if (symmetric and not nat.get_precise()) else 1e-10
    assert np.max(np.abs(pot - pr_) / np.abs(pr_)) < lim
    assert np.max(np.linalg.norm(acc - ar, axis=1) / np.linalg.norm(ar, axis=1)) < lim


def test_sharded_tree_multirank(gpu):
    """ShardedTree over 3 ranks for two steps (the second balanced on the
    first's all-gathered costs): every target's potential / acceleration
    equals the one-rank walk's bit for bit (identical decisions and order per
    target), the summed profile equals the one-rank profile to rounding."""
    from pynbodyext._engine import Octree

    n, world = 60_000, 3
    pos, mass = plummer(n, seed=17)
    edges = np.logspace(np.log10(0.01), np.log10(50.0), 65)

    def leaf_to_orig(tree, first, count, vals):
        idx = nat.DeviceArray(8 * max(count, 1))
        tree._leaf_particles_device(first, count, None, None, idx.ptr)
        order = idx.download(np.empty(count, dtype=np.int64))
        idx.free()
        return order

    def rank_fn(comm):
        d_pos = nat.DeviceArray.from_host(pos)
        d_mass = nat.DeviceArray.from_host(mass)
        s = ShardedTree(comm, n, d_pos, d_mass, 8, 3, 0.5)
        steps = []
        try:
            for _ in range(2):
                mom = s.step(None, edges)
                first, count = s.ranges[comm.rank]
                pot = s.d_pot.download(np.empty(count)) if count else np.empty(0)
                acc = s.d_acc.download(np.empty((count, 3))) if count else np.empty((0, 3))
                order = leaf_to_orig(s.tree, first, count, pot)
                steps.append((list(s.ranges), order, pot, acc, mom))
        finally:
            s.close()
            d_pos.free()
            d_mass.free()
        return steps

    out = ThreadLoopback(world).run(rank_fn)
    # the same steps on one rank (no communicator): the reference walk
    d_pos = nat.DeviceArray.from_host(pos)
    d_mass = nat.DeviceArray.from_host(mass)
    ref = ShardedTree(None, n, d_pos, d_mass, 8, 3, 0.5)
    try:
        mom1 = ref.step(None, edges)
        p1 = ref.d_pot.download(np.empty(n))
        a1 = ref.d_acc.download(np.empty((n, 3)))
        order1 = leaf_to_orig(ref.tree, 0, n, p1)
    finally:
        ref.close()
        d_pos.free()
        d_mass.free()
    pot1 = np.empty(n)
    acc1 = np.empty((n, 3))
    pot1[order1] = p1
    acc1[order1] = a1
    # and against the Octree API (same tree, same decisions: rounding only)
    t = Octree(pos, mass, leaf_capacity=8, multipole_order=3)
    try:
        pp = t.compute_potentials(0.5)
    finally:
        t.close()
    assert np.max(np.abs(pp - pot1) / np.abs(pp)) < 1e-12
    for step in range(2):
        ranges = out[0][step][0]
        assert all(o[step][0] == ranges for o in out)
        assert sum(c for _, c in ranges) == n
        pot = np.full(n, np.nan)
        acc = np.full((n, 3), np.nan)
        for o in out:
            _, order, p, a, mom = o[step]
            pot[order] = p
            acc[order] = a
            np.testing.assert_allclose(mom, mom1, rtol=1e-12, atol=1e-300)
        assert np.array_equal(pot, pot1)
        assert np.array_equal(acc, acc1)
    # the second step's ranges come from the first step's costs
    assert out[0][1][0] != [(lo, hi - lo) for lo, hi in all_shards(n, world)]


def test_host_communicator_reports_transport_errors(gpu):
    """A transport that raises: the library call fails with RuntimeError and
    the communicator keeps the transport's exception."""

    class Broken:
        def allreduce(self, a, op):
            raise KeyError("boom")

        def allgatherv(self, buf, counts, displs):
            raise KeyError("boom")

    comm = HostCommunicator(1, 0, Broken())
    try:
        d = nat.DeviceArray.from_host(np.zeros(4))
        with pytest.raises(RuntimeError, match="host collective"):
            comm.allreduce_sum_f64(d.ptr, d.ptr, 4)
        assert isinstance(comm.error, KeyError)
    finally:
        comm.destroy()
