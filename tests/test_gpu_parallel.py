"""RCCL leg of the sharded direct sum on the GPU box (world = 1 communicator).

The single-GPU box can only host one RCCL rank per GPU; the world>1 data
path is exercised by the driver's 8-GPU bench, and its bookkeeping by
tests/test_dist_gloo.py on CPU.
"""
import numpy as np
import pytest

from oracle import gravity as og
from pynbodyext import _native as nat
from pynbodyext.parallel import Communicator, ShardedDirect
from pynbodyext.synthetic import plummer

pytestmark = pytest.mark.gpu


def test_rccl_world1_collectives(gpu):
    comm = Communicator(1, 0, Communicator.unique_id())
    try:
        a = np.arange(10, dtype=np.float64)
        d = nat.DeviceArray.from_host(a)
        comm.allreduce_sum_f64(d.ptr, d.ptr, 10)
        comm.allgather_inplace(d.ptr, 80)
        out = np.empty(10)
        d.download(out)
        assert np.array_equal(out, a)
        ai = np.arange(5, dtype=np.int64)
        di = nat.DeviceArray.from_host(ai)
        comm.allreduce_sum_i64(di.ptr, di.ptr, 5)
        oi = np.empty(5, dtype=np.int64)
        di.download(oi)
        assert np.array_equal(oi, ai)
    finally:
        comm.destroy()


def test_sharded_direct_world1(gpu):
    pos, mass = plummer(3000, seed=4)
    comm = Communicator(1, 0, Communicator.unique_id())
    try:
        s = ShardedDirect(comm, len(pos), pos, mass)
        s.step()
        nat.synchronize()
        pot, acc = s.results()
    finally:
        comm.destroy()
    pr = og.direct_potentials(pos, mass)
    ar = og.direct_accelerations(pos, mass)
    assert np.max(np.abs(pot - pr) / np.abs(pr)) < 1e-10
    assert np.max(np.linalg.norm(acc - ar, axis=1) / np.linalg.norm(ar, axis=1)) < 1e-10


def test_sharded_solve_of_one_shard_matches_oracle(gpu):
    """Simulate rank 1 of 3 on one GPU: records of all ranks in place, solve
    only the local targets with self offset lo (what each rank does)."""
    from pynbodyext.parallel import shard_bounds

    n, world, rank = 2501, 3, 1
    pos, mass = plummer(n, seed=6)
    lo, hi = shard_bounds(n, world, rank)
    s = ShardedDirect(None, n, pos, mass)  # world-1 instance to hold all records
    s.gather_sources()
    d_tgt = nat.DeviceArray.from_host(np.ascontiguousarray(pos[lo:hi]))
    d_pot = nat.DeviceArray(8 * (hi - lo))
    d_acc = nat.DeviceArray(24 * (hi - lo))
    nat.call("pbx_direct_dev", s.d_rec.ptr, None, n, d_tgt.ptr, None, hi - lo, lo,
             nat.KERNEL_NONE, 3, d_pot.ptr, d_acc.ptr)
    pot = d_pot.download(np.empty(hi - lo))
    acc = d_acc.download(np.empty((hi - lo, 3)))
    pr, ar = og.direct_subset(pos, mass, np.arange(lo, hi))
    assert np.max(np.abs(pot - pr) / np.abs(pr)) < 1e-10
    assert np.max(np.linalg.norm(acc - ar, axis=1) / np.linalg.norm(ar, axis=1)) < 1e-10


def test_symmetric_units_split_across_ranks(gpu):
    """Multi-GPU symmetric direct sum on one GPU: the unit triangle split into
    3 weight-balanced ranges (what 3 ranks run), accumulators summed (what the
    RCCL all-reduce does), each rank's shard finished."""
    import ctypes

    from pynbodyext.parallel import balanced_ranges, shard_bounds

    n, world = 20_000, 3
    pos, mass = plummer(n, seed=8)
    s = ShardedDirect(None, n, pos, mass, symmetric=True)
    s.gather_sources()
    npad, nunits = ctypes.c_int64(), ctypes.c_int64()
    nat.call("pbx_direct_sym_plan", n, ctypes.byref(npad), ctypes.byref(nunits), None)
    w = np.zeros(nunits.value, dtype=np.int64)
    nat.call("pbx_direct_sym_plan", n, None, None, w.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
    total = np.zeros(4 * npad.value)
    d_acc4 = nat.DeviceArray(32 * npad.value)
    for first, count in balanced_ranges(w, world):
        nat.call("pbx_memset", d_acc4.ptr, 0, ctypes.c_size_t(32 * npad.value))
        nat.call("pbx_direct_sym_accumulate", s.d_rec.ptr, n, first, first + count, 3, d_acc4.ptr)
        part = np.empty(4 * npad.value)
        d_acc4.download(part)
        total += part
    d_acc4.upload(total)
    pr = og.direct_potentials(pos, mass)
    ar = og.direct_accelerations(pos, mass)
    for rank in range(world):
        lo, hi = shard_bounds(n, world, rank)
        d_pot, d_acc = nat.DeviceArray(8 * (hi - lo)), nat.DeviceArray(24 * (hi - lo))
        nat.call("pbx_direct_sym_finish", d_acc4.ptr, lo, hi, 3, d_pot.ptr, d_acc.ptr)
        pot = d_pot.download(np.empty(hi - lo))
        acc = d_acc.download(np.empty((hi - lo, 3)))
        lim = 1e-10 if nat.get_precise() else 1e-6  # fast mode: raw v_rsq_f64
        assert np.max(np.abs(pot - pr[lo:hi]) / np.abs(pr[lo:hi])) < lim
        assert np.max(np.linalg.norm(acc - ar[lo:hi], axis=1) /
                      np.linalg.norm(ar[lo:hi], axis=1)) < lim


def test_sharded_direct_symmetric_world1(gpu):
    pos, mass = plummer(12_000, seed=9)
    comm = Communicator(1, 0, Communicator.unique_id())
    try:
        s = ShardedDirect(comm, len(pos), pos, mass)
        assert s.symmetric
        s.step()
        nat.synchronize()
        pot, acc = s.results()
    finally:
        comm.destroy()
    pr = og.direct_potentials(pos, mass)
    assert np.max(np.abs(pot - pr) / np.abs(pr)) < (1e-10 if nat.get_precise() else 1e-6)


def _emulated_ranks_equaln(devs, nbins, lo=None, hi=None):
    """The distributed equaln protocol with R ranks emulated on one GPU: the
    'all-reduce' of every level's histogram is a host sum over the handles."""
    import ctypes

    kr = [d.key_range() for d in devs]
    kmin, kmax = min(k[0] for k in kr), max(k[1] for k in kr)
    levels = [d.msel_begin(nbins, lo, hi, kmin, kmax) for d in devs]
    assert len(set(levels)) == 1
    for level in range(levels[0]):
        hs = [d.msel_hist(level) for d in devs]
        tot = None
        for ptr, cnt in hs:
            h = np.empty(cnt, dtype=np.uint32)
            nat.call("pbx_memcpy_dtoh", h.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr),
                     ctypes.c_size_t(h.nbytes))
            tot = h.astype(np.uint64) if tot is None else tot + h
        tot = tot.astype(np.uint32)
        for ptr, _ in hs:
            nat.call("pbx_memcpy_htod", ctypes.c_void_p(ptr), tot.ctypes.data_as(ctypes.c_void_p),
                     ctypes.c_size_t(tot.nbytes))
        for d in devs:
            d.msel_resolve(level)
    return [d.msel_edges() for d in devs]


@pytest.mark.parametrize("case", ["halves", "uneven", "empty_rank", "bounds", "nan", "dups"])
def test_distributed_equaln_emulated_ranks(gpu, case):
    """Edges from rank-local radix-select histograms summed over ranks equal
    the single-process equaln of the concatenated x (bins.py:720-746)."""
    from oracle import profile_ref as pr
    from pynbodyext.profiles._device import DeviceBins

    rng = np.random.default_rng(21)
    x = rng.lognormal(0.0, 1.5, 300_000)
    nb, lo, hi, cuts = 128, None, None, [150_000]
    if case == "uneven":
        cuts = [1000, 250_000]
    elif case == "empty_rank":
        cuts = [0, 100_000]
    elif case == "bounds":
        lo, hi, cuts = 0.05, 20.0, [50_000, 120_000, 290_000]
    elif case == "nan":
        x[::97] = np.nan
    elif case == "dups":
        x = rng.choice(np.array([0.5, 1.0, 1.0000000000000002, 3.0]), 300_000)
        nb = 256
    parts = np.split(x, cuts)
    devs = [DeviceBins.from_x(p) if p.size else DeviceBins.from_x(np.zeros(0)) for p in parts]
    try:
        got = _emulated_ranks_equaln(devs, nb, lo, hi)
    finally:
        for d in devs:
            d.close()
    want = pr.edges_equaln(x, nb, lo, hi)
    for g in got:
        assert np.array_equal(g, want, equal_nan=True), case


def test_sharded_profile_world1_matches_single(gpu):
    """ShardedProfile through a 1-rank RCCL communicator (the all-reduce
    plumbing of the multi-GPU profile) = the single-device profile."""
    from pynbodyext.parallel import ShardedProfile
    from pynbodyext.profiles._device import SRC_W, SRC_X, DeviceBins

    pos, mass = plummer(200_000, seed=31)
    comm = Communicator(1, 0, Communicator.unique_id())
    a = DeviceBins.select(pos, mass, sphere=((0.0, 0.0, 0.0), 10.0), ndim=3)
    b = DeviceBins.select(pos, mass, sphere=((0.0, 0.0, 0.0), 10.0), ndim=3)
    try:
        sp = ShardedProfile(comm, a, offset=0)
        e = sp.edges_equaln(128)
        assert np.array_equal(e, b.edges_equaln(128))
        c = sp.assign(e)
        assert np.array_equal(c, b.assign(e))
        m = sp.moments(SRC_X, SRC_W)
        np.testing.assert_allclose(m, b.moments(SRC_X, SRC_W), rtol=1e-12)
        perm, offs, start = sp.csr()
        p2, o2 = b.csr()
        assert np.array_equal(offs, o2) and np.array_equal(start, o2[:-1])
        assert np.array_equal(perm, p2)
    finally:
        a.close()
        b.close()
        comm.destroy()


@pytest.mark.parametrize("case", ["small", "tiled", "family", "clip", "nan", "single", "many_stats",
                                  "wide", "nothing_kept", "empty_window"])
def test_radial_equaln_comm_world1_matches_single(gpu, case):
    """pbx_profile_radial_equaln_comm through a 1-rank RCCL communicator (the
    distributed pipeline: key-range / digit-histogram / group-key / result
    all-reduces between the kernels, the segment sized from the mid-call
    read-back) = the single-device pbx_profile_radial_equaln: edges, counts,
    CSR bit-identical, sums to rounding, same errors; local counts = global."""
    from pynbodyext.parallel import ShardedProfile
    from pynbodyext.profiles._device import SRC_NONE, SRC_W, SRC_X, DeviceBins

    rng = np.random.default_rng(41)
    n = 4_400_000 if case == "tiled" else 300_000
    pos = rng.normal(scale=3.0, size=(n, 3))
    mass = rng.uniform(0.5, 1.5, n)
    kw = dict(nbins=128, sphere=None, families=None, bin_min=None, bin_max=None,
              stats=[(SRC_W, SRC_NONE, 1 << 3), (SRC_X, SRC_W, 0b11)])
    if case == "family":
        kw.update(sphere=((0.3, 0.0, -0.1), 6.0), families=[(1_000, 120_000), (150_000, 290_000)])
    elif case == "clip":
        kw.update(bin_min=0.5, bin_max=6.0)
    elif case == "nan":
        pos[::61] = np.nan
    elif case == "single":
        kw.update(bin_min=1.0, bin_max=1.0)
        pos[9] = [1.0, 0.0, 0.0]
    elif case == "many_stats":
        kw.update(nbins=64, stats=[(SRC_W, SRC_NONE, 1 << 3), (SRC_X, SRC_W, 0b11),
                                   (SRC_X, SRC_NONE, 0x7f), (SRC_W, SRC_W, 0x7f),
                                   (SRC_X, SRC_W, 0x7f), (SRC_W, SRC_NONE, 0x18)])
    elif case == "wide":
        kw.update(nbins=300)
    elif case == "nothing_kept":
        kw.update(sphere=((1e6, 0.0, 0.0), 1.0))
    elif case == "empty_window":
        kw.update(bin_min=1e9, bin_max=2e9)
    comm = Communicator(1, 0, Communicator.unique_id())
    a, b = DeviceBins(), DeviceBins()
    try:
        sp = ShardedProfile(comm, a, offset=0)
        if case in ("nothing_kept", "empty_window"):
            exc = IndexError if case == "empty_window" else ValueError
            with pytest.raises(exc) as e1:
                sp.radial_equaln(pos, mass, **kw)
            with pytest.raises(exc) as e2:
                DeviceBins.radial_equaln(pos, mass, into=b, **kw)
            assert str(e1.value) == str(e2.value)
            return
        for _ in range(2):  # the second call reuses the handle's buffers
            e1, c1, m1 = sp.radial_equaln(pos, mass, **kw)
            _, e2, c2, m2 = DeviceBins.radial_equaln(pos, mass, into=b, **kw)
            assert np.array_equal(e1, e2, equal_nan=True)
            assert np.array_equal(c1, c2) and np.array_equal(a.counts, c2)
            assert a.n == b.n and a.n_valid == b.n_valid
            for u, v in zip(m1, m2):
                np.testing.assert_allclose(u, v, rtol=1e-12, atol=1e-300)
            p1, o1 = a.csr()
            p2, o2 = b.csr()
            assert np.array_equal(p1, p2) and np.array_equal(o1, o2)
    finally:
        a.close()
        b.close()
        comm.destroy()
