"""N>1 host logic on CPU: world_size-2 gloo processes.

Runs the host logic of pynbodyext.parallel.ShardedDirect / ShardedTree
unchanged in 2 gloo processes: balanced contiguous shards, the all-gather-v
of the 32-byte source records with uneven shards, self-skip offsets, the
weight-split symmetric triangle + accumulator all-reduce, cost-balanced
tree ranges with the cost all-gather, the profile all-reduce.  The device
layer is replaced by oracle stand-ins and the collectives by gloo
(tests/_mock_device.py); the real kernels over real collectives at world
2-4 are tests/test_gpu_multirank.py (ranks as threads on one GPU).
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

from pynbodyext.parallel import all_shards, shard_bounds

ROOT = Path(__file__).resolve().parent.parent


def test_shard_bounds_cover_and_balance():
    for n in (0, 1, 7, 10, 1_000_003):
        for w in (1, 2, 3, 8):
            sh = all_shards(n, w)
            assert sh[0][0] == 0 and sh[-1][1] == n
            assert all(sh[i][1] == sh[i + 1][0] for i in range(w - 1))
            sizes = [h - lo for lo, h in sh]
            assert max(sizes) - min(sizes) <= 1
            assert shard_bounds(n, w, w - 1) == sh[-1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, symmetric, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd"), str(ROOT / "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    import _mock_device as md
    from pynbodyext import parallel
    from pynbodyext.synthetic import plummer

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        parallel.nat = md.make_nat()      # device layer -> numpy / oracle stand-ins
        comm = md.GlooHostComm(dist, torch)
        pos, mass = plummer(n, seed=77)
        lo, hi = parallel.shard_bounds(n, world, rank)
        # ShardedDirect's own host logic: shards, record all-gather-v, the
        # weight-balanced unit ranges + accumulator all-reduce, finish
        s = parallel.ShardedDirect(comm, n, pos[lo:hi], mass[lo:hi], symmetric=symmetric)
        s.step()
        rec = md.view(s.d_rec.ptr, 32 * n, np.float64).reshape(n, 4)
        assert np.array_equal(rec[:, :3], pos) and np.array_equal(rec[:, 3], mass)
        pot, acc = s.results()
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.barrier()
        q.put((rank, lo, hi, pot, acc, float(t.item()), s.units if symmetric else None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("symmetric", [False, True])
def test_sharded_direct_world2_matches_unsharded(symmetric):
    """ShardedDirect (pynbodyext.parallel) over 2 gloo ranks with uneven
    shards: its host logic unchanged, the device calls replaced by the oracle
    (tests/_mock_device.py), the collectives by gloo = the unsharded oracle."""
    import multiprocessing as mp

    from oracle import gravity as og
    from pynbodyext.synthetic import plummer

    n, world = 1003, 2          # uneven shards: 502 + 501
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, symmetric, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pos, mass = plummer(n, seed=77)
    pot_ref = og.direct_potentials(pos, mass)
    acc_ref = og.direct_accelerations(pos, mass)
    res.sort(key=lambda r: r[0])
    if symmetric:  # the two ranks' unit ranges tile the triangle
        assert res[0][6][0] == 0 and res[0][6][1] == res[1][6][0]
        assert res[1][6][1] == (n + 63) // 64
    for rank, lo, hi, pot, acc, tmax, _ in res:
        assert tmax == float(world)
        if symmetric:  # every unordered pair once, summed in another order
            np.testing.assert_allclose(pot, pot_ref[lo:hi], rtol=1e-12)
            np.testing.assert_allclose(acc, acc_ref[lo:hi], rtol=1e-9, atol=1e-12)
        else:
            np.testing.assert_array_equal(pot, pot_ref[lo:hi])
            np.testing.assert_array_equal(acc, acc_ref[lo:hi])


def _rdzv_worker(rank, world, d, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]
    from pynbodyext.parallel import FileRendezvous

    r = FileRendezvous(rank, world, directory=d, key="k", timeout=60)
    q.put((rank, r.broadcast(b"unique-id-bytes" if rank == 0 else None)))


def test_file_rendezvous_world3(tmp_path):
    """The out-of-band RCCL unique-id exchange of bench.py (no torch import)."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rdzv_worker, args=(r, 3, str(tmp_path), q)) for r in (2, 1, 0)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=60) for _ in range(3))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert got == {0: b"unique-id-bytes", 1: b"unique-id-bytes", 2: b"unique-id-bytes"}


# --- Barnes-Hut: replicated tree, cost-balanced leaf-order target ranges ---
def test_balanced_ranges():
    from pynbodyext.parallel import balanced_ranges

    rng = np.random.default_rng(3)
    for n in (0, 1, 5, 1000):
        cost = rng.integers(1, 5000, n)
        for w in (1, 2, 3, 8):
            rr = balanced_ranges(cost, w)
            assert len(rr) == w
            assert sum(c for _, c in rr) == n
            assert all(rr[i][0] + rr[i][1] == rr[i + 1][0] for i in range(w - 1))
            if n >= 100 and w > 1:
                loads = [cost[f:f + c].sum() for f, c in rr]
                assert max(loads) <= cost.sum() / w + cost.max()


def _tree_worker(rank, world, port, n, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd"), str(ROOT / "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    import _mock_device as md
    from pynbodyext import _engine, parallel
    from pynbodyext.synthetic import plummer

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        parallel.nat = md.make_nat()
        _engine.Octree = md.MockOctree        # the oracle tree behind the Octree surface
        comm = md.GlooHostComm(dist, torch)
        pos, mass = plummer(n, seed=91)
        d_pos, d_mass = md.DeviceArray.from_host(pos), md.DeviceArray.from_host(mass)
        edges = np.logspace(np.log10(0.01), np.log10(50.0), 33)
        s = parallel.ShardedTree(comm, n, d_pos, d_mass, 8, 3, 0.5)
        steps = []
        for _ in range(2):  # step 2 balances on step 1's all-gathered costs
            mom = s.step(None, edges)
            first, count = s.ranges[rank]
            pot = md.view(s.d_pot.ptr, 8 * count, np.float64).copy()
            steps.append((list(s.ranges), s.tree.perm[first:first + count].copy(), pot, mom))
        q.put((rank, steps))
    finally:
        dist.destroy_process_group()


def test_sharded_tree_world2_profile_matches_unsharded():
    """ShardedTree (pynbodyext.parallel) over 2 gloo ranks, two steps: its
    host logic unchanged (ranges, cost all-gather-v -> original order ->
    balance, profile all-reduce), the tree = oracle/tree_ref.c behind the
    Octree surface (tests/_mock_device.py).  Every target's potential equals
    the unsharded oracle walk's, the all-reduced profile the unsharded one."""
    import multiprocessing as mp

    from oracle import tree as ot
    from pynbodyext.parallel import all_shards
    from pynbodyext.synthetic import plummer

    n, world = 3000, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tree_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pos, mass = plummer(n, seed=91)
    pot_ref = ot.RefOctree(pos, mass, 8, 3).compute_potentials(0.5)
    r = np.sqrt((pos[:, 0] * pos[:, 0] + pos[:, 1] * pos[:, 1]) + pos[:, 2] * pos[:, 2])
    edges = np.logspace(np.log10(0.01), np.log10(50.0), 33)
    b = np.searchsorted(edges, r, side="left") - 1
    ok = (b >= 0) & (b < 32)
    full = np.zeros((32, 2))
    np.add.at(full[:, 0], b[ok], mass[ok])
    np.add.at(full[:, 1], b[ok], mass[ok] * pot_ref[ok])
    for step in range(2):
        ranges = res[0][step][0]
        assert res[1][step][0] == ranges
        assert ranges[0][0] == 0 and sum(c for _, c in ranges) == n
        pot = np.full(n, np.nan)
        for rank in range(world):
            _, idx, p, mom = res[rank][step]
            pot[idx] = p
            np.testing.assert_allclose(mom[:, :2], full, rtol=1e-12, atol=1e-15)
        np.testing.assert_array_equal(pot, pot_ref)
    assert res[0][1][0] != [(lo, hi - lo) for lo, hi in all_shards(n, world)]


def _equaln_worker(rank, world, port, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd"), str(ROOT / "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from _msel_mock import GlooComm, NumpyMsel
    from pynbodyext.parallel import distributed_equaln

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(5)
        x = rng.lognormal(0.0, 2.0, 20_000)
        x[::101] = np.nan
        parts = np.split(x, [3000, 3000, 11_000])  # rank 1 holds nothing
        comm = GlooComm(dist, torch)
        out = {}
        for key, nb, lo, hi in (("plain", 64, None, None), ("clip", 100, 0.1, 30.0)):
            out[key] = distributed_equaln(NumpyMsel(parts[rank]), comm, nb, lo, hi)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_distributed_equaln_world4_protocol():
    """The distributed equaln protocol (parallel.distributed_equaln) over 4
    gloo ranks with uneven shards and an empty rank: every rank's edges equal
    the single-process equaln of the concatenation (bins.py:720-746).  The
    per-rank radix select is the numpy restatement of the device stages."""
    import multiprocessing as mp

    from oracle import profile_ref as pr

    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_equaln_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(5)
    x = rng.lognormal(0.0, 2.0, 20_000)
    x[::101] = np.nan
    want = {"plain": pr.edges_equaln(x, 64), "clip": pr.edges_equaln(x, 100, 0.1, 30.0)}
    for _, out in res:
        for key in want:
            assert np.array_equal(out[key], want[key], equal_nan=True), key


def test_distributed_equaln_rejects_u32_overflow():
    """The digit histograms are u32: a global kept count of 2**32 or more is
    refused before any histogram is summed (it would wrap silently)."""
    from pynbodyext.parallel import distributed_equaln

    class Dev:
        n = 1 << 31

        def key_range(self):
            raise AssertionError("must not be reached")

    class Comm:  # three ranks of 2**31 kept particles each
        def allreduce_host(self, a, op=0):
            return a * 3

    with pytest.raises(ValueError, match="u32"):
        distributed_equaln(Dev(), Comm(), 128)
