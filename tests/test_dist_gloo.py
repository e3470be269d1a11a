"""N>1 host logic on CPU: world_size-2 gloo processes.

Covers the multi-GPU bookkeeping of pynbodyext.parallel (balanced
contiguous shards, all-gather-v of the 32-byte source records with uneven
shards, self-skip offsets of the sharded solve) and the bench control plane
(barrier, max over ranks).  The device all-gather itself is RCCL on the GPU
box; here the same record layout is gathered with gloo and each rank's
targets are solved by the oracle, then compared with the unsharded oracle.
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


def _worker(rank, world, port, n, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from oracle import gravity as og
    from pynbodyext.parallel import all_shards, shard_bounds
    from pynbodyext.synthetic import plummer

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pos, mass = plummer(n, seed=77)
        lo, hi = shard_bounds(n, world, rank)
        # pack the local shard exactly like pbx_pack_sources: {x, y, z, m}
        rec_local = np.concatenate([pos[lo:hi], mass[lo:hi, None]], axis=1)
        shards = all_shards(n, world)
        maxn = max(h - l for l, h in shards)
        buf = torch.zeros((maxn, 4), dtype=torch.float64)
        buf[: hi - lo] = torch.from_numpy(rec_local)
        parts = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf)
        rec = np.concatenate([parts[r][: h - l].numpy() for r, (l, h) in enumerate(shards)])
        assert np.array_equal(rec[:, :3], pos) and np.array_equal(rec[:, 3], mass)
        # this rank's targets against all sources, self-skip at global index lo + t
        pot, acc = og.direct_subset(np.ascontiguousarray(rec[:, :3]), np.ascontiguousarray(rec[:, 3]),
                                    np.arange(lo, hi))
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.barrier()
        q.put((rank, lo, hi, pot, acc, float(t.item())))
    finally:
        dist.destroy_process_group()


def test_sharded_direct_world2_matches_unsharded():
    import multiprocessing as mp

    from oracle import gravity as og
    from pynbodyext.synthetic import plummer

    n, world = 1003, 2          # uneven shards: 502 + 501
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pos, mass = plummer(n, seed=77)
    pot_ref = og.direct_potentials(pos, mass)
    acc_ref = og.direct_accelerations(pos, mass)
    for rank, lo, hi, pot, acc, tmax in res:
        assert tmax == float(world)
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
    sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from oracle import tree as ot
    from pynbodyext.parallel import balanced_ranges
    from pynbodyext.synthetic import plummer

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pos, mass = plummer(n, seed=91)
        ref = ot.RefOctree(pos, mass, 8, 3)       # every rank builds the tree
        e = ref.export()
        order = e["perm"]                          # leaf order -> original index
        # costs of a first walk, then this rank's balanced leaf-order range
        _, _, nn, npp = ref.compute_subset(order, 0.5)
        first, count = balanced_ranges(nn + npp, world)[rank]
        idx = order[first:first + count]
        pot, _, _, _ = ref.compute_subset(idx, 0.5)
        r = np.sqrt((pos[idx] ** 2).sum(1))
        edges = np.logspace(np.log10(0.01), np.log10(50.0), 33)
        b = np.searchsorted(edges, r, side="left") - 1
        ok = (b >= 0) & (b < 32)
        part = np.zeros((32, 2))
        np.add.at(part[:, 0], b[ok], mass[idx][ok])
        np.add.at(part[:, 1], b[ok], mass[idx][ok] * pot[ok])
        t = torch.from_numpy(part)
        dist.all_reduce(t)                         # RCCL all-reduce on the GPU box
        q.put((rank, first, count, t.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_sharded_tree_world2_profile_matches_unsharded():
    import multiprocessing as mp

    from oracle import tree as ot
    from pynbodyext.synthetic import plummer

    n, world = 3000, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tree_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert res[0][1] == 0 and res[0][2] + res[1][2] == n and res[1][1] == res[0][2]
    pos, mass = plummer(n, seed=91)
    pot = ot.RefOctree(pos, mass, 8, 3).compute_potentials(0.5)
    r = np.sqrt((pos ** 2).sum(1))
    edges = np.logspace(np.log10(0.01), np.log10(50.0), 33)
    b = np.searchsorted(edges, r, side="left") - 1
    ok = (b >= 0) & (b < 32)
    full = np.zeros((32, 2))
    np.add.at(full[:, 0], b[ok], mass[ok])
    np.add.at(full[:, 1], b[ok], mass[ok] * pot[ok])
    for _, _, _, part in res:
        np.testing.assert_allclose(part, full, rtol=1e-12, atol=1e-15)


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
