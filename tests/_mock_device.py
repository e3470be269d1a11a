"""CPU stand-ins for libpbx's device layer, so the HOST LOGIC of
pynbodyext.parallel.ShardedDirect / ShardedTree runs unchanged in gloo
processes without a GPU (tests/test_dist_gloo.py).  Test infrastructure
only — never imported by the product path.

* ``MockNat`` replaces the ``nat`` module that parallel.py calls: device
  arrays are numpy buffers at fake addresses (``.ptr`` / ``.offset()``
  behave like device pointers), and the handful of pbx_* entry points the
  sharded solvers call are restated with the oracle: pbx_pack_sources (the
  32-byte {x, y, z, m} records), pbx_direct_dev (oracle direct_subset, self
  pair at lo + t), and a symmetric-triangle plan of 64-row units whose
  accumulate / finish have the ABI meaning of pbx_direct_sym_* (each
  unordered pair once, credited to both particles).
* ``MockOctree`` stands for _engine.Octree over oracle/tree_ref.c's
  RefOctree (leaf order = its export's perm; costs = accepted nodes + leaf
  pairs; balance = parallel.balanced_ranges, which pbx_octree_balance
  reproduces, include/pbx.h).
* ``GlooHostComm`` is the Communicator surface parallel.py uses
  (allgatherv / allreduce_sum_f64 / allreduce) staged exactly like
  pbx_comm_init_host's host transport, over torch.distributed (gloo).
"""
from __future__ import annotations

import bisect
import ctypes
import types

import numpy as np

_BLOCKS: dict[int, np.ndarray] = {}
_BASES: list[int] = []
_NEXT = [1 << 44]


def _addr(p) -> int:
    if isinstance(p, ctypes.c_void_p):
        return int(p.value)
    return int(p)


def view(p, nbytes: int, dtype=np.uint8) -> np.ndarray:
    """numpy view of nbytes at mock device address p."""
    a = _addr(p)
    i = bisect.bisect_right(_BASES, a) - 1
    base = _BASES[i]
    off = a - base
    blk = _BLOCKS[base]
    if off + nbytes > blk.size:
        raise IndexError("mock device access out of bounds")
    return blk[off:off + nbytes].view(dtype)


class DeviceArray:
    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        base = _NEXT[0]
        _NEXT[0] += (max(self.nbytes, 16) // 4096 + 2) * 4096
        _BLOCKS[base] = np.zeros(max(self.nbytes, 16), dtype=np.uint8)
        bisect.insort(_BASES, base)
        self.ptr = ctypes.c_void_p(base)

    @classmethod
    def from_host(cls, a):
        a = np.ascontiguousarray(a)
        d = cls(a.nbytes)
        d.upload(a)
        return d

    def upload(self, a):
        a = np.ascontiguousarray(a)
        view(self.ptr, a.nbytes)[:] = a.view(np.uint8).reshape(-1)

    def download(self, out):
        out.view(np.uint8).reshape(-1)[:] = view(self.ptr, out.nbytes)
        return out

    def offset(self, nbytes: int):
        return ctypes.c_void_p(self.ptr.value + int(nbytes))

    def free(self):
        pass


SYM_ROWS = 64  # rows of the mock symmetric unit


def _byref_obj(r):
    return getattr(r, "_obj", r)


def _pack_sources(d_pos, d_mass, n, d_out):
    pos = view(d_pos, 24 * n, np.float64).reshape(n, 3)
    rec = view(d_out, 32 * n, np.float64).reshape(n, 4)
    rec[:, :3] = pos
    rec[:, 3] = 1.0 if d_mass is None else view(d_mass, 8 * n, np.float64)


def _sym_plan(n, p_npad, p_nunits, w):
    nunits = (int(n) + SYM_ROWS - 1) // SYM_ROWS
    if p_npad is not None:
        _byref_obj(p_npad).value = int(n)
        _byref_obj(p_nunits).value = nunits
    if w is not None:
        ww = np.ctypeslib.as_array(w, shape=(nunits,))
        for u in range(nunits):
            lo, hi = u * SYM_ROWS, min(n, (u + 1) * SYM_ROWS)
            ww[u] = sum(n - 1 - i for i in range(lo, hi))  # pairs (i, j > i)


def _sym_accumulate(d_rec, n, u0, u1, want, d_acc4):
    rec = view(d_rec, 32 * n, np.float64).reshape(n, 4)
    acc = view(d_acc4, 32 * n, np.float64).reshape(n, 4)
    for i in range(u0 * SYM_ROWS, min(n, u1 * SYM_ROWS)):
        d = rec[i + 1:, :3] - rec[i, :3]
        r2 = (d * d).sum(1)
        inv = 1.0 / np.sqrt(r2)
        inv3 = inv / r2
        acc[i, 0] -= (rec[i + 1:, 3] * inv).sum()
        acc[i + 1:, 0] -= rec[i, 3] * inv
        acc[i, 1:] += (rec[i + 1:, 3, None] * inv3[:, None] * d).sum(0)
        acc[i + 1:, 1:] -= rec[i, 3] * inv3[:, None] * d


def _sym_finish(d_acc4, lo, hi, want, pot, acc):
    a = view(d_acc4, 32 * hi, np.float64).reshape(hi, 4)[lo:hi]
    if pot is not None:
        view(pot, 8 * (hi - lo), np.float64)[:] = a[:, 0]
    if acc is not None:
        view(acc, 24 * (hi - lo), np.float64).reshape(-1, 3)[:] = a[:, 1:]


def _direct_dev(d_rec, d_soft, n_src, d_tgt, d_tsoft, m, self_lo, kernel, want, pot, acc):
    from oracle import gravity as og

    rec = view(d_rec, 32 * n_src, np.float64).reshape(n_src, 4)
    p, a = og.direct_subset(np.ascontiguousarray(rec[:, :3]), np.ascontiguousarray(rec[:, 3]),
                            np.arange(self_lo, self_lo + m))
    if pot is not None:
        view(pot, 8 * m, np.float64)[:] = p
    if acc is not None:
        view(acc, 24 * m, np.float64).reshape(m, 3)[:] = a


def _memset(p, value, nbytes):
    nb = nbytes.value if hasattr(nbytes, "value") else int(nbytes)
    view(p, nb)[:] = value


_CALLS = {
    "pbx_pack_sources": _pack_sources,
    "pbx_direct_sym_plan": _sym_plan,
    "pbx_direct_sym_accumulate": _sym_accumulate,
    "pbx_direct_sym_finish": _sym_finish,
    "pbx_direct_dev": _direct_dev,
    "pbx_memset": _memset,
}


def make_nat():
    """A stand-in for pynbodyext._native as parallel.py uses it."""
    from pynbodyext import _native as real

    m = types.SimpleNamespace()
    m.DeviceArray = DeviceArray
    m.WANT_POT, m.WANT_ACC, m.KERNEL_NONE = real.WANT_POT, real.WANT_ACC, real.KERNEL_NONE
    m.call = lambda name, *args: _CALLS[name](*args)
    m.synchronize = lambda: None
    return m


class MockOctree:
    """_engine.Octree's device-resident surface over the oracle tree."""

    def __init__(self, pos, mass, leaf, order):
        from oracle import tree as ot

        self.pos, self.mass = pos, mass
        self.ref = ot.RefOctree(pos, mass, leaf, order)
        self.perm = self.ref.export()["perm"].astype(np.int64)  # leaf order -> original
        self.n = len(pos)
        self._info = {}

    @classmethod
    def _from_device(cls, d_pos, n, d_mass, leaf, order):
        pos = view(d_pos, 24 * n, np.float64).reshape(n, 3).copy()
        mass = view(d_mass, 8 * n, np.float64).copy()
        return cls(pos, mass, leaf, order)

    def _set_cost_kind(self, kind):
        self.kind = kind

    def _set_walk_counters(self, enabled=True):
        # instrumentation only on the device: recorded
        self.counters = bool(enabled)

    def _rebuild_device(self, d_pos, n, d_mass):
        self.__init__(view(d_pos, 24 * n, np.float64).reshape(n, 3).copy(),
                      view(d_mass, 8 * n, np.float64).copy(), 8, 3)

    def _balance_device(self, d_cost_orig, world):
        from pynbodyext.parallel import balanced_ranges

        cost = view(d_cost_orig, 4 * self.n, np.int32)
        return balanced_ranges(cost[self.perm], world)

    def _compute_range_device(self, theta, want, first, count, compact, d_pot=None, d_acc=None,
                              d_cost=None):
        assert compact == 1
        idx = self.perm[first:first + count]
        pot, acc, nn, npp = self.ref.compute_subset(idx, theta)
        view(d_pot, 8 * count, np.float64)[:] = pot
        view(d_acc, 24 * count, np.float64).reshape(count, 3)[:] = acc
        if d_cost is not None:
            view(d_cost, 4 * count, np.int32)[:] = nn + npp
        self._info = {"node_interactions": int(nn.sum()), "leaf_pairs": int(npp.sum())}

    def info(self):
        return dict(self._info)

    def _cost_to_orig_device(self, d_cost_leaf, d_cost_orig):
        leaf = view(d_cost_leaf, 4 * self.n, np.int32)
        view(d_cost_orig, 4 * self.n, np.int32)[self.perm] = leaf

    def _moments(self, first, count, f, edges):
        idx = self.perm[first:first + count]
        p = self.pos[idx]
        r = np.sqrt((p[:, 0] * p[:, 0] + p[:, 1] * p[:, 1]) + p[:, 2] * p[:, 2])
        nb = len(edges) - 1
        b = np.searchsorted(edges, r, side="left") - 1
        b[r == edges[0]] = 0
        b[r == edges[-1]] = nb - 1
        ok = (b >= 0) & (b < nb)
        w = self.mass[idx]
        cols = [w, f * w, f * f * w, f, f * f, np.abs(f) * w, np.abs(f)]
        counts = np.bincount(b[ok], minlength=nb).astype(np.int64)
        mom = np.stack([np.bincount(b[ok], weights=c[ok], minlength=nb) for c in cols], axis=1)
        return counts, mom

    def _radial_moments_device(self, first, count, d_f, edges):
        return self._moments(first, count, view(d_f, 8 * count, np.float64), np.asarray(edges))

    def _radial_moments_into(self, first, count, d_f, edges, d_out):
        counts, mom = self._moments(first, count, view(d_f, 8 * count, np.float64),
                                    np.asarray(edges))
        nb = len(counts)
        view(d_out, 8 * nb, np.int64)[:] = counts
        view(ctypes.c_void_p(_addr(d_out) + 8 * nb), 56 * nb, np.float64).reshape(nb, 7)[:] = mom

    def close(self):
        pass


class GlooHostComm:
    """Communicator surface of parallel.py over torch.distributed (gloo),
    staged through host arrays like pbx_comm_init_host: device bytes ->
    host -> collective -> device."""

    def __init__(self, dist, torch):
        self.dist, self.torch = dist, torch
        self.nranks, self.rank = dist.get_world_size(), dist.get_rank()

    def allgatherv(self, d_buf, counts, displs):
        t = self.torch
        maxc = max(counts)
        mine = np.zeros(maxc, dtype=np.uint8)
        c, d = counts[self.rank], displs[self.rank]
        mine[:c] = view(ctypes.c_void_p(_addr(d_buf) + d), c)
        parts = [t.zeros(maxc, dtype=t.uint8) for _ in range(self.nranks)]
        self.dist.all_gather(parts, t.from_numpy(mine))
        for r in range(self.nranks):
            if counts[r]:
                view(ctypes.c_void_p(_addr(d_buf) + displs[r]), counts[r])[:] = \
                    parts[r].numpy()[:counts[r]]

    def allreduce(self, d_send, d_recv, count, dtype, op=0):
        dt = (np.float64, np.int64, np.uint64, np.uint32)[dtype]
        nb = count * np.dtype(dt).itemsize
        a = view(d_send, nb, dt).copy()
        ten = self.torch.from_numpy(a.astype(np.float64 if dtype == 0 else np.int64))
        red = {0: self.dist.ReduceOp.SUM, 1: self.dist.ReduceOp.MIN, 2: self.dist.ReduceOp.MAX}[op]
        self.dist.all_reduce(ten, op=red)
        view(d_recv, nb, dt)[:] = ten.numpy().astype(dt)

    def allreduce_sum_f64(self, d_send, d_recv, count):
        self.allreduce(d_send, d_recv, count, 0)
