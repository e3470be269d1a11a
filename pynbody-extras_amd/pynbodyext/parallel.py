"""Multi-GPU execution: one process per GPU, RCCL over xGMI.

The reference is single-process (rayon threads over targets);
this module is the MI355X scale-out of the same solve:

* direct summation shards the TARGETS: rank r owns particles
  [lo_r, hi_r) (contiguous, balanced); every rank packs its particles into
  32-byte source records, one all-gather-v (RCCL broadcasts in a group)
  gives every rank all N records, and each rank runs the direct-sum kernel
  for its own targets with self-skip offset lo_r.  Outputs stay sharded.
* profile partials (int64 counts, f64 per-bin sums) are summed with one
  all-reduce.
* profiles over particles sharded across ranks (ShardedProfile): equaln
  edges are the global order statistics, found by the device radix select
  with its per-level digit histograms summed over ranks (u32 all-reduce:
  64 KB at level 0, nbins+1 rows of 16 KB after); counts, per-bin sums and
  the global CSR offsets are all-reduced.

The control plane (unique-id exchange, barriers) is the caller's, e.g.
torch.distributed with the gloo backend; the data path is RCCL only.
"""
from __future__ import annotations

import ctypes
from ctypes import c_int64, c_void_p

import os

import numpy as np

from . import _native as nat


SYM_MIN_N = 8192  # all-particles solves of at least this size use direct_sym.hip

# pbx_comm_allreduce dtypes / ops
DT_F64, DT_I64, DT_U64, DT_U32 = 0, 1, 2, 3
OP_SUM, OP_MIN, OP_MAX = 0, 1, 2


def shard_bounds(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous balanced shard [lo, hi) of rank (first n % world ranks get +1)."""
    base, extra = divmod(int(n_total), int(world))
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def all_shards(n_total: int, world: int) -> list[tuple[int, int]]:
    return [shard_bounds(n_total, world, r) for r in range(world)]


class Communicator:
    """RCCL communicator of libpbx (device buffers, library stream)."""

    def __init__(self, nranks: int, rank: int, uid: bytes):
        self.nranks, self.rank = int(nranks), int(rank)
        h = c_void_p()
        nat.call("pbx_comm_init", ctypes.byref(h), self.nranks, self.rank, bytes(uid))
        self.handle = h

    @staticmethod
    def unique_id() -> bytes:
        lib = nat.load()
        size = lib.pbx_comm_unique_id_size()
        buf = ctypes.create_string_buffer(size)
        nat.call("pbx_comm_unique_id", buf, size)
        return buf.raw

    def allgatherv(self, d_buf, counts_bytes, displs_bytes) -> None:
        c = np.ascontiguousarray(counts_bytes, dtype=np.int64)
        d = np.ascontiguousarray(displs_bytes, dtype=np.int64)
        nat.call("pbx_comm_allgatherv", self.handle, d_buf, c.ctypes.data_as(ctypes.POINTER(c_int64)),
                 d.ctypes.data_as(ctypes.POINTER(c_int64)))

    def allgather_inplace(self, d_buf, bytes_per_rank: int) -> None:
        counts = [bytes_per_rank] * self.nranks
        displs = [r * bytes_per_rank for r in range(self.nranks)]
        self.allgatherv(d_buf, counts, displs)

    def allreduce_sum_f64(self, d_send, d_recv, count: int) -> None:
        nat.call("pbx_comm_allreduce_f64", self.handle, d_send, d_recv, int(count))

    def allreduce_sum_i64(self, d_send, d_recv, count: int) -> None:
        nat.call("pbx_comm_allreduce_i64", self.handle, d_send, d_recv, int(count))

    def allreduce(self, d_send, d_recv, count: int, dtype: int, op: int = OP_SUM) -> None:
        """Device all-reduce (dtype DT_*, op OP_*), e.g. in place."""
        nat.call("pbx_comm_allreduce", self.handle, d_send, d_recv, int(count), int(dtype),
                 int(op))

    def allreduce_host(self, a: np.ndarray, op: int = OP_SUM) -> np.ndarray:
        """All-reduce of a small host array (f64 / i64 / u64 / u32) through the
        communicator's persistent HBM staging (one call, one stream sync)."""
        out = np.array(a, copy=True, order="C")
        dt = {np.dtype(np.float64): DT_F64, np.dtype(np.int64): DT_I64,
              np.dtype(np.uint64): DT_U64, np.dtype(np.uint32): DT_U32}[out.dtype]
        nat.call("pbx_comm_allreduce_host", self.handle, out.ctypes.data_as(c_void_p), out.size,
                 dt, int(op))
        return out

    def barrier(self) -> None:
        nat.call("pbx_comm_barrier", self.handle)

    def max(self, value: float) -> float:
        out = ctypes.c_double(0.0)
        nat.call("pbx_comm_max_f64", self.handle, float(value), ctypes.byref(out))
        return out.value

    def destroy(self) -> None:
        if self.handle is not None and self.handle.value:
            nat.call("pbx_comm_destroy", self.handle)
        self.handle = c_void_p()


_NP_DTYPES = (np.float64, np.int64, np.uint64, np.uint32)  # pbx_comm_allreduce dtype codes


class HostCommunicator(Communicator):
    """A communicator whose collectives run over a HOST transport instead of
    RCCL (pbx_comm_init_host): the library stages every collective's device
    bytes through pinned memory and calls ``transport``, an object with

    * ``allreduce(a: np.ndarray, op: int)`` — reduce ``a`` over the ranks in
      place (OP_SUM / OP_MIN / OP_MAX);
    * ``allgatherv(buf: np.ndarray[uint8], counts, displs)`` — fill in the
      other ranks' byte segments of ``buf`` (this rank's is in place).

    Every library path that takes a communicator (ShardedDirect, ShardedTree,
    ShardedProfile, the one-call distributed profile) runs over it unchanged;
    :class:`ThreadLoopback` is the transport for several ranks as threads of
    one process on one GPU."""

    def __init__(self, nranks: int, rank: int, transport):
        self.nranks, self.rank = int(nranks), int(rank)
        self.transport = transport

        def fn(_ctx, kind, buf, count, dtype, op, counts, displs):
            try:
                if kind == nat.COLL_ALLREDUCE:
                    dt = np.dtype(_NP_DTYPES[dtype])
                    a = np.ctypeslib.as_array(
                        (ctypes.c_uint8 * (int(count) * dt.itemsize)).from_address(buf)).view(dt)
                    transport.allreduce(a, int(op))
                elif kind == nat.COLL_ALLGATHERV:
                    c = [int(counts[r]) for r in range(self.nranks)]
                    d = [int(displs[r]) for r in range(self.nranks)]
                    size = max((d[r] + c[r] for r in range(self.nranks) if c[r]), default=0)
                    b = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(buf))
                    transport.allgatherv(b, c, d)
                else:
                    return 2
                return 0
            except BaseException as e:  # noqa: BLE001 - reported as a status to C
                self.error = e
                abort = getattr(transport, "abort", None)
                if abort is not None:
                    abort()
                return 1

        self.error = None
        self._fn = nat.HOST_COLLECTIVE_FN(fn)  # kept alive as long as the handle
        h = c_void_p()
        nat.call("pbx_comm_init_host", ctypes.byref(h), self.nranks, self.rank, self._fn, None)
        self.handle = h


class ThreadLoopback:
    """Host transport for ``world`` ranks that are threads of ONE process
    sharing one device: what a multi-GPU job does, on one GPU (the library
    releases its device lock while a rank waits in a collective).  Sums are
    taken in rank order; a rank that fails aborts the group so no rank waits
    forever.  ``run(fn)`` calls ``fn(comm)`` on one thread per rank and
    returns the per-rank results (re-raising the first failure)."""

    def __init__(self, world: int, timeout: float = 120.0):
        import threading

        self.world = int(world)
        self._barrier = threading.Barrier(self.world, timeout=timeout)
        self._slots = [None] * self.world
        self._rank = threading.local()

    def abort(self) -> None:
        self._barrier.abort()

    def _exchange(self, item):
        self._slots[self._rank.value] = item
        self._barrier.wait()
        return list(self._slots)

    def allreduce(self, a: np.ndarray, op: int) -> None:
        parts = self._exchange(a.copy())
        if len({(p.shape, p.dtype.str) for p in parts}) > 1:
            raise RuntimeError("all-reduce of different sizes / types across ranks: "
                               f"{[(p.shape, p.dtype.str) for p in parts]}")
        if op == OP_SUM:
            acc = parts[0].copy()
            for p in parts[1:]:
                acc += p  # rank order (u32: wraps like the RCCL sum)
        elif op == OP_MIN:
            acc = np.minimum.reduce(parts)
        else:
            acc = np.maximum.reduce(parts)
        self._barrier.wait()  # every rank read the slots before any overwrites them
        a[...] = acc

    def allgatherv(self, buf: np.ndarray, counts, displs) -> None:
        r = self._rank.value
        mine = buf[displs[r]:displs[r] + counts[r]].copy()
        parts = self._exchange((list(counts), list(displs), mine))
        if any(p[0] != parts[0][0] or p[1] != parts[0][1] for p in parts):
            raise RuntimeError("all-gather-v with different segment tables across ranks")
        self._barrier.wait()
        for q, (_, _, seg) in enumerate(parts):
            if q != r and counts[q]:
                buf[displs[q]:displs[q] + counts[q]] = seg

    def run(self, fn):
        """fn(comm) on one thread per rank; returns [result of rank r]."""
        import threading

        out = [None] * self.world
        errs = [None] * self.world

        def body(r):
            self._rank.value = r
            comm = None
            try:
                comm = HostCommunicator(self.world, r, self)
                out[r] = fn(comm)
            except BaseException as e:  # noqa: BLE001
                errs[r] = (comm.error if comm is not None else None) or e
                self.abort()
            finally:
                if comm is not None:
                    comm.destroy()

        ts = [threading.Thread(target=body, args=(r,)) for r in range(self.world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for e in errs:
            if e is not None and not isinstance(e, threading.BrokenBarrierError):
                raise e
        for e in errs:
            if e is not None:
                raise e
        return out


class FileRendezvous:
    """Out-of-band exchange of the RCCL unique id between the ranks of ONE
    node, through a file in a local directory.

    The launch key is (MASTER_ADDR, MASTER_PORT, parent pid): every rank of
    one ``torch.distributed.run`` launch is a child of the same agent, so
    concurrent or stale launches never share a file.  No torch import is
    needed in the worker (the launcher only sets the environment).
    """

    def __init__(self, rank: int, world: int, directory: str | None = None,
                 key: str | None = None, timeout: float = 600.0):
        import os
        import tempfile

        self.rank, self.world, self.timeout = int(rank), int(world), float(timeout)
        if key is None:
            key = "{}_{}_{}".format(os.environ.get("MASTER_ADDR", "local"),
                                    os.environ.get("MASTER_PORT", "0"), os.getppid())
        d = directory or os.environ.get("PBX_RDZV_DIR") or tempfile.gettempdir()
        self.path = os.path.join(d, f"pbx_rdzv_{key}.uid")

    def broadcast(self, payload: bytes | None) -> bytes:
        import os
        import time

        if self.rank == 0:
            tmp = f"{self.path}.tmp{os.getpid()}"
            with open(tmp, "wb") as f:
                f.write(payload)
            os.replace(tmp, self.path)
            return payload
        t0 = time.monotonic()
        while True:
            try:
                with open(self.path, "rb") as f:
                    data = f.read()
                if data:
                    return data
            except FileNotFoundError:
                pass
            if time.monotonic() - t0 > self.timeout:
                raise TimeoutError(f"rank {self.rank}: no rendezvous file {self.path}")
            time.sleep(0.05)

    def cleanup(self) -> None:
        import os

        if self.rank == 0:
            try:
                os.remove(self.path)
            except FileNotFoundError:
                pass


class ShardedDirect:
    """Direct-sum gravity over particles sharded across ranks (device-resident).

    ``comm`` is a :class:`Communicator` (or None for a single rank).  The
    local shard (positions, masses) lives in HBM; ``step`` computes the
    potential and acceleration of the local particles due to ALL particles.
    """

    def __init__(self, comm, n_total: int, pos_local: np.ndarray, mass_local: np.ndarray | None,
                 symmetric: bool | None = None):
        self.comm = comm
        world = comm.nranks if comm is not None else 1
        rank = comm.rank if comm is not None else 0
        # each unordered pair once (csrc/direct_sym.hip): the work units of the
        # pair triangle are split across ranks by weight, one RCCL all-reduce
        # of the per-particle accumulator, each rank converts its own shard
        self.symmetric = (n_total >= SYM_MIN_N) if symmetric is None else bool(symmetric)
        self.n_total = int(n_total)
        self.shards = all_shards(self.n_total, world)
        self.lo, self.hi = self.shards[rank]
        self.n_loc = self.hi - self.lo
        if pos_local.shape != (self.n_loc, 3):
            raise ValueError(f"rank {rank} expects {self.n_loc} local particles")
        self.d_pos = nat.DeviceArray.from_host(np.ascontiguousarray(pos_local, dtype=np.float64))
        self.d_mass = (nat.DeviceArray.from_host(np.ascontiguousarray(mass_local, dtype=np.float64))
                       if mass_local is not None else None)
        self.d_rec = nat.DeviceArray(32 * self.n_total)
        self.d_pot = nat.DeviceArray(8 * max(self.n_loc, 1))
        self.d_acc = nat.DeviceArray(24 * max(self.n_loc, 1))
        self._counts = [32 * (h - lo) for lo, h in self.shards]
        self._displs = [32 * lo for lo, _ in self.shards]
        if self.symmetric:
            npad, nunits = ctypes.c_int64(), ctypes.c_int64()
            nat.call("pbx_direct_sym_plan", self.n_total, ctypes.byref(npad), ctypes.byref(nunits),
                     None)
            w = np.zeros(nunits.value, dtype=np.int64)
            nat.call("pbx_direct_sym_plan", self.n_total, None, None,
                     w.ctypes.data_as(ctypes.POINTER(c_int64)))
            first, count = balanced_ranges(w, world)[rank]
            self.units = (first, first + count)
            self.npad = npad.value
            self.d_acc4 = nat.DeviceArray(32 * self.npad)

    def gather_sources(self) -> None:
        nat.call("pbx_pack_sources", self.d_pos.ptr, self.d_mass.ptr if self.d_mass else None,
                 self.n_loc, self.d_rec.offset(32 * self.lo))
        if self.comm is not None and self.comm.nranks > 1:
            self.comm.allgatherv(self.d_rec.ptr, self._counts, self._displs)

    def solve(self, want: int = nat.WANT_POT | nat.WANT_ACC) -> None:
        pot = self.d_pot.ptr if want & nat.WANT_POT else None
        acc = self.d_acc.ptr if want & nat.WANT_ACC else None
        if not self.symmetric:
            nat.call("pbx_direct_dev", self.d_rec.ptr, None, self.n_total, self.d_pos.ptr, None,
                     self.n_loc, self.lo, nat.KERNEL_NONE, want, pot, acc)
            return
        nat.call("pbx_memset", self.d_acc4.ptr, 0, ctypes.c_size_t(32 * self.npad))
        nat.call("pbx_direct_sym_accumulate", self.d_rec.ptr, self.n_total, self.units[0],
                 self.units[1], want, self.d_acc4.ptr)
        if self.comm is not None:
            self.comm.allreduce_sum_f64(self.d_acc4.ptr, self.d_acc4.ptr, 4 * self.npad)
        nat.call("pbx_direct_sym_finish", self.d_acc4.ptr, self.lo, self.hi, want, pot, acc)

    def step(self, want: int = nat.WANT_POT | nat.WANT_ACC) -> None:
        self.gather_sources()
        self.solve(want)

    def results(self) -> tuple[np.ndarray, np.ndarray]:
        pot = np.empty(self.n_loc)
        acc = np.empty((self.n_loc, 3))
        if self.n_loc:
            self.d_pot.download(pot)
            self.d_acc.download(acc)
        return pot, acc


def balanced_ranges(cost: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Split targets (in the tree's leaf order) into ``world`` contiguous
    ranges of about equal summed ``cost`` (interactions per target from a
    previous walk).  Returns [(first, count)] per rank."""
    c = np.asarray(cost, dtype=np.float64).reshape(-1)
    n = c.shape[0]
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, 0)] * max(world - 1, 0)
    cum = np.cumsum(np.maximum(c, 1.0))
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(cum, total * r / world, side="left")) + 1)
    cuts.append(n)
    cuts = np.minimum(np.maximum.accumulate(np.asarray(cuts)), n)
    return [(int(cuts[r]), int(cuts[r + 1] - cuts[r])) for r in range(world)]


def align_ranges(ranges, n: int, q: int):
    """Contiguous (first, count) ranges with every inner cut rounded to a
    multiple of q (monotone, the last range ending at n)."""
    cuts = [0]
    for first, count in ranges[1:]:
        c = min(n, max(cuts[-1], int(round(first / q)) * q))
        cuts.append(c)
    cuts.append(n)
    return [(a, b - a) for a, b in zip(cuts[:-1], cuts[1:])]


class ShardedTree:
    """Barnes-Hut solve + radial potential profile, one rank per GPU.

    Every rank builds the full octree from the (replicated, HBM-resident)
    particle set and walks its own contiguous range of the leaf-ordered
    targets.  One step (all of it timed by bench.py) =

    * ``build()``   — device octree + payloads (identical on every rank);
    * ``balance()`` — the ranges: contiguous leaf-order pieces of equal
      summed cost, where a target's cost is its interaction count in the
      PREVIOUS step's walk, carried in original particle order (so a
      changed snapshot / leaf order still maps); before any walk, equal
      target counts.  Device-side (two small kernels, one (world+1)-int
      read-back) — no extra walk;
    * ``walk()``    — this rank's targets, writing their costs (the work of
      each target's wave: node steps + 4-record leaf rounds, what the walk's
      time follows); the costs are all-gathered (RCCL, 4 bytes per particle)
      and moved to original order for the next step;
    * ``profile()`` — per-bin partial moments of this rank's targets, one
      RCCL all-reduce of nbins x 7 doubles.

    Strong scaling: the particle set is fixed.  The reference has no
    multi-process path; its rayon pool splits the targets of one process
    (tree.rs:1443-1556).
    """

    def __init__(self, comm, n: int, d_pos, d_mass, leaf_capacity: int = 8,
                 multipole_order: int = 3, theta: float = 0.5):
        self.comm = comm
        self.world = comm.nranks if comm is not None else 1
        self.rank = comm.rank if comm is not None else 0
        self.n, self.d_pos, self.d_mass = int(n), d_pos, d_mass
        self.leaf, self.order, self.theta = leaf_capacity, multipole_order, theta
        self.ranges = None
        self.tree = None
        cap = self.n  # worst-case shard
        self.d_pot = nat.DeviceArray(8 * max(cap, 1))
        self.d_acc = nat.DeviceArray(24 * max(cap, 1))
        self.d_cost = nat.DeviceArray(4 * max(cap, 1))       # leaf order, last walk
        self.d_cost_orig = nat.DeviceArray(4 * max(cap, 1))  # original order, carried
        self.have_costs = False
        self.info = None
        self.count_walks = True  # walk statistics (set_walk_counters)
        self.d_prof = None  # [counts | moments] of the profile all-reduce

    def build(self):
        from ._engine import Octree

        if self.tree is None:
            self.tree = Octree._from_device(self.d_pos.ptr, self.n, self.d_mass.ptr, self.leaf,
                                            self.order)
            self.tree._set_cost_kind(1)
            self.tree._set_walk_counters(self.count_walks)
        else:  # next step / snapshot: same handle, HBM buffers reused
            self.tree._rebuild_device(self.d_pos.ptr, self.n, self.d_mass.ptr)

    def set_walk_counters(self, enabled: bool) -> None:
        """Walk statistics on / off for the later walks (info keeps the last
        counted walk's); the walk's decisions and sums do not change."""
        self.count_walks = bool(enabled)
        if self.tree is not None:
            self.tree._set_walk_counters(self.count_walks)

    def balance(self):
        """This step's target ranges (see the class docstring)."""
        if self.world == 1:
            self.ranges = [(0, self.n)]
        elif self.have_costs:
            self.ranges = self.tree._balance_device(self.d_cost_orig.ptr, self.world)
        else:
            self.ranges = [(lo, hi - lo) for lo, hi in all_shards(self.n, self.world)]
        return self.ranges

    def walk(self, want: int = nat.WANT_POT | nat.WANT_ACC, share: bool = True):
        """This rank's targets; ``share`` then runs share_costs()."""
        if self.ranges is None:
            self.balance()
        first, count = self.ranges[self.rank]
        multi = self.world > 1
        self.tree._compute_range_device(self.theta, want, first, count, 1, self.d_pot.ptr,
                                        self.d_acc.ptr,
                                        self.d_cost.offset(4 * first) if multi else None)
        info = self.tree.info()
        if self.count_walks or self.info is None:  # (uncounted walks report zeros)
            self.info = info
        if multi and share:
            self.share_costs()
        return first, count

    def share_costs(self):
        """All-gather every rank's walk costs, then to original order."""
        if self.world == 1:
            return
        if self.comm is not None and self.world > 1:
            self.comm.allgatherv(self.d_cost.ptr, [4 * c for _, c in self.ranges],
                                 [4 * f for f, _ in self.ranges])
        self.tree._cost_to_orig_device(self.d_cost.ptr, self.d_cost_orig.ptr)
        self.have_costs = True

    def profile(self, dev_bins, edges) -> np.ndarray:
        """Per-bin moments (nbins, 7) of this rank's targets, summed over ranks
        (RadialProfile ndim=3 of the potential with the mass as weight: the
        pbx_profile_moments columns, f = potential).  One fused device pass
        over the leaf-ordered records and this rank's potentials
        (pbx_octree_radial_moments); the summed bin counts are left in
        ``dev_bins.counts`` when a DeviceBins is given."""
        first, count = self.ranges[self.rank] if self.ranges else (0, self.n)
        if self.comm is not None:
            # the partial profile stays on the device: [counts | moments]
            # all-reduced in place (RCCL), one read-back
            nb = len(edges) - 1
            if self.d_prof is None or self.d_prof.nbytes < 64 * nb:
                if self.d_prof is not None:
                    self.d_prof.free()
                self.d_prof = nat.DeviceArray(64 * nb)
            self.tree._radial_moments_into(first, count, self.d_pot.ptr, edges, self.d_prof.ptr)
            self.comm.allreduce(self.d_prof.ptr, self.d_prof.ptr, nb, DT_I64)
            self.comm.allreduce(self.d_prof.offset(8 * nb), self.d_prof.offset(8 * nb), 7 * nb,
                                DT_F64)
            flat = np.empty(8 * nb)
            self.d_prof.download(flat)
            counts = flat[:nb].view(np.int64).copy()
            mom = flat[nb:].reshape(nb, 7)
        else:
            counts, mom = self.tree._radial_moments_device(first, count, self.d_pot.ptr, edges)
        if dev_bins is not None:
            dev_bins.counts = counts
            dev_bins.nbins = len(counts)
        return mom

    def step(self, dev_bins, edges, want: int = nat.WANT_POT | nat.WANT_ACC) -> np.ndarray:
        self.build()
        self.balance()
        self.walk(want)
        return self.profile(dev_bins, edges)

    def close(self):
        if self.tree is not None:
            self.tree.close()
            self.tree = None
        for a in (self.d_pot, self.d_acc, self.d_cost, self.d_cost_orig, self.d_prof):
            if a is not None:
                a.free()
        self.d_prof = None


def distributed_equaln(dev, comm, nbins: int, bin_min=None, bin_max=None) -> np.ndarray:
    """Global equaln edges of the x values held by all ranks (bins.py:720-746
    on the concatenation), every rank the same.  ``dev`` offers the staged
    radix select (DeviceBins.key_range / msel_*); ``comm`` the all-reduces
    (Communicator: allreduce_host for the key range, allreduce in place on
    the device histogram).  The histograms are summed before every resolve,
    so each rank picks the same digits and no particle moves.

    The digit histograms (and the window counts the resolve derives from
    them) are u32: the global kept count is all-reduced in i64 first and a
    total that does not fit u32 is rejected instead of silently wrapping."""
    total = int(comm.allreduce_host(np.array([int(dev.n)], dtype=np.int64))[0])
    if total >= 1 << 32:
        raise ValueError(f"distributed equaln over {total} particles: the u32 radix-select "
                         "histograms hold at most 2**32 - 1")
    kmin, kmax = dev.key_range()
    kmin = int(comm.allreduce_host(np.array([kmin], dtype=np.uint64), OP_MIN)[0])
    kmax = int(comm.allreduce_host(np.array([kmax], dtype=np.uint64), OP_MAX)[0])
    levels = dev.msel_begin(nbins, bin_min, bin_max, kmin, kmax)
    for level in range(levels):
        ptr, count = dev.msel_hist(level)
        comm.allreduce(ptr, ptr, count, DT_U32, OP_SUM)
        dev.msel_resolve(level)
    return dev.msel_edges()


class ShardedProfile:
    """RadialProfile over particles sharded across ranks:
    each rank selects and bins its own particles; edges (equaln: distributed
    radix select), counts and per-bin sums are global.  ``offset`` is this
    rank's first global particle index (for the global binind)."""

    def __init__(self, comm, dev, offset: int = 0):
        self.comm, self.dev, self.offset = comm, dev, int(offset)
        self.world = comm.nranks if comm is not None else 1
        self.rank = comm.rank if comm is not None else 0

    def radial_equaln(self, pos, mass=None, **kw):
        """The whole equaln radial profile of the sharded particles in one
        call per rank (DeviceBins.radial_equaln with the communicator:
        selection, global edges, assignment, CSR, global counts and sums with
        device all-reduces between the kernels).  Returns (global edges,
        global counts, global per-statistic sums); this rank's counts and CSR
        stay in ``self.dev``."""
        from .profiles._device import DeviceBins

        _, edges, counts, mom = DeviceBins.radial_equaln(pos, mass, into=self.dev, comm=self.comm,
                                                         **kw)
        return edges, counts, mom

    def edges_equaln(self, nbins: int, bin_min=None, bin_max=None) -> np.ndarray:
        if self.comm is None:
            return self.dev.edges_equaln(nbins, bin_min, bin_max)
        return distributed_equaln(self.dev, self.comm, nbins, bin_min, bin_max)

    def assign(self, edges) -> np.ndarray:
        """Global per-bin counts (this rank's stay in dev.counts)."""
        local = self.dev.assign(edges)
        return local.copy() if self.comm is None else self.comm.allreduce_host(local)

    def moments(self, field, weights, cols: int = (1 << 7) - 1) -> np.ndarray:
        local = self.dev.moments(field, weights, cols)
        return local if self.comm is None else self.comm.allreduce_host(local)

    def csr(self) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(global particle indices of this rank's members, global offsets
        (nbins + 1), start of this rank's run inside every bin).  Bin b of
        the global binind = the ranks' runs in rank order."""
        perm, _ = self.dev.csr()
        local = self.dev.counts
        nb = local.shape[0]
        table = np.zeros((self.world, nb), dtype=np.int64)
        table[self.rank] = local
        if self.comm is not None:
            table = self.comm.allreduce_host(table)
        glob = table.sum(0)
        offs = np.zeros(nb + 1, dtype=np.int64)
        np.cumsum(glob, out=offs[1:])
        start = offs[:-1] + table[:self.rank].sum(0)
        return perm + self.offset, offs, start
