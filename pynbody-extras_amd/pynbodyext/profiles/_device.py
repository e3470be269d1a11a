"""Device state of one binning (libpbx profile handle, HBM-resident).

Thin ctypes wrapper of the pbx_profile_* entry points (include/pbx.h):
the binned quantity x (and, after a fused selection, the selection mass
and original indices) stays in HBM; edges, counts, CSR and per-bin sums are
computed by the HIP kernels of csrc/profile.hip.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_double, c_int, c_int64, c_uint32, c_uint64, c_void_p

import numpy as np

from .. import _native as nat

NMOM = 7  # Σw, Σf·w, Σf²·w, Σf, Σf², Σ|f|·w, Σ|f|
ALL_COLS = (1 << NMOM) - 1
SRC_X, SRC_W, SRC_HOST, SRC_DEVICE, SRC_NONE = 0, 1, 2, 3, -1
PBX_F64, PBX_F32 = 0, 1  # element types of pbx_profile_select_typed

_i64p = ctypes.POINTER(c_int64)


def _i64(a: np.ndarray):
    return a.ctypes.data_as(_i64p)


_REQ_CACHE = 8  # argument sets kept per handle (radial_equaln on device pointers)


def _addr(p):
    """A device pointer argument as a hashable address (None stays None)."""
    if p is None:
        return None
    v = getattr(p, "value", p)  # (ctypes pointers)
    return int(v) if v is not None else 0

class DeviceBins:
    """One binned quantity on the GPU and the results derived from it."""

    def __init__(self):
        h = c_void_p()
        nat.call("pbx_profile_create", byref(h))
        self._h = h
        self.n = 0
        self.nbins = None
        self.n_valid = 0
        self.has_selection = False
        self._csr = None

    # -- construction -------------------------------------------------------
    @classmethod
    def from_x(cls, x) -> "DeviceBins":
        d = cls()
        d.set_x(x)
        return d

    def set_x(self, x) -> None:
        a = np.ascontiguousarray(np.asarray(x), dtype=np.float64).reshape(-1)
        nat.call("pbx_profile_set_x", self._h, nat.dptr(a), a.shape[0])
        self.n = a.shape[0]
        self.has_selection = False
        self.nbins = None
        self._csr = None

    @classmethod
    def select(cls, pos, mass=None, *, sphere=None, families=None, ndim: int = 3,
               on_device: bool = False, n: int | None = None,
               into: "DeviceBins | None" = None) -> "DeviceBins":
        """Fused mask + x + compaction.

        pos / mass: host (N,3) / (N,) float64 or float32 arrays (float32 is
        passed as is: r in float32 arithmetic, like numpy on a float32
        snapshot), or float64 device pointers (``on_device=True``, then ``n``
        is required).  sphere: (cen, radius)
        or None.  families: list of (start, stop) index ranges or None.
        ``into`` reuses an existing handle (and its HBM buffers).
        """
        d = into if into is not None else cls()
        d.nbins, d._csr = None, None
        # float32 snapshots stay float32 (no host up-cast; pbx_profile_select_typed)
        d._pos_dt = PBX_F32 if (not on_device and np.asarray(pos).dtype == np.float32) else PBX_F64
        d._mass_dt = (PBX_F32 if (not on_device and mass is not None and
                                  np.asarray(mass).dtype == np.float32) else PBX_F64)
        args, keep = cls._select_args(pos, mass, sphere, families, ndim, on_device, n,
                                      native_f32=True)
        kept = c_int64(0)
        p_pos, p_mass, n_part, *rest = args
        nat.call("pbx_profile_select_typed", d._h, p_pos, d._pos_dt, p_mass, d._mass_dt, n_part,
                 *rest, byref(kept))
        del keep
        d.n = kept.value
        d.has_selection = True
        return d

    @staticmethod
    def _select_args(pos, mass, sphere, families, ndim, on_device, n, native_f32=False):
        """ctypes arguments of a selection (pbx_profile_select order) and the
        host arrays to keep alive during the call."""
        if on_device:
            p_pos, p_mass, n_part = pos, mass, int(n)
            keep = ()
        else:
            pos = np.asarray(pos)
            f32 = native_f32 and pos.dtype == np.float32
            pos = np.ascontiguousarray(pos, dtype=np.float32 if f32 else np.float64)
            if pos.ndim != 2 or pos.shape[1] != 3:
                raise ValueError("pos must be (N,3)")
            n_part = pos.shape[0]
            if mass is not None:
                mass = np.asarray(mass)
                mf32 = native_f32 and mass.dtype == np.float32
                mass = np.ascontiguousarray(mass, dtype=np.float32 if mf32 else np.float64)
            p_pos = pos.ctypes.data_as(c_void_p)
            p_mass = None if mass is None else mass.ctypes.data_as(c_void_p)
            keep = (pos, mass)
        sph = np.zeros(4)
        if sphere is not None:
            cen, radius = sphere
            radius = float(radius)
            sph[:3] = np.asarray(cen, dtype=np.float64).reshape(3)
            sph[3] = radius * radius
        fam = np.zeros(2, dtype=np.int64)
        nfam = 0
        if families is not None:
            fam = np.ascontiguousarray(np.asarray(families, dtype=np.int64).reshape(-1, 2))
            nfam = fam.shape[0]
            if nfam == 0:  # an empty family set keeps nothing
                fam = np.array([[0, 0]], dtype=np.int64)
                nfam = 1
        keep = keep + (sph, fam)
        args = (p_pos, p_mass, n_part, int(on_device), int(sphere is not None), nat.dptr(sph),
                _i64(fam), nfam, int(ndim))
        return args, keep

    @classmethod
    def radial_equaln(cls, pos, mass=None, *, nbins: int, sphere=None, families=None,
                      ndim: int = 3, bin_min=None, bin_max=None, stats=(), csr=True,
                      on_device: bool = False, n: int | None = None,
                      into: "DeviceBins | None" = None, comm=None):
        """select() followed by binned_equaln() with ONE host round trip
        (pbx_profile_radial_equaln).  Returns (handle, edges, counts, moments)
        with the same values and errors as the two calls.

        ``comm`` (a parallel.Communicator): this rank's share of a profile
        sharded over the ranks (pbx_profile_radial_equaln_comm) — global
        edges, counts and sums, device all-reduces between the kernels; the
        handle keeps this rank's selection, counts (``.counts``) and CSR.

        With ``on_device=True`` the selection is lazy: the weights of the kept
        particles are read from the caller's ``mass`` device array by the
        first later call that needs them (moments(), selection(w=True),
        weighted percentiles) and held by the handle from then on, so that
        array must stay alive and unchanged until that call or the next
        selection on this handle (pbx.h, pbx_profile_radial_equaln).  After
        ``set_source_stable(True)`` so must ``pos``: a repeated large call
        may then bin with the stored table and keep no copy of x, the first
        later reader of x (selection(x=True), statistics of x, percentiles)
        recomputing it from ``pos``.  Host arrays are staged into the handle
        and carry no such contract."""
        if comm is None and not on_device and (
                np.asarray(pos).dtype == np.float32 or
                (mass is not None and np.asarray(mass).dtype == np.float32)):
            # float32 snapshots: r in float32 arithmetic exactly as select()
            # computes it (the one-sync kernels read float64 only), then the
            # same binning pass — identical to select() + binned_equaln()
            d = cls.select(pos, mass, sphere=sphere, families=families, ndim=ndim, into=into)
            edges, counts, mom = d.binned_equaln(nbins, bin_min, bin_max, stats, csr)
            return d, edges, counts, [m.copy() for m in mom]
        d = into if into is not None else cls()
        d.nbins, d._csr = None, None
        nq = int(nbins) + 1
        k = len(stats)
        # The selection and statistics arguments of a repeated call on device
        # pointers, and the staging arrays the results land in, are rebuilt
        # only when they change (host-side cost of a 1M-particle step); the
        # returned arrays are fresh copies every call.
        key = None
        if on_device:
            key = (d._h.value if d._h is not None else None, _addr(pos), _addr(mass),
                   None if sphere is None else (tuple(sphere[0]), float(sphere[1])),
                   None if families is None else tuple(map(tuple, families)), ndim, n,
                   tuple(map(tuple, stats)), nbins, bin_min, bin_max, bool(csr),
                   None if comm is None else comm.handle.value)
        # (a few argument sets per handle: a handle cycling through several
        # snapshots' device arrays keeps each one's)
        reqs = d.__dict__.setdefault("_reqs", {})
        cached = reqs.get(key) if key is not None else None
        prep = None
        if cached is not None:
            args, keep, fs, ws, cs, head, refs, outs, prep = cached
        else:
            args, keep = cls._select_args(pos, mass, sphere, families, ndim, on_device, n)
            fs = (c_int * max(k, 1))(*[int(s[0]) for s in stats])
            ws = (c_int * max(k, 1))(*[int(s[1]) for s in stats])
            cs = (c_uint32 * max(k, 1))(*[int(s[2]) & ALL_COLS for s in stats])
            head = (int(nbins), int(bin_min is not None),
                    float(bin_min) if bin_min is not None else 0.0, int(bin_max is not None),
                    float(bin_max) if bin_max is not None else 0.0, int(bool(csr)), k, fs, ws, cs)
            refs = (c_int64(0), c_int64(0), c_int64(0))
            e_buf, c_buf = np.empty(nq), np.zeros(nbins, dtype=np.int64)
            m_buf = np.zeros((max(k, 1), nbins, NMOM))
            kept, ne, nv = refs
            if comm is None:
                outs = (e_buf, c_buf, m_buf, (byref(kept), nat.dptr(e_buf), byref(ne), _i64(c_buf),
                                              byref(nv), nat.dptr(m_buf)), None)
            else:
                cl_buf = np.zeros(nbins, dtype=np.int64)
                outs = (e_buf, c_buf, m_buf, (byref(kept), nat.dptr(e_buf), byref(ne), _i64(c_buf),
                                              _i64(cl_buf), byref(nv), nat.dptr(m_buf)), cl_buf)
            if key is not None:  # the whole argument list, converted once
                optrs_ = outs[3]
                prep = nat.Prepared("pbx_profile_radial_equaln", d._h, *args, *head, *optrs_) \
                    if comm is None else \
                    nat.Prepared("pbx_profile_radial_equaln_comm", comm.handle, d._h, *args, *head,
                                 *optrs_)
                if len(reqs) >= _REQ_CACHE:
                    reqs.pop(next(iter(reqs)))  # (the oldest)
                reqs[key] = (args, keep, fs, ws, cs, head, refs, outs, prep)
        kept, ne, nv = refs
        edges, counts, mom, optrs, local = outs
        try:
            if prep is not None:
                prep()
            elif comm is None:
                nat.call("pbx_profile_radial_equaln", d._h, *args, *head, *optrs)
            else:
                nat.call("pbx_profile_radial_equaln_comm", comm.handle, d._h, *args, *head, *optrs)
        except ValueError as e:
            if str(e).startswith("index 0 is out of bounds"):
                raise IndexError(str(e)) from None
            raise
        finally:
            del keep
            d.n = kept.value
            d.has_selection = True
        nb = ne.value - 1
        d.nbins = nb
        d.n_valid = nv.value
        if nb != nbins:  # degenerate: one bin, compact layout [k][1][7]
            mom = mom.reshape(-1)[: max(k, 1) * NMOM].reshape(max(k, 1), 1, NMOM)
            counts = counts[:1]
            local = local[:1] if local is not None else None
        counts = counts.copy()  # (the staging arrays are reused by the next call)
        d.counts = counts if local is None else local.copy()  # this rank's (CSR lengths)
        return d, edges[: ne.value].copy(), counts, [mom[i].copy() for i in range(k)]

    def path_stats(self) -> dict:
        """Which path radial_equaln took on this handle: one-launch calls,
        of them discarded at a grid barrier (re-run by the multi-kernel path),
        multi-kernel calls (pbx_profile_path_stats)."""
        out = np.zeros(3, dtype=np.int64)
        nat.call("pbx_profile_path_stats", self._h, _i64(out))
        return {"mono": int(out[0]), "mono_discarded": int(out[1]), "multi": int(out[2])}

    def mono_stats(self) -> dict:
        """One-launch radial_equaln calls on this handle, and of them those
        whose level-0 digits were counted with the previous one-launch call's
        geometry (one grid barrier less), and of them those that found the
        previous call's edges at their ranks (no order statistics, three
        barriers less; pbx_profile_mono_stats)."""
        out = np.zeros(3, dtype=np.int64)
        nat.call("pbx_profile_mono_stats", self._h, _i64(out))
        return {"mono": int(out[0]), "hinted": int(out[1]), "edge_hits": int(out[2])}

    def level0_stats(self) -> dict:
        """Tiled multi-kernel radial_equaln calls on this handle, and of them
        those whose level-0 digit histogram the selection kernel counted with
        the previous tiled call's geometry (no second read of x;
        pbx_profile_level0_stats)."""
        out = np.zeros(2, dtype=np.int64)
        nat.call("pbx_profile_level0_stats", self._h, _i64(out))
        return {"tiled": int(out[0]), "hinted": int(out[1])}

    def spec_stats(self) -> dict:
        """Tiled radial_equaln calls whose selection kernel also binned the
        keys with the stored bin table, of them the hits (the assignment
        pass skipped), and of those the edge hits (the previous call's edges
        held: no deferred keys, no finish; pbx_profile_spec_stats)."""
        out = np.zeros(3, dtype=np.int64)
        nat.call("pbx_profile_spec_stats", self._h, _i64(out))
        return {"speculated": int(out[0]), "hits": int(out[1]), "edge_hits": int(out[2])}

    def set_level0_hint(self, enabled: bool) -> None:
        """False: every tiled radial_equaln call on this handle re-reads x for
        its level-0 histogram (no geometry it did not derive itself); True
        (default): reuse the previous call's digit geometry when it holds,
        and on a first call one sampled from the keys.  Same results either
        way (pbx_profile_set_level0_hint)."""
        nat.call("pbx_profile_set_level0_hint", self._h, 1 if enabled else 0)

    def set_source_stable(self, stable: bool) -> None:
        """True: the DEVICE positions (and masses) this handle's
        radial_equaln calls are given stay alive and unchanged until the next
        selection on it, so a repeated call may speculate and keep no copy of
        x (rebuilt from the positions for a later reader).  False (default):
        on-device calls do not speculate and store x
        (pbx_profile_set_source_stable).  Host arrays are staged into the
        handle and speculate either way."""
        nat.call("pbx_profile_set_source_stable", self._h, 1 if stable else 0)

    def forget_history(self) -> None:
        """The next call runs as this handle's first: no earlier level-0
        geometry (a first tiled call samples one), no speculation state
        (pbx_profile_set_level0_hint mode 2).  Same results."""
        nat.call("pbx_profile_set_level0_hint", self._h, 2)

    def selection(self, idx=True, x=True, w=True):
        """(original indices int64, x, weights) of the fused selection."""
        oi = np.empty(self.n, dtype=np.int64) if idx else None
        ox = np.empty(self.n) if x else None
        ow = np.empty(self.n) if w else None
        nat.call("pbx_profile_get_selection", self._h, None if oi is None else _i64(oi),
                 nat.dptr(ox), nat.dptr(ow))
        return oi, ox, ow

    # -- edges --------------------------------------------------------------
    def minmax(self) -> tuple[float, float]:
        lo, hi = c_double(), c_double()
        nat.call("pbx_profile_minmax", self._h, byref(lo), byref(hi))
        return lo.value, hi.value

    def edges_equaln(self, nbins: int, bin_min=None, bin_max=None) -> np.ndarray:
        out = np.empty(int(nbins) + 1)
        ne = c_int64(0)
        try:
            nat.call("pbx_profile_edges_equaln", self._h, int(nbins), int(bin_min is not None),
                     float(bin_min) if bin_min is not None else 0.0, int(bin_max is not None),
                     float(bin_max) if bin_max is not None else 0.0, nat.dptr(out), byref(ne))
        except ValueError as e:
            if str(e).startswith("index 0 is out of bounds"):
                raise IndexError(str(e)) from None
            raise
        return out[: ne.value].copy()

    # -- staged equaln (distributed radix select, parallel.distributed_equaln)
    def key_range(self) -> tuple[int, int]:
        """Local (min, max) order-preserving u64 keys of x ((2^64-1, 0) if empty)."""
        lo, hi = c_uint64(), c_uint64()
        nat.call("pbx_profile_key_range", self._h, byref(lo), byref(hi))
        return lo.value, hi.value

    def msel_begin(self, nbins: int, bin_min, bin_max, kmin: int, kmax: int) -> int:
        lv = c_int(0)
        try:
            nat.call("pbx_profile_msel_begin", self._h, int(nbins), int(bin_min is not None),
                     float(bin_min) if bin_min is not None else 0.0, int(bin_max is not None),
                     float(bin_max) if bin_max is not None else 0.0, int(kmin), int(kmax),
                     byref(lv))
        except ValueError as e:
            if str(e).startswith("index 0 is out of bounds"):
                raise IndexError(str(e)) from None
            raise
        self._msel_nq = int(nbins) + 1
        return lv.value

    def msel_hist(self, level: int) -> tuple[int, int]:
        """(device pointer, u32 count) of this rank's digit histogram."""
        ptr, cnt = c_void_p(), c_int64()
        nat.call("pbx_profile_msel_hist", self._h, int(level), byref(ptr), byref(cnt))
        return ptr.value, cnt.value

    def msel_resolve(self, level: int) -> None:
        nat.call("pbx_profile_msel_resolve", self._h, int(level))

    def msel_edges(self) -> np.ndarray:
        out = np.empty(self._msel_nq)
        ne = c_int64(0)
        try:
            nat.call("pbx_profile_msel_edges", self._h, nat.dptr(out), byref(ne))
        except ValueError as e:
            if str(e).startswith("index 0 is out of bounds"):
                raise IndexError(str(e)) from None
            raise
        return out[: ne.value].copy()

    def binned_equaln(self, nbins: int, bin_min=None, bin_max=None, stats=(), csr=True):
        """equaln edges + assignment (+ CSR) + per-bin sums in one pass with a
        single host round trip.  stats: (field, weights, cols) with field in
        {SRC_X, SRC_W} and weights in {SRC_X, SRC_W, SRC_NONE}.  Returns
        (edges, counts, [moments (nbins, 7) per stat]) exactly as
        edges_equaln / assign / moments would."""
        nq = int(nbins) + 1
        k = len(stats)
        fs = (c_int * max(k, 1))(*[int(s[0]) for s in stats])
        ws = (c_int * max(k, 1))(*[int(s[1]) for s in stats])
        cs = (c_uint32 * max(k, 1))(*[int(s[2]) & ALL_COLS for s in stats])
        edges = np.empty(nq)
        counts = np.zeros(nbins, dtype=np.int64)
        mom = np.zeros((max(k, 1), nbins, NMOM))
        ne, nv = c_int64(0), c_int64(0)
        try:
            nat.call("pbx_profile_binned_equaln", self._h, int(nbins), int(bin_min is not None),
                     float(bin_min) if bin_min is not None else 0.0, int(bin_max is not None),
                     float(bin_max) if bin_max is not None else 0.0, int(bool(csr)), k, fs, ws,
                     cs, nat.dptr(edges), byref(ne), _i64(counts), byref(nv), nat.dptr(mom))
        except ValueError as e:
            if str(e).startswith("index 0 is out of bounds"):
                raise IndexError(str(e)) from None
            raise
        nb = ne.value - 1
        self.nbins = nb
        self.n_valid = nv.value
        self._csr = None
        if nb != nbins:  # degenerate: one bin, compact layout [k][1][7]
            flat = mom.reshape(-1)[: max(k, 1) * NMOM].reshape(max(k, 1), 1, NMOM)
            mom = flat
            counts = counts[:1].copy()
        self.counts = counts
        return edges[: ne.value].copy(), counts, [mom[i] for i in range(k)]

    # -- assignment ---------------------------------------------------------
    def assign(self, edges) -> np.ndarray:
        e = np.ascontiguousarray(np.asarray(edges), dtype=np.float64).reshape(-1)
        nb = e.shape[0] - 1
        counts = np.zeros(max(nb, 0), dtype=np.int64)
        nv = c_int64(0)
        nat.call("pbx_profile_assign", self._h, nat.dptr(e), e.shape[0], _i64(counts), byref(nv))
        self.nbins = nb
        self.n_valid = nv.value
        self._csr = None
        self.counts = counts
        return counts

    def csr(self) -> tuple[np.ndarray, np.ndarray]:
        """(perm, offsets): the per-bin ascending index lists, concatenated."""
        if self._csr is None:
            perm = np.empty(self.n_valid, dtype=np.int64)
            offs = np.empty(self.nbins + 1, dtype=np.int64)
            nat.call("pbx_profile_csr", self._h, _i64(perm), _i64(offs))
            self._csr = (perm, offs)
        return self._csr

    def build_csr_on_device(self) -> None:
        """Build the CSR in HBM without downloading it."""
        nat.call("pbx_profile_csr", self._h, None, None)

    # -- reductions ---------------------------------------------------------
    def _src(self, v):
        if isinstance(v, (int, np.integer)) and not isinstance(v, bool):
            return int(v), None
        if isinstance(v, nat.DeviceArray):  # per original particle, in HBM
            return SRC_DEVICE, v.ptr
        a = np.ascontiguousarray(np.asarray(v), dtype=np.float64).reshape(-1)
        if a.shape[0] != self.n:
            raise ValueError(f"array length {a.shape[0]} != {self.n}")
        return SRC_HOST, a

    @staticmethod
    def _ptr(a):
        return a if isinstance(a, ctypes.c_void_p) else nat.vptr(a)

    def percentiles(self, q, field=SRC_X, weights=SRC_NONE, absval: bool = False) -> np.ndarray:
        """Per-bin percentiles (nbins, len(q)), q = p/100 fractions: the
        reference's Percentile per bin (np.argsort, np.cumsum of the weights
        or np.linspace, np.interp); empty bins NaN."""
        if self.nbins is None:
            raise ValueError("assign() first")
        qa = np.ascontiguousarray(np.atleast_1d(np.asarray(q, dtype=np.float64)))
        fs, fa = self._src(field)
        ws, wa = self._src(weights) if weights is not None else (SRC_NONE, None)
        out = np.zeros((self.nbins, qa.shape[0]))
        nat.call("pbx_profile_percentiles", self._h, fs, self._ptr(fa), ws, self._ptr(wa),
                 int(bool(absval)), qa.shape[0], nat.dptr(qa), nat.dptr(out))
        return out

    def moments(self, field=SRC_X, weights=SRC_NONE, cols: int = ALL_COLS) -> np.ndarray:
        """Per-bin sums (nbins, 7): Σw, Σf·w, Σf²·w, Σf, Σf², Σ|f|·w, Σ|f|.

        field / weights: SRC_X, SRC_W (selection mass), a host array of
        length n, or (weights only) SRC_NONE.  cols: bit mask of the columns
        to accumulate (the others come back 0).
        """
        if self.nbins is None:
            raise ValueError("assign() first")

        def src(v):
            if isinstance(v, (int, np.integer)) and not isinstance(v, bool):
                return int(v), None
            if isinstance(v, nat.DeviceArray):  # per original particle, in HBM
                return SRC_DEVICE, v.ptr
            a = np.ascontiguousarray(np.asarray(v), dtype=np.float64).reshape(-1)
            if a.shape[0] != self.n:
                raise ValueError(f"array length {a.shape[0]} != {self.n}")
            return SRC_HOST, a

        fs, fa = src(field)
        ws, wa = src(weights) if weights is not None else (SRC_NONE, None)
        out = np.zeros((self.nbins, NMOM))
        def ptr(a):
            return a if isinstance(a, ctypes.c_void_p) else nat.vptr(a)

        nat.call("pbx_profile_moments_cols", self._h, fs, ptr(fa), ws, ptr(wa), int(cols) & ALL_COLS,
                 nat.dptr(out))
        return out

    def close(self) -> None:
        if self._h is not None and self._h.value and nat._lib is not None:
            try:
                nat.call("pbx_profile_destroy", self._h)
            except Exception:
                pass
        self._h = c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
