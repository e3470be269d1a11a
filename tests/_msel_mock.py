"""Host stand-ins for the distributed-equaln protocol test on CPU (gloo).

NumpyMsel restates, in numpy, the staged radix select that
csrc/profile.hip runs on the device (same key map, level widths, rank
formula and digit choice), exposing the DeviceBins staged interface
(key_range / msel_begin / msel_hist / msel_resolve / msel_edges).
GlooComm offers the Communicator calls parallel.distributed_equaln uses,
over torch.distributed (gloo) on host arrays.  Test infrastructure only.
"""
import numpy as np

MS0_BITS, MS_BITS = 14, 12
SIGN = np.uint64(1 << 63)


def dkey(x):
    b = np.ascontiguousarray(x, dtype=np.float64).view(np.uint64)
    neg = (b & SIGN) != 0
    return np.where(neg, ~b, b | SIGN)


def dkey_inv(k):
    k = np.uint64(k)
    b = (k ^ SIGN) if (k & SIGN) else ~k
    return float(np.array([b], dtype=np.uint64).view(np.float64)[0])


class NumpyMsel:
    def __init__(self, x):
        self.k = dkey(x)
        self.n = self.k.size

    def key_range(self):
        if self.k.size == 0:
            return (1 << 64) - 1, 0
        return int(self.k.min()), int(self.k.max())

    def msel_begin(self, nbins, bin_min, bin_max, kmin, kmax):
        ka, kb, empty = 0, (1 << 64) - 1, False
        if bin_min is not None or bin_max is not None:
            kb = (1 << 64) - 2
            if bin_min is not None:
                empty |= bin_min != bin_min
                ka = 0 if empty else int(dkey([bin_min])[0])
            if bin_max is not None:
                empty |= bin_max != bin_max
                if bin_max == bin_max:
                    kb = min(kb, int(dkey([bin_max])[0]))
        lo, hi = max(ka, kmin), min(kb, kmax)
        if empty or lo > hi:
            raise IndexError("index 0 is out of bounds for axis 0 with size 0")
        span = hi - lo
        self.B = span.bit_length() if span else 1
        self.wd = [min(self.B, MS0_BITS)]
        rem = self.B - self.wd[0]
        while rem > 0:
            self.wd.append(min(rem, MS_BITS))
            rem -= MS_BITS
        self.nq, self.nbins = nbins + 1, nbins
        kk = self.k[(self.k >= np.uint64(ka)) & (self.k <= np.uint64(kb))]
        self.offa = (kk - np.uint64(lo)).astype(np.uint64)
        self.lo = lo
        return len(self.wd)

    def _shift(self, level):
        return self.B - sum(self.wd[: level + 1])

    def msel_hist(self, level):
        s = self._shift(level)
        d = (self.offa >> np.uint64(s)) & np.uint64((1 << self.wd[level]) - 1)
        if level == 0:
            self.H = np.bincount(d.astype(np.int64), minlength=1 << MS0_BITS).astype(np.uint32)
        else:
            pref = self.offa >> np.uint64(s + self.wd[level])
            self.H = np.zeros((self.nq, 1 << MS_BITS), dtype=np.uint32)
            g = np.searchsorted(self.groups, pref)
            ok = (g < len(self.groups)) & (self.groups[np.minimum(g, len(self.groups) - 1)] == pref)
            np.add.at(self.H, (g[ok], d[ok].astype(np.int64)), 1)
            self.H = self.H.reshape(-1)
        return self.H, self.H.size

    def msel_resolve(self, level):
        w = self.wd[level]
        if level == 0:
            incl = np.cumsum(self.H.astype(np.int64))
            m = int(incl[-1])
            self.m = m
            self.rr = np.array([0 if m < 2 else (m - 1 if q == self.nq - 1 else int((q * m) / self.nbins))
                                for q in range(self.nq)], dtype=np.int64)
            self.prefix = np.zeros(self.nq, dtype=np.uint64)
            rows = [incl]
            grp = np.zeros(self.nq, dtype=np.int64)
        else:
            rows = np.cumsum(self.H.reshape(self.nq, -1).astype(np.int64), axis=1)
            grp = self.grp
        for q in range(self.nq):
            inc = rows[grp[q]][: 1 << w]
            a = int(np.searchsorted(inc, self.rr[q], side="right"))
            self.rr[q] -= int(inc[a - 1]) if a else 0
            self.prefix[q] = (self.prefix[q] << np.uint64(w)) | np.uint64(a)
        self.groups, self.grp = np.unique(self.prefix, return_inverse=True)

    def msel_edges(self):
        if self.m == 0:
            raise IndexError("index 0 is out of bounds for axis 0 with size 0")
        e = np.array([dkey_inv(self.lo + int(p)) for p in self.prefix])
        return e[:2] if self.m < 2 else e


class GlooComm:
    """The Communicator calls of parallel.distributed_equaln over gloo."""

    def __init__(self, dist, torch):
        self.dist, self.torch = dist, torch

    def allreduce_host(self, a, op=0):
        t = self.torch
        a = np.ascontiguousarray(a)
        if a.dtype == np.uint64:  # order-preserving map into int64
            v = t.from_numpy((a ^ SIGN).view(np.int64).copy())
        else:
            v = t.from_numpy(a.astype(np.int64 if a.dtype.kind in "iu" else np.float64))
        red = {0: self.dist.ReduceOp.SUM, 1: self.dist.ReduceOp.MIN, 2: self.dist.ReduceOp.MAX}[op]
        self.dist.all_reduce(v, op=red)
        out = v.numpy()
        if a.dtype == np.uint64:
            return out.view(np.uint64) ^ SIGN
        return out.astype(a.dtype)

    def allreduce(self, buf, _buf, count, dtype, op=0):
        buf[:count] = self.allreduce_host(buf[:count].astype(np.int64), op).astype(buf.dtype)
