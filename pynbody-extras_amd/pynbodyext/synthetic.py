"""Synthetic Plummer-sphere particle sets.

G = M = a = 1, equal masses m = 1/N, radii r = (X^(-2/3) - 1)^(-1/2) with
X ~ U(0, 1) re-drawn while r > ``rmax`` (default 50), isotropic directions.
Families are contiguous blocks in gadget order used by the survey:
dm 60 %, gas 30 %, star 10 %.  Seeds used by the configs: 1001 (10k),
1002 (1M), 1003 (4M), 1004 (8M).
"""
from __future__ import annotations

import numpy as np

FAMILY_FRACTIONS = (("dm", 0.6), ("gas", 0.3), ("star", 0.1))


def plummer_radii(n: int, rng: np.random.Generator, rmax: float = 50.0) -> np.ndarray:
    r = np.empty(n, dtype=np.float64)
    todo = np.arange(n)
    while todo.size:
        x = rng.random(todo.size)
        with np.errstate(divide="ignore", invalid="ignore"):
            rr = (x ** (-2.0 / 3.0) - 1.0) ** -0.5
        ok = np.isfinite(rr) & (rr <= rmax)
        r[todo[ok]] = rr[ok]
        todo = todo[~ok]
    return r


def plummer(n: int, seed: int = 1002, rmax: float = 50.0):
    """(pos (n,3) float64 C-order, mass (n,) float64)."""
    rng = np.random.default_rng(seed)
    r = plummer_radii(n, rng, rmax)
    cost = rng.uniform(-1.0, 1.0, n)
    phi = rng.uniform(0.0, 2.0 * np.pi, n)
    sint = np.sqrt(1.0 - cost * cost)
    pos = np.empty((n, 3), dtype=np.float64)
    pos[:, 0] = r * sint * np.cos(phi)
    pos[:, 1] = r * sint * np.sin(phi)
    pos[:, 2] = r * cost
    mass = np.full(n, 1.0 / n, dtype=np.float64)
    return pos, mass


def plummer_chunked(n: int, seed: int, chunk: int = 1 << 22, threads: int = 16,
                    rmax: float = 50.0):
    """A Plummer sphere drawn in independent chunks on a thread pool (numpy
    releases the GIL in its kernels): chunk k holds particles
    [k·chunk, (k+1)·chunk) drawn by plummer()'s rule from the k-th child of
    SeedSequence(seed).  A different particle set than plummer(n, seed) —
    used where many large snapshots are needed (the bench's changing-input
    rows), ~10x faster than one stream."""
    from concurrent.futures import ThreadPoolExecutor

    nch = max(1, -(-n // chunk))
    seqs = np.random.SeedSequence(seed).spawn(nch)
    pos = np.empty((n, 3), dtype=np.float64)

    def fill(k):
        lo, hi = k * chunk, min(n, (k + 1) * chunk)
        rng = np.random.default_rng(seqs[k])
        m = hi - lo
        r = plummer_radii(m, rng, rmax)
        cost = rng.uniform(-1.0, 1.0, m)
        phi = rng.uniform(0.0, 2.0 * np.pi, m)
        sint = np.sqrt(1.0 - cost * cost)
        pos[lo:hi, 0] = r * sint * np.cos(phi)
        pos[lo:hi, 1] = r * sint * np.sin(phi)
        pos[lo:hi, 2] = r * cost

    with ThreadPoolExecutor(max_workers=max(1, threads)) as ex:
        list(ex.map(fill, range(nch)))
    return pos, np.full(n, 1.0 / n, dtype=np.float64)


def family_slices(n: int) -> dict:
    out, start = {}, 0
    for i, (name, frac) in enumerate(FAMILY_FRACTIONS):
        stop = n if i == len(FAMILY_FRACTIONS) - 1 else start + int(round(frac * n))
        out[name] = slice(start, stop)
        start = stop
    return out


def plummer_snapshot(n: int, seed: int = 1002):
    """A SimSnap of a Plummer sphere with dm/gas/star families."""
    from .simcore import new_snapshot

    pos, mass = plummer(n, seed)
    return new_snapshot(pos, mass, families=family_slices(n),
                        units_map={"pos": "kpc", "mass": "1e10 Msol"})
