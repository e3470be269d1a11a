"""ORACLE — numpy restatement of the reference radial-profile path.

Test infrastructure only (tests/, __graft_entry__.smoke(), bench.py's
cpu_baseline leg); never the product path.

Restates, operation for operation:
  * edge algorithms        pynbodyext/profiles/bins.py:689-746
  * particle assignment    bins.py:346-395 (digitize(right=True) - 1 ==
                           searchsorted(side="left") - 1, the two extrema
                           fix-ups, keep 0 <= bin < nbins, stable grouping)
  * area calculators       bins.py:750-789
  * per-bin statistics     proarray.py:272-334 and the StatisticBase
                           plug-ins :632-860 (same numpy expressions, so the
                           same pairwise-summation rounding)
Pinned bit-for-bit against fixtures produced by the reference's own code
(tests/golden/make_golden.py -> tests/golden/*.npz), see
tests/test_oracle_profile.py.

Also times the reference-equivalent pipeline for bench.py's CPU baseline of
the profile workload (mask + r + edges + assignment + sums, one core).
"""
from __future__ import annotations

import re

import numpy as np


# ---------------------------------------------------------------- edges
def edges_lin(x, nbins, bin_min=None, bin_max=None):
    lo = np.min(x) if bin_min is None else bin_min
    hi = np.max(x) if bin_max is None else bin_max
    return np.linspace(lo, hi, nbins + 1)


def edges_log(x, nbins, bin_min=None, bin_max=None):
    lo = np.min(x) if bin_min is None else bin_min
    hi = np.max(x) if bin_max is None else bin_max
    if lo <= 0:
        raise ValueError("Logarithmic bins require xmin to be non-negative")
    return np.logspace(np.log10(lo), np.log10(hi), nbins + 1)


def edges_equaln(x, nbins, bin_min=None, bin_max=None):
    s = np.sort(x)
    if s.size == 0:
        raise ValueError("Cannot create bins: input array is empty")
    if bin_min is not None:
        s = s[s >= bin_min]
    if bin_max is not None:
        s = s[s <= bin_max]
    if s.size < 2:
        return np.array([s[0], s[0]], dtype=float)
    n = len(s)
    picks = [0] + [int(i * n / nbins) for i in range(1, nbins)] + [n - 1]
    return np.array([s[k] for k in picks])


EDGE_ALGORITHMS = {"lin": edges_lin, "log": edges_log, "equaln": edges_equaln}


# ---------------------------------------------------------------- assign
def bin_ids(x, edges):
    """Bin id of every element (nbins = invalid), Appendix B of SURVEY.md."""
    x = np.asarray(x)
    e = np.asarray(edges)
    nb = len(e) - 1
    b = np.searchsorted(e, x, side="left") - 1
    b[x == e[0]] = 0
    b[x == e[-1]] = nb - 1
    b[(b < 0) | (b >= nb)] = nb
    return b


def assign(x, edges):
    """(perm, offsets, counts): CSR of the reference's binind lists."""
    e = np.asarray(edges)
    nb = len(e) - 1
    if nb <= 0:
        return np.zeros(0, np.int64), np.zeros(1, np.int64), np.zeros(0, np.int64)
    b = bin_ids(x, e)
    counts = np.bincount(b, minlength=nb + 1)[:nb].astype(np.int64)
    order = np.argsort(b, kind="stable")
    nvalid = int(counts.sum())
    perm = order[:nvalid].astype(np.int64)
    offsets = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    return perm, offsets, counts


def binind_lists(perm, offsets):
    return [perm[offsets[i]:offsets[i + 1]] for i in range(len(offsets) - 1)]


# ---------------------------------------------------------------- areas
def area_length(edges):
    return edges[1:] - edges[:-1]


def area_annulus(edges):
    return np.pi * (edges[1:] ** 2 - edges[:-1] ** 2)


def area_spherical_shell(edges):
    return 4 / 3 * np.pi * (edges[1:] ** 3 - edges[:-1] ** 3)


# ---------------------------------------------------------------- statistics
def _mean(a, w):
    return (a * w).sum() / w.sum() if w is not None else a.mean()


def _sum(a, w):
    return a.sum()


def _sum_w(a, w):
    return (a * w).sum() if w is not None else a.sum()


def _percentile(q):
    def f(a, w):
        if len(a) == 0:
            return np.nan
        idx = np.argsort(a)
        s = a[idx]
        if w is None:
            cdf = np.linspace(0, 1, len(s))
        else:
            cdf = w[idx].cumsum()
            cdf -= cdf[0]
            cdf /= cdf[-1]
        return np.interp(q / 100, cdf, s)
    return f


def _rms(a, w):
    if len(a) == 0:
        return np.nan
    if w is not None:
        return np.sqrt((a ** 2 * w).sum() / w.sum())
    return np.sqrt((a ** 2).mean())


def _disp(a, w):
    if len(a) == 0:
        return np.nan
    if w is not None:
        ws = float(np.asarray(w.sum()))
        if ws == 0:
            return np.nan
        sq = float(np.asarray((a ** 2 * w).sum() / ws))
        mn = float(np.asarray((a * w).sum() / ws)) ** 2
    else:
        sq = float(np.asarray((a ** 2).mean()))
        mn = float(np.asarray(a.mean())) ** 2
    d = sq - mn
    if -1e-12 < d < 0:
        d = 0.0
    return float(np.sqrt(d)) if d >= 0 else np.nan


def statistic(key: str):
    """(canonical key, callable(arr, weight)) like ProfileArray.get_statistic."""
    k = key.lower()
    if k == "mean":
        return "mean", _mean
    if k == "sum":
        return "sum", _sum
    if k == "sum_w":
        return "sum_w", _sum_w
    m = re.match(r"^p(\d{1,3})$", k)
    if m and 0 <= int(m.group(1)) <= 100:
        return k, _percentile(int(m.group(1)))
    if k == "rms":
        return "rms", _rms
    if k in ("med", "median"):
        return "median", _percentile(50)
    if k in ("abs", "abs_") or k.startswith("abs_"):
        sub = "mean" if k in ("abs", "abs_") else k[4:]
        got = statistic(sub)
        if got is None:
            return None
        canon, fn = got
        return "abs_" + canon, (lambda a, w, fn=fn: fn(np.abs(a), w))
    if k in ("dispersion", "disp"):
        return "disp", _disp
    return None


def compute(field, weights, perm, offsets, key: str):
    """Per-bin statistic over the CSR, proarray.py:304-334 semantics
    (empty bin -> NaN for every statistic, including sum)."""
    got = statistic(key)
    if got is None:
        raise ValueError(f"Statistic '{key}' not found")
    canon, fn = got
    nb = len(offsets) - 1
    vals = np.zeros(nb)
    for i in range(nb):
        ind = perm[offsets[i]:offsets[i + 1]]
        if len(ind) == 0:
            vals[i] = np.nan
            continue
        vals[i] = fn(field[ind], None if weights is None else weights[ind])
    return vals, canon


# ---------------------------------------------------------------- pipeline
def radial_r(pos):
    x, y, z = pos[:, 0], pos[:, 1], pos[:, 2]
    return np.sqrt((x * x + y * y) + z * z)


def sphere_mask(pos, radius, cen=(0.0, 0.0, 0.0)):
    dx = pos[:, 0] - cen[0]
    dy = pos[:, 1] - cen[1]
    dz = pos[:, 2] - cen[2]
    return ((dx * dx + dy * dy) + dz * dz) < radius * radius


def radial_profile(pos, mass, mask, bins_type="equaln", nbins=128, bin_min=None, bin_max=None):
    """Reference semantics of RadialProfileBuilder(ndim=3, weight='mass')
    on sim[mask]: returns edges, counts, perm, offsets, mass sums, mean r."""
    p = pos[mask]
    m = mass[mask]
    r = radial_r(p)
    edges = EDGE_ALGORITHMS[bins_type](r, nbins, bin_min, bin_max)
    perm, offsets, counts = assign(r, edges)
    msum, _ = compute(m, m, perm, offsets, "sum")
    rmean, _ = compute(r, m, perm, offsets, "mean")
    return {"edges": edges, "counts": counts, "perm": perm, "offsets": offsets,
            "mass_sum": msum, "r_mean": rmean, "x": r, "w": m}
