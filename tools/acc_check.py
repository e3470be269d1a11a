"""Accuracy of the all-particles direct sum (symmetric kernel) against the C
oracle on a 1M Plummer sphere: 4096 random targets + the 64 innermost ones.
Run with PBX_AB_LIBRARY=... to check a variant build (GPU box diagnostic)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from oracle import gravity as og  # noqa: E402
from pynbodyext import _rust  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
pos, mass = bench.plummer(n, seed=bench.SEEDS.get(n, 1002))
pot = _rust.direct_potentials_py(pos, mass)
acc = _rust.direct_accelerations_py(pos, mass)
r = np.sqrt((pos ** 2).sum(1))
rng = np.random.default_rng(0)
idx = np.unique(np.concatenate([rng.choice(n, 4096, replace=False), np.argsort(r)[:64]]))
rp, ra = og.direct_subset(pos, mass, idx)
ep = np.abs(pot[idx] - rp) / np.abs(rp)
ea = np.linalg.norm(acc[idx] - ra, axis=1) / np.linalg.norm(ra, axis=1)
w = np.argmax(ea)
print(f"lib={os.environ.get('PBX_AB_LIBRARY', 'default')} n={n}")
print(f"pot rel err: max {ep.max():.3e}  p99.9 {np.quantile(ep, 0.999):.3e}  median {np.median(ep):.3e}")
print(f"acc rel err: max {ea.max():.3e}  p99.9 {np.quantile(ea, 0.999):.3e}  median {np.median(ea):.3e}"
      f"  (worst at r={r[idx][w]:.3e}, |a|={np.linalg.norm(ra[w]):.3e})")
