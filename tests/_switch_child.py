"""Child process of tests/test_gpu_switches.py: one fixed workload through
the library under whatever PBX_* runtime variables the parent set (they are
read once per process), results saved to the .npz named by argv[1].

Workload: radial equal-number profiles (a tiled 4.4M-particle point set and
a one-launch 300k one, each called three times on one handle so the hinted
and speculating paths run), a 200k order-3 octree walk, a 10k direct sum."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]

from pynbodyext import _engine  # noqa: E402
from pynbodyext import _native as nat  # noqa: E402
from pynbodyext.profiles._device import SRC_NONE, SRC_W, SRC_X, DeviceBins  # noqa: E402
from pynbodyext.synthetic import plummer  # noqa: E402


def main(out: str) -> None:
    nat.load()
    nat.set_device(0)
    res = {}
    stats = [(SRC_W, SRC_NONE, 1 << 3), (SRC_X, SRC_W, 0b11)]
    rng = np.random.default_rng(77)
    for tag, n in (("tiled", 4_400_000), ("mono", 300_000)):
        pos = rng.normal(scale=3.0, size=(n, 3))
        mass = rng.uniform(0.5, 1.5, n)
        h = DeviceBins()
        try:
            for k in range(3):
                _, e, c, m = DeviceBins.radial_equaln(pos, mass, nbins=128, stats=stats, into=h,
                                                      bin_min=0.3, bin_max=8.0)
                perm, off = h.csr()
                res[f"{tag}{k}/edges"], res[f"{tag}{k}/counts"] = e, c
                res[f"{tag}{k}/perm"], res[f"{tag}{k}/off"] = perm, off
                for j, a in enumerate(m):
                    res[f"{tag}{k}/m{j}"] = np.asarray(a)
        finally:
            h.close()
    pos, mass = plummer(200_000, seed=1003)
    t = _engine.Octree(pos, mass, 8, 3)
    try:
        res["tree/pot"] = t.compute_potentials(0.5)
        res["tree/acc"] = t.compute_accelerations(0.5)
    finally:
        t.close()
    pos, mass = plummer(10_000, seed=1001)
    res["direct/pot"] = _engine.direct_potentials_py(pos, mass)
    res["direct/acc"] = _engine.direct_accelerations_py(pos, mass)
    np.savez(out, **res)


if __name__ == "__main__":
    main(sys.argv[1])
