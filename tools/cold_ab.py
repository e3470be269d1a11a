"""First-call (cold) timing of the tiled radial profile: the bench's config-3
step (Sphere(10) & dm family, equaln 128, mass sum + mean r, CSR) on
device-resident positions, each timed call made a handle's first.
mode "forget": forget_history() before every call (the sampled level-0
geometry of a first call); mode "off": set_level0_hint(False) (every call
re-reads x for its level-0 histogram — a first call before the sampler).
usage: python tools/cold_ab.py N mode [reps]   (COLD_STATS=none|w: fewer sums)"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]

from pynbodyext import _native as nat  # noqa: E402
from pynbodyext.profiles._device import SRC_NONE, SRC_W, SRC_X, DeviceBins  # noqa: E402
from pynbodyext.synthetic import family_slices, plummer  # noqa: E402

n = int(sys.argv[1])
mode = sys.argv[2]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 15
nat.load()
nat.set_device(0)
pos, mass = plummer(n, seed=1002)
dm = family_slices(n)["dm"]
d_pos, d_mass = nat.DeviceArray.from_host(pos), nat.DeviceArray.from_host(mass)
stats = [(SRC_W, SRC_NONE, 1 << 3), (SRC_X, SRC_W, (1 << 0) | (1 << 1))]
# COLD_STATS (diagnostic): "none" (counts only) or "w" (the mass sum only)
stats = {"none": [], "w": [(SRC_W, SRC_NONE, 1 << 3)]}.get(os.environ.get("COLD_STATS", ""), stats)
h = DeviceBins()
e0, e1 = nat.Event(), nat.Event()


def step():
    return DeviceBins.radial_equaln(d_pos.ptr, d_mass.ptr, nbins=128, sphere=((0.0, 0.0, 0.0), 10.0),
                                    families=[(dm.start, dm.stop)], ndim=3, stats=stats, csr=True,
                                    on_device=True, n=n, into=h)


for _ in range(3):
    step()
if mode == "off":
    h.set_level0_hint(False)
ts = []
for _ in range(reps):
    if mode == "forget":
        h.forget_history()
    nat.synchronize()
    e0.record()
    step()
    e1.record()
    nat.synchronize()
    ts.append(e0.elapsed_ms(e1))
print(json.dumps({"n": n, "mode": mode, "cold_stream_ms": float(np.median(ts)),
                  "min_ms": float(np.min(ts)), "level0": h.level0_stats()}))
