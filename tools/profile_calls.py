"""One kind of radial-profile call, repeated, for rocprofv3 kernel traces /
A-B timing on the box: the bench's config-3 step (Sphere(10) & dm family,
equaln 128, mass sum + mean r, CSR) on device-resident positions.

mode "identical": the same snapshot every call (the handle speculates);
mode "cold": forget_history() before every call (each call a first one);
mode "changing": a handle cycling through 4 snapshots (bench.changing_snapshots'
seeds), every call a different snapshot than the previous one.
usage: python tools/profile_calls.py N mode [calls]"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]

import bench  # noqa: E402
from pynbodyext import _native as nat  # noqa: E402
from pynbodyext.profiles._device import SRC_NONE, SRC_W, SRC_X, DeviceBins  # noqa: E402
from pynbodyext.synthetic import family_slices, plummer, plummer_chunked  # noqa: E402

n = int(sys.argv[1])
mode = sys.argv[2]
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 40
nat.load()
nat.set_device(0)
seed = bench.SEEDS.get(n, 1002)
snaps = []
for k in range(bench.N_CHANGING if mode == "changing" else 1):
    pos, mass = plummer(n, seed=seed) if k == 0 else plummer_chunked(n, seed + 104729 * k)
    snaps.append((nat.DeviceArray.from_host(pos), nat.DeviceArray.from_host(mass)))
    del pos, mass
dm = family_slices(n)["dm"]
stats = [(SRC_W, SRC_NONE, 1 << 3), (SRC_X, SRC_W, (1 << 0) | (1 << 1))]
h = DeviceBins()
h.set_source_stable(True)
e0, e1 = nat.Event(), nat.Event()


def step(i):
    p, m = snaps[i % len(snaps)]
    return DeviceBins.radial_equaln(p.ptr, m.ptr, nbins=128, sphere=((0.0, 0.0, 0.0), 10.0),
                                    families=[(dm.start, dm.stop)], ndim=3, stats=stats, csr=True,
                                    on_device=True, n=n, into=h)


for i in range(2 * len(snaps)):
    step(i)
nat.synchronize()
s0 = h.spec_stats()
ts = []
for i in range(calls):
    if mode == "cold":
        h.forget_history()
    e0.record()
    step(i)
    e1.record()
    nat.synchronize()
    ts.append(e0.elapsed_ms(e1))
s1 = h.spec_stats()
print(json.dumps({"n": n, "mode": mode, "calls": calls, "stream_ms": float(np.median(ts)),
                  "min_ms": float(np.min(ts)), "p90_ms": float(np.percentile(ts, 90)),
                  "spec": {k: s1[k] - s0[k] for k in s0}, "level0": h.level0_stats(),
                  "mono": h.mono_stats()}))
