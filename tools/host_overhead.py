"""Host time around a 1M changing-input radial_equaln call (bench.py's
changing rows): the wall per call of the bench's loop, of the library call
alone (the handle's prepared argument set, no Python wrapper), and of the
wrapper's argument-key lookup; the kernel time comes from rocprof.
usage: python tools/host_overhead.py [calls]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]

import bench  # noqa: E402
from pynbodyext import _native as nat  # noqa: E402
from pynbodyext.profiles._device import SRC_NONE, SRC_W, SRC_X, DeviceBins  # noqa: E402
from pynbodyext.synthetic import family_slices, plummer_chunked  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 400
n = 1_000_000
nat.load()
nat.set_device(0)
dm = family_slices(n)["dm"]
snaps = []
for k in range(4):
    p, m = plummer_chunked(n, seed=1002 + 104729 * k)
    snaps.append((nat.DeviceArray.from_host(p), nat.DeviceArray.from_host(m)))
stats = ((SRC_W, SRC_NONE, 1 << 3), (SRC_X, SRC_W, 0b11))
h = DeviceBins()
h.set_source_stable(True)


def single(pp, mp):
    return DeviceBins.radial_equaln(pp, mp, nbins=128, sphere=((0.0, 0.0, 0.0), 10.0),
                                    families=[(dm.start, dm.stop)], ndim=3, stats=stats, csr=True,
                                    on_device=True, n=n, into=h)


for i in range(16):
    single(snaps[i % 4][0].ptr, snaps[i % 4][1].ptr)
nat.synchronize()
e0, e1 = nat.Event(), nat.Event()
out = {}
# 1: the bench's loop (events + sync around every call)
t = []
for i in range(calls):
    pp, mp = snaps[i % 4]
    t0 = time.perf_counter()
    e0.record()
    single(pp.ptr, mp.ptr)
    e1.record()
    nat.synchronize()
    t.append(time.perf_counter() - t0)
out["bench_loop_us"] = float(np.median(t)) * 1e6
# 2: the wrapper alone, no events / sync
t = []
for i in range(calls):
    pp, mp = snaps[i % 4]
    t0 = time.perf_counter()
    single(pp.ptr, mp.ptr)
    t.append(time.perf_counter() - t0)
out["wrapper_us"] = float(np.median(t)) * 1e6
# 3: the library call alone through each snapshot's prepared argument set
preps = [v[8] for v in h._reqs.values()]
t = []
for i in range(calls):
    prep = preps[i % len(preps)]
    t0 = time.perf_counter()
    prep()
    t.append(time.perf_counter() - t0)
out["library_call_us"] = float(np.median(t)) * 1e6
# 4: an empty synchronize
t = []
for i in range(calls):
    t0 = time.perf_counter()
    nat.synchronize()
    t.append(time.perf_counter() - t0)
out["sync_us"] = float(np.median(t)) * 1e6
print(json.dumps(out))
