"""Same-process A/B of the 4M octree walk (theta 0.5, leaf 8, order 3, fast
mode, force + potential): walk statistics on vs off
(pbx_octree_set_walk_counters), alternating, HIP events around each walk;
full walk and one cost-balanced 1/8 range (8 waves per SIMD).
usage: python tools/walk_ab.py [n] [reps]"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]

from pynbodyext import _native as nat  # noqa: E402
from pynbodyext._engine import Octree  # noqa: E402
from pynbodyext.synthetic import plummer  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
nat.load()
nat.set_device(0)
pos, mass = plummer(n, seed=1003)
d_pos, d_mass = nat.DeviceArray.from_host(pos), nat.DeviceArray.from_host(mass)
d_pot, d_acc = nat.DeviceArray(8 * n), nat.DeviceArray(24 * n)
d_cost, d_orig = nat.DeviceArray(4 * n), nat.DeviceArray(4 * n)
tree = Octree._from_device(d_pos.ptr, n, d_mass.ptr, 8, 3)
tree._set_cost_kind(1)
want = nat.WANT_POT | nat.WANT_ACC
ev = [nat.Event(), nat.Event()]


def walk(first, count, cost=None):
    ev[0].record()
    tree._compute_range_device(0.5, want, first, count, 1, d_pot.ptr, d_acc.ptr, cost)
    ev[1].record()
    nat.synchronize()
    return ev[0].elapsed_ms(ev[1])


walk(0, n, d_cost.ptr)
tree._cost_to_orig_device(d_cost.ptr, d_orig.ptr)
first, count = tree._balance_device(d_orig.ptr, 8)[4]
out = {}
for label, (f, c) in (("full", (0, n)), ("range4of8", (first, count))):
    t = {True: [], False: []}
    for r in range(reps):
        for on in (True, False):
            tree._set_walk_counters(on)
            walk(f, c)
            t[on].append(walk(f, c))
    tree._set_walk_counters(True)
    out[label] = {"counters_on_ms": float(np.median(t[True])),
                  "counters_off_ms": float(np.median(t[False])),
                  "on": t[True], "off": t[False]}
print(json.dumps(out), flush=True)
