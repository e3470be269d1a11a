"""The 8-GPU bound of config 5 measured on one GPU: the 4M-particle octree
(theta 0.5, leaf 8, order 3) is built, walked once in full with per-target
costs, split into `world` cost-balanced leaf-order ranges exactly as
ShardedTree does (pbx_octree_balance over the previous walk's costs), and
each range is walked alone (compact outputs) and timed with HIP events on
the library stream.  Cases: ranges balanced on interaction counts (cost
kind 0), on wave work (kind 1, ShardedTree's), and equal target counts.
An 8-rank step is bounded by build + max(range walk) + profile (+ the cost
all-gather / all-reduce, not timed here).
usage: python tools/range_walks.py [n] [world] [reps]"""
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
world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
nat.load()
nat.set_device(0)
pos, mass = plummer(n, seed=1003)
d_pos, d_mass = nat.DeviceArray.from_host(pos), nat.DeviceArray.from_host(mass)
d_pot, d_acc = nat.DeviceArray(8 * n), nat.DeviceArray(24 * n)
d_cost, d_cost_orig = nat.DeviceArray(4 * n), nat.DeviceArray(4 * n)
want = nat.WANT_POT | nat.WANT_ACC
ev = [nat.Event() for _ in range(2)]


def timed(fn):
    ms = []
    for _ in range(reps):
        ev[0].record()
        fn()
        ev[1].record()
        nat.synchronize()
        ms.append(ev[0].elapsed_ms(ev[1]))
    return float(np.median(ms))


tree = Octree._from_device(d_pos.ptr, n, d_mass.ptr, 8, 3)
build_ms = timed(lambda: tree._rebuild_device(d_pos.ptr, n, d_mass.ptr))
out = {"n": n, "world": world, "build_ms": build_ms}
costs = {}
for kind, label in ((0, "interactions"), (1, "wave_work")):
    tree._set_cost_kind(kind)
    ms = timed(lambda: tree._compute_range_device(0.5, want, 0, n, 1, d_pot.ptr, d_acc.ptr,
                                                  d_cost.ptr))
    out["full_walk_ms" if kind == 0 else "full_walk_ms_k1"] = ms
    c = nat.DeviceArray(4 * n)
    tree._cost_to_orig_device(d_cost.ptr, c.ptr)
    costs[label] = c
full_ms = out["full_walk_ms"]
cases = [("cost_balanced", "interactions"), ("wave_balanced", "wave_work"),
         ("equal_count", None)]
for label, ckey in cases:
    if ckey is None:
        ranges = [((n * r) // world, (n * (r + 1)) // world - (n * r) // world) for r in range(world)]
    else:
        ranges = tree._balance_device(costs[ckey].ptr, world)
    walks = []
    for first, count in ranges:
        walks.append(timed(lambda f=first, c=count: tree._compute_range_device(
            0.5, want, f, c, 1, d_pot.ptr, d_acc.ptr, None)))
    mx, mean = max(walks), float(np.mean(walks))
    out[label] = {"ranges": ranges, "walk_ms": walks, "max_ms": mx, "mean_ms": mean,
                  "max_over_mean": mx / mean, "sum_ms": float(np.sum(walks)),
                  "bound_speedup_vs_full": (build_ms + full_ms) / (build_ms + mx)}
print(json.dumps(out), flush=True)
tree.close()
