"""Walk statistics of the 4M config-5 tree: interactions, wave steps, lane
efficiency, time per wave step (GPU box diagnostic, not a test)."""
import sys
import time

import numpy as np

import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from pynbodyext._engine import Octree  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
pos, mass = bench.plummer(n, seed=bench.SEEDS.get(n, 1003))
t = Octree(pos, mass, leaf_capacity=8, multipole_order=3)
from pynbodyext import _native as nat  # noqa: E402

d_pot = nat.DeviceArray.empty((n,)) if hasattr(nat.DeviceArray, "empty") else nat.DeviceArray.from_host(np.zeros(n))
d_acc = nat.DeviceArray.from_host(np.zeros((n, 3)))
for _ in range(3):
    t0 = time.perf_counter()
    t._compute_device(0.5, nat.WANT_POT | nat.WANT_ACC, d_pot.ptr, d_acc.ptr)
    nat.synchronize()
    dt = time.perf_counter() - t0
print(f"walk {dt * 1e3:.2f} ms")
inf = t.info()
ws, al = inf["wave_steps"], inf["active_lane_steps"]
print(inf)
print(f"lane eff {al / ws / 64:.3f}  wave steps/target-wave {ws / (n / 64):.0f}  "
      f"lane steps/target {al / n:.0f}  nodes/target {inf['node_interactions'] / n:.0f}  "
      f"pairs/target {inf['leaf_pairs'] / n:.0f}")
lws, lal, dws = inf["leaf_wave_steps"], inf["leaf_active_lanes"], inf["descend_wave_steps"]
print(f"leaf wave steps {lws / ws:.3f} of steps, leaf lane eff {lal / max(lws, 1) / 64:.3f}; "
      f"node steps lane eff {(al - lal) / max(ws - lws, 1) / 64:.3f}; descending steps {dws / ws:.3f}")
