"""Concurrency of a PBX_WALK_TRACE dump (last launch): waves in flight."""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 3).astype(np.int64)
nw = int(sys.argv[2])  # waves per launch
t = a[-nw:]
ok = t[:, 1] > 0
s, e = (t[ok, 0] - t[ok, 0].min()) / 100.0, (t[ok, 1] - t[ok, 0].min()) / 100.0
T = e.max()
conc = [np.sum((s <= g) & (e > g)) for g in np.linspace(0.05 * T, 0.95 * T, 19)]
print(f"span {T:.0f} us, waves in flight median {np.median(conc):.0f} (min {min(conc)}, max {max(conc)})")
