"""Per-wave timeline of octree range walks (PBX_WALK_TRACE: start, end,
steps per wave from s_memrealtime, 100 MHz): how much of a range walk is
the tail after most waves are done.  usage: python tools/walk_tail.py"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]
trace = "/tmp/walk_trace.bin"
os.environ["PBX_WALK_TRACE"] = trace

from pynbodyext import _native as nat  # noqa: E402
from pynbodyext._engine import Octree  # noqa: E402
from pynbodyext.synthetic import plummer  # noqa: E402

n = 4_000_000
nat.load()
nat.set_device(0)
pos, mass = plummer(n, seed=1003)
d_pos, d_mass = nat.DeviceArray.from_host(pos), nat.DeviceArray.from_host(mass)
d_pot, d_acc = nat.DeviceArray(8 * n), nat.DeviceArray(24 * n)
tree = Octree._from_device(d_pos.ptr, n, d_mass.ptr, 8, 3)
want = nat.WANT_POT | nat.WANT_ACC
for label, first, count in [("full", 0, n), ("full", 0, n), ("range", 0, n // 8), ("range", 3 * n // 8, n // 8)]:
    if os.path.exists(trace):
        os.remove(trace)
    tree._compute_range_device(0.5, want, first, count, 1, d_pot.ptr, d_acc.ptr, None)
    nat.synchronize()
    h = np.fromfile(trace, dtype=np.uint64).reshape(-1, 3)
    h = h[h[:, 1] > 0]
    s, e, st = h[:, 0].astype(np.int64), h[:, 1].astype(np.int64), h[:, 2]
    t0 = s.min()
    s, e = (s - t0) / 100.0, (e - t0) / 100.0  # us
    d = e - s
    span = e.max()
    ends = np.sort(e)
    out = {"walk": label, "waves": int(len(d)), "span_us": float(span),
           "wave_us_mean": float(d.mean()), "p50": float(np.median(d)),
           "p99": float(np.percentile(d, 99)), "max": float(d.max()),
           "last_start_us": float(s.max()),
           "t90_us": float(ends[int(0.9 * len(ends))]), "t99_us": float(ends[int(0.99 * len(ends))]),
           "steps_mean": float(st.mean()), "steps_max": int(st.max()),
           "corr_dur_steps": float(np.corrcoef(d, st.astype(float))[0, 1]),
           "mean_concurrency": float(d.sum() / span),
           "starts_per_us_mid": float(np.sum((s > 0.25 * span) & (s < 0.75 * span)) / (0.5 * span))}
    # concurrency over time (waves running at 20 sample points)
    ts = np.linspace(0, span, 21)[1:-1]
    out["concurrency_samples"] = [int(np.sum((s <= x) & (e > x))) for x in ts]
    print(json.dumps(out), flush=True)
tree.close()
