"""Critical path of config 5 at 8 GPUs, measured on one GPU: the 4M octree
(theta 0.5, leaf 8, order 3) walked in full once for the per-target wave
costs (ShardedTree's cost kind 1), split into `world` cost-balanced
leaf-order ranges exactly as ShardedTree.balance does, and every range
walked alone with the per-wave timeline (PBX_WALK_TRACE: start, end and
node steps of every wave, s_memrealtime at 100 MHz).

walk_ms includes the trace read-back (host
fwrite between the events); span_us (first wave start to last wave end) is
the kernel's own critical path.

A range walk cannot end before its longest wave: a wave walks the UNION of
its 64 targets' reference walks as one dependent chain of node steps (each
step's next node depends on the ballot of the previous one), so its time is
steps x (time per step when its SIMD is shared).  A range holds ~1.1 waves
per wave slot (8k waves, ~7.2k resident), so all its waves start together
and the range's time is its longest wave's.  This tool prints, per range:
walk time (HIP events), the longest wave's duration and steps, ns per step
of that wave, and the bound build + max(range) + profile it implies.

usage: python tools/critical_path.py [n] [world]"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]
trace = "/tmp/walk_trace_cp.bin"
os.environ["PBX_WALK_TRACE"] = trace

from pynbodyext import _native as nat  # noqa: E402
from pynbodyext._engine import Octree  # noqa: E402
from pynbodyext.synthetic import plummer  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
nat.load()
nat.set_device(0)
pos, mass = plummer(n, seed=1003)
d_pos, d_mass = nat.DeviceArray.from_host(pos), nat.DeviceArray.from_host(mass)
d_pot, d_acc = nat.DeviceArray(8 * n), nat.DeviceArray(24 * n)
d_cost, d_cost_orig = nat.DeviceArray(4 * n), nat.DeviceArray(4 * n)
want = nat.WANT_POT | nat.WANT_ACC
ev = [nat.Event() for _ in range(2)]


def walk(first, count, cost=None):
    if os.path.exists(trace):
        os.remove(trace)
    ev[0].record()
    tree._compute_range_device(0.5, want, first, count, 1, d_pot.ptr, d_acc.ptr, cost)
    ev[1].record()
    nat.synchronize()
    ms = ev[0].elapsed_ms(ev[1])
    h = np.fromfile(trace, dtype=np.uint64).reshape(-1, 3)
    h = h[h[:, 1] > 0]
    s, e, st = h[:, 0].astype(np.int64), h[:, 1].astype(np.int64), h[:, 2].astype(np.int64)
    d = (e - s) / 100.0  # us
    k = int(np.argmax(d))
    return ms, {"waves": int(len(d)), "wave_us_max": float(d[k]), "steps_of_longest": int(st[k]),
                "ns_per_step_longest": float(d[k] * 1e3 / max(st[k], 1)),
                "steps_max": int(st.max()), "wave_us_p99": float(np.percentile(d, 99)),
                "wave_us_mean": float(d.mean()),
                "span_us": float((e.max() - s.min()) / 100.0)}


tree = Octree._from_device(d_pos.ptr, n, d_mass.ptr, 8, 3)
tree._set_cost_kind(1)
ev[0].record()
tree._rebuild_device(d_pos.ptr, n, d_mass.ptr)
ev[1].record()
nat.synchronize()
build_ms = ev[0].elapsed_ms(ev[1])
full_ms, full = walk(0, n, d_cost.ptr)
full_ms, full = walk(0, n, d_cost.ptr)
tree._cost_to_orig_device(d_cost.ptr, d_cost_orig.ptr)
ranges = tree._balance_device(d_cost_orig.ptr, world)
rows = []
for first, count in ranges:
    walk(first, count)  # warm
    ms, info = walk(first, count)
    rows.append({"first": first, "count": count, "walk_ms": ms, **info})
mx = max(r["walk_ms"] for r in rows)
out = {"n": n, "world": world, "build_ms": build_ms, "full_walk_ms": full_ms, "full": full,
       "ranges": rows, "max_range_ms": mx,
       "max_range_over_longest_wave": mx / (max(r["wave_us_max"] for r in rows) / 1e3),
       "max_span_us": max(r["span_us"] for r in rows),
       "bound_speedup_spans": (build_ms + full["span_us"] / 1e3)
       / (build_ms + max(r["span_us"] for r in rows) / 1e3),
       "bound_speedup_excl_profile": (build_ms + full_ms) / (build_ms + mx),
       "note": "range time ~= its longest wave (steps x ns/step); bound = (build + full walk) / "
               "(build + max range), the replicated build counted on every rank"}
print(json.dumps(out), flush=True)
tree.close()
