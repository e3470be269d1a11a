"""Config 5 at 8 GPUs, measured on one GPU, with PREORDER PIECES
(pbx_octree_set_walk_pieces): the 4M octree (theta 0.5, leaf 8, order 3)
walked in full for the wave costs, split into `world` cost-balanced
leaf-order ranges aligned to 64 targets (ShardedTree.balance with pieces),
and every range walked alone with the per-wave timeline (PBX_WALK_TRACE)
— first plain, then under each pieces setting "permille,kmax": a range is
walked three times (the first records its groups' steps and node
checkpoints, the second is cut at them and records its pieces' own, the
third — timed, without the walk statistics like the bench's timed steps —
is cut at those), each checked against the full walk
(interaction counts identical, values to 1e-12).

Prints one JSON object: per setting the max range span (first wave start to
last wave end: the kernel's own critical path), the longest wave, and the
bound (build + full walk) / (build + max span) — DESIGN §4.

usage: python tools/critical_path_pieces.py [n] [world] [settings]
       settings: "500,2;400,3;300,4" (default)"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]
trace = "/tmp/walk_trace_cpp.bin"
os.environ["PBX_WALK_TRACE"] = trace

from pynbodyext import _native as nat  # noqa: E402
from pynbodyext._engine import Octree  # noqa: E402
from pynbodyext.parallel import align_ranges  # noqa: E402
from pynbodyext.synthetic import plummer  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
settings = [tuple(int(v) for v in s.split(",")) for s in
            (sys.argv[3] if len(sys.argv) > 3 else "500,2;400,3;300,4").split(";")]
nat.load()
nat.set_device(0)
pos, mass = plummer(n, seed=1003)
d_pos, d_mass = nat.DeviceArray.from_host(pos), nat.DeviceArray.from_host(mass)
d_pot, d_acc = nat.DeviceArray(8 * n), nat.DeviceArray(24 * n)
d_cost, d_cost_orig = nat.DeviceArray(4 * n), nat.DeviceArray(4 * n)
want = nat.WANT_POT | nat.WANT_ACC
ev = [nat.Event() for _ in range(2)]


def walk(first, count, cost=None, counted=True):
    """One range walk; ``counted=False``: without the walk statistics (the
    fast kernel the timed ShardedTree steps run), counts then reported from
    the last counted walk."""
    if os.path.exists(trace):
        os.remove(trace)
    tree._set_walk_counters(counted)
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
    info = tree.info() if counted else last_info[0]
    last_info[0] = info
    return ms, {"waves": int(len(d)), "wave_us_max": float(d[k]), "steps_of_longest": int(st[k]),
                "steps_max": int(st.max()), "wave_us_p99": float(np.percentile(d, 99)),
                "wave_us_mean": float(d.mean()),
                "span_us": float((e.max() - s.min()) / 100.0),
                "counts": (info["node_interactions"], info["leaf_pairs"])}


last_info = [None]


def outputs(count):
    p, a = np.empty(count), np.empty((count, 3))
    d_pot.download(p)
    d_acc.download(a)
    return p, a


tree = Octree._from_device(d_pos.ptr, n, d_mass.ptr, 8, 3)
tree._set_cost_kind(1)
ev[0].record()
tree._rebuild_device(d_pos.ptr, n, d_mass.ptr)
ev[1].record()
nat.synchronize()
build_ms = ev[0].elapsed_ms(ev[1])
walk(0, n, d_cost.ptr)
full_ms, full = walk(0, n, d_cost.ptr, counted=False)
p_full, a_full = outputs(n)
tree._cost_to_orig_device(d_cost.ptr, d_cost_orig.ptr)
ranges = align_ranges(tree._balance_device(d_cost_orig.ptr, world), n, 64)


def run_ranges(label, reps):
    rows, worst = [], 0.0
    for first, count in ranges:
        for _ in range(reps - 1):
            walk(first, count, d_cost.offset(4 * first))
        ms, info = walk(first, count, d_cost.offset(4 * first), counted=False)
        p, a = outputs(count)
        rp = float(np.max(np.abs(p - p_full[first:first + count]) / np.abs(p_full[first:first + count])))
        ra = float(np.max(np.linalg.norm(a - a_full[first:first + count], axis=1)
                          / np.linalg.norm(a_full[first:first + count], axis=1)))
        worst = max(worst, rp, ra)
        rows.append({"first": first, "count": count, "walk_ms": ms, **info})
    span = max(r["span_us"] for r in rows)
    print(f"{label}: max span {span:.0f} us, longest wave {max(r['wave_us_max'] for r in rows):.0f} us, "
          f"waves {sum(r['waves'] for r in rows)}, max rel vs full {worst:.2e}", file=sys.stderr,
          flush=True)
    return {"max_range_ms": max(r["walk_ms"] for r in rows), "max_span_us": span,
            "max_wave_us": max(r["wave_us_max"] for r in rows), "max_rel_vs_full": worst,
            "bound_speedup_spans": (build_ms + full["span_us"] / 1e3) / (build_ms + span / 1e3),
            "ranges": rows}


res = {"plain": run_ranges("plain", 2)}
for pm, kmax in settings:
    tree._set_walk_pieces(pm, kmax)
    res[f"pieces_{pm}_{kmax}"] = run_ranges(f"pieces {pm},{kmax}", 3)
    tree._set_walk_pieces(-1, 2)
# interaction counts summed over the ranges equal the full walk's
for k, v in res.items():
    tot = tuple(sum(r["counts"][i] for r in v["ranges"]) for i in range(2))
    v["counts_equal_full"] = tot == tuple(full["counts"])
out = {"n": n, "world": world, "build_ms": build_ms, "full_walk_ms": full_ms, "full": full,
       "ranges": [list(r) for r in ranges], "results": res,
       "note": "span = first wave start to last wave end of a range walk (its critical path); "
               "bound = (build + full span) / (build + max range span), the replicated build "
               "counted on every rank"}
print(json.dumps(out), flush=True)
tree.close()
