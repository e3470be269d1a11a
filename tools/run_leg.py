"""Run one bench leg alone (for rocprofv3 traces / A-B timing on the box).
usage: python tools/run_leg.py profile N[,N...] [steps]
       python tools/run_leg.py tree N [steps]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]

import bench  # noqa: E402
from pynbodyext import _native as nat  # noqa: E402

leg = sys.argv[1]
sizes = [int(s) for s in sys.argv[2].split(",")]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
nat.load()
nat.set_device(0)
if leg == "profile":
    out = bench.bench_profile(sizes, steps=steps, warmup=2, cpu=False)
    for r in out:
        d = {k: r[k] for k in ("n", "ms", "stream_ms", "hbm_gbs_algorithmic")}
        d["changing_stream_ms"] = (r.get("changing") or {}).get("stream_ms")
        d["cold_stream_ms"] = r.get("cold_stream_ms")
        print(json.dumps(d))
elif leg == "tree":
    d = bench.Dist()
    out = bench.bench_tree(d, sizes[0], steps=steps, warmup=1, cpu=False, cpu_seconds=0)
    print(json.dumps({k: out[k] for k in ("ms_per_step", "phases_ms", "interactions", "roofline")}))
