"""Where the user-facing profile call spends its time: bench.py's
profile.api_level call — RadialProfileBuilder(ndim=3, weight="mass",
equaln, 128).filter(Sphere(10) & FamilyFilter("dm"))(sim) on host numpy
arrays, then prof["mass"]["sum"] and prof["r"] — warmed twice, then one call
under cProfile (top functions by cumulative time) and the wall time of
reps more.  GRAVITY_TIMING=1 adds the library's per-call timings.
usage: python tools/api_breakdown.py N [reps]"""
import cProfile
import io
import json
import pstats
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]

from pynbodyext import _native as nat  # noqa: E402
from pynbodyext.filters import FamilyFilter, Sphere  # noqa: E402
from pynbodyext.profiles import RadialProfileBuilder  # noqa: E402
from pynbodyext.synthetic import plummer_snapshot  # noqa: E402

n = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
nat.load()
nat.set_device(0)
sim = plummer_snapshot(n, seed=1002)
builder = RadialProfileBuilder(ndim=3, weight="mass", bins_type="equaln",
                               nbins=128).filter(Sphere(10.0) & FamilyFilter("dm"))


def call():
    prof = builder(sim)
    return prof, np.asarray(prof["mass"]["sum"]), np.asarray(prof["r"])


call()
call()
pr = cProfile.Profile()
pr.enable()
call()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(30)
print(s.getvalue())
ts = []
for _ in range(reps):
    t0 = time.perf_counter()
    call()
    ts.append(time.perf_counter() - t0)
print(json.dumps({"n": n, "builder_ms_median": float(np.median(ts)) * 1e3,
                  "builder_ms_min": float(np.min(ts)) * 1e3}))
