import sys, ctypes, gc
sys.path[:0] = ['.', 'pynbody-extras_amd']
import numpy as np
from pynbodyext import _native as nat
from pynbodyext.filters import FamilyFilter, Sphere
from pynbodyext.profiles import RadialProfileBuilder
from pynbodyext.synthetic import plummer_snapshot
nat.load(); nat.set_device(0)
def stats():
    out = (ctypes.c_int64 * 4)(); nat.call("pbx_device_pool_stats", out); return list(out)
sim = plummer_snapshot(2_000_000, seed=1008)
b = RadialProfileBuilder(ndim=3, weight="mass", bins_type="equaln", nbins=64).filter(Sphere(10.0) & FamilyFilter("dm"))
print('start', stats())
for k in range(3):
    prof = b(sim); np.asarray(prof["mass"]["sum"]); prof.bins.binind.csr
    print(k, stats())
    del prof; gc.collect()
    print(k, 'after free', stats())
