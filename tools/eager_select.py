"""Time the eager (stepwise) selection of the bench's config-3 input at N
particles (the multi-rank bench path's select): python tools/eager_select.py N [steps]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]
from bench import plummer  # noqa: E402
from pynbodyext import _native as nat  # noqa: E402
from pynbodyext.profiles._device import DeviceBins  # noqa: E402
from pynbodyext.synthetic import family_slices  # noqa: E402

n = int(sys.argv[1])
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
nat.load()
nat.set_device(0)
pos, mass = plummer(n, seed=1002)
dm = family_slices(n)["dm"]
d_pos, d_mass = nat.DeviceArray.from_host(pos), nat.DeviceArray.from_host(mass)
dev = DeviceBins()
for _ in range(steps):
    DeviceBins.select(d_pos.ptr, d_mass.ptr, sphere=((0.0, 0.0, 0.0), 10.0),
                      families=[(dm.start, dm.stop)], ndim=3, on_device=True, n=n, into=dev)
nat.synchronize()
print("kept", dev.n)
dev.close()
