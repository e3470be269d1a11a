"""pynbodyext (MI355X-native hot path).

A from-scratch MI355X (gfx950) implementation of pynbody-extras' particle
analysis hot path: the direct-sum / Barnes-Hut gravity solve
(:mod:`pynbodyext.gravity`) and the radial-profile binning / per-bin
reduction (:mod:`pynbodyext.profiles`), behind the reference's Python API.
The compute runs in hand-written HIP kernels (libpbx.so, C ABI in
include/pbx.h) called through ctypes.
"""
__version__ = "0.1.0"
