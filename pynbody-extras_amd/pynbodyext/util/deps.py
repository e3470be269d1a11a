"""Feature flags (mirrors pynbodyext/util/deps.py:14-19 of the reference).

``GRAVITY_RUST_AVAILABLE`` keeps its reference name: it is True when the
native gravity engine (here libpbx.so, HIP/gfx950) is built and loadable.
"""
from __future__ import annotations

import importlib.util


def _native_available() -> bool:
    try:
        from pynbodyext import _native
        _native.load()
        return True
    except Exception:
        return False


GRAVITY_RUST_AVAILABLE: bool = _native_available()
GRAVITY_NATIVE_AVAILABLE: bool = GRAVITY_RUST_AVAILABLE
PYNBODY_AVAILABLE: bool = importlib.util.find_spec("pynbody") is not None
DASK_AVAILABLE: bool = importlib.util.find_spec("dask") is not None
