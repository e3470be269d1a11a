"""pynbody when it is installed, else the in-package stand-in (simcore)."""
from __future__ import annotations

try:  # pragma: no cover - pynbody is absent in this image
    import pynbody as _pynbody
    from pynbody import filt, units
    from pynbody.array import IndexedSimArray, SimArray
    from pynbody.family import Family, get_family
    from pynbody.snapshot import SimSnap

    HAVE_PYNBODY = True
except ImportError:
    from .simcore import (  # noqa: F401
        Family,
        IndexedSimArray,
        SimArray,
        SimSnap,
        filt,
        get_family,
        units,
    )

    HAVE_PYNBODY = False

__all__ = ["SimArray", "IndexedSimArray", "SimSnap", "Family", "get_family", "units", "filt",
           "HAVE_PYNBODY"]
