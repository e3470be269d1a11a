"""pynbodyext.gravity — direct-sum and Barnes-Hut gravity on MI355X.

Exports follow the reference (pynbodyext/gravity/__init__.py:15-30): the
``GRAVITY_RUST_AVAILABLE`` flag always; ``Gravity``, ``KernelKind``,
``calculate_potential`` and ``calculate_acceleration`` when the native
engine (libpbx.so) is built.
"""
from pynbodyext.util.deps import GRAVITY_RUST_AVAILABLE

__all__ = ["GRAVITY_RUST_AVAILABLE"]

if GRAVITY_RUST_AVAILABLE:
    from .base import Gravity, KernelKind, TreeOptions
    from .pyn_gravity import calculate_acceleration, calculate_potential

    __all__ += ["Gravity", "KernelKind", "TreeOptions", "calculate_potential",
                "calculate_acceleration"]
else:
    import warnings

    warnings.warn(
        "pynbodyext.gravity: native HIP engine (libpbx.so) not available; "
        "gravity calculations will be unavailable.",
        ImportWarning,
        stacklevel=2,
    )
