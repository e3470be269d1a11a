"""Drop-in name for the reference's native module.

The reference's gravity front end imports ``pynbodyext._rust``
(pynbodyext/gravity/base.py:50-62, crates/pynbodyext-rust/src/lib.rs:10-27).
This module exposes the same surface, computed on MI355X by libpbx.so, so a
caller that kept the reference's Python front end unchanged still works.
"""
from ._engine import *  # noqa: F401,F403
from ._engine import __all__  # noqa: F401
