import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "pynbody-extras_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP path")
    config.addinivalue_line("markers", "fast: runs the default fast-precision mode (tree tests default to precise)")


@pytest.fixture(scope="session")
def gpu():
    """Fail (not skip) a gpu-marked test when the HIP path cannot run."""
    from pynbodyext import _native

    _native.load()
    n = _native.device_count()
    assert n >= 1, "no GPU visible to libpbx"
    return n
