"""The C-ABI library loads and exports every symbol include/pbx.h declares."""
import re
import subprocess
from pathlib import Path

import pytest

from pynbodyext import _native

HEADER = Path(__file__).resolve().parent.parent / "include" / "pbx.h"


def declared_symbols():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"\b(pbx_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_are_bound():
    decl = declared_symbols()
    assert decl, "no symbols parsed from pbx.h"
    assert sorted(decl) == _native.exported_symbols()


def test_library_exports_symbols():
    path = _native.lib_path()
    assert path.exists(), "libpbx.so not built"
    out = subprocess.run(["nm", "-D", "--defined-only", str(path)], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\b(pbx_[a-z0-9_]+)\b", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    lib = _native.load()
    assert lib.pbx_version() == 100


def test_library_is_gfx950_code_object():
    path = _native.lib_path()
    out = subprocess.run(["strings", str(path)], capture_output=True, text=True).stdout
    assert "gfx950" in out


def test_no_cpu_fallback_without_gpu():
    """On a machine without a GPU the engine must raise, never compute on CPU."""
    import numpy as np

    from pynbodyext import _engine

    try:
        n = _native.device_count()
    except RuntimeError:
        n = 0
    if n:
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no HIP device"):
        _engine.direct_potentials_py(np.zeros((4, 3)))
