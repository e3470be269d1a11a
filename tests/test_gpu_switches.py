"""The library's remaining runtime variables (INTEGRATION.md "Runtime
variables") — PBX_PRECISE (the precise arithmetic for every call of the
process), GRAVITY_TIMING (per-call timing lines on stderr) and the
diagnostic traces PBX_MONO_TRACE / PBX_WALK_TRACE — are read once per
process.  tests/_switch_child.py runs one fixed workload in a child process
with the defaults and under each of them; the results are compared with the
defaults' (which the other GPU tests check against the oracle):

* timing and traces: every result bit-identical (profiles: sums to 1e-12;
  the direct sum to 1e-12: its float atomics make the last bits vary);
* PBX_PRECISE=1: profiles bit-identical; the walk and the direct sum move by
  the fast reciprocal square root's rounding only — within the fast mode's
  1e-6 relative per particle (vector norm for the accelerations).
"""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
CHILD = Path(__file__).resolve().parent / "_switch_child.py"

GROUPS = {
    "timing": ({"GRAVITY_TIMING": "1"}, True),
    "traces": ({"PBX_MONO_TRACE": "1", "PBX_WALK_TRACE": "{tmp}/walk_trace.bin"}, True),
    "precise": ({"PBX_PRECISE": "1"}, False),
}


def run_child(tmp_path, tag, env_extra):
    out = tmp_path / f"{tag}.npz"
    env = {k: v for k, v in os.environ.items()
           if not (k.startswith("PBX_") or k == "GRAVITY_TIMING") or k == "PBX_LIBRARY"}
    env.update({k: v.format(tmp=tmp_path) for k, v in env_extra.items()})
    r = subprocess.run([sys.executable, str(CHILD), str(out)], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, f"{tag}: rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    with np.load(out) as z:
        return {k: z[k] for k in z.files}, r.stderr


@pytest.fixture(scope="module")
def defaults(gpu, tmp_path_factory):
    return run_child(tmp_path_factory.mktemp("sw"), "defaults", {})[0]


@pytest.mark.parametrize("group", sorted(GROUPS))
def test_runtime_variables_same_results(defaults, tmp_path, group):
    env, exact = GROUPS[group]
    got, err = run_child(tmp_path, group, env)
    assert sorted(got) == sorted(defaults)
    if group == "timing":
        assert "pbx." in err  # ScopedTimer lines
    if group == "traces":
        assert "[mono]" in err and (tmp_path / "walk_trace.bin").stat().st_size > 0
    for k, ref in defaults.items():
        v = got[k]
        if k.startswith("direct/") or (k.startswith("tree/") and not exact):
            # (the direct sum adds its per-particle partials with float
            # atomics: the last bits follow the arrival order, run to run)
            d = np.abs(v - ref) if v.ndim == 1 else np.linalg.norm(v - ref, axis=1)
            nrm = np.abs(ref) if ref.ndim == 1 else np.linalg.norm(ref, axis=1)
            assert float(np.max(d / nrm)) < (1e-12 if exact else 1e-6), k
        elif "/m" in k:
            np.testing.assert_allclose(v, ref, rtol=1e-12, atol=1e-300, err_msg=k)
        else:  # edges, counts, CSR, tree and direct outputs
            assert np.array_equal(v, ref, equal_nan=True), k
