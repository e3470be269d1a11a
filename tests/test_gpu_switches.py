"""The library's runtime A/B switches (INTEGRATION.md "Runtime variables")
select alternatives that were measured slower; each must still compute the
same results.  tests/_switch_child.py runs one fixed workload in a child
process (the switches are read once per process) with the defaults and
under each group of switches; the results are compared with the defaults'
(which the other GPU tests check against the oracle):

* profiles: edges, counts and CSR bit-identical, per-bin sums to 1e-12;
* octree walk: the same tree and the same per-target walks — bit-identical;
* direct sum: the ordered-pair kernel in place of the pairwise-symmetric one
  (another use of the fast reciprocal square root) — the fast-mode 1e-6
  relative per particle (vector norm for the accelerations).
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
    "profile_a": {"PBX_SPEC": "0", "PBX_MONO_EDGE": "0", "PBX_MONO_HINT": "0",
                  "PBX_MONO_SPIN": "0", "PBX_SEL_TAILFILL": "1", "PBX_SCAN_TICKET": "1",
                  "PBX_PACK_MAPPED": "0", "PBX_TREE_LEVEL_BUILD": "1",
                  "PBX_WALK_XCD_CHUNK": "0", "PBX_DIRECT_T": "1", "PBX_DIRECT_SYM": "0"},
    "profile_b": {"PBX_AGATHER": "0", "PBX_SEL_BT": "256", "PBX_RADIAL_MONO": "0",
                  "PBX_WALK_TPB": "256", "PBX_WALK_W8": "0", "PBX_DIRECT_T": "2"},
    "profile_c": {"PBX_SEL_HINT": "0", "PBX_WALK_W8": "1"},
    "profile_d": {"PBX_RADIAL_EAGER": "1", "PBX_EQUALN": "sort"},
}


def run_child(tmp_path, tag, env_extra):
    out = tmp_path / f"{tag}.npz"
    env = {k: v for k, v in os.environ.items() if not k.startswith("PBX_") or k == "PBX_LIBRARY"}
    env.update(env_extra)
    r = subprocess.run([sys.executable, str(CHILD), str(out)], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, f"{tag}: rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    with np.load(out) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def defaults(gpu, tmp_path_factory):
    return run_child(tmp_path_factory.mktemp("sw"), "defaults", {})


@pytest.mark.parametrize("group", sorted(GROUPS))
def test_runtime_switches_same_results(defaults, tmp_path, group):
    got = run_child(tmp_path, group, GROUPS[group])
    assert sorted(got) == sorted(defaults)
    for k, ref in defaults.items():
        v = got[k]
        if k.startswith("direct/"):  # per particle, the vector norm for accelerations
            d = np.abs(v - ref) if v.ndim == 1 else np.linalg.norm(v - ref, axis=1)
            nrm = np.abs(ref) if ref.ndim == 1 else np.linalg.norm(ref, axis=1)
            assert float(np.max(d / nrm)) < 1e-6, k
        elif "/m" in k:
            np.testing.assert_allclose(v, ref, rtol=1e-12, atol=1e-300, err_msg=k)
        else:  # edges, counts, CSR, tree outputs
            assert np.array_equal(v, ref, equal_nan=True), k
