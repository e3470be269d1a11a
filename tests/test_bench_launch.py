"""bench.py's multi-GPU launch contract (CPU; no GPU call is made):
``--gpus N`` without a launcher starts N rank processes itself (one per
GPU, torch.distributed.run, before any GPU call), and a rank whose
WORLD_SIZE differs from ``--gpus`` exits non-zero."""
import json
import os
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(PBX_BENCH_DRYRUN="1", **kw)
    return env


def test_bench_gpus2_spawns_two_ranks():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    # the ranks print concurrently: their lines may interleave
    ranks = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", r.stdout)]
    assert sorted(x["rank"] for x in ranks) == [0, 1]
    assert all(x["world"] == 2 for x in ranks)
    assert sorted(x["local_rank"] for x in ranks) == [0, 1]


def test_bench_world_size_mismatch_fails():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"],
                       env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE 3" in r.stderr


def test_bench_default_is_one_gpu():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py")], env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["world"] == 1
