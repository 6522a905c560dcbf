"""bench.py --gpus N launcher (CPU, gloo): without a torchrun environment `bench.py --gpus N` must start N ranks
itself (distinct RANK / LOCAL_RANK, WORLD_SIZE = N) and print exactly one JSON line (rank 0)."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       env=env, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return lines


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks(n):
    lines = _run(["--gpus", str(n), "--launcher-probe"])
    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    assert d["n_gpus"] == n
    ranks = sorted(tuple(r) for r in d["ranks"])
    assert ranks == [(i, i, n) for i in range(n)]


def test_launcher_single_rank_runs_in_process():
    lines = _run(["--gpus", "1", "--launcher-probe"])
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d == {"n_gpus": 1, "ranks": [[0, 0, 1]]}
