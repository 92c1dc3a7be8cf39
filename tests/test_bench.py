"""bench.py's multi-rank launch (no GPU): with --gpus N and no launcher it starts N rank processes
itself (RANK / WORLD_SIZE / MASTER_* set, before any HIP call), they rendezvous, and rank 0 reports
the ranks it saw; a WORLD_SIZE that disagrees with --gpus is refused (exit 2) instead of silently
measuring another N."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    e.update(kw)
    return e


@pytest.mark.parametrize("n", [2, 4])
def test_bench_launches_n_ranks_itself(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--check-launch"], capture_output=True, text=True,
                       timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["ranks_seen"] == n and line["world"] == n


def test_bench_refuses_a_wrong_world_size():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--check-launch"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                                             MASTER_PORT="29512"))
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_bench_launcher_stops_when_a_rank_dies():
    """a rank that dies before the rendezvous must not leave rank 0 waiting for it; the
    launcher kills the others and exits with the failed rank's code."""
    import time
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--check-launch", "--check-launch-fail-rank", "1"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 5, (r.returncode, r.stderr[-2000:])
    assert time.monotonic() - t0 < 200
