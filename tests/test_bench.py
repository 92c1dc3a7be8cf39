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


def test_traffic_only_from_a_profile_of_this_build(tmp_path):
    """roofline.traffic is read from a committed PMC summary only when that summary was
    taken with the libbos.so this process loaded (its sha256); otherwise it is null."""
    sys.path.insert(0, ROOT)
    import bench
    import bos
    bench.bos = bos
    mine = bench.lib_sha256()
    for label, sha in (("instep", mine), ("warm", "0" * 64)):
        with open(tmp_path / f"{bench.PROFILE_TAG}_pmc_linearize_fp32_{label}.json", "w") as f:
            json.dump({"hbm_bytes_per_launch": 123.0, "libbos_sha256": sha}, f)
    t, why = bench.traffic_from_profile(bos.BOS_FP32, str(tmp_path))
    assert t == {"instep": 123.0, "warm": None}
    assert "another libbos.so" in why["warm"]
    t, why = bench.traffic_from_profile(bos.BOS_FP64, str(tmp_path))
    assert t == {"instep": None, "warm": None}


LADDER_CASES = [
    # (world, failures, expected mode, expected failed attempts)
    (2, "", "p2p", []),
    (2, "p2p:setup@1", "rccl", ["p2p"]),
    (2, "p2p:run@0,rccl:setup@*", "gloo", ["p2p", "rccl"]),
    (8, "p2p:run@5", "rccl", ["p2p"]),
    (8, "p2p:setup@3,rccl:run@7", "gloo", ["p2p", "rccl"]),
    (8, "p2p:setup@*,rccl:run@1,gloo:run@6", None, ["p2p", "rccl", "gloo"]),
]


@pytest.mark.parametrize("world,fails,mode,failed", LADDER_CASES)
def test_exchange_ladder_every_rank_takes_the_same_decision(world, fails, mode, failed):
    """the N > 1 bench falls back p2p -> RCCL -> gloo host exchange when a mode
    fails on any rank (at setup or in its run), every rank agreeing on each step (gloo collectives),
    and rank 0 prints a line whatever fails, naming the failing ranks' reasons. The stand-in modes
    fail at the listed rank and stage and make the real run's collective calls after the failure."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(world), "--check-launch", "--check-ladder", fails],
                       capture_output=True, text=True, timeout=600, env=_env())
    assert r.returncode == (0 if mode else 4), r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["ranks_seen"] == world
    d = line["exchange_decision"]
    assert d["mode"] == mode
    assert [a["mode"] for a in d["attempts"] if not a["ok"]] == failed
    for a in d["attempts"]:
        if not a["ok"]:   # the reason of every rank that failed, and only of those
            spec = [f for f in fails.split(",") if f.startswith(a["mode"] + ":")][0]
            who = spec.split("@")[1]
            assert set(a["why"]) == ({str(q) for q in range(world)} if who == "*" else {who}), a
            assert a["stage"] == spec.split(":")[1].split("@")[0]
