"""bench.py's launcher (CPU, no GPU): `python bench.py --gpus 2` with no WORLD_SIZE starts two
ranks itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* on 127.0.0.1), they rendezvous over
gloo, time with barrier + max over ranks, and rank 0 prints exactly one JSON line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=180)


def test_launcher_spawns_world_2():
    r = _run(["--gpus", "2", "--plumbing"])
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_ranks"] == 2 and d["ranks_seen"] == 2
    assert d["check"] == (1 << 16) * ((1 << 16) - 1) // 2
    assert d["t_max"] >= 1e-3  # the max over ranks includes rank 1's offset


def test_launcher_single_rank():
    r = _run(["--gpus", "1", "--plumbing"])
    assert r.returncode == 0, r.stderr
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_ranks"] == 1


def test_world_mismatch_fails():
    r = _run(["--gpus", "2", "--plumbing"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
