"""bench.py's launcher (CPU, no GPU work): `--gpus N` starts N rank processes itself when no launcher
did (torchrun's per-rank environment, rendezvous on 127.0.0.1), and refuses a rank count it cannot
honour rather than printing a line whose n_gpus misstates the run."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, capture_output=True,
                          text=True, timeout=240)


def test_gpus_2_starts_two_ranks():
    r = _bench(["--gpus", "2", "--check-launch"], LK_BENCH_BACKEND="gloo")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["ranks_seen"] == 2 and line["spawned"] is True
    assert line["master"].startswith("127.0.0.1:")


def test_gpus_disagreeing_with_world_size_is_refused():
    r = _bench(["--gpus", "2", "--check-launch"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr


def test_more_gpus_than_visible_is_refused():
    # this container has no GPU: an RCCL run of 2 ranks cannot be honoured, and nothing is spawned
    r = _bench(["--gpus", "2"])
    assert r.returncode == 2
    assert "visible" in r.stderr
