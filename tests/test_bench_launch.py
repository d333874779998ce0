"""bench.py's own N-rank launcher (CPU, no GPU call): ``--gpus N`` without WORLD_SIZE starts N
rank processes with distinct RANK / LOCAL_RANK, one shared MASTER_ADDR / MASTER_PORT and
WORLD_SIZE = N, and fails when a rank fails.  ``--dry-launch`` stops every rank before it
imports vaex_amd."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(*extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, BENCH, *extra], capture_output=True, text=True, env=env, timeout=120)


def test_launcher_starts_n_ranks():
    r = _run("--gpus", "4", "--dry-launch")
    assert r.returncode == 0, r.stderr
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(l["rank"] for l in lines) == [0, 1, 2, 3]
    assert sorted(l["local_rank"] for l in lines) == [0, 1, 2, 3]
    assert {l["world"] for l in lines} == {4}
    assert {l["master_addr"] for l in lines} == {"127.0.0.1"}
    assert len({l["master_port"] for l in lines}) == 1
    assert len({l["pid"] for l in lines}) == 4 and os.getpid() not in {l["pid"] for l in lines}


def test_launcher_fails_when_a_rank_fails():
    r = _run("--gpus", "3", "--dry-launch", "--dry-launch-fail-rank", "2")
    assert r.returncode != 0
    assert "rank 2 exited" in r.stderr


def test_single_gpu_runs_in_process():
    r = _run("--gpus", "1", "--dry-launch")
    assert r.returncode == 0
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and lines[0]["world"] == 1 and lines[0]["rank"] == 0


def test_under_an_external_launcher_no_relaunch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="1", LOCAL_RANK="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-launch"], capture_output=True, text=True,
                       env=env, timeout=120)
    assert r.returncode == 0
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and lines[0]["rank"] == 1 and lines[0]["world"] == 2
