"""bench.py's own launcher (no torchrun): `python bench.py --gpus 2` must start two rank processes
that rendezvous over 127.0.0.1, and rank 0 must report n_gpus = 2. Runs on the CPU with gloo
(--rehearse-launch skips the GPU workload); the GPU path is the same launch with backend nccl."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=300, env=e, cwd=ROOT)


def test_bench_spawns_ranks_for_gpus_2():
    p = _run("--gpus", "2", "--rehearse-launch")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["ranks_seen"] == [0, 1]


def test_bench_single_rank_default():
    p = _run("--rehearse-launch")
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_bench_rejects_mismatched_world():
    p = _run("--gpus", "4", "--rehearse-launch", env={"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr
