"""bench.py --gpus N without a launcher starts its own N rank processes (missing 1):
each child gets the torch.distributed.run environment (RANK, LOCAL_RANK, WORLD_SIZE, a shared
127.0.0.1 rendezvous).  CPU only: the children stop at PANO_BENCH_SPAWN_PROBE, before any GPU
call."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_spawns_its_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PANO_BENCH_SPAWN_PROBE"] = "1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    got = [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert sorted(int(g["RANK"]) for g in got) == [0, 1, 2]
    assert all(g["WORLD_SIZE"] == "3" and g["LOCAL_RANK"] == g["RANK"] for g in got)
    assert all(g["MASTER_ADDR"] == "127.0.0.1" for g in got)
    assert len({g["MASTER_PORT"] for g in got}) == 1


def test_bench_rank_failure_is_the_exit_status():
    """A rank that fails (here: no GPU in this container) makes the launcher exit non-zero."""
    import torch
    if torch.cuda.is_available():
        return
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                             "PANO_BENCH_SPAWN_PROBE")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0
