"""bench.py's multi-GPU launch plan, on the CPU: `--gpus N` without WORLD_SIZE starts N ranks under
torch.distributed.run as a child process, and every rank checks WORLD_SIZE == N (dry run: the ranks
print their plan and exit before any GPU call)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=300, env=e, cwd=ROOT)


def test_gpus_2_spawns_two_ranks():
    r = run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    plans = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert sorted(p["rank"] for p in plans) == [0, 1]
    assert all(p["world_size"] == 2 for p in plans)
    assert sorted(p["device"] for p in plans) == [0, 1]
    assert all(p["master"].startswith("127.0.0.1:") for p in plans)


def test_world_size_must_match_gpus():
    r = run(["--gpus", "4", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in (r.stderr + r.stdout)


def test_single_gpu_dry_run():
    r = run(["--dry-run"])
    assert r.returncode == 0
    plan = json.loads(r.stdout.strip().splitlines()[-1])
    assert plan["world_size"] == 1 and plan["rank"] == 0
