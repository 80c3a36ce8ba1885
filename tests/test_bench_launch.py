"""bench.py's own rank launcher (`--gpus N` without an outside torchrun), run
on the CPU through its gloo dry run: N rank processes come up under a
torch.distributed.run child, rank 0's key/table reach every rank by
broadcast, and the line reports n_gpus = world.  A WORLD_SIZE that disagrees
with --gpus is refused.  No GPU, no packets."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout,
                          env=env, cwd=ROOT)


@pytest.mark.parametrize("world", [2, 3])
def test_launcher_starts_world_ranks(world):
    r = _run(["--gpus", str(world), "--dry-run", "--workload", "c3", "--packets", "512", "--steps", "3",
              "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == world and d["dry_run"] and d["steps"] == 3
    assert [p["rank"] for p in d["per_rank"]] == list(range(world))
    assert all(p["rss_config_broadcast_ok"] for p in d["per_rank"])  # ranks > 0 started from zeros
    assert sum(p["packets"] for p in d["per_rank"]) == d["config"]["job_packets"] == 512 * world
    assert d["job_queue_hits_ok"]


def test_launcher_one_gpu_stays_in_process():
    r = _run(["--gpus", "1", "--dry-run", "--steps", "2", "--packets", "64"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert d["n_gpus"] == 1 and "launching" not in r.stderr


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "3", "--dry-run"], env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "refusing" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]
