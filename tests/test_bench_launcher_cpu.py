"""bench.py's multi-GPU launch, checked on the CPU (no GPU, no library).

`python bench.py --gpus N` without WORLD_SIZE must start N rank processes
itself (one per GPU; the driver may instead start them with
torch.distributed.run, which sets WORLD_SIZE), and only rank 0 prints the JSON
line.  --dry-run runs the same launcher, process group (gloo here), barriers
and max-over-ranks timing with a CPU stand-in step."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None):
    env = dict(os.environ)
    for key in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(key, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=300, env=env)


def test_gpus_2_spawns_two_ranks_one_json_line():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]  # (gloo logs its connections)
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["ranks_seen"] == [0, 1] and line["pids_differ"]
    assert line["steps"] == 3 and line["scaling"] == "strong"


def test_gpus_1_runs_in_process():
    r = _run(["--gpus", "1", "--dry-run", "--steps", "2", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["ranks_seen"] == [0]


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "1"], {"WORLD_SIZE": "3", "RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr
