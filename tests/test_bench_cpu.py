"""bench.py's multi-rank launcher on CPU (gloo): `--gpus N` outside torchrun spawns N rank
processes before anything touches a GPU, shards the tasks contiguously and
reduces the timing with a max over ranks; a --gpus / WORLD_SIZE mismatch is an error."""

from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=e, timeout=240)


def _line(p):
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, (p.returncode, p.stdout, p.stderr[-2000:])
    return json.loads(lines[0])


def test_gpus2_spawns_two_ranks_with_25_25_shards():
    d = _line(_run(["--gpus", "2", "--dry-run"]))
    assert d["n_gpus"] == 2 and d["nranks"] == 2 and d["max_over_ranks"] == 2.0
    assert d["config"]["task_shards"] == [[0, 25], [25, 25]]
    assert d["config"]["parallelism"] == "task-shard2" and d["scaling"] == "strong"
    assert d["config"]["allreduce_bytes_per_step"] == 102_990_856  # 68.7 MB critic + 34.3 MB actor trunk


def test_gpus8_mt50_split():
    d = _line(_run(["--gpus", "8", "--dry-run"]))
    assert [c for _, c in d["config"]["task_shards"]] == [7, 7, 6, 6, 6, 6, 6, 6]
    assert d["max_over_ranks"] == 8.0


def test_gpus1_is_single_rank():
    d = _line(_run(["--dry-run"]))
    assert d["n_gpus"] == 1 and d["config"]["task_shards"] == [[0, 50]] and d["config"]["allreduce_bytes_per_step"] == 0


def test_world_size_mismatch_is_an_error():
    p = _run(["--gpus", "2", "--dry-run"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2 and "WORLD_SIZE" in p.stderr
