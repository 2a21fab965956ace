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


def test_pmc_traffic_takes_the_newest_round_summary(tmp_path, monkeypatch):
    """The roofline's `traffic` comes from the newest committed PMC summary of the workload: rounds in
    order, then a..z, aa..zz (r5x before r5bb), not plain name order."""
    sys.path.insert(0, ROOT)
    import bench

    prof = tmp_path / "profiles"
    prof.mkdir()
    for name, v in (("r4zz", 1.0), ("r5x", 2.0), ("r5bb", 3.0), ("r3final3", 0.5)):
        (prof / f"{name}_pmc_traffic.json").write_text(json.dumps({"split2h": {"0": {"hbm_bytes_per_launch": v}}}))
    (prof / "r9_pmc_traffic.json").write_text(json.dumps({"workload": "mt10_w400",
                                                           "split2h": {"0": {"hbm_bytes_per_launch": 9.0}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    v, src = bench.pmc_traffic("split2h", 0, "mt50_w2048")
    assert v == 3.0 and src.endswith("r5bb_pmc_traffic.json")
    assert bench.pmc_traffic("split2h", 0, "mt10_w400")[0] == 9.0
    assert bench.pmc_traffic("bf16", 0, "mt50_w2048") == (None, None)
