"""Hardware queues for the engine's streams.

HIP maps streams beyond GPU_MAX_HW_QUEUES (its default is 4) onto shared hardware queues, and with
shared queues the engine's experimental 5-lane form (MTSAC_LANES=1) was even less reproducible
("Lanes and hardware queues").  The engine grants the lanes only if the
process STARTED with enough queues for every live engine's 5 lanes + 3 reserved (engine.cpp
relane, reading /proc/self/environ: the runtime reads the variable once, so a value set from
inside the process is not trusted).  Tests of the lane form run in child processes started with
``child_env()``."""

from __future__ import annotations

import os

WANT = 16  # 5 engine lanes + null stream + torch + RCCL, with room for a second engine


def start_hw_queues() -> int:
    """GPU_MAX_HW_QUEUES in the environment this process started with (HIP's default 4)."""
    try:
        with open("/proc/self/environ", "rb") as f:
            for kv in f.read().split(b"\0"):
                if kv.startswith(b"GPU_MAX_HW_QUEUES="):
                    v = int(kv.split(b"=", 1)[1] or b"0")
                    return v if v > 0 else 4
    except (OSError, ValueError):
        pass
    return 4


def child_env(n: int = WANT, lanes: bool = True) -> dict:
    """Environment for a child process started with n hardware queues (and the lane form)."""
    env = dict(os.environ)
    env["GPU_MAX_HW_QUEUES"] = str(max(n, start_hw_queues()))
    if lanes:
        env["MTSAC_LANES"] = "1"
    return env
