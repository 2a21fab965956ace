"""mtrl/types.py:30-35,85-99 (the types the MTSAC path exchanges)."""

from typing import Any, NamedTuple, TypedDict

import numpy as np

LogDict = dict[str, float]


class ReplayBufferSamples(NamedTuple):
    observations: np.ndarray
    actions: np.ndarray
    next_observations: np.ndarray
    dones: np.ndarray
    rewards: np.ndarray


class AtariReplayBufferSamples(NamedTuple):  # mtrl/types.py:38-45
    observations: np.ndarray  # uint8 [B][C][H][W]
    actions: np.ndarray
    next_observations: np.ndarray
    truncations: np.ndarray
    dones: np.ndarray
    rewards: np.ndarray
    task_ids: np.ndarray


class CheckpointMetadata(TypedDict):
    timestamp: str
    step: int
    episodes_ended: int


class ReplayBufferCheckpoint(TypedDict):
    data: dict[str, Any]
    rng_state: Any
