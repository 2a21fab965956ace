"""mtrl/rl/algorithms/__init__.py:9-19 -- dispatch on the config type."""

from ...config.rl import AlgorithmConfig
from .base import Algorithm, OffPolicyAlgorithm
from .mtsac import MTSAC, MTSACConfig


def get_algorithm_for_config(config: AlgorithmConfig) -> type[Algorithm]:
    if type(config) is MTSACConfig:
        return MTSAC
    raise ValueError(f"Invalid config type: {type(config)} (only MTSACConfig runs on the MI355X engine)")


__all__ = ["Algorithm", "OffPolicyAlgorithm", "MTSAC", "MTSACConfig", "get_algorithm_for_config"]
