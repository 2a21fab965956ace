"""mtrl/rl/algorithms/__init__.py:9-19 -- dispatch on the config type."""

from ...config.rl import AlgorithmConfig
from .base import Algorithm, OffPolicyAlgorithm
from .drqeps import DrQ, DrQConfig
from .mtsac import MTSAC, MTSACConfig


def get_algorithm_for_config(config: AlgorithmConfig) -> type[Algorithm]:
    if type(config) is MTSACConfig:
        return MTSAC
    if type(config) is DrQConfig:
        return DrQ
    raise ValueError(f"Invalid config type: {type(config)} (MTSACConfig and DrQConfig run on the MI355X engines)")


__all__ = ["Algorithm", "OffPolicyAlgorithm", "DrQ", "DrQConfig", "MTSAC", "MTSACConfig", "get_algorithm_for_config"]
