"""mtrl/config/networks.py:6-31."""

from dataclasses import dataclass

from .nn import NeuralNetworkConfig, VanillaNetworkConfig


@dataclass(frozen=True)
class ContinuousActionPolicyConfig:
    network_config: NeuralNetworkConfig = VanillaNetworkConfig(width=400, depth=3)
    squash_tanh: bool = True
    log_std_min: float = -20.0
    log_std_max: float = 2.0


@dataclass(frozen=True)
class QValueFunctionConfig:
    network_config: NeuralNetworkConfig = VanillaNetworkConfig(width=400, depth=3)
    use_classification: bool = False
    num_atoms: int | None = None
    dueling: bool = False
