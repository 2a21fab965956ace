"""mtrl/config/networks.py:6-31."""

from dataclasses import dataclass

from .nn import ImpalaEncoderConfig, NeuralNetworkConfig, TaskEmbeddingConfig, VanillaNetworkConfig


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


@dataclass(frozen=True)
class ImpalaDQNConfig:  # mtrl/config/networks.py:37-42
    impala_config: ImpalaEncoderConfig = ImpalaEncoderConfig()
    q_function_config: QValueFunctionConfig = QValueFunctionConfig(use_classification=True, num_atoms=101)
    task_embed_config: TaskEmbeddingConfig = TaskEmbeddingConfig()
    use_layer_norm: bool = True
