"""Network configs of mtrl/config/nn.py:8-31,63 (only the multi-head MLP path)."""

from dataclasses import dataclass

from .optim import OptimizerConfig
from .utils import Activation, Initializer


@dataclass(frozen=True, kw_only=True)
class NeuralNetworkConfig:
    width: int = 400
    depth: int = 3
    kernel_init: Initializer = Initializer.HE_UNIFORM
    bias_init: Initializer = Initializer.ZEROS
    use_bias: bool = True
    activation: Activation = Activation.ReLU
    optimizer: OptimizerConfig = OptimizerConfig()


@dataclass(frozen=True, kw_only=True)
class VanillaNetworkConfig(NeuralNetworkConfig):
    use_skip_connections: bool = False
    use_layer_norm: bool = False


@dataclass(frozen=True, kw_only=True)
class MultiHeadConfig(NeuralNetworkConfig):
    num_tasks: int


@dataclass(frozen=True, kw_only=True)
class ImpalaEncoderConfig(NeuralNetworkConfig):  # mtrl/config/nn.py:47-52
    use_layer_norm: bool = False
    scale: int = 1
    blocks: int = 2
    stacks: tuple[int, ...] = (8, 16, 16)
    num_critics: int = 1


@dataclass(frozen=True, kw_only=True)
class TaskEmbeddingConfig:  # mtrl/config/nn.py:54-59
    num_tasks: int = 26
    embed_dim: int = 32
