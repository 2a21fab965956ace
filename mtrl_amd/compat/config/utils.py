"""Enums of mtrl/config/utils.py:14-59 (names only; the HIP engine implements the
ReLU / he_uniform / zeros / Adam members the MTSAC path uses)."""

import enum


class Initializer(enum.Enum):
    ZEROS = "zeros"
    HE_NORMAL = "he_normal"
    HE_UNIFORM = "he_uniform"
    XAVIER_NORMAL = "xavier_normal"
    XAVIER_UNIFORM = "xavier_uniform"
    CONSTANT = "constant"
    UNIFORM = "uniform"


class Activation(enum.Enum):
    ReLU = "relu"
    Tanh = "tanh"
    LeakyReLU = "leaky_relu"
    PReLU = "prelu"
    ReLU6 = "relu6"
    SiLU = "silu"
    GELU = "gelu"
    GLU = "glu"


class Optimizer(enum.Enum):
    Adam = "adam"
    AdamW = "adamw"
    RMSProp = "rmsprop"
    SGD = "sgd"


class Metrics(enum.Enum):
    NONE = 0
    DORMANT_NEURONS = 1
    SRANK = 2
    ALL = 3

    def is_enabled(self, other: "Metrics") -> bool:
        return self.value & other.value == other.value
