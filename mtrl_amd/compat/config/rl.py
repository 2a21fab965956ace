"""mtrl/config/rl.py:16-50 (AlgorithmConfig, TrainingConfig, OffPolicyTrainingConfig)."""

from dataclasses import dataclass

from .utils import Metrics


@dataclass(frozen=True)
class AlgorithmConfig:
    num_tasks: int
    gamma: float = 0.99
    weights_critic_loss: bool = False
    weights_actor_loss: bool = False
    weights_qf_vals: bool = False
    clip: bool = False


@dataclass(frozen=True, kw_only=True)
class TrainingConfig:
    total_steps: int
    evaluation_frequency: int = 200_000 // 500
    compute_network_metrics: Metrics = Metrics.ALL
    reward_filter: str | None = None
    reward_filter_sigma: float | None = None
    reward_filter_alpha: float | None = None
    reward_filter_delta: float | None = None
    reward_filter_mode: str | None = None
    sampler_type: str | None = None
    update_weights_every: int = 500
    weights_critic_loss: bool = False
    weights_actor_loss: bool = False
    weights_qf_vals: bool = False
    state_coverage: bool = False
    normalize_rewards: bool = False
    returns_normalization: bool = False


@dataclass(frozen=True)
class OffPolicyTrainingConfig(TrainingConfig):
    warmstart_steps: int = int(4e3)
    buffer_size: int = int(1e6)
    batch_size: int = 1280
