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


@dataclass(frozen=True)
class DrQTrainingConfig(OffPolicyTrainingConfig):  # mtrl/config/rl.py:53-79 (the fields the DrQ path reads)
    warmstart_steps: int = 1_000
    buffer_size: int = 100_000
    batch_size: int = 256
    num_critics: int = 2
    tau: float = 0.005
    eps_start: float = 1.0
    eps_end: float = 0.01
    eps_decay_steps: int = 5_000
    v_min: float = -10.0
    v_max: float = 10.0
    num_tasks: int = 26
    normalize_rewards: bool = True
    nstep: int = 3
    replay_ratio: int = 2
    eval_step_frequency: int = 10_000
