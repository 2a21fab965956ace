"""OptimizerConfig (mtrl/config/optim.py:14-43): optax.chain(clip_by_global_norm, adam(eps=1e-5))
is executed by the engine's optimizer kernels (mtrl_amd/csrc/optim.hip)."""

from dataclasses import dataclass

from .utils import Optimizer


@dataclass(frozen=True, kw_only=True)
class OptimizerConfig:
    lr: float = 3e-4
    optimizer: Optimizer = Optimizer.Adam
    max_grad_norm: float | None = None
    eps: float | None = None
    weight_decay: float | None = None

    @property
    def requires_split_task_losses(self) -> bool:
        return False

    @property
    def adam_eps(self) -> float:  # config/optim.py:29-32
        return self.eps if self.eps is not None else 1e-5
