"""EnvConfig (mtrl/envs/base.py:16-38)."""

import abc
from dataclasses import dataclass


@dataclass(frozen=True)
class EnvConfig(abc.ABC):
    env_id: str
    use_one_hot: bool = True
    max_episode_steps: int = 500
    evaluation_num_episodes: int = 50
    terminate_on_success: bool = False

    @property
    @abc.abstractmethod
    def action_space(self): ...

    @property
    @abc.abstractmethod
    def observation_space(self): ...

    @abc.abstractmethod
    def spawn(self, seed: int = 1): ...

    @abc.abstractmethod
    def evaluate(self, envs, agent) -> tuple[float, float, dict[str, float]]: ...
