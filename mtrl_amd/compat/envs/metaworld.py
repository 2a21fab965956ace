"""MetaworldConfig (mtrl/envs/metaworld.py:16-178).

Spaces are reproduced exactly (obs = 39 features + one-hot of T tasks, actions in
[-1, 1]^4).  Env stepping stays on the host (north star) and needs gymnasium +
metaworld, which this image does not ship: ``spawn``/``evaluate`` raise a clear
ImportError without them.
"""

from dataclasses import dataclass

import numpy as np

from .base import EnvConfig
from .spaces import Box

_NUM_TASKS = {"MT10": 10, "MT25": 25, "MT50": 50, "MT1": 1}


@dataclass(frozen=True)
class MetaworldConfig(EnvConfig):
    reward_func_version: str = "v2"
    num_eval_episodes: int = 50
    num_goals: int = 50
    reward_normalization_method: str | None = None
    task_name: str | None = None

    @property
    def num_tasks(self) -> int:
        return _NUM_TASKS.get(self.env_id, 1)

    @property
    def action_space(self):
        return Box(np.full(4, -1.0, np.float32), np.full(4, 1.0, np.float32), dtype=np.float32)

    @property
    def observation_space(self):
        hand_lo, hand_hi = np.array([-0.525, 0.348, -0.0525]), np.array([0.525, 1.025, 0.7])
        goal_lo = np.array([-0.1, 0.85, 0.0]) + np.array([0, -0.083, 0.2499])
        goal_hi = np.array([0.1, 0.9 + 1e-7, 0.0]) + np.array([0, -0.083, 0.2501])
        obj = np.full(14, np.inf)
        lo = np.hstack((hand_lo, -1.0, -obj, hand_lo, -1.0, -obj, goal_lo))
        hi = np.hstack((hand_hi, 1.0, obj, hand_hi, 1.0, obj, goal_hi))
        if self.use_one_hot and self.env_id != "MT1":
            lo = np.concatenate([lo, np.zeros(self.num_tasks)])
            hi = np.concatenate([hi, np.ones(self.num_tasks)])
        return Box(lo, hi, dtype=np.float64)

    def spawn(self, seed: int = 1):  # pragma: no cover - needs metaworld
        try:
            import gymnasium as gym
            import metaworld  # noqa: F401
        except ImportError as e:
            raise ImportError("MetaworldConfig.spawn needs gymnasium + metaworld (not in this image)") from e
        return gym.make_vec(
            f"Meta-World/{self.env_id}", seed=seed, use_one_hot=self.use_one_hot,
            terminate_on_success=self.terminate_on_success, max_episode_steps=self.max_episode_steps,
            vector_strategy="async", reward_function_version=self.reward_func_version,
            num_goals=self.num_goals, reward_normalization_method=self.reward_normalization_method,
        )

    def evaluate(self, envs, agent):  # pragma: no cover - needs metaworld
        from metaworld.evaluation import evaluation

        return evaluation(agent, envs, num_episodes=self.num_eval_episodes)[:3]
