"""A gymnasium-shaped synthetic multi-task vector env (gymnasium/metaworld are not in
this image).  Observations are 39 features + the one-hot task id, like Meta-World
with use_one_hot (mtrl/envs/metaworld.py:83-98); episodes truncate after
``max_steps`` with ``final_obs`` / ``final_info`` like gymnasium's autoreset."""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from mtrl_amd.compat.envs import MetaworldConfig
from mtrl_amd.compat.envs.spaces import Box


class FakeMTVecEnv:
    def __init__(self, num_tasks: int, max_steps: int = 20, seed: int = 0):
        self.num_envs = num_tasks
        self.T = num_tasks
        self.max_steps = max_steps
        self.rng = np.random.default_rng(seed)
        self.action_space = Box(-1.0, 1.0, shape=(num_tasks, 4), dtype=np.float32, seed=seed)
        self.t = np.zeros(num_tasks, int)
        self.ret = np.zeros(num_tasks)

    def _obs(self):
        o = np.zeros((self.T, 39 + self.T), np.float64)
        o[:, :39] = self.rng.standard_normal((self.T, 39))
        o[np.arange(self.T), 39 + np.arange(self.T)] = 1.0
        return o

    def reset(self, seed=None):
        self.t[:] = 0
        self.ret[:] = 0
        return self._obs(), {}

    def step(self, actions):
        actions = np.asarray(actions)
        assert actions.shape == (self.T, 4)
        self.t += 1
        r = 1.0 - np.abs(actions).mean(axis=1)
        self.ret += r
        obs = self._obs()
        trunc = self.t >= self.max_steps
        term = np.zeros(self.T, bool)
        infos = {}
        if trunc.any():
            infos["final_obs"] = np.array([obs[i].copy() if trunc[i] else None for i in range(self.T)], dtype=object)
            infos["final_info"] = {"episode": {"r": self.ret.copy(), "l": self.t.copy()}}
            obs = obs.copy()
            obs[trunc, :39] = self.rng.standard_normal((int(trunc.sum()), 39))
            self.t[trunc] = 0
            self.ret[trunc] = 0
        return obs, r, term, trunc, infos


@dataclass(frozen=True)
class FakeMetaworldConfig(MetaworldConfig):
    """MetaworldConfig spaces; evaluation = mean return of eval_action on fresh obs."""

    def evaluate(self, envs, agent):
        obs, _ = envs.reset()
        a = agent.eval_action(obs)
        assert a.shape == (envs.num_envs, 4) and np.all(np.abs(a) <= 1.0)
        return 0.0, float(1.0 - np.abs(a).mean()), {f"task{i}": 0.0 for i in range(envs.num_envs)}
