"""Shared synthetic-input helpers for the tests (SURVEY.md §8d input recipe)."""

from __future__ import annotations

import numpy as np


def synthetic_batch(num_tasks: int, batch: int, obs_feat: int = 39, action_dim: int = 4, seed: int = 0,
                    dtype=np.float64):
    """A batch laid out like ``MultiTaskReplayBuffer.sample``: row = i*T + t,
    obs = [39 N(0,1) features | one-hot(t)], actions U(-1,1), rewards U(0,10),
    dones Bernoulli(1/500) (forced to contain at least one 1 for coverage)."""
    rng = np.random.default_rng(seed)
    T = num_tasks
    t = np.arange(batch) % T
    def obs_block():
        o = np.zeros((batch, obs_feat + T))
        o[:, :obs_feat] = rng.standard_normal((batch, obs_feat))
        o[np.arange(batch), obs_feat + t] = 1.0
        return o
    obs = obs_block()
    nobs = obs_block()
    act = rng.uniform(-1, 1, (batch, action_dim))
    rew = rng.uniform(0, 10, (batch, 1))
    done = (rng.uniform(size=(batch, 1)) < 1 / 500).astype(np.float64)
    done[min(3, batch - 1)] = 1.0
    return tuple(x.astype(dtype) for x in (obs, act, nobs, done, rew))


def synthetic_eps(batch: int, action_dim: int = 4, seed: int = 0, dtype=np.float64):
    rng = np.random.default_rng(seed + 1000)
    return (rng.standard_normal((batch, action_dim)).astype(dtype),
            rng.standard_normal((batch, action_dim)).astype(dtype))
