"""ORACLE (test infrastructure only) -- restatement of ``MultiTaskReplayBuffer``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module.

Follows ``mtrl/rl/buffers.py``:
* ``__init__`` / ``reset``: ``buffers.py:235-306`` (capacity = total // T,
  zero-filled float32 arrays ``(cap, T, dim)``, ``pos = 0``, ``full = False``,
  ``default_rng(seed)``)
* ``_advance_position``: ``buffers.py:337-343`` (same logic as the single-task
  ``buffers.py:83-93`` the reference test pins, ``tests/test_rl_buffers.py:21-62``)
* ``add``: ``buffers.py:426-474`` (one slot for all T tasks; min/max reward
  tracking when ``normalize_rewards``)
* ``sample(int)``: ``buffers.py:494-549`` int branch ``520-549``: one shared
  index vector of length ``B // T``; rows come out ``row = i*T + t``.
* ``checkpoint`` / ``load_checkpoint``: ``buffers.py:308-335``.
* return normalisation (``returns_normalization=True``): ``_compute_discounted_returns``,
  ``_update_return_stats``, ``_normalize_rewards_by_return`` (``buffers.py:347-422``), called from
  ``add`` (``:464-472``) and ``sample`` (``:531-533``, before the min-max branch).

The index stream is drawn through :mod:`oracle.pcg64` (pinned bit-exact against
``numpy.random.default_rng`` by ``tests/test_oracle_pcg64.py``).
"""

from __future__ import annotations

import numpy as np

from .pcg64 import PCG64State


class MultiTaskReplayBufferOracle:
    def __init__(self, total_capacity: int, num_tasks: int, obs_dim: int, action_dim: int,
                 seed=None, normalize_rewards: bool = False, reward_norm_eps: float = 1e-8,
                 returns_normalization: bool = False, discount: float = 0.99, v_max: float = 10.0):
        assert total_capacity % num_tasks == 0, "Total capacity must be divisible by the number of tasks."
        self.capacity = total_capacity // num_tasks
        self.num_tasks = num_tasks
        self._obs_shape = obs_dim
        self._action_shape = action_dim
        self.rng = PCG64State.from_seed(seed)
        self.full = False
        self.normalize_rewards = normalize_rewards
        self.reward_norm_eps = reward_norm_eps
        self._min_rewards = np.full(num_tasks, np.inf, dtype=np.float64)
        self._max_rewards = np.full(num_tasks, -np.inf, dtype=np.float64)
        self.use_return_normalization = returns_normalization
        self.discount, self.v_max = discount, v_max
        self.effective_horizon = 1.0 / (1.0 - discount)
        self._returns_min = np.full(num_tasks, np.inf, dtype=np.float64)
        self._returns_max = np.full(num_tasks, -np.inf, dtype=np.float64)
        self._episode_rewards = [[] for _ in range(num_tasks)]
        self.reset()

    def reset(self) -> None:
        c, T = self.capacity, self.num_tasks
        self.obs = np.zeros((c, T, self._obs_shape), dtype=np.float32)
        self.actions = np.zeros((c, T, self._action_shape), dtype=np.float32)
        self.rewards = np.zeros((c, T, 1), dtype=np.float32)
        self.next_obs = np.zeros((c, T, self._obs_shape), dtype=np.float32)
        self.dones = np.zeros((c, T, 1), dtype=np.float32)
        self.pos = 0

    def _advance_position(self, steps: int) -> None:
        if steps <= 0:
            return
        new_pos = self.pos + steps
        if new_pos >= self.capacity:
            self.full = True
        self.pos = new_pos % self.capacity

    def _compute_discounted_returns(self, rewards, truncated):  # buffers.py:347-366
        values = np.zeros(len(rewards), dtype=np.float64)
        bootstrap = float(rewards.mean()) * self.effective_horizon if truncated else 0.0
        for i in reversed(range(len(rewards))):
            values[i] = rewards[i] + self.discount * bootstrap
            bootstrap = values[i]
        return float(values.min()), float(values.max())

    def _update_return_stats(self, rewards, terminal, truncated):  # buffers.py:368-390
        for t in range(self.num_tasks):
            self._episode_rewards[t].append(float(rewards[t]))
            if bool(terminal[t]) or bool(truncated[t]):
                lo, hi = self._compute_discounted_returns(np.array(self._episode_rewards[t], dtype=np.float64),
                                                          truncated=bool(truncated[t]))
                self._returns_min[t] = min(self._returns_min[t], lo)
                self._returns_max[t] = max(self._returns_max[t], hi)
                self._episode_rewards[t] = []

    def return_denominator(self):  # buffers.py:406-418
        no_data = np.isinf(self._returns_min) | np.isinf(self._returns_max)
        den = np.where(self._returns_max >= np.abs(self._returns_min), self._returns_max, np.abs(self._returns_min))
        den = den / self.v_max
        return np.where(no_data | (den < self.reward_norm_eps), 1.0, den)

    def add(self, obs, next_obs, action, reward, done, terminal=None, truncated=None) -> None:
        obs, next_obs, action = np.asarray(obs), np.asarray(next_obs), np.asarray(action)
        reward, done = np.asarray(reward), np.asarray(done)
        assert obs.ndim == 2 and action.ndim == 2 and reward.ndim <= 2 and done.ndim <= 2
        assert obs.shape[0] == action.shape[0] == reward.shape[0] == done.shape[0] == self.num_tasks
        self.obs[self.pos] = obs
        self.actions[self.pos] = action
        self.next_obs[self.pos] = next_obs
        self.dones[self.pos] = done.reshape(-1, 1)
        self.rewards[self.pos] = reward.reshape(-1, 1)
        if self.normalize_rewards:
            self._min_rewards = np.minimum(self._min_rewards, reward.reshape(-1))
            self._max_rewards = np.maximum(self._max_rewards, reward.reshape(-1))
        if self.use_return_normalization:
            term = terminal if terminal is not None else done
            trunc = truncated if truncated is not None else np.zeros_like(done)
            self._update_return_stats(reward.flatten(), np.asarray(term).flatten().astype(bool),
                                      np.asarray(trunc).flatten().astype(bool))
        self._advance_position(1)

    def sample_indices(self, batch_size: int) -> np.ndarray:
        assert batch_size % self.num_tasks == 0
        n = batch_size // self.num_tasks
        high = max(self.pos if not self.full else self.capacity, n)
        return self.rng.integers(high, n)

    def gather(self, idx: np.ndarray):
        n = idx.shape[0]
        rewards = self.rewards[idx]
        if self.use_return_normalization:
            rewards = rewards / self.return_denominator()[np.newaxis, :, np.newaxis]
        elif self.normalize_rewards:
            mn = self._min_rewards[np.newaxis, :, np.newaxis]
            mx = self._max_rewards[np.newaxis, :, np.newaxis]
            rewards = (rewards - mn) / (mx - mn + self.reward_norm_eps)
        batch = (self.obs[idx], self.actions[idx], self.next_obs[idx], self.dones[idx], rewards)
        B = n * self.num_tasks
        return tuple(x.reshape(B, *x.shape[2:]) for x in batch)

    def sample(self, batch_size: int):
        return self.gather(self.sample_indices(batch_size))

    def checkpoint(self) -> dict:
        """buffers.py:308-324.  ``rng_state`` is ``self._rng.__getstate__()`` (:323); under the pinned
        numpy 2.2.4 (2.2.6 here) ``Generator.__getstate__()`` returns ``None`` -- the stream is NOT
        persisted by the reference (tests/test_buffer_checkpoint_cpu.py pins this)."""
        return {
            "data": {
                "obs": self.obs, "actions": self.actions, "rewards": self.rewards,
                "next_obs": self.next_obs, "dones": self.dones, "pos": self.pos, "full": self.full,
                "returns_min": self._returns_min, "returns_max": self._returns_max,
            },
            "rng_state": None,
        }

    def load_checkpoint(self, ckpt: dict) -> None:
        """buffers.py:326-335.  ``self._rng.__setstate__(ckpt["rng_state"])`` (:335) with numpy 2.2's
        ``Generator.__setstate__``: ``None`` leaves the stream where it is (a resumed reference run
        continues from the fresh ``default_rng(seed)`` of ``spawn_replay_buffer``, base.py:148); a
        ``bit_generator.state`` dict (numpy's legacy pickle form) sets it."""
        for key in ["data", "rng_state"]:
            assert key in ckpt
        d = ckpt["data"]
        for key in ["obs", "actions", "rewards", "next_obs", "dones", "pos", "full"]:
            assert key in d
            setattr(self, key, d[key])
        self._returns_min = d.get("returns_min", self._returns_min)
        self._returns_max = d.get("returns_max", self._returns_max)
        if ckpt["rng_state"] is not None:
            self.rng = PCG64State.from_numpy_state(ckpt["rng_state"])
