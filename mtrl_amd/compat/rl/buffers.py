"""MultiTaskReplayBuffer (mtrl/rl/buffers.py:221-549) backed by the engine's
device-resident buffer: same add / sample / checkpoint / load_checkpoint API, same
index stream (numpy PCG64 reproduced on the device), same row layout (row = i*T + t).

Return normalisation (``returns_normalization=True``, buffers.py:347-422) keeps the reference's
per-episode bookkeeping here on the host (float64, the reward values as passed to ``add``); the
per-task denominator goes to the engine (normalize_rewards mode 2) whenever an episode end moves
it, and the device gather divides the sampled rewards by it."""

from __future__ import annotations

import numpy as np

from ..types import ReplayBufferSamples


class MultiTaskReplayBuffer:
    # checkpoint()'s "rng_state": the reference stores self._rng.__getstate__() (buffers.py:323), which
    # numpy 2.2 (the pinned 2.2.4) returns as None -- its resumed runs restart the index stream from the
    # fresh default_rng(seed).  False (default): write None too, so a resumed run draws the reference's
    # indices bit for bit.  True: write the device stream's bit_generator.state dict (numpy's own
    # Generator.__setstate__ accepts it as well), so a resumed run continues the interrupted stream --
    # the uninterrupted run's indices, NOT the reference's ("Checkpoints").
    persist_rng_state: bool = False

    def __init__(self, total_capacity: int, num_tasks: int, env_obs_space=None, env_action_space=None,
                 seed: int | None = None, max_steps: int = 500, normalize_rewards: bool = False,
                 reward_norm_eps: float = 1e-8, reward_filter=None, sigma=None, alpha=None, delta=None,
                 filter_mode=None, returns_normalization: bool = False, discount: float = 0.99, v_max: float = 10.0,
                 *, engine=None):
        assert total_capacity % num_tasks == 0, "Total capacity must be divisible by the number of tasks."
        # buffers.py:245-249 accepts the filter arguments but never reads them
        del reward_filter, sigma, alpha, delta, filter_mode
        if engine is None:
            raise ValueError("the device buffer lives in an MTSAC engine: use MTSAC.spawn_replay_buffer")
        self.engine = engine
        self.capacity = total_capacity // num_tasks
        self.num_tasks = num_tasks
        self.normalize_rewards = normalize_rewards
        self._min_rewards = np.full(num_tasks, np.inf)
        self._max_rewards = np.full(num_tasks, -np.inf)
        self.reward_norm_eps = reward_norm_eps
        self.use_return_normalization = returns_normalization
        self.discount, self.v_max = discount, v_max
        self.effective_horizon = 1.0 / (1.0 - discount)
        self._returns_min = np.full(num_tasks, np.inf, dtype=np.float64)
        self._returns_max = np.full(num_tasks, -np.inf, dtype=np.float64)
        self._episode_rewards: list[list[float]] = [[] for _ in range(num_tasks)]
        if returns_normalization and engine.config.normalize_rewards != 2:
            raise ValueError("return normalisation needs an engine created with normalize_rewards = 2")
        self.engine.seed_rng(seed)  # np.random.default_rng(seed), buffers.py:260

    # pos / full mirror buffers.py:306,337-343 (kept on the host, size uploaded to HBM)
    @property
    def pos(self) -> int:
        return self.engine.buffer_state()[0]

    @property
    def full(self) -> bool:
        return self.engine.buffer_state()[1]

    def reset(self) -> None:
        self.engine.set_buffer_state(0, False)

    # ---- return normalisation (buffers.py:347-422), host bookkeeping
    def _compute_discounted_returns(self, rewards: np.ndarray, truncated: bool) -> tuple[float, float]:
        values = np.zeros(len(rewards), dtype=np.float64)
        bootstrap = float(rewards.mean()) * self.effective_horizon if truncated else 0.0
        for i in reversed(range(len(rewards))):
            values[i] = rewards[i] + self.discount * bootstrap
            bootstrap = values[i]
        return float(values.min()), float(values.max())

    def _update_return_stats(self, rewards, terminal, truncated) -> bool:
        moved = False
        for t in range(self.num_tasks):
            self._episode_rewards[t].append(float(rewards[t]))
            if bool(terminal[t]) or bool(truncated[t]):
                lo, hi = self._compute_discounted_returns(np.array(self._episode_rewards[t], dtype=np.float64),
                                                          truncated=bool(truncated[t]))
                self._returns_min[t] = min(self._returns_min[t], lo)
                self._returns_max[t] = max(self._returns_max[t], hi)
                self._episode_rewards[t] = []
                moved = True
        return moved

    def return_denominator(self) -> np.ndarray:
        """_normalize_rewards_by_return's per-task denominator (buffers.py:406-418)."""
        no_data = np.isinf(self._returns_min) | np.isinf(self._returns_max)
        den = np.where(self._returns_max >= np.abs(self._returns_min), self._returns_max, np.abs(self._returns_min))
        den = den / self.v_max
        return np.where(no_data | (den < self.reward_norm_eps), 1.0, den)

    def _push_denominator(self) -> None:
        self.engine.set_reward_stats(np.zeros(self.num_tasks), self.return_denominator())

    def add(self, obs, next_obs, action, reward, done, terminal=None, truncated=None) -> None:
        obs = np.asarray(obs, np.float32)
        assert obs.ndim == 2 and obs.shape[0] == self.num_tasks
        raw_reward = np.asarray(reward).reshape(-1)
        reward = np.asarray(reward, np.float32).reshape(-1)
        self.engine.buffer_add(obs, np.asarray(next_obs, np.float32), np.asarray(action, np.float32), reward,
                               np.asarray(done, np.float32).reshape(-1))
        if self.normalize_rewards:
            self._min_rewards = np.minimum(self._min_rewards, reward)
            self._max_rewards = np.maximum(self._max_rewards, reward)
        if self.use_return_normalization:  # buffers.py:465-472
            d = np.asarray(done).reshape(-1)
            term = np.asarray(terminal).reshape(-1) if terminal is not None else d
            trunc = np.asarray(truncated).reshape(-1) if truncated is not None else np.zeros_like(d)
            if self._update_return_stats(raw_reward, term.astype(bool), trunc.astype(bool)):
                self._push_denominator()

    def sample(self, batch_size: int) -> ReplayBufferSamples:
        assert batch_size % self.num_tasks == 0
        assert batch_size // self.num_tasks == self.engine.config.batch_per_task
        _, (obs, act, nobs, done, rew) = self.engine.sample()
        return ReplayBufferSamples(obs, act, nobs, done, rew)

    def checkpoint(self) -> dict:
        obs, nobs, act, rew, done = self.engine.buffer_read(0, self.capacity)
        pos, full = self.engine.buffer_state()
        return {
            "data": {"obs": obs, "actions": act, "rewards": rew[..., None], "next_obs": nobs,
                     "dones": done[..., None], "pos": pos, "full": full,
                     "returns_min": self._returns_min.copy(), "returns_max": self._returns_max.copy()},
            "rng_state": self.engine.get_rng_state() if self.persist_rng_state else None,
        }

    def load_checkpoint(self, ckpt: dict) -> None:
        for key in ["data", "rng_state"]:
            assert key in ckpt
        d = ckpt["data"]
        for key in ["obs", "actions", "rewards", "next_obs", "dones", "pos", "full"]:
            assert key in d
        T = self.num_tasks
        # buffers.py:333-334 (backwards-compatible: absent keys keep the current statistics)
        self._returns_min = np.asarray(d.get("returns_min", self._returns_min), np.float64).copy()
        self._returns_max = np.asarray(d.get("returns_max", self._returns_max), np.float64).copy()
        if self.use_return_normalization:
            self._push_denominator()
        self.engine.buffer_write(0, np.asarray(d["obs"]).reshape(-1, d["obs"].shape[-1]),
                                 np.asarray(d["next_obs"]).reshape(-1, d["next_obs"].shape[-1]),
                                 np.asarray(d["actions"]).reshape(-1, d["actions"].shape[-1]),
                                 np.asarray(d["rewards"]).reshape(-1), np.asarray(d["dones"]).reshape(-1))
        self.engine.set_buffer_state(int(d["pos"]), bool(d["full"]))
        # buffers.py:335, numpy 2.2 Generator.__setstate__: None leaves the stream (seeded by __init__
        # like the reference's fresh default_rng(seed)); a bit_generator.state dict sets it
        if ckpt["rng_state"] is not None:
            self.engine.set_rng_state(ckpt["rng_state"])
        assert T == self.num_tasks
