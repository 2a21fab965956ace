"""MultiTaskReplayBuffer (mtrl/rl/buffers.py:221-549) backed by the engine's
device-resident buffer: same add / sample / checkpoint / load_checkpoint API, same
index stream (numpy PCG64 reproduced on the device), same row layout (row = i*T + t)."""

from __future__ import annotations

import numpy as np

from ..types import ReplayBufferSamples


class MultiTaskReplayBuffer:
    def __init__(self, total_capacity: int, num_tasks: int, env_obs_space=None, env_action_space=None,
                 seed: int | None = None, max_steps: int = 500, normalize_rewards: bool = False,
                 reward_norm_eps: float = 1e-8, *, engine=None, **unsupported):
        assert total_capacity % num_tasks == 0, "Total capacity must be divisible by the number of tasks."
        if unsupported.get("returns_normalization") or unsupported.get("reward_filter"):
            raise NotImplementedError("return-based normalization / reward filters are not on the MTSAC path")
        if engine is None:
            raise ValueError("the device buffer lives in an MTSAC engine: use MTSAC.spawn_replay_buffer")
        self.engine = engine
        self.capacity = total_capacity // num_tasks
        self.num_tasks = num_tasks
        self.normalize_rewards = normalize_rewards
        self._min_rewards = np.full(num_tasks, np.inf)
        self._max_rewards = np.full(num_tasks, -np.inf)
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

    def add(self, obs, next_obs, action, reward, done, terminal=None, truncated=None) -> None:
        obs = np.asarray(obs, np.float32)
        assert obs.ndim == 2 and obs.shape[0] == self.num_tasks
        reward = np.asarray(reward, np.float32).reshape(-1)
        self.engine.buffer_add(obs, np.asarray(next_obs, np.float32), np.asarray(action, np.float32), reward,
                               np.asarray(done, np.float32).reshape(-1))
        if self.normalize_rewards:
            self._min_rewards = np.minimum(self._min_rewards, reward)
            self._max_rewards = np.maximum(self._max_rewards, reward)

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
                     # return-normalisation statistics (buffers.py:319-321); return normalisation
                     # is not on the MTSAC path, so they keep their initial values (:281-282)
                     "returns_min": np.full(self.num_tasks, np.inf), "returns_max": np.full(self.num_tasks, -np.inf)},
            "rng_state": self.engine.get_rng_state(),
        }

    def load_checkpoint(self, ckpt: dict) -> None:
        for key in ["data", "rng_state"]:
            assert key in ckpt
        d = ckpt["data"]
        for key in ["obs", "actions", "rewards", "next_obs", "dones", "pos", "full"]:
            assert key in d
        T = self.num_tasks
        for key, init in (("returns_min", np.inf), ("returns_max", -np.inf)):  # buffers.py:333-334
            if key in d and not np.all(np.asarray(d[key]) == init):
                raise NotImplementedError(f"checkpoint carries {key} statistics: return normalisation is not "
                                          "on the MTSAC path")
        self.engine.buffer_write(0, np.asarray(d["obs"]).reshape(-1, d["obs"].shape[-1]),
                                 np.asarray(d["next_obs"]).reshape(-1, d["next_obs"].shape[-1]),
                                 np.asarray(d["actions"]).reshape(-1, d["actions"].shape[-1]),
                                 np.asarray(d["rewards"]).reshape(-1), np.asarray(d["dones"]).reshape(-1))
        self.engine.set_buffer_state(int(d["pos"]), bool(d["full"]))
        self.engine.set_rng_state(ckpt["rng_state"])
        assert T == self.num_tasks
