"""CPU restatement of MemoryEfficientAtariMultiTaskReplayBuffer -- TEST INFRASTRUCTURE ONLY (the
checker for the device buffer of include/drq.h).  Reference: mtrl/rl/buffers.py:949-1229 (add with
the n-step ring and _get_nstep_info, _sample_indices with the guard window, sample with per-task
min-max reward normalisation).  numpy, same dtypes and operation order as the reference, so the
device path is compared bit for bit (indices from numpy's own Generator).

sample_unbalanced restates buffers.py:1230-1279 (Dirichlet task sizes, per-task gathers).
kind=1 restates AtariMultiTaskReplayBuffer (buffers.py:710-947) instead: its own next_obs array,
indices in [0, max(pos or capacity, n)) with no guard window, and the reward normalisation as one
float64 expression (no in-place float32 rounding in between).

Kept from the reference: the sampled rows are (sample i, task t) in i-major order (obs[idx] of shape
[n][T] flattened), while task_ids = repeat(arange(T), n) lists tasks in task-major order
(buffers.py:1213-1227) -- the two orders differ whenever n > 1."""

from __future__ import annotations

import numpy as np


class AtariBuffer:
    def __init__(self, capacity: int, num_tasks: int, obs_shape, seed: int, nstep: int = 3, gamma: float = 0.99,
                 normalize_rewards: bool = False, reward_norm_eps: float = 1e-8, kind: int = 0):
        self.kind = kind
        self.capacity, self.T, self.nstep, self.gamma = capacity, num_tasks, nstep, gamma
        self.normalize_rewards, self.eps = normalize_rewards, reward_norm_eps
        self.rng = np.random.default_rng(seed)
        T = num_tasks
        self.ns_obs = np.zeros((nstep, T, *obs_shape), np.uint8)
        self.ns_next = np.zeros((nstep, T, *obs_shape), np.uint8)
        self.ns_act = np.zeros((nstep, T), np.int32)
        self.ns_rew = np.zeros((nstep, T), np.float32)
        self.ns_trunc = np.zeros((nstep, T), np.float32)
        self.ns_done = np.zeros((nstep, T), np.float32)
        self.ns_pos = self.ns_count = 0
        self.min_r = np.full(T, np.inf)
        self.max_r = np.full(T, -np.inf)
        self.obs = np.zeros((capacity, T, *obs_shape), np.uint8)
        if kind == 1:
            self.next_obs = np.zeros((capacity, T, *obs_shape), np.uint8)
        self.actions = np.zeros((capacity, T), np.int32)
        self.rewards = np.zeros((capacity, T, 1), np.float32)
        self.dones = np.zeros((capacity, T, 1), np.float32)
        self.truncations = np.zeros((capacity, T, 1), np.float32)
        self.pos, self.full = 0, False

    def _nstep_info(self):  # buffers.py:1048-1080
        n = self.nstep
        oldest = self.ns_pos
        newest = (self.ns_pos - 1) % n
        r = self.ns_rew[newest].copy()
        d = self.ns_done[newest].copy()
        nxt = self.ns_next[newest].copy()
        for k in range(1, n):
            i = (self.ns_pos - 1 - k) % n
            r *= self.gamma
            r *= (1.0 - self.ns_done[i])
            r += self.ns_rew[i]
            mask = self.ns_done[i] > 0.0
            if mask.any():
                np.copyto(nxt, self.ns_next[i], where=mask[:, None, None, None])
                np.copyto(d, self.ns_done[i], where=mask)
        return self.ns_obs[oldest], self.ns_act[oldest], r, self.ns_trunc[oldest], d, nxt

    def add(self, obs, next_obs, action, reward, truncate, done):  # buffers.py:1138-1186
        s = self.ns_pos
        self.ns_obs[s] = obs
        self.ns_next[s] = next_obs
        self.ns_act[s] = action
        self.ns_rew[s] = np.asarray(reward, np.float32).reshape(-1)
        self.ns_trunc[s] = np.asarray(truncate, np.float32).reshape(-1)
        self.ns_done[s] = np.asarray(done, np.float32).reshape(-1)
        self.ns_pos = (s + 1) % self.nstep
        self.ns_count = min(self.ns_count + 1, self.nstep)
        if self.ns_count < self.nstep:
            return
        o, a, r, tr, d, nxt = self._nstep_info()
        p = self.pos
        self.obs[p] = o
        if self.kind == 1:
            self.next_obs[p] = nxt  # buffers.py:836
        else:
            self.obs[(p + self.nstep) % self.capacity] = nxt
        self.actions[p] = a
        self.rewards[p] = r.reshape(-1, 1)
        self.dones[p] = d.reshape(-1, 1)
        self.truncations[p] = tr.reshape(-1, 1)
        if self.normalize_rewards:
            np.minimum(self.min_r, r, out=self.min_r)
            np.maximum(self.max_r, r, out=self.max_r)
        self.pos = (p + 1) % self.capacity
        if self.pos == 0:
            self.full = True

    def sample_indices(self, n):  # buffers.py:1082-1105
        if self.kind == 1:  # buffers.py:863-869
            return self.rng.integers(0, max(self.pos if not self.full else self.capacity, n), size=(n,))
        if not self.full:
            return self.rng.integers(0, max(self.pos - self.nstep, 1), size=(n,))
        guard = self.nstep + 6
        excluded = set(int((self.pos + k) % self.capacity) for k in range(guard))
        valid = np.array([i for i in range(self.capacity) if i not in excluded], dtype=np.int64)
        return valid[self.rng.integers(0, len(valid), size=(n,))]

    def sample(self, batch_size):  # buffers.py:1188-1227
        n = batch_size // self.T
        idx = self.sample_indices(n)
        nidx = (idx + self.nstep) % self.capacity
        rewards = self.rewards[idx].copy()
        if self.kind == 1:  # buffers.py:872-892
            if self.normalize_rewards:
                mn = self.min_r[None, :, None]
                mx = self.max_r[None, :, None]
                rewards = (rewards - mn) / (mx - mn + self.eps)
            task_ids = np.repeat(np.arange(self.T), n)
            f = lambda a: a.reshape(batch_size, *a.shape[2:])
            return (f(self.obs[idx]), f(self.actions[idx]), f(self.next_obs[idx]), f(self.truncations[idx]),
                    f(self.dones[idx]), f(rewards), task_ids)
        if self.normalize_rewards:
            mn = self.min_r[None, :, None]
            mx = self.max_r[None, :, None]
            rewards -= mn
            rewards /= (mx - mn + self.eps)
        task_ids = np.repeat(np.arange(self.T), n)
        f = lambda a: a.reshape(batch_size, *a.shape[2:])
        return (f(self.obs[idx]), f(self.actions[idx]), f(self.obs[nidx]), f(self.truncations[idx]),
                f(self.dones[idx]), f(rewards), task_ids)

    def sample_unbalanced(self, batch_size):  # buffers.py:1230-1279
        weights = self.rng.dirichlet([1] * self.T)
        task_sizes = np.floor(weights * batch_size).astype(np.int32)
        remainder = batch_size - task_sizes.sum()
        if remainder > 0:
            task_sizes[np.argsort(-weights)[:remainder]] += 1
        shp = self.obs.shape[2:]
        out_obs = np.empty((batch_size, *shp), np.uint8)
        out_next = np.empty((batch_size, *shp), np.uint8)
        out_act = np.empty((batch_size,), np.int32)
        out_tr = np.empty((batch_size, 1), np.float32)
        out_d = np.empty((batch_size, 1), np.float32)
        out_r = np.empty((batch_size, 1), np.float32)
        out_t = np.empty((batch_size,), np.int32)
        cursor = 0
        for i in range(self.T):
            n = task_sizes[i]
            if n == 0:
                continue
            sl = slice(cursor, cursor + n)
            if self.kind == 1:  # buffers.py:922-937
                idx = self.rng.integers(0, self.pos if not self.full else self.capacity, size=(n,))
                out_next[sl] = self.next_obs[idx, i]
            else:
                idx = self.sample_indices(n)
                out_next[sl] = self.obs[(idx + self.nstep) % self.capacity, i]
            out_obs[sl] = self.obs[idx, i]
            out_act[sl] = self.actions[idx, i]
            out_tr[sl] = self.truncations[idx, i]
            out_d[sl] = self.dones[idx, i]
            out_t[sl] = i
            r = self.rewards[idx, i]
            if self.normalize_rewards and self.kind == 1:
                r = (r - self.min_r[i]) / (self.max_r[i] - self.min_r[i] + self.eps)
            elif self.normalize_rewards:
                r = r.copy()
                r -= self.min_r[i]
                r /= (self.max_r[i] - self.min_r[i] + self.eps)
            out_r[sl] = r
            cursor += n
        return out_obs, out_act, out_next, out_tr, out_d, out_r, out_t
