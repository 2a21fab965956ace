"""Host mirror of the DrQ-eps update (experiments/atari.py, mtrl/rl/algorithms/drqeps.py) on the
HIP engine of include/drq.h.  The product path: there is no CPU fallback (the library must load).

``DrQEngine.update(batch, aug)`` runs DrQ.update (drqeps.py:337-343): augmentation of obs and
next_obs with the given draws, then _update_inner (drqeps.py:268-335) -- C51 target from the online
greedy action and the target network at s', cross entropy at the taken action, optax.adamw, Polyak.
Parameters are flat float32 vectors in flax ravel order (oracle/drq.py:param_spec)."""

from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib as L


@dataclass(frozen=True)
class DrQSettings:
    num_tasks: int = 26
    n_actions: int = 18
    n_atoms: int = 51
    in_ch: int = 4
    hw: int = 84
    scale: int = 1
    embed_dim: int = 32
    n_hidden: int = 512
    batch: int = 256
    nstep: int = 3
    gamma: float = 0.99
    v_min: float = -10.0
    v_max: float = 10.0
    tau: float = 0.005
    lr: float = 1e-4
    b1: float = 0.9
    b2: float = 0.999
    eps: float = 1.5e-4
    weight_decay: float = 0.05
    ln_eps: float = 1e-6
    capacity: int = 0  # device replay slots per task (0: none)
    normalize_rewards: int = 0
    buffer_kind: int = 0  # 0: MemoryEfficientAtariMultiTaskReplayBuffer, 1: AtariMultiTaskReplayBuffer


def _ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def _drq_check(rc: int) -> int:
    if rc < 0:
        msg = L.load().drq_last_error()
        raise L.MTSACError(f"libmtsac drq error {rc}: {msg.decode() if msg else ''}")
    return rc


def unbalanced_rows(rng: np.random.Generator, num_tasks: int, batch: int, pos: int, full: bool, capacity: int,
                    nstep: int, kind: int = 0):
    """The host draws of sample_unbalanced (buffers.py:1235-1257) with _sample_indices
    (buffers.py:1082-1100): Dirichlet(1, ..., 1) task weights, floor(w * batch) rows per task plus
    the remainder to the largest weights, then each task's slots from the same Generator.  The
    guard window's valid[k] is computed arithmetically (no list of the capacity).  kind 1
    (AtariMultiTaskReplayBuffer.sample_unbalanced, buffers.py:896-947): slots in [0, pos or capacity).
    Returns (slots int64 [batch], task ids int32 [batch]) in the reference's row order."""
    weights = rng.dirichlet([1] * num_tasks)
    sizes = np.floor(weights * batch).astype(np.int32)
    rem = batch - sizes.sum()
    if rem > 0:
        sizes[np.argsort(-weights)[:rem]] += 1
    slots = np.empty(batch, np.int64)
    tasks = np.empty(batch, np.int32)
    guard = nstep + 6
    c = 0
    for i in range(num_tasks):
        n = int(sizes[i])
        if n == 0:
            continue
        if kind == 1:
            idx = rng.integers(0, capacity if full else pos, size=(n,))
        elif not full:
            idx = rng.integers(0, max(pos - nstep, 1), size=(n,))
        else:
            k = rng.integers(0, capacity - guard, size=(n,))
            idx = np.where(k < pos, k, k + guard) if pos + guard <= capacity else k + (pos + guard - capacity)
        slots[c:c + n] = idx
        tasks[c:c + n] = i
        c += n
    return slots, tasks


class DrQEngine:
    def __init__(self, s: DrQSettings = DrQSettings(), device: int = 0):
        self.lib = L.load()
        self.s = s
        c = L.DrqConfig(**{k: getattr(s, k) for k, _ in L.DrqConfig._fields_})
        h = ctypes.c_void_p()
        _drq_check(self.lib.drq_create(ctypes.byref(c), device, ctypes.byref(h)))
        self.h = h
        self.n = int(self.lib.drq_num_params(h))
        self._keep = []
        # the buffer's Generator: drawn on the device by sample(), on the host by sample_unbalanced();
        # one stream either way (the side that draws next first takes the other's state)
        self._rng = np.random.Generator(np.random.PCG64())
        self._rng_on_device = True

    def close(self):
        if self.h:
            self.lib.drq_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def set_params(self, which: int, flat):
        a = np.ascontiguousarray(flat, np.float32)
        assert a.size == self.n, (a.size, self.n)
        _drq_check(self.lib.drq_set_params(self.h, which, _ptr(a), self.n))

    def get_params(self, which: int = L.DRQ_PARAMS) -> np.ndarray:
        out = np.empty(self.n, np.float32)
        _drq_check(self.lib.drq_get_params(self.h, which, _ptr(out), self.n))
        return out

    def set_step(self, count: int):
        _drq_check(self.lib.drq_set_step(self.h, int(count)))

    def get_step(self) -> int:
        c = ctypes.c_int()
        _drq_check(self.lib.drq_get_step(self.h, ctypes.byref(c)))
        return c.value

    @staticmethod
    def _batch_arrays(batch, aug):
        obs, act, nobs, done, rew, task = batch
        co, no, cn, nn = aug
        return [np.ascontiguousarray(obs, np.uint8), np.ascontiguousarray(act, np.int32),
                np.ascontiguousarray(nobs, np.uint8), np.ascontiguousarray(done, np.float32),
                np.ascontiguousarray(rew, np.float32), np.ascontiguousarray(task, np.int32),
                np.ascontiguousarray(co, np.int32), np.ascontiguousarray(no, np.float32),
                np.ascontiguousarray(cn, np.int32), np.ascontiguousarray(nn, np.float32)]

    def task_gradient(self, batch, aug, slot: int, num_slots: int) -> None:
        """compute_weights' per_task_loss gradient (drqeps.py:385-410, 454-460) of one task group
        (this engine's `batch` rows), kept on the device as row `slot` in flax ravel order."""
        arrs = self._batch_arrays(batch, aug)
        b = L.DrqBatch(*[a.ctypes.data for a in arrs])
        _drq_check(self.lib.drq_task_gradient(self.h, ctypes.byref(b), int(slot), int(num_slots)))
        self._keep = arrs
        self.synchronize()

    def get_task_gradient(self, slot: int) -> np.ndarray:
        out = np.empty(self.n, np.float32)
        _drq_check(self.lib.drq_get_task_gradient(self.h, int(slot), _ptr(out), self.n))
        return out

    def project_task_gradients(self, num_slots: int, proj_dim: int = 10_000, chunk: int = 500_000,
                               seed: int = 42) -> np.ndarray:
        """project_grad (drqeps.py:428-448) of the stored task gradients -> [num_slots][proj_dim]."""
        out = np.empty((num_slots, proj_dim), np.float32)
        _drq_check(self.lib.drq_project_task_gradients(self.h, int(num_slots), int(proj_dim), int(chunk), int(seed),
                                                       _ptr(out)))
        return out

    def update(self, batch, aug) -> None:
        """batch = (obs u8 [B][C][H][W], actions, next_obs u8, dones, rewards, task_ids);
        aug = (crop_obs int [B][2], noise_obs [B], crop_next, noise_next)."""
        obs, act, nobs, done, rew, task = batch
        co, no, cn, nn = aug
        arrs = [np.ascontiguousarray(obs, np.uint8), np.ascontiguousarray(act, np.int32),
                np.ascontiguousarray(nobs, np.uint8), np.ascontiguousarray(done, np.float32),
                np.ascontiguousarray(rew, np.float32), np.ascontiguousarray(task, np.int32),
                np.ascontiguousarray(co, np.int32), np.ascontiguousarray(no, np.float32),
                np.ascontiguousarray(cn, np.int32), np.ascontiguousarray(nn, np.float32)]
        b = L.DrqBatch(*[a.ctypes.data for a in arrs])
        _drq_check(self.lib.drq_update(self.h, ctypes.byref(b)))
        self._keep = arrs  # alive until the copies on the engine's stream have run
        self.synchronize()

    def q_values(self, obs, task_ids, crop, noise) -> np.ndarray:
        """Expected Q [n][A] of the online network on augmented observations (n <= batch)."""
        o = np.ascontiguousarray(obs, np.uint8)
        t = np.ascontiguousarray(task_ids, np.int32)
        c = np.ascontiguousarray(crop, np.int32)
        z = np.ascontiguousarray(noise, np.float32)
        n = o.shape[0]
        q = np.empty((n, self.s.n_actions), np.float32)
        _drq_check(self.lib.drq_q_values(self.h, _ptr(o), _ptr(t), _ptr(c), _ptr(z), n, _ptr(q)))
        return q

    # ---- device replay buffer (MemoryEfficientAtariMultiTaskReplayBuffer)
    def buffer_add(self, obs, next_obs, action, reward, truncate, done):
        arrs = [np.ascontiguousarray(obs, np.uint8), np.ascontiguousarray(next_obs, np.uint8),
                np.ascontiguousarray(action, np.int32).reshape(-1), np.ascontiguousarray(reward, np.float32).reshape(-1),
                np.ascontiguousarray(truncate, np.float32).reshape(-1), np.ascontiguousarray(done, np.float32).reshape(-1)]
        _drq_check(self.lib.drq_buffer_add(self.h, *[_ptr(a) for a in arrs]))

    def buffer_state(self):
        pos, full = ctypes.c_int64(), ctypes.c_int32()
        _drq_check(self.lib.drq_buffer_state(self.h, ctypes.byref(pos), ctypes.byref(full)))
        return int(pos.value), bool(full.value)

    def seed_rng(self, seed: int):
        """numpy.random.default_rng(seed)'s PCG64 state (buffers.py:981)."""
        st = np.random.default_rng(seed).bit_generator.state
        self.set_rng_state(st)

    def set_rng_state(self, st: dict):
        s_, inc = st["state"]["state"], st["state"]["inc"]
        m = (1 << 64) - 1
        _drq_check(self.lib.drq_rng_set(self.h, s_ >> 64, s_ & m, inc >> 64, inc & m, int(st["has_uint32"]),
                                        int(st["uinteger"])))
        self._rng.bit_generator.state = st
        self._rng_on_device = False

    def get_rng_state(self) -> dict:
        if not self._rng_on_device:
            return self._rng.bit_generator.state
        o = np.zeros(6, np.uint64)
        _drq_check(self.lib.drq_rng_get(self.h, _ptr(o)))
        v = [int(x) for x in o]
        return {"bit_generator": "PCG64", "state": {"state": (v[0] << 64) | v[1], "inc": (v[2] << 64) | v[3]},
                "has_uint32": v[4], "uinteger": v[5]}

    def _host_rng(self) -> np.random.Generator:
        if self._rng_on_device:
            self._rng.bit_generator.state = self.get_rng_state()
            self._rng_on_device = False
        return self._rng

    def _push_rng(self):
        self.set_rng_state(self._rng.bit_generator.state)

    def seed_augment(self, seed: int):
        """seed of the device augmentation draws of sample_update / sample_unbalanced_update."""
        _drq_check(self.lib.drq_seed_augment(self.h, int(seed) & ((1 << 64) - 1)))

    def sample(self):
        """sample(batch) (buffers.py:1188-1227), indices drawn on the device."""
        _drq_check(self.lib.drq_sample(self.h))
        self._rng_on_device = True

    def sample_update(self, steps: int = 1):
        _drq_check(self.lib.drq_sample_update(self.h, int(steps)))
        self._rng_on_device = True

    def _rows(self, steps):
        pos, full = self.buffer_state()
        if pos == 0 and not full:
            raise L.MTSACError("libmtsac drq error -22: empty buffer")
        rng = self._host_rng()
        s = self.s
        rows = [unbalanced_rows(rng, s.num_tasks, s.batch, pos, full, s.capacity, s.nstep, s.buffer_kind)
                for _ in range(steps)]
        slots = np.ascontiguousarray(np.concatenate([r[0] for r in rows]))
        tasks = np.ascontiguousarray(np.concatenate([r[1] for r in rows]))
        self._push_rng()
        return slots, tasks

    def gather_rows(self, slots, tasks):
        """Rows (slot, task) of the device buffer in batches of this engine's size -> host arrays
        (obs, actions, next_obs, truncations, dones, rewards, task ids), any number of rows."""
        slots = np.asarray(slots, np.int64)
        tasks = np.asarray(tasks, np.int32)
        R, B = slots.size, self.s.batch
        parts = []
        for r0 in range(0, R, B):
            k = min(B, R - r0)
            s_ = np.zeros(B, np.int64)
            t_ = np.zeros(B, np.int32)
            s_[:k], t_[:k] = slots[r0:r0 + k], tasks[r0:r0 + k]
            _drq_check(self.lib.drq_sample_rows(self.h, _ptr(s_), _ptr(t_)))
            parts.append([a[:k] for a in self.read_batch()])
        return tuple(np.concatenate([p[i] for p in parts]) for i in range(7))

    def sample_balanced_host(self, batch_size: int):
        """sample(batch_size) (buffers.py:1188-1227) for any multiple of num_tasks (compute_weights'
        metrics batch, base.py:280): the indices from the buffer's Generator on the host (same
        stream as the device draws), the rows gathered on the device."""
        s = self.s
        T = s.num_tasks
        if batch_size % T:
            raise ValueError("batch_size must be a multiple of num_tasks")
        n = batch_size // T
        pos, full = self.buffer_state()
        rng = self._host_rng()
        guard = s.nstep + 6
        if s.buffer_kind == 1:
            idx = rng.integers(0, max(pos if not full else s.capacity, n), size=(n,))
        elif not full:
            idx = rng.integers(0, max(pos - s.nstep, 1), size=(n,))
        else:
            k = rng.integers(0, s.capacity - guard, size=(n,))
            idx = np.where(k < pos, k, k + guard) if pos + guard <= s.capacity else k + (pos + guard - s.capacity)
        self._push_rng()
        slots = np.repeat(idx, T)  # row i * T + t
        tasks = np.tile(np.arange(T, dtype=np.int32), n)
        o, a, no, tr, d, r, _ = self.gather_rows(slots, tasks)
        return o, a, no, tr, d, r, np.repeat(np.arange(T, dtype=np.int32), n)  # task ids as the reference lists them

    def sample_unbalanced(self):
        """sample_unbalanced(batch) (buffers.py:1230-1279): rows drawn on the host, gathered on the device."""
        slots, tasks = self._rows(1)
        _drq_check(self.lib.drq_sample_rows(self.h, _ptr(slots), _ptr(tasks)))

    def sample_unbalanced_update(self, steps: int = 1):
        """`steps` x (sample_unbalanced + update): OffPolicyAlgorithm.train's inner loop (base.py:213-221)."""
        if steps <= 0:
            return
        slots, tasks = self._rows(steps)
        _drq_check(self.lib.drq_sample_rows_update(self.h, _ptr(slots), _ptr(tasks), int(steps)))

    def read_batch(self):
        B, C, H = self.s.batch, self.s.in_ch, self.s.hw
        obs = np.empty((B, C, H, H), np.uint8)
        nobs = np.empty_like(obs)
        act = np.empty(B, np.int32)
        rew, done, trunc = (np.empty(B, np.float32) for _ in range(3))
        task = np.empty(B, np.int32)
        _drq_check(self.lib.drq_read_batch(self.h, _ptr(obs), _ptr(nobs), _ptr(act), _ptr(rew), _ptr(done),
                                           _ptr(trunc), _ptr(task)))
        return obs, act, nobs, trunc, done, rew, task

    def update_resident(self, steps: int):
        _drq_check(self.lib.drq_update_resident(self.h, int(steps)))

    def logs(self) -> dict:
        out = np.zeros(L.DRQ_NUM_LOGS, np.float32)
        _drq_check(self.lib.drq_get_logs(self.h, _ptr(out)))
        return dict(zip(L.DRQ_LOG_KEYS, (float(v) for v in out)))

    def set_timing(self, on: bool):
        _drq_check(self.lib.drq_set_timing(self.h, int(on)))

    def timing(self):
        """(ms, launches, flops) of the conv-forward launches since set_timing(True)."""
        ms, n, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        _drq_check(self.lib.drq_timing(self.h, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl)))
        return ms.value, n.value, fl.value

    def synchronize(self):
        _drq_check(self.lib.drq_synchronize(self.h))
