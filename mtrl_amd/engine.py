"""Python handle of one HIP MTSAC engine (``libmtsac.so``, include/mtsac.h).

Thin, allocation-free wrapper: it converts arrays to contiguous fp32 host
buffers (numpy) or passes device pointers through (torch CUDA tensors), calls the
C-ABI, and turns negative return codes into :class:`MTSACError`.
"""

from __future__ import annotations

import ctypes
from typing import Any

import numpy as np

from . import _lib
from ._lib import LOG_KEYS, Batch, Config, MTSACError, check


def _ptr(x) -> tuple[int, Any]:
    """(address, keep-alive) of a host numpy array or a torch tensor (host or device)."""
    if x is None:
        return 0, None
    if hasattr(x, "data_ptr") and hasattr(x, "is_contiguous"):
        import torch

        t = x
        if t.dtype != torch.float32 or not t.is_contiguous():
            t = t.to(torch.float32).contiguous()
        return t.data_ptr(), t
    a = np.ascontiguousarray(x, dtype=np.float32)
    return a.ctypes.data, a


def default_config(num_tasks: int) -> Config:
    c = Config()
    _lib.load().mtsac_default_config(ctypes.byref(c), num_tasks)
    return c


def make_config(**kw) -> Config:
    """Config with the C defaults (mtsac_default_config) overridden by ``kw``."""
    c = default_config(int(kw["num_tasks"]))
    for k, v in kw.items():
        if k == "actor_max_grad_norm" or k == "critic_max_grad_norm" or k == "alpha_max_grad_norm":
            v = -1.0 if v is None else v  # None: no clip_by_global_norm in the chain
        setattr(c, k, v)
    return c


class MTSACEngine:
    """One engine per GPU: device-resident replay buffer + MTSAC update."""

    def __init__(self, config: Config, device: int = 0):
        self.lib = _lib.load()
        self.config = config
        self.device = device
        h = ctypes.c_void_p()
        check(self.lib.mtsac_create(ctypes.byref(config), device, ctypes.byref(h)))
        self._h = h
        c = config
        self.T_l = c.task_count
        self.B = c.batch_per_task * c.task_count
        self.obs_dim = c.obs_dim
        self.action_dim = c.action_dim

    # ------------------------------------------------------------------ lifecycle
    def close(self) -> None:
        if getattr(self, "_h", None):
            self.lib.mtsac_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ parameters
    def param_count(self, which: int) -> int:
        return check(self.lib.mtsac_param_count(self._h, which))

    def set_params(self, which: int, values) -> None:
        n = self.param_count(which)
        p, keep = _ptr(np.asarray(values, dtype=np.float32).reshape(-1))
        check(self.lib.mtsac_set_params(self._h, which, p, n))

    def get_params(self, which: int) -> np.ndarray:
        n = self.param_count(which)
        out = np.empty(n, dtype=np.float32)
        check(self.lib.mtsac_get_params(self._h, which, out.ctypes.data, n))
        return out

    def set_adam_count(self, which: int, count: int) -> None:
        check(self.lib.mtsac_set_adam_count(self._h, which, count))

    def get_adam_count(self, which: int) -> int:
        c = ctypes.c_int32()
        check(self.lib.mtsac_get_adam_count(self._h, which, ctypes.byref(c)))
        return c.value

    # ------------------------------------------------------------------ replay buffer
    def buffer_add(self, obs, next_obs, actions, rewards, dones) -> None:
        """Non-blocking add.  Device (torch) tensors are read in the order of torch's current
        stream, which then waits for the read (mtsac_buffer_add_stream): they may be reused or
        freed as soon as this returns."""
        args = [_ptr(x) for x in (obs, next_obs, actions, rewards, dones)]
        stream = None
        if getattr(obs, "is_cuda", False):
            import torch

            stream = torch.cuda.current_stream(obs.device).cuda_stream
        check(self.lib.mtsac_buffer_add_stream(self._h, *[a[0] for a in args], stream))

    def buffer_write(self, slot_begin: int, obs, next_obs, actions, rewards, dones) -> None:
        n = int(np.asarray(rewards).size) // self.T_l  # slots (rows are slot-major, T_l per slot)
        args = [_ptr(x) for x in (obs, next_obs, actions, rewards, dones)]
        check(self.lib.mtsac_buffer_write(self._h, slot_begin, n, *[a[0] for a in args]))

    def buffer_read(self, slot_begin: int, n_slots: int):
        T, D, A = self.T_l, self.obs_dim, self.action_dim
        obs = np.empty((n_slots, T, D), np.float32)
        nobs = np.empty((n_slots, T, D), np.float32)
        act = np.empty((n_slots, T, A), np.float32)
        rew = np.empty((n_slots, T), np.float32)
        done = np.empty((n_slots, T), np.float32)
        check(self.lib.mtsac_buffer_read(self._h, slot_begin, n_slots, obs.ctypes.data, nobs.ctypes.data,
                                         act.ctypes.data, rew.ctypes.data, done.ctypes.data))
        return obs, nobs, act, rew, done

    def buffer_fill_synthetic(self, seed: int = 1234) -> None:
        check(self.lib.mtsac_buffer_fill_synthetic(self._h, seed))

    def buffer_state(self) -> tuple[int, bool]:
        pos, full = ctypes.c_int64(), ctypes.c_int32()
        check(self.lib.mtsac_buffer_get_state(self._h, ctypes.byref(pos), ctypes.byref(full)))
        return pos.value, bool(full.value)

    def set_buffer_state(self, pos: int, full: bool) -> None:
        check(self.lib.mtsac_buffer_set_state(self._h, pos, 1 if full else 0))

    def set_reward_stats(self, min_r, max_r) -> None:
        mn = np.ascontiguousarray(min_r, dtype=np.float64)
        mx = np.ascontiguousarray(max_r, dtype=np.float64)
        check(self.lib.mtsac_buffer_set_reward_stats(self._h, mn.ctypes.data_as(_lib.PD), mx.ctypes.data_as(_lib.PD)))

    def reward_stats(self) -> tuple[np.ndarray, np.ndarray]:
        mn, mx = np.empty(self.T_l, np.float64), np.empty(self.T_l, np.float64)
        check(self.lib.mtsac_buffer_get_reward_stats(self._h, mn.ctypes.data_as(_lib.PD), mx.ctypes.data_as(_lib.PD)))
        return mn, mx

    def set_rng_state(self, st: dict) -> None:
        """Load a numpy ``PCG64`` ``bit_generator.state`` dict (buffers.py:335)."""
        assert st["bit_generator"] == "PCG64"
        s, inc = int(st["state"]["state"]), int(st["state"]["inc"])
        m = (1 << 64) - 1
        check(self.lib.mtsac_rng_set(self._h, s >> 64, s & m, inc >> 64, inc & m, int(st["has_uint32"]),
                                     int(st["uinteger"])))

    def get_rng_state(self) -> dict:
        v = [ctypes.c_uint64() for _ in range(4)]
        has, u = ctypes.c_int32(), ctypes.c_uint32()
        check(self.lib.mtsac_rng_get(self._h, *[ctypes.byref(x) for x in v], ctypes.byref(has), ctypes.byref(u)))
        return {
            "bit_generator": "PCG64",
            "state": {"state": (v[0].value << 64) | v[1].value, "inc": (v[2].value << 64) | v[3].value},
            "has_uint32": has.value,
            "uinteger": u.value,
        }

    def seed_rng(self, seed) -> None:
        """Seed the index stream exactly like ``np.random.default_rng(seed)`` (buffers.py:260)."""
        self.set_rng_state(np.random.default_rng(seed).bit_generator.state)

    def sample(self):
        n = self.config.batch_per_task
        B, D, A = self.B, self.obs_dim, self.action_dim
        idx = np.empty(n, np.int64)
        obs, nobs = np.empty((B, D), np.float32), np.empty((B, D), np.float32)
        act, done, rew = np.empty((B, A), np.float32), np.empty((B, 1), np.float32), np.empty((B, 1), np.float32)
        check(self.lib.mtsac_sample(self._h, idx.ctypes.data, obs.ctypes.data, act.ctypes.data, nobs.ctypes.data,
                                    done.ctypes.data, rew.ctypes.data))
        return idx, (obs, act, nobs, done, rew)

    # ------------------------------------------------------------------ update
    def update(self, batch=None, eps_next=None, eps_cur=None) -> None:
        keep = []
        bp = None
        if batch is not None:
            obs, act, nobs, done, rew = batch
            ptrs = [_ptr(x) for x in (obs, act, nobs, done, rew)]
            keep.extend(ptrs)
            b = Batch(*[p[0] for p in ptrs])
            bp = ctypes.byref(b)
        en, ec = _ptr(eps_next), _ptr(eps_cur)
        keep.extend([en, ec])
        check(self.lib.mtsac_update(self._h, bp, en[0] or None, ec[0] or None))

    # ------------------------------------------------------------------ gradient-conflict metrics
    def task_gradients(self, batch=None, eps_next=None, eps_cur=None) -> None:
        """Per-task gradients on the current parameters (include/mtsac.h, mtsac_task_gradients)."""
        keep = []
        bp = None
        if batch is not None:
            ptrs = [_ptr(x) for x in batch]
            keep.extend(ptrs)
            b = Batch(*[p[0] for p in ptrs])
            bp = ctypes.byref(b)
        en, ec = _ptr(eps_next), _ptr(eps_cur)
        keep.extend([en, ec])
        check(self.lib.mtsac_task_gradients(self._h, bp, en[0] or None, ec[0] or None))

    def task_gradient_size(self, which: int) -> int:
        return check(self.lib.mtsac_task_gradient_size(self._h, which))

    def get_task_gradients(self, which: int) -> np.ndarray:
        P = self.task_gradient_size(which)
        out = np.empty((self.T_l, P), np.float32)
        check(self.lib.mtsac_get_task_gradients(self._h, which, out.ctypes.data, out.size))
        return out

    def set_task_gradients(self, which: int, G) -> None:
        G = np.ascontiguousarray(G, np.float32)
        check(self.lib.mtsac_set_task_gradients(self._h, which, G.ctypes.data, G.size))

    def task_gradient_select(self, which: int, ranks) -> np.ndarray:
        r = np.ascontiguousarray(ranks, np.int64).reshape(self.T_l, 2)
        out = np.empty((self.T_l, 2), np.float32)
        check(self.lib.mtsac_task_gradient_select(self._h, which, r.ctypes.data, out.ctypes.data))
        return out

    def task_gradient_stats(self, which: int, thresholds, eps: float, tau: float) -> dict:
        T = self.T_l
        thr = np.ascontiguousarray(thresholds, np.float32).reshape(T)
        gram, l1 = np.empty((T, T), np.float64), np.empty(T, np.float64)
        counts, nz = np.empty((4, T, T), np.int64), np.empty(T, np.int64)
        check(self.lib.mtsac_task_gradient_stats(self._h, which, thr.ctypes.data, eps, tau, gram.ctypes.data,
                                                 l1.ctypes.data, counts.ctypes.data, nz.ctypes.data))
        return {"gram": gram, "l1": l1, "conflict": counts[0], "intersection": counts[1], "genuine": counts[2],
                "mismatch": counts[3], "near_zero": nz}

    def update_many(self, steps: int) -> None:
        check(self.lib.mtsac_update_many(self._h, steps))

    def logs(self) -> dict[str, float]:
        out = np.empty(_lib.NUM_LOGS, np.float32)
        check(self.lib.mtsac_get_logs(self._h, out.ctypes.data))
        return {k: float(v) for k, v in zip(LOG_KEYS, out)}

    def enable_graph(self, on: bool) -> None:
        check(self.lib.mtsac_enable_graph(self._h, 1 if on else 0))

    def synchronize(self) -> None:
        check(self.lib.mtsac_synchronize(self._h))

    # ------------------------------------------------------------------ rollout
    def eval_action(self, obs) -> np.ndarray:
        obs = np.ascontiguousarray(obs, dtype=np.float32)
        out = np.empty((obs.shape[0], self.action_dim), np.float32)
        check(self.lib.mtsac_eval_action(self._h, obs.ctypes.data, obs.shape[0], out.ctypes.data))
        return out

    def sample_action(self, obs, eps) -> np.ndarray:
        obs = np.ascontiguousarray(obs, dtype=np.float32)
        eps = np.ascontiguousarray(eps, dtype=np.float32)
        out = np.empty((obs.shape[0], self.action_dim), np.float32)
        check(self.lib.mtsac_sample_action(self._h, obs.ctypes.data, obs.shape[0], eps.ctypes.data, out.ctypes.data))
        return out

    # ------------------------------------------------------------------ multi-GPU
    @staticmethod
    def comm_unique_id() -> bytes:
        lib = _lib.load()
        n = lib.mtsac_comm_unique_id_size()
        buf = ctypes.create_string_buffer(n)
        check(lib.mtsac_comm_get_unique_id(buf))
        return buf.raw

    def comm_init(self, unique_id: bytes, nranks: int, rank: int, timeout_s: float = 0.0) -> None:
        """Join the RCCL communicator; timeout_s > 0 raises MTSACError (-110) when the peers have
        not all joined by then (include/mtsac.h, mtsac_comm_init_timeout)."""
        buf = ctypes.create_string_buffer(bytes(unique_id), len(unique_id))
        check(self.lib.mtsac_comm_init_timeout(self._h, buf, nranks, rank, float(timeout_s)))

    def noise_state(self) -> tuple[int, int]:
        s, c = ctypes.c_uint64(), ctypes.c_uint64()
        check(self.lib.mtsac_get_noise_state(self._h, ctypes.byref(s), ctypes.byref(c)))
        return s.value, c.value

    def set_noise_state(self, seed: int, counter: int) -> None:
        check(self.lib.mtsac_set_noise_state(self._h, seed, counter))

    def comm_nranks(self) -> int:
        n = ctypes.c_int32()
        check(self.lib.mtsac_comm_nranks(self._h, ctypes.byref(n)))
        return n.value

    def set_allreduce_hook(self, fn) -> None:
        """``fn(device_ptr: int, count: int)`` must leave the SUM over shards in the buffer."""
        if fn is None:
            self._hook = None
            check(self.lib.mtsac_set_allreduce_hook(self._h, None, None))
            return

        def tramp(_user, ptr, count):
            try:
                fn(ptr, count)
                return 0
            except Exception:  # pragma: no cover - reported through the engine
                import traceback

                traceback.print_exc()
                return -1

        self._hook = _lib.ALLREDUCE_FN(tramp)
        check(self.lib.mtsac_set_allreduce_hook(self._h, ctypes.cast(self._hook, ctypes.c_void_p), None))

    def set_collective_hook(self, fn, rank: int, world: int) -> None:
        """``fn(op, device_ptr, count)``: op 0 all-reduce (sum), 1 reduce-scatter in place (this rank's
        shard [rank count / world, (rank + 1) count / world) must hold the sum), 2 all-gather in place
        (include/mtsac.h mtsac_set_collective_hook)."""
        if fn is None:
            self._hook = None
            check(self.lib.mtsac_set_collective_hook(self._h, None, None, 0, 1))
            return

        def tramp(_user, op, ptr, count):
            try:
                fn(op, ptr, count)
                return 0
            except Exception:  # pragma: no cover - reported through the engine
                import traceback

                traceback.print_exc()
                return -1

        self._hook = _lib.COLLECTIVE_FN(tramp)
        check(self.lib.mtsac_set_collective_hook(self._h, ctypes.cast(self._hook, ctypes.c_void_p), None, rank, world))

    def set_sharded_optimizer(self, on: bool) -> None:
        """ZeRO-1-style sharded trunk optimizer for task-sharded runs (include/mtsac.h
        mtsac_set_sharded_optimizer): reduce-scatter, Adam on 1/world of the trunk, all-gather."""
        check(self.lib.mtsac_set_sharded_optimizer(self._h, 1 if on else 0))

    # ------------------------------------------------------------------ measurement
    def set_timing(self, on: bool, serial: bool = False) -> None:
        """HIP-event timing of every GEMM launch of the next update call(s); serial=True runs
        the step on one stream (solo kernel durations), else the step keeps its streams."""
        check(self.lib.mtsac_set_timing(self._h, (2 if serial else 1) if on else 0))

    def timing_kernel(self, family: int) -> str:
        buf = ctypes.create_string_buffer(256)
        check(self.lib.mtsac_get_timing_kernel(self._h, family, buf, 256))
        return buf.value.decode()

    def timing(self, family: int) -> tuple[float, int, float]:
        ms, n, fl = ctypes.c_double(), ctypes.c_int32(), ctypes.c_double()
        check(self.lib.mtsac_get_timing(self._h, family, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl)))
        return ms.value, n.value, fl.value


def debug_gemm(kind: int, epi: int, A, B, C, M: int, N: int, K: int, batch: int = 1, a_shared: bool = False,
               bias=None, mask=None, want_db: bool = False, precision: int = 0, splits: int = 1):
    """Run one device GEMM (include/mtsac_debug.h) on host arrays; returns (C, db)."""
    lib = _lib.load()
    A = np.ascontiguousarray(A, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    C = np.ascontiguousarray(C, np.float32).copy()
    lda, ldb, ldc = A.shape[-1], B.shape[-1], C.shape[-1]
    bias_a = None if bias is None else np.ascontiguousarray(bias, np.float32)
    mask_a = None if mask is None else np.ascontiguousarray(mask, np.float32)
    db = np.zeros((batch, N), np.float32) if want_db else None
    check(lib.mtsac_debug_gemm(precision | (splits << 8), kind, epi, batch, M, N, K, A.ctypes.data, lda, 1 if a_shared else 0, B.ctypes.data,
                               ldb, C.ctypes.data, ldc, None if bias_a is None else bias_a.ctypes.data,
                               None if mask_a is None else mask_a.ctypes.data,
                               0 if mask_a is None else mask_a.shape[-1], None if db is None else db.ctypes.data))
    return C, db
