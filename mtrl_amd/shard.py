"""Task sharding across GPUs.

Every row's loss depends only on the shared trunks plus its own task's head and
log-alpha (mtrl/nn/multi_head.py:65-66, mtsac.py:60-63), and the replay buffer
draws ONE index vector shared by all tasks (mtrl/rl/buffers.py:523-527).  So the
tasks split contiguously over ranks, every rank runs the same PCG64 index stream
(no communication for sampling), and only the trunk gradients (plus a scalar tail)
are summed over RCCL once per network per step.
"""

from __future__ import annotations

import threading

import numpy as np

from . import _lib


def shard_tasks(num_tasks: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous split: MT50 over 8 ranks -> 7,7,6,6,6,6,6,6."""
    if not 0 <= rank < world or world > num_tasks:
        raise ValueError("need 0 <= rank < world <= num_tasks")
    base, rem = divmod(num_tasks, world)
    begin = rank * base + min(rank, rem)
    return begin, base + (1 if rank < rem else 0)


def local_rows(num_tasks: int, batch_per_task: int, begin: int, count: int) -> np.ndarray:
    """Global row ids of a shard's batch, in the shard's order.

    The reference lays the batch out ``row = i*T + t`` (buffers.py:547-548); the
    shard holding tasks [begin, begin+count) sees ``row_local = i*count + (t-begin)``.
    """
    i = np.repeat(np.arange(batch_per_task), count)
    t = np.tile(np.arange(begin, begin + count), batch_per_task)
    return i * num_tasks + t


class InProcessAllReduce:
    """Sum-all-reduce between engines driven from threads of ONE process.

    Used with :meth:`MTSACEngine.set_allreduce_hook` to run several task shards on
    one device (tests, or a host without RCCL peers).  Host-staged; not a fast path.
    """

    def __init__(self, world: int):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.bufs: list[np.ndarray | None] = [None] * world
        self.total: np.ndarray | None = None

    def hook(self, rank: int):
        lib = _lib.load()

        def fn(ptr: int, count: int) -> None:
            host = np.empty(count, np.float32)
            _lib.check(lib.mtsac_memcpy(host.ctypes.data, ptr, count * 4))
            self.bufs[rank] = host
            if self.barrier.wait() == 0:
                acc = self.bufs[0].copy()
                for b in self.bufs[1:]:
                    acc += b
                self.total = acc
            self.barrier.wait()
            _lib.check(lib.mtsac_memcpy(ptr, self.total.ctypes.data, count * 4))
            self.barrier.wait()

        return fn


class InProcessCollectives(InProcessAllReduce):
    """All-reduce, reduce-scatter and all-gather between engines on threads of one process, for
    :meth:`MTSACEngine.set_collective_hook` (the sharded optimizer's collectives).  Host-staged."""

    def collective_hook(self, rank: int):
        lib = _lib.load()
        world = self.world

        def fn(op: int, ptr: int, count: int) -> None:
            host = np.empty(count, np.float32)
            _lib.check(lib.mtsac_memcpy(host.ctypes.data, ptr, count * 4))
            self.bufs[rank] = host
            if self.barrier.wait() == 0:
                if op == 2:  # all-gather: shard r from rank r
                    sh = count // world
                    acc = np.empty(count, np.float32)
                    for r, b in enumerate(self.bufs):
                        acc[r * sh:(r + 1) * sh] = b[r * sh:(r + 1) * sh]
                else:  # all-reduce / reduce-scatter: the sum (rank order), written whole
                    acc = self.bufs[0].copy()
                    for b in self.bufs[1:]:
                        acc += b
                self.total = acc
            self.barrier.wait()
            _lib.check(lib.mtsac_memcpy(ptr, self.total.ctypes.data, count * 4))
            self.barrier.wait()

        return fn


def allreduce_floats_per_step(obs_dim: int, action_dim: int, actor_width: int, actor_depth: int, critic_width: int,
                              critic_depth: int, num_critics: int) -> int:
    """Floats one rank all-reduces per gradient step: each network's contiguous trunk range
    (leaves 64-float aligned, engine.cpp Net::layout) plus its 128-float scalar tail, and the
    2 floats of head |p|^2 (engine.cpp step())."""
    def trunk(in_dim, width, depth, ens):
        n, fan = 0, in_dim
        for _ in range(depth):
            n += -(-width * ens // 64) * 64 + -(-fan * width * ens // 64) * 64
            fan = width
        return n

    return (trunk(obs_dim, actor_width, actor_depth, 1) + 128
            + trunk(obs_dim + action_dim, critic_width, critic_depth, num_critics) + 128 + 2)
