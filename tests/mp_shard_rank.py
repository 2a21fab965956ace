"""One rank of the process-per-GPU task-sharded update (run as a child process by
tests/test_gpu_multiprocess.py; not a test module).

Layout of the multi-GPU bench (bench.py --gpus N): one fresh process per rank, each owning a
contiguous task shard (mtrl_amd/shard.py) with its own engine.  On one GPU box
every rank's engine sits on device 0 and RCCL cannot form (it refuses two ranks on one
device), so the trunk gradients are summed by a host-staged gloo all-reduce installed through
mtsac_set_allreduce_hook: the engine calls it at the RCCL path's own points and in its order
(one bucket per hidden layer as its weight gradient lands, then layer 0 + the scalar tail).

Usage: python mp_shard_rank.py <problem.npz> <out.npz> <device_steps>   (RANK, WORLD_SIZE,
MASTER_ADDR, MASTER_PORT in the environment).
"""

from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def gloo_hook(dist, torch, lib):
    """fn(device_ptr, count): device -> host, gloo sum over ranks, host -> device."""
    from mtrl_amd import _lib

    calls = []

    def fn(ptr: int, count: int) -> None:
        host = np.empty(count, np.float32)
        _lib.check(lib.mtsac_memcpy(host.ctypes.data, ptr, count * 4))
        t = torch.from_numpy(host)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        _lib.check(lib.mtsac_memcpy(ptr, host.ctypes.data, count * 4))
        calls.append(count)

    return fn, calls


def main() -> int:
    import torch
    import torch.distributed as dist

    prob_path, out_path, device_steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    from mtrl_amd import _lib as L
    from mtrl_amd.engine import MTSACEngine, make_config
    from mtrl_amd.init import slice_heads
    from mtrl_amd.shard import local_rows, shard_tasks

    p = np.load(prob_path)
    T, W, n, clip, precision = (int(p[k]) for k in ("T", "W", "n", "clip", "precision"))
    D = 39 + T
    b0, c0 = shard_tasks(T, world, rank)
    cfg = make_config(num_tasks=T, task_begin=b0, task_count=c0, obs_dim=D, actor_width=W, critic_width=W,
                      batch_per_task=n, capacity=max(n, 256), clip=clip, precision=precision)
    e = MTSACEngine(cfg, device=0)
    e.enable_graph(False)
    e.set_params(L.ACTOR, slice_heads(p["actor"], D, W, 3, T, 8, None, b0, c0))
    e.set_params(L.CRITIC, slice_heads(p["critic"], D + 4, W, 3, T, 1, 2, b0, c0))
    e.set_params(L.CRITIC_TARGET, slice_heads(p["critic_target"], D + 4, W, 3, T, 1, 2, b0, c0))
    e.set_params(L.LOG_ALPHA, p["log_alpha"])
    hook, calls = gloo_hook(dist, torch, e.lib)
    e.set_allreduce_hook(hook)
    rows = local_rows(T, n, b0, c0)
    batch = tuple(p[k][rows] for k in ("obs", "act", "nobs", "done", "rew"))
    e.update(batch, p["eps_next"][rows], p["eps_cur"][rows])
    logs1 = e.logs()
    first = {w: e.get_params(w) for w in (L.ACTOR, L.CRITIC, L.CRITIC_TARGET, L.LOG_ALPHA)}
    calls_per_step = len(calls)
    # more steps on the device-sampled path the bench times (same index stream on every rank)
    e.buffer_fill_synthetic(1234)
    e.seed_rng(1)
    e.update_many(device_steps)
    logs2 = e.logs()
    out = {f"p{w}": v for w, v in first.items()}
    out.update({f"q{w}": e.get_params(w) for w in (L.ACTOR, L.CRITIC)})
    out["logs1"] = np.array([logs1[k] for k in L.LOG_KEYS], np.float32)
    out["logs2"] = np.array([logs2[k] for k in L.LOG_KEYS], np.float32)
    out["bucket_counts"] = np.array(calls[:calls_per_step], np.int64)
    out["calls_total"] = np.array(len(calls))
    out["shard"] = np.array([b0, c0])
    np.savez(out_path, **out)
    e.close()
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
