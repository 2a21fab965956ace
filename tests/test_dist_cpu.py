"""world_size-2 gloo tests of the multi-GPU (task-sharded) path, on CPU.

Covers the host-side control plane bench.py uses for N>1 (task split, identical
trunk init on every rank, row permutation, max-over-ranks timing reduction) and
the gradient decomposition the engine's RCCL all-reduce relies on: per-rank
critic gradients with the GLOBAL 1/(C*B) normalisation, summed over ranks on the
trunk leaves and kept local on the head leaves, equal the single-process oracle
gradient; the clip norm is sqrt(sum trunk^2 + sum_r head_r^2).
"""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ret):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from helpers import synthetic_batch, synthetic_eps
        from mtrl_amd.init import init_mtsac, leaf_shapes
        from mtrl_amd.shard import local_rows, shard_tasks
        from oracle import mtsac as om

        T, W, n = 5, 16, 4
        D, B = 39 + T, 4 * 5
        b0, c = shard_tasks(T, world, rank)
        counts = [None] * world
        dist.all_gather_object(counts, (b0, c))
        assert sorted(t for bb, cc in counts for t in range(bb, bb + cc)) == list(range(T))

        a_loc, c_loc = init_mtsac(T, D, 4, W, 3, W, 3, 2, seed=7, task_begin=b0, task_count=c)
        a_full, c_full = init_mtsac(T, D, 4, W, 3, W, 3, 2, seed=7)
        sh_loc = leaf_shapes(D, W, 3, c, 8, None)
        n_head = sum(int(np.prod(s)) for k, s in sh_loc if k.startswith("head"))
        trunk = torch.from_numpy(a_loc[n_head:].copy())
        gathered = [torch.zeros_like(trunk) for _ in range(world)]
        dist.all_gather(gathered, trunk)
        assert all(torch.equal(g, gathered[0]) for g in gathered)

        rows = local_rows(T, n, b0, c)
        allrows = [None] * world
        dist.all_gather_object(allrows, rows.tolist())
        assert sorted(sum(allrows, [])) == list(range(B))

        # critic-gradient decomposition with the global normalisation
        cfg = om.OracleConfig(num_tasks=T, obs_dim=D, actor_width=W, critic_width=W)
        csh = om.critic_leaf_shapes(cfg)
        pc = om.unflatten(c_full.astype(np.float64), csh)
        batch = synthetic_batch(T, B, seed=3)
        en, _ = synthetic_eps(B, seed=4)
        obs, act = batch[0][rows], batch[1][rows]
        y = np.random.default_rng(5).standard_normal((B, 1))[rows]
        q, caches = om.critic_forward(pc, np.concatenate([act, obs], 1), cfg)
        dq = 2.0 * (q - y[None]) / (cfg.num_critics * B)  # GLOBAL B
        grads = {}
        for k in range(cfg.num_critics):
            hs, t = caches[k]
            g, _ = om.mh_backward(om.ens_slice(pc, k), hs, t, dq[k], cfg.critic_depth)
            for name, v in g.items():
                grads.setdefault(name, []).append(v)
        grads = {k: np.stack(v) for k, v in grads.items()}
        head_sq = sum(float((grads[k][:, b0:b0 + c] ** 2).sum()) for k in ("head_b", "head_W"))
        tail = [grads[k] for k, _ in csh if not k.startswith("head")]
        vec = torch.from_numpy(np.concatenate([x.reshape(-1) for x in tail] + [np.array([head_sq])]))
        dist.all_reduce(vec)  # the engine's single RCCL all-reduce per network
        # single-process reference
        qf, cf = om.critic_forward(pc, np.concatenate([batch[1], batch[0]], 1), cfg)
        yf = np.random.default_rng(5).standard_normal((B, 1))
        dqf = 2.0 * (qf - yf[None]) / (cfg.num_critics * B)
        gf = {}
        for k in range(cfg.num_critics):
            hs, t = cf[k]
            g, _ = om.mh_backward(om.ens_slice(pc, k), hs, t, dqf[k], cfg.critic_depth)
            for name, v in g.items():
                gf.setdefault(name, []).append(v)
        gf = {k: np.stack(v) for k, v in gf.items()}
        want_tail = np.concatenate([gf[k].reshape(-1) for k, _ in csh if not k.startswith("head")])
        np.testing.assert_allclose(vec[:-1].numpy(), want_tail, rtol=1e-10, atol=1e-14)
        for k in ("head_b", "head_W"):
            np.testing.assert_allclose(grads[k][:, b0:b0 + c], gf[k][:, b0:b0 + c], rtol=1e-10, atol=1e-14)
        full_norm = np.sqrt(sum(float((gf[k] ** 2).sum()) for k in gf))
        got_norm = np.sqrt(float((vec[:-1] ** 2).sum()) + float(vec[-1]))
        assert abs(full_norm - got_norm) < 1e-10 * full_norm

        # bench.py: max-over-ranks timing reduction
        t = torch.tensor([1.0 + rank], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        assert t.item() == float(world)
        ret[rank] = "ok"
    except Exception as e:  # pragma: no cover
        ret[rank] = repr(e)
        raise
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_sharded_decomposition():
    world = 2
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), ret), nprocs=world, join=True)
    assert dict(ret) == {0: "ok", 1: "ok"}


def test_shard_split_mt50_over_8():
    from mtrl_amd.shard import shard_tasks

    assert [shard_tasks(50, 8, r)[1] for r in range(8)] == [7, 7, 6, 6, 6, 6, 6, 6]
    assert [shard_tasks(10, 8, r)[1] for r in range(8)] == [2, 2, 1, 1, 1, 1, 1, 1]
    with pytest.raises(ValueError):
        shard_tasks(4, 8, 0)
