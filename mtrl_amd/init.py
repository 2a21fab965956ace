"""Parameter initialisation of the multi-head actor / twin critic (host, numpy).

Follows MTSAC.initialize (mtrl/rl/algorithms/mtsac.py:153-284): trunk kernels
he_uniform ``U(+-sqrt(6 / fan_in))`` (mtrl/config/nn.py:192 + jax he_uniform),
zero trunk biases (config/nn.py:196), head kernel and bias ``uniform(1e-3)`` for
the actor (mtrl/rl/networks.py:33-34) and ``uniform(3e-3)`` for the critic
(networks.py:65-66), ``target_params = params`` (mtsac.py:238-243),
``log_alpha = log(initial_temperature)`` (mtsac.py:52-58).  The distributions are
the reference's; the random stream is numpy's (JAX threefry is not reproduced).

Vectors come out in flax leaf order (ravel_pytree): head bias, head kernel,
layer_0 bias, layer_0 kernel, ... -- the order of ``mtsac_set_params``.
"""

from __future__ import annotations

import math

import numpy as np


def leaf_shapes(in_dim: int, width: int, depth: int, num_tasks: int, head_dim: int, ens: int | None):
    pre = () if ens is None else (ens,)
    shapes = [("head_b", pre + (num_tasks, head_dim)), ("head_W", pre + (num_tasks, width, head_dim))]
    fan = in_dim
    for i in range(depth):
        shapes.append((f"b{i}", pre + (width,)))
        shapes.append((f"W{i}", pre + (fan, width)))
        fan = width
    return shapes


def init_flat(rng: np.random.Generator, shapes, head_bound: float) -> dict[str, np.ndarray]:
    out = {}
    for k, s in shapes:
        if k in ("head_W", "head_b"):
            out[k] = rng.uniform(-head_bound, head_bound, size=s).astype(np.float32)
        elif k.startswith("W"):
            lim = math.sqrt(6.0 / s[-2])
            out[k] = rng.uniform(-lim, lim, size=s).astype(np.float32)
        else:
            out[k] = np.zeros(s, np.float32)
    return out


def slice_tasks(p: dict[str, np.ndarray], begin: int, count: int, ens: bool) -> dict[str, np.ndarray]:
    """Keep the heads of tasks [begin, begin+count) (task sharding)."""
    q = dict(p)
    ax = 1 if ens else 0
    for k in ("head_b", "head_W"):
        q[k] = np.take(p[k], np.arange(begin, begin + count), axis=ax)
    return q


def flatten(p: dict[str, np.ndarray], shapes) -> np.ndarray:
    return np.concatenate([np.ascontiguousarray(p[k]).reshape(-1) for k, _ in shapes]).astype(np.float32)


def init_mtsac(num_tasks: int, obs_dim: int, action_dim: int, actor_width: int, actor_depth: int, critic_width: int,
               critic_depth: int, num_critics: int, seed: int = 1, task_begin: int = 0, task_count: int | None = None):
    """Return (actor_flat, critic_flat) for the local task range; identical trunks on every shard."""
    task_count = num_tasks if task_count is None else task_count
    rng = np.random.default_rng(seed)
    ash = leaf_shapes(obs_dim, actor_width, actor_depth, num_tasks, 2 * action_dim, None)
    csh = leaf_shapes(action_dim + obs_dim, critic_width, critic_depth, num_tasks, 1, num_critics)
    pa = init_flat(rng, ash, 1e-3)
    pc = init_flat(rng, csh, 3e-3)
    ash_l = leaf_shapes(obs_dim, actor_width, actor_depth, task_count, 2 * action_dim, None)
    csh_l = leaf_shapes(action_dim + obs_dim, critic_width, critic_depth, task_count, 1, num_critics)
    pa = slice_tasks(pa, task_begin, task_count, False)
    pc = slice_tasks(pc, task_begin, task_count, True)
    return flatten(pa, ash_l), flatten(pc, csh_l)


def slice_heads(flat, in_dim: int, width: int, depth: int, num_tasks: int, head_dim: int, ens: int | None,
                begin: int, count: int) -> np.ndarray:
    """A full-task flat parameter vector (flax leaf order) cut down to the heads of tasks
    [begin, begin+count): the vector a task shard's engine holds."""
    flat = np.asarray(flat).reshape(-1)
    shapes = leaf_shapes(in_dim, width, depth, num_tasks, head_dim, ens)
    if begin == 0 and count == num_tasks:
        return flat
    p, o = {}, 0
    for k, s in shapes:
        m = int(np.prod(s))
        p[k] = flat[o:o + m].reshape(s)
        o += m
    q = slice_tasks(p, begin, count, ens is not None)
    return np.concatenate([np.ascontiguousarray(q[k]).reshape(-1)
                           for k, _ in leaf_shapes(in_dim, width, depth, count, head_dim, ens)])
