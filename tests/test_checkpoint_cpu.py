"""Flax-named agent state (mtrl_amd/compat/checkpoint.py) on CPU: the engine's flat
vectors are the ravel_pytree order of the reference's flax trees."""

from __future__ import annotations

import numpy as np
import pytest

from mtrl_amd.compat import checkpoint as C
from mtrl_amd.init import leaf_shapes


def _tree_flatten_sorted(tree: dict) -> list[np.ndarray]:
    """jax.tree_util order for nested dicts: keys sorted, depth first."""
    out = []
    for k in sorted(tree):
        v = tree[k]
        out.extend(_tree_flatten_sorted(v) if isinstance(v, dict) else [np.asarray(v)])
    return out


def _random_tree(rng, in_dim, width, depth, T, head_dim, ens):
    pre = () if ens is None else (ens,)
    net = {"VmapDense_0": {"bias": rng.standard_normal(pre + (T, head_dim)),
                           "kernel": rng.standard_normal(pre + (T, width, head_dim))}}
    fan = in_dim
    for i in range(depth):
        net[f"layer_{i}"] = {"bias": rng.standard_normal(pre + (width,)),
                             "kernel": rng.standard_normal(pre + (fan, width))}
        fan = width
    return net


@pytest.mark.parametrize("depth,ens", [(3, None), (2, 2), (3, 2)])
def test_flat_order_is_ravel_pytree_order(depth, ens):
    rng = np.random.default_rng(depth)
    T, W, I, hd = 5, 16, 49, 8 if ens is None else 1
    net = _random_tree(rng, I, W, depth, T, hd, ens)
    root = C._ACTOR_ROOT if ens is None else C._CRITIC_ROOT
    tree = {root[0]: net} if len(root) == 1 else {root[0]: {root[1]: net}}
    shapes = leaf_shapes(I, W, depth, T, hd, ens)
    flat = C.from_flax_tree(tree, shapes, root)
    ref = np.concatenate([a.reshape(-1) for a in _tree_flatten_sorted(tree)]).astype(np.float32)
    np.testing.assert_array_equal(flat, ref)
    back = C.to_flax_tree(flat, shapes, root)
    np.testing.assert_array_equal(np.concatenate([a.reshape(-1) for a in _tree_flatten_sorted(back)]), ref)


def test_shape_and_size_errors():
    shapes = leaf_shapes(10, 8, 2, 3, 8, None)
    with pytest.raises(ValueError):
        C.to_flax_tree(np.zeros(5, np.float32), shapes, C._ACTOR_ROOT)
    tree = C.to_flax_tree(np.zeros(sum(int(np.prod(s)) for _, s in shapes), np.float32), shapes, C._ACTOR_ROOT)
    tree["MultiHeadNetwork_0"]["layer_1"]["kernel"] = np.zeros((3, 3))
    with pytest.raises(ValueError):
        C.from_flax_tree(tree, shapes, C._ACTOR_ROOT)
    del tree["MultiHeadNetwork_0"]["layer_0"]
    with pytest.raises(KeyError):
        C.from_flax_tree(tree, shapes, C._ACTOR_ROOT)


class _FakeEngine:
    """Host stand-in for MTSACEngine's parameter API (no compute)."""

    def __init__(self, sizes):
        rng = np.random.default_rng(0)
        self.p = {w: rng.standard_normal(n).astype(np.float32) for w, n in sizes.items()}
        self.counts = [3, 4, 5]

    def get_params(self, w):
        return self.p[w].copy()

    def set_params(self, w, v):
        assert v.size == self.p[w].size
        self.p[w] = np.asarray(v, np.float32).reshape(-1).copy()

    def get_adam_count(self, i):
        return self.counts[i]

    def set_adam_count(self, i, c):
        self.counts[i] = c


def test_agent_state_round_trip_paths():
    from mtrl_amd import _lib as L

    kw = dict(num_tasks=4, task_count=4, obs_dim=43, action_dim=4, actor_width=16, actor_depth=3,
              critic_width=16, critic_depth=3, num_critics=2)
    na = sum(int(np.prod(s)) for _, s in C.network_shapes(kw, "actor"))
    nc = sum(int(np.prod(s)) for _, s in C.network_shapes(kw, "critic"))
    sizes = {L.ACTOR: na, L.ACTOR_ADAM_MU: na, L.ACTOR_ADAM_NU: na, L.CRITIC: nc, L.CRITIC_TARGET: nc,
             L.CRITIC_ADAM_MU: nc, L.CRITIC_ADAM_NU: nc, L.LOG_ALPHA: 4, L.ALPHA_ADAM_MU: 4, L.ALPHA_ADAM_NU: 4}

    class Algo:
        pass

    a = Algo()
    a.engine, a._cfg_kwargs = _FakeEngine(sizes), kw
    st = C.agent_state(a)
    assert st["critic/target_params/VmapQValueFunction_0/MultiHeadNetwork_0/layer_1/kernel"].shape == (2, 16, 16)
    assert st["actor/params/MultiHeadNetwork_0/VmapDense_0/kernel"].shape == (4, 16, 8)
    assert st["alpha/params/log_alpha"].shape == (4,)
    assert int(st["critic/opt_state/count"]) == 4
    b = Algo()
    b.engine, b._cfg_kwargs = _FakeEngine(sizes), kw
    b.engine.p = {w: np.zeros_like(v) for w, v in b.engine.p.items()}
    C.load_agent_state(b, st)
    for w in sizes:
        np.testing.assert_array_equal(b.engine.p[w], a.engine.p[w])
    assert b.engine.counts == a.engine.counts
