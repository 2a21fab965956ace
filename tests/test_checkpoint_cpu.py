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
    tree = net
    for k in reversed(root):
        tree = {k: tree}
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
    tree["params"]["MultiHeadNetwork_0"]["layer_1"]["kernel"] = np.zeros((3, 3))
    with pytest.raises(ValueError):
        C.from_flax_tree(tree, shapes, C._ACTOR_ROOT)
    del tree["params"]["MultiHeadNetwork_0"]["layer_0"]
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


def _expected_keys(T, I, W, depth, E):
    """The reference agent pytree written out by hand (not from the module's constants):
    MTSAC fields actor / critic / alpha / key (mtsac.py:130-134); TrainState fields params,
    opt_state, step (+ target_params, CriticTrainState mtsac.py:66-67); params = the flax
    variables dict {"params": ...} (mtsac.py:109,720); ContinuousActionPolicy wraps a
    MultiHeadNetwork (networks.py:28-34) whose trunk Denses are layer_i and heads a vmapped
    Dense (multi_head.py:29-62); the critic is Ensemble(QValueFunction) -> VmapQValueFunction_0
    (sac.py:419); opt_state of chain(clip_by_global_norm, adam) = (EmptyState,
    (ScaleByAdamState(count, mu, nu), EmptyState)); of plain adam = (ScaleByAdamState, EmptyState)."""
    def net(prefix, ens, hd, fan0):
        e = (ens,) if ens else ()
        out = {f"{prefix}/VmapDense_0/bias": e + (T, hd), f"{prefix}/VmapDense_0/kernel": e + (T, W, hd)}
        fan = fan0
        for i in range(depth):
            out[f"{prefix}/layer_{i}/bias"] = e + (W,)
            out[f"{prefix}/layer_{i}/kernel"] = e + (fan, W)
            fan = W
        return out

    keys = {}
    a = "params/MultiHeadNetwork_0"
    c = "params/VmapQValueFunction_0/MultiHeadNetwork_0"
    for top, path, ens, hd, fan0, extra in (("actor", a, None, 8, I, ()), ("critic", c, E, 1, I + 4,
                                                                            ("target_params",))):
        for coll in ("params",) + extra:
            keys.update(net(f"{top}/{coll}/{path}", ens, hd, fan0))
        for mom in ("mu", "nu"):
            keys.update(net(f"{top}/opt_state/1/0/{mom}/{path}", ens, hd, fan0))
        keys[f"{top}/opt_state/1/0/count"] = ()
        keys[f"{top}/step"] = ()
    keys["alpha/params/params/log_alpha"] = (T,)
    keys["alpha/opt_state/0/mu/params/log_alpha"] = (T,)
    keys["alpha/opt_state/0/nu/params/log_alpha"] = (T,)
    keys["alpha/opt_state/0/count"] = ()
    keys["alpha/step"] = ()
    keys["key"] = (2,)
    return keys


def _sizes(kw):
    from mtrl_amd import _lib as L

    na = sum(int(np.prod(s)) for _, s in C.network_shapes(kw, "actor"))
    nc = sum(int(np.prod(s)) for _, s in C.network_shapes(kw, "critic"))
    T = kw["num_tasks"]
    return {L.ACTOR: na, L.ACTOR_ADAM_MU: na, L.ACTOR_ADAM_NU: na, L.CRITIC: nc, L.CRITIC_TARGET: nc,
            L.CRITIC_ADAM_MU: nc, L.CRITIC_ADAM_NU: nc, L.LOG_ALPHA: T, L.ALPHA_ADAM_MU: T, L.ALPHA_ADAM_NU: T}


class _Algo:
    def __init__(self, engine, kw):
        self.engine, self._cfg_kwargs = engine, kw
        self.key = np.array([7, 123], np.uint32)

    def noise_key(self):
        return self.key

    def set_noise_key(self, k):
        self.key = np.asarray(k, np.uint32)


KW = dict(num_tasks=4, task_count=4, obs_dim=43, action_dim=4, actor_width=16, actor_depth=3, critic_width=16,
          critic_depth=3, num_critics=2, actor_max_grad_norm=1.0, critic_max_grad_norm=1.0, alpha_max_grad_norm=None)


def test_agent_state_matches_hand_written_reference_tree():
    st = C.agent_state(_Algo(_FakeEngine(_sizes(KW)), KW))
    want = _expected_keys(4, 43, 16, 3, 2)
    assert set(st) == set(want), (sorted(set(st) - set(want)), sorted(set(want) - set(st)))
    for k, s in want.items():
        assert st[k].shape == s, (k, st[k].shape, s)
    assert int(st["critic/opt_state/1/0/count"]) == 4 and int(st["actor/step"]) == 3
    assert int(st["alpha/opt_state/0/count"]) == 5


def test_agent_state_round_trip_paths():
    a = _Algo(_FakeEngine(_sizes(KW)), KW)
    st = C.agent_state(a)
    b = _Algo(_FakeEngine(_sizes(KW)), KW)
    b.engine.p = {w: np.zeros_like(v) for w, v in b.engine.p.items()}
    b.engine.counts = [0, 0, 0]
    b.key = np.zeros(2, np.uint32)
    C.load_agent_state(b, st)
    for w in _sizes(KW):
        np.testing.assert_array_equal(b.engine.p[w], a.engine.p[w])
    assert b.engine.counts == a.engine.counts
    np.testing.assert_array_equal(b.key, a.key)


def test_unclipped_networks_use_plain_adam_prefix():
    kw = dict(KW, actor_max_grad_norm=None, critic_max_grad_norm=0.0, alpha_max_grad_norm=1.0)
    st = C.agent_state(_Algo(_FakeEngine(_sizes(kw)), kw))
    # None: plain adam; 0.0 still chains clip_by_global_norm (optim.py:38 tests `is not None`)
    assert "actor/opt_state/0/count" in st and "critic/opt_state/1/0/count" in st
    assert "alpha/opt_state/1/0/count" in st
    with pytest.raises(KeyError):  # a clipped checkpoint does not load into an unclipped config
        C.load_agent_state(_Algo(_FakeEngine(_sizes(KW)), KW), st)
