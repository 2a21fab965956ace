"""Flax-named agent state for checkpoint interop.

The reference saves one orbax ``Composite`` per checkpoint (mtrl/checkpoint.py:54-109,
called from mtrl/experiment.py:119-168) whose ``agent`` item is the MTSAC flax struct:
actor / critic / alpha TrainStates with params, optax Adam state and critic target
params.  orbax is not in this image; ``compat.experiment.NpzCheckpointManager`` writes
the Composite as one npz (loads with ``allow_pickle=False``), and this module names the
agent leaves in it by their flax tree path, ``MTSAC.state_dict()`` being
``agent_state``.

Agent keys follow the flax auto-names of the reference networks (SURVEY.md §8 a16,
mtrl/nn/multi_head.py:20-68, mtrl/rl/networks.py:21-67,208-222):

    actor/params/params/MultiHeadNetwork_0/{VmapDense_0,layer_i}/{bias,kernel}
    critic/params/params/VmapQValueFunction_0/MultiHeadNetwork_0/...  (leading axis = ensemble)
    critic/target_params/params/VmapQValueFunction_0/MultiHeadNetwork_0/...
    {actor,critic}/opt_state/1/0/{mu,nu}/<params path>, .../opt_state/1/0/count   (clipped Adam)
    alpha/params/params/log_alpha, alpha/opt_state/0/{mu,nu}/params/log_alpha, .../0/count
    {actor,critic,alpha}/step, key

(TrainState.params is the whole flax variables dict, hence ``params/params``; the optax
state nesting follows ``OptimizerConfig.spawn``: see ``opt_prefix``.)

so a converter from a reference orbax tree is a key rename at most.  The engine's flat
vectors are in ravel_pytree order of exactly these trees (include/mtsac.h), which
``to_flax_tree`` / ``from_flax_tree`` make explicit.
"""

from __future__ import annotations

import numpy as np

from .. import _lib as L
from ..init import leaf_shapes

# params of every TrainState are the flax variables dict, so the collection name comes first
# (``alpha.params["params"]["log_alpha"]``, mtsac.py:109,720,730; ``critic_state["intermediates"]
# ["VmapQValueFunction_0"]``, sac.py:419)
_ACTOR_ROOT = ("params", "MultiHeadNetwork_0")
_CRITIC_ROOT = ("params", "VmapQValueFunction_0", "MultiHeadNetwork_0")


def opt_prefix(max_grad_norm) -> tuple[str, ...]:
    """Path of the Adam state inside a TrainState's opt_state (config/optim.py:26-43):
    ``optax.chain(clip_by_global_norm, adam)`` when max_grad_norm is set -> (EmptyState,
    (ScaleByAdamState, EmptyState)) -> ``1/0``; plain ``adam`` (the temperature optimizer,
    max_grad_norm=None, mtsac.py:120) -> (ScaleByAdamState, EmptyState) -> ``0``."""
    return ("1", "0") if max_grad_norm is not None else ("0",)


def _leaf_path(name: str) -> tuple[str, str]:
    if name == "head_b":
        return ("VmapDense_0", "bias")
    if name == "head_W":
        return ("VmapDense_0", "kernel")
    return (f"layer_{name[1:]}", "bias" if name[0] == "b" else "kernel")


def network_shapes(kw: dict, which: str):
    """Leaf shapes (flat order) of the local actor or critic from engine config kwargs."""
    T = kw.get("task_count", kw["num_tasks"])
    if which == "actor":
        return leaf_shapes(kw["obs_dim"], kw["actor_width"], kw["actor_depth"], T, 2 * kw["action_dim"], None)
    return leaf_shapes(kw["action_dim"] + kw["obs_dim"], kw["critic_width"], kw["critic_depth"], T, 1,
                       kw["num_critics"])


def to_flax_tree(flat: np.ndarray, shapes, root: tuple[str, ...]) -> dict:
    """Flat engine vector -> nested dict keyed like the reference flax params."""
    flat = np.asarray(flat, np.float32).reshape(-1)
    need = sum(int(np.prod(s)) for _, s in shapes)
    if flat.size != need:
        raise ValueError(f"flat vector has {flat.size} values, the tree needs {need}")
    tree: dict = {}
    off = 0
    for name, s in shapes:
        n = int(np.prod(s))
        node = tree
        for k in root + _leaf_path(name)[:-1]:
            node = node.setdefault(k, {})
        node[_leaf_path(name)[-1]] = flat[off:off + n].reshape(s).copy()
        off += n
    return tree


def from_flax_tree(tree: dict, shapes, root: tuple[str, ...]) -> np.ndarray:
    """Nested reference-style params -> flat engine vector (ravel_pytree order)."""
    parts = []
    for name, s in shapes:
        node = tree
        for k in root + _leaf_path(name):
            if k not in node:
                raise KeyError(f"missing leaf {'/'.join(root + _leaf_path(name))}")
            node = node[k]
        a = np.asarray(node, np.float32)
        if a.shape != tuple(s):
            raise ValueError(f"leaf {'/'.join(root + _leaf_path(name))}: shape {a.shape}, expected {tuple(s)}")
        parts.append(a.reshape(-1))
    return np.concatenate(parts).astype(np.float32)


def _flatten_paths(tree: dict, prefix: str, out: dict) -> None:
    for k, v in tree.items():
        p = f"{prefix}/{k}" if prefix else k
        if isinstance(v, dict):
            _flatten_paths(v, p, out)
        else:
            out[p] = v


def _unflatten_paths(flat: dict, prefix: str) -> dict:
    tree: dict = {}
    for key, v in flat.items():
        if not key.startswith(prefix + "/"):
            continue
        node = tree
        parts = key[len(prefix) + 1:].split("/")
        for k in parts[:-1]:
            node = node.setdefault(k, {})
        node[parts[-1]] = v
    return tree


def agent_tree(kw: dict, get, count, key=None) -> dict[str, np.ndarray]:
    """The MTSAC pytree (mtsac.py:130-151: actor / critic / alpha TrainStates + key) as
    {flax path: array}.  ``get(which)`` returns an engine flat vector (include/mtsac.h ids),
    ``count(i)`` the Adam count of actor (0) / critic (1) / alpha (2)."""
    ash, csh = network_shapes(kw, "actor"), network_shapes(kw, "critic")

    def state(which_p, which_mu, which_nu, shapes, root, i, clip, extra=None):
        n = np.int32(count(i))
        adam = {"count": n, "mu": to_flax_tree(get(which_mu), shapes, root),
                "nu": to_flax_tree(get(which_nu), shapes, root)}
        opt: dict = {}
        node = opt
        pre = opt_prefix(clip)
        for k in pre[:-1]:
            node = node.setdefault(k, {})
        node[pre[-1]] = adam
        ts = {"params": to_flax_tree(get(which_p), shapes, root), "opt_state": opt, "step": n}
        ts.update(extra or {})
        return ts

    tree = {
        "actor": state(L.ACTOR, L.ACTOR_ADAM_MU, L.ACTOR_ADAM_NU, ash, _ACTOR_ROOT, 0,
                       kw.get("actor_max_grad_norm")),
        "critic": state(L.CRITIC, L.CRITIC_ADAM_MU, L.CRITIC_ADAM_NU, csh, _CRITIC_ROOT, 1,
                        kw.get("critic_max_grad_norm"),
                        {"target_params": to_flax_tree(get(L.CRITIC_TARGET), csh, _CRITIC_ROOT)}),
        "alpha": {"params": {"params": {"log_alpha": np.asarray(get(L.LOG_ALPHA), np.float32)}},
                  "step": np.int32(count(2))},
    }
    a_opt: dict = {}
    node = a_opt
    pre = opt_prefix(kw.get("alpha_max_grad_norm"))
    for k in pre[:-1]:
        node = node.setdefault(k, {})
    node[pre[-1]] = {"count": np.int32(count(2)),
                     "mu": {"params": {"log_alpha": np.asarray(get(L.ALPHA_ADAM_MU), np.float32)}},
                     "nu": {"params": {"log_alpha": np.asarray(get(L.ALPHA_ADAM_NU), np.float32)}}}
    tree["alpha"]["opt_state"] = a_opt
    if key is not None:
        tree["key"] = np.asarray(key, np.uint32)
    out: dict = {}
    _flatten_paths(tree, "", out)
    return {k: np.asarray(v) for k, v in out.items()}


def agent_state(algo) -> dict[str, np.ndarray]:
    """The agent pytree of an engine-backed MTSAC as {flax path: array}.  ``key`` holds the
    engine's action-noise stream position in place of the JAX PRNG key (threefry is not
    reproduced): [noise seed, draws so far]."""
    eng = algo.engine
    return agent_tree(algo._cfg_kwargs, eng.get_params, eng.get_adam_count, key=algo.noise_key())


def load_agent_tree(kw: dict, flat: dict, put, set_count) -> None:
    """Inverse of ``agent_tree``: ``put(which, flat_vector)``, ``set_count(i, n)``."""
    ash, csh = network_shapes(kw, "actor"), network_shapes(kw, "critic")
    a = _unflatten_paths(flat, "actor")
    c = _unflatten_paths(flat, "critic")
    al = _unflatten_paths(flat, "alpha")

    def adam(ts, clip, what):
        node = ts["opt_state"]
        for k in opt_prefix(clip):
            if k not in node:
                raise KeyError(f"{what}/opt_state/{'/'.join(opt_prefix(clip))}: missing (max_grad_norm={clip})")
            node = node[k]
        return node

    aa = adam(a, kw.get("actor_max_grad_norm"), "actor")
    ca = adam(c, kw.get("critic_max_grad_norm"), "critic")
    la = adam(al, kw.get("alpha_max_grad_norm"), "alpha")
    put(L.ACTOR, from_flax_tree(a["params"], ash, _ACTOR_ROOT))
    put(L.ACTOR_ADAM_MU, from_flax_tree(aa["mu"], ash, _ACTOR_ROOT))
    put(L.ACTOR_ADAM_NU, from_flax_tree(aa["nu"], ash, _ACTOR_ROOT))
    put(L.CRITIC, from_flax_tree(c["params"], csh, _CRITIC_ROOT))
    put(L.CRITIC_TARGET, from_flax_tree(c["target_params"], csh, _CRITIC_ROOT))
    put(L.CRITIC_ADAM_MU, from_flax_tree(ca["mu"], csh, _CRITIC_ROOT))
    put(L.CRITIC_ADAM_NU, from_flax_tree(ca["nu"], csh, _CRITIC_ROOT))
    put(L.LOG_ALPHA, np.asarray(al["params"]["params"]["log_alpha"], np.float32))
    put(L.ALPHA_ADAM_MU, np.asarray(la["mu"]["params"]["log_alpha"], np.float32))
    put(L.ALPHA_ADAM_NU, np.asarray(la["nu"]["params"]["log_alpha"], np.float32))
    for i, st in enumerate((aa, ca, la)):
        set_count(i, int(st["count"]))


def load_agent_state(algo, flat: dict) -> None:
    """Inverse of ``agent_state``: push every leaf back into the engine."""
    eng = algo.engine
    load_agent_tree(algo._cfg_kwargs, flat, eng.set_params, eng.set_adam_count)
    if "key" in flat:
        algo.set_noise_key(np.asarray(flat["key"]))
