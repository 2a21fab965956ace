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

    actor/params/MultiHeadNetwork_0/{VmapDense_0,layer_i}/{bias,kernel}
    critic/params/VmapQValueFunction_0/MultiHeadNetwork_0/...      (leading axis = ensemble)
    critic/target_params/VmapQValueFunction_0/MultiHeadNetwork_0/...
    {actor,critic}/opt_state/{mu,nu}/<same path as params>, .../opt_state/count
    alpha/params/log_alpha, alpha/opt_state/{mu,nu}/log_alpha, alpha/opt_state/count

so a converter from a reference orbax tree is a key rename at most.  The engine's flat
vectors are in ravel_pytree order of exactly these trees (include/mtsac.h), which
``to_flax_tree`` / ``from_flax_tree`` make explicit.
"""

from __future__ import annotations

import numpy as np

from .. import _lib as L
from ..init import leaf_shapes

_ACTOR_ROOT = ("MultiHeadNetwork_0",)
_CRITIC_ROOT = ("VmapQValueFunction_0", "MultiHeadNetwork_0")


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


def agent_state(algo) -> dict[str, np.ndarray]:
    """The agent pytree of an engine-backed MTSAC as {flax path: array}."""
    eng, kw = algo.engine, algo._cfg_kwargs
    ash, csh = network_shapes(kw, "actor"), network_shapes(kw, "critic")
    tree = {
        "actor": {"params": to_flax_tree(eng.get_params(L.ACTOR), ash, _ACTOR_ROOT),
                  "opt_state": {"mu": to_flax_tree(eng.get_params(L.ACTOR_ADAM_MU), ash, _ACTOR_ROOT),
                                "nu": to_flax_tree(eng.get_params(L.ACTOR_ADAM_NU), ash, _ACTOR_ROOT),
                                "count": np.int32(eng.get_adam_count(0))}},
        "critic": {"params": to_flax_tree(eng.get_params(L.CRITIC), csh, _CRITIC_ROOT),
                   "target_params": to_flax_tree(eng.get_params(L.CRITIC_TARGET), csh, _CRITIC_ROOT),
                   "opt_state": {"mu": to_flax_tree(eng.get_params(L.CRITIC_ADAM_MU), csh, _CRITIC_ROOT),
                                 "nu": to_flax_tree(eng.get_params(L.CRITIC_ADAM_NU), csh, _CRITIC_ROOT),
                                 "count": np.int32(eng.get_adam_count(1))}},
        "alpha": {"params": {"log_alpha": eng.get_params(L.LOG_ALPHA)},
                  "opt_state": {"mu": {"log_alpha": eng.get_params(L.ALPHA_ADAM_MU)},
                                "nu": {"log_alpha": eng.get_params(L.ALPHA_ADAM_NU)},
                                "count": np.int32(eng.get_adam_count(2))}},
    }
    out: dict = {}
    _flatten_paths(tree, "", out)
    return {k: np.asarray(v) for k, v in out.items()}


def load_agent_state(algo, flat: dict) -> None:
    """Inverse of ``agent_state``: push every leaf back into the engine."""
    eng, kw = algo.engine, algo._cfg_kwargs
    ash, csh = network_shapes(kw, "actor"), network_shapes(kw, "critic")
    a = _unflatten_paths(flat, "actor")
    c = _unflatten_paths(flat, "critic")
    al = _unflatten_paths(flat, "alpha")
    eng.set_params(L.ACTOR, from_flax_tree(a["params"], ash, _ACTOR_ROOT))
    eng.set_params(L.ACTOR_ADAM_MU, from_flax_tree(a["opt_state"]["mu"], ash, _ACTOR_ROOT))
    eng.set_params(L.ACTOR_ADAM_NU, from_flax_tree(a["opt_state"]["nu"], ash, _ACTOR_ROOT))
    eng.set_params(L.CRITIC, from_flax_tree(c["params"], csh, _CRITIC_ROOT))
    eng.set_params(L.CRITIC_TARGET, from_flax_tree(c["target_params"], csh, _CRITIC_ROOT))
    eng.set_params(L.CRITIC_ADAM_MU, from_flax_tree(c["opt_state"]["mu"], csh, _CRITIC_ROOT))
    eng.set_params(L.CRITIC_ADAM_NU, from_flax_tree(c["opt_state"]["nu"], csh, _CRITIC_ROOT))
    eng.set_params(L.LOG_ALPHA, np.asarray(al["params"]["log_alpha"], np.float32))
    eng.set_params(L.ALPHA_ADAM_MU, np.asarray(al["opt_state"]["mu"]["log_alpha"], np.float32))
    eng.set_params(L.ALPHA_ADAM_NU, np.asarray(al["opt_state"]["nu"]["log_alpha"], np.float32))
    for i, part in enumerate((a, c, al)):
        eng.set_adam_count(i, int(part["opt_state"]["count"]))
