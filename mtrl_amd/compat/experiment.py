"""Experiment (mtrl/experiment.py:30-237) on the MI355X engine.

Same dataclass fields and ``enable_wandb`` / ``run`` flow: device check, env spawn,
``get_algorithm_for_config(...).initialize``, RNG seeding, optional resume, ``train``.
orbax is not in this image, so checkpoints are ``.npz`` files holding the same items
(agent tensors + Adam state, buffer arrays + PCG64 state, metadata, python/numpy RNG
states, the agent's noise streams) -- written by :class:`NpzCheckpointManager`; ``restore``
reinstates the RNG states like experiment.py:157-161.
"""

from __future__ import annotations

import json
import pathlib
import random
import time
from dataclasses import dataclass

import numpy as np

from .config.rl import AlgorithmConfig, TrainingConfig
from .envs import EnvConfig
from .rl.algorithms import OffPolicyAlgorithm, get_algorithm_for_config


def _rng_arrays(agent) -> dict:
    """The reference's ``rngs`` item (checkpoint.py:76-79: python ``random`` state, numpy global
    MT19937 state) plus the agent's action-noise Generator, as plain arrays (reloadable with
    ``allow_pickle=False``)."""
    ver, st, gauss = random.getstate()
    name, keys, pos, has_gauss, cached = np.random.get_state()
    out = {"rngs/python/version": np.int64(ver), "rngs/python/state": np.asarray(st, np.int64),
           "rngs/python/gauss": np.float64(np.nan if gauss is None else gauss),
           "rngs/numpy/keys": np.asarray(keys, np.uint32),
           "rngs/numpy/pos_gauss": np.array([pos, has_gauss], np.int64), "rngs/numpy/cached": np.float64(cached)}
    if hasattr(agent, "rng_state"):
        st = agent.rng_state()
        out["rngs/agent"] = np.array(json.dumps({**st, "state": {k: str(v) for k, v in st["state"].items()}}))
    return out


def _restore_rngs(z, agent) -> None:
    g = float(z["rngs/python/gauss"])
    random.setstate((int(z["rngs/python/version"]), tuple(int(v) for v in z["rngs/python/state"]),
                     None if np.isnan(g) else g))
    pos, has_gauss = (int(v) for v in z["rngs/numpy/pos_gauss"])
    np.random.set_state(("MT19937", z["rngs/numpy/keys"], pos, has_gauss, float(z["rngs/numpy/cached"])))
    if "rngs/agent" in z.files and hasattr(agent, "set_rng_state"):
        st = json.loads(str(z["rngs/agent"]))
        st["state"] = {k: int(v) for k, v in st["state"].items()}
        agent.set_rng_state(st)


class NpzCheckpointManager:
    def __init__(self, directory: pathlib.Path, max_to_keep: int = 5):
        self.dir = pathlib.Path(directory)
        self.dir.mkdir(parents=True, exist_ok=True)
        self.max_to_keep = max_to_keep

    def _steps(self):
        return sorted(int(p.stem.split("_")[1]) for p in self.dir.glob("ckpt_*.npz"))

    def latest_step(self):
        s = self._steps()
        return s[-1] if s else None

    def save(self, step: int, agent, buffer=None, metadata=None, metrics=None) -> None:
        arrays = {f"agent/{k}": v for k, v in agent.state_dict().items()}
        if buffer is not None:
            ck = buffer.checkpoint()
            arrays.update({f"buffer/{k}": np.asarray(v) for k, v in ck["data"].items()})
            st = ck["rng_state"]  # None (the reference's numpy 2.2 value) or a bit_generator.state dict
            arrays["buffer/rng"] = np.array(json.dumps(
                None if st is None else {**st, "state": {k: str(v) for k, v in st["state"].items()}}))
        arrays["metadata"] = np.array(json.dumps(metadata or {}))
        arrays["metrics"] = np.array(json.dumps(metrics or {}))
        arrays.update(_rng_arrays(agent))
        np.savez(self.dir / f"ckpt_{step}.npz", **arrays)
        for old in self._steps()[: -self.max_to_keep]:
            (self.dir / f"ckpt_{old}.npz").unlink(missing_ok=True)

    def restore(self, step: int, agent, buffer=None):
        z = np.load(self.dir / f"ckpt_{step}.npz", allow_pickle=False)
        agent.load_state_dict({k[len("agent/"):]: z[k] for k in z.files if k.startswith("agent/")})
        buf_ckpt = None
        if buffer is not None and "buffer/obs" in z.files:
            st = json.loads(str(z["buffer/rng"]))
            if st is not None:
                st["state"] = {k: int(v) for k, v in st["state"].items()}
            buf_ckpt = {"data": {k[len("buffer/"):]: z[k] for k in z.files if k.startswith("buffer/") and k != "buffer/rng"},
                        "rng_state": st}
            buf_ckpt["data"]["pos"] = int(buf_ckpt["data"]["pos"])
            buf_ckpt["data"]["full"] = bool(buf_ckpt["data"]["full"])
        if "rngs/python/state" in z.files:
            _restore_rngs(z, agent)
        return json.loads(str(z["metadata"])), buf_ckpt


@dataclass
class Experiment:
    exp_name: str
    seed: int
    data_dir: pathlib.Path
    env: EnvConfig
    algorithm: AlgorithmConfig
    training_config: TrainingConfig
    checkpoint: bool = True
    max_checkpoints_to_keep: int = 5
    best_checkpoint_metric: str = "mean_success_rate"
    resume: bool = False

    def __post_init__(self) -> None:
        self._wandb_enabled = False
        self._timestamp = str(int(time.time()))

    def _get_data_dir(self) -> pathlib.Path:
        return pathlib.Path(self.data_dir) / f"{self.exp_name}_{self.seed}"

    def enable_wandb(self, **wandb_kwargs) -> None:
        import wandb

        self._wandb_enabled = True
        wandb.init(dir=str(self._get_data_dir()), id=f"{self._timestamp}_{self.exp_name}_{self.seed}",
                   name=self.exp_name, **wandb_kwargs)

    def run(self, envs=None, eval_envs=None) -> OffPolicyAlgorithm:
        from .. import _lib

        _lib.load()  # fails loudly without the HIP engine (mirrors the device check, experiment.py:94-97)
        envs = envs if envs is not None else self.env.spawn(seed=self.seed)
        algorithm_cls = get_algorithm_for_config(self.algorithm)
        algorithm = algorithm_cls.initialize(self.algorithm, self.env, seed=self.seed)
        random.seed(self.seed)
        np.random.seed(self.seed)
        manager, metadata, buffer_ckpt = None, None, None
        if self.checkpoint:
            manager = NpzCheckpointManager(self._get_data_dir() / "checkpoints", self.max_checkpoints_to_keep)
            if self.resume and manager.latest_step() is not None:
                rb = algorithm.spawn_replay_buffer(self.env, self.training_config, self.seed)
                metadata, buffer_ckpt = manager.restore(manager.latest_step(), algorithm, rb)
                self._timestamp = metadata.get("timestamp", self._timestamp) or self._timestamp
                print(f"Loaded checkpoint at step {metadata['step']}")
        if self._wandb_enabled:
            import wandb

            wandb.config.update(algorithm.get_num_params())
        return algorithm.train(config=self.training_config, envs=envs, eval_envs=eval_envs, env_config=self.env,
                               run_timestamp=self._timestamp, seed=self.seed, track=self._wandb_enabled,
                               checkpoint_manager=manager, checkpoint_metadata=metadata,
                               buffer_checkpoint=buffer_ckpt)
