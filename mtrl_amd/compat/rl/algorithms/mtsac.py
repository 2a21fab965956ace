"""MTSAC on the MI355X engine -- the drop-in for mtrl/rl/algorithms/mtsac.py.

``MTSACConfig`` has the reference's fields (mtsac.py:116-127 + AlgorithmConfig);
``MTSAC.initialize / update / sample_action / eval_action / get_num_params`` keep the
reference's functional signatures (``self, logs = self.update(data)``) while the state
lives in one ``MTSACEngine`` (device memory, mutated in place; methods return ``self``).
Supported: multi-head MLP actor/critic (MultiHeadConfig or VanillaNetworkConfig with
num_tasks from the algorithm config), MSE critic, Adam optimizers -- the north-star path.
"""

from __future__ import annotations

import dataclasses
from collections.abc import Mapping

import numpy as np

from .... import _lib as L
from ....engine import MTSACEngine, make_config
from ....init import init_mtsac
from ...config.networks import ContinuousActionPolicyConfig, QValueFunctionConfig
from ...config.optim import OptimizerConfig
from ...config.rl import AlgorithmConfig
from ...config.utils import Activation, Initializer, Optimizer
from ..buffers import MultiTaskReplayBuffer
from .base import OffPolicyAlgorithm


@dataclasses.dataclass(frozen=True)
class MTSACConfig(AlgorithmConfig):
    actor_config: ContinuousActionPolicyConfig = ContinuousActionPolicyConfig()
    critic_config: QValueFunctionConfig = QValueFunctionConfig()
    temperature_optimizer_config: OptimizerConfig = OptimizerConfig(max_grad_norm=None)
    initial_temperature: float = 1.0
    num_critics: int = 2
    tau: float = 0.005
    use_task_weights: bool = False
    v_min: float = -10.0
    v_max: float = 10.0
    n_atoms: int = 51


class _DeviceLogs(Mapping):
    """The update's LogDict, fetched from the device on first access (like jax.device_get)."""

    def __init__(self, engine: MTSACEngine):
        self._engine, self._d = engine, None

    def _get(self):
        if self._d is None:
            self._d = self._engine.logs()
        return self._d

    def __getitem__(self, k):
        return self._get()[k]

    def __iter__(self):
        return iter(self._get())

    def __len__(self):
        return len(L.LOG_KEYS)


def _check_supported(net, what: str):
    if getattr(net, "activation", Activation.ReLU) is not Activation.ReLU:
        raise NotImplementedError(f"{what}: only ReLU trunks run on the engine")
    if getattr(net, "kernel_init", Initializer.HE_UNIFORM) is not Initializer.HE_UNIFORM:
        raise NotImplementedError(f"{what}: only he_uniform trunk init is implemented")
    if not getattr(net, "use_bias", True):
        raise NotImplementedError(f"{what}: use_bias=False is not implemented")
    if net.optimizer.optimizer is not Optimizer.Adam or net.optimizer.requires_split_task_losses:
        raise NotImplementedError(f"{what}: only plain Adam (optax.adam + clip_by_global_norm)")


class MTSAC(OffPolicyAlgorithm):
    def __init__(self, config: MTSACConfig, env_config, seed: int, engine: MTSACEngine, cfg_kwargs: dict):
        self.config = config
        self.env_config = env_config
        self.num_tasks = config.num_tasks
        self.engine = engine
        self._cfg_kwargs = cfg_kwargs
        self._rng = np.random.default_rng(seed)  # action noise (replaces jax.random keys, mtsac.py:70-77)
        self._buffer = None  # the replay buffer living in this engine, once spawned
        self.gamma, self.tau = config.gamma, config.tau
        self.target_entropy = -float(np.prod(env_config.action_space.shape))

    # ------------------------------------------------------------------ construction
    @staticmethod
    def initialize(config: MTSACConfig, env_config, seed: int = 1, *, precision: str = "split2h",
                   device: int = 0) -> "MTSAC":
        if config.critic_config.use_classification:
            raise NotImplementedError("classification critics are outside the MTSAC MSE path")
        net_a, net_c = config.actor_config.network_config, config.critic_config.network_config
        _check_supported(net_a, "actor")
        _check_supported(net_c, "critic")
        T = config.num_tasks
        obs_dim = int(np.prod(env_config.observation_space.shape))
        act_dim = int(np.prod(env_config.action_space.shape))
        kw = dict(
            num_tasks=T, task_count=T, obs_dim=obs_dim, action_dim=act_dim,
            actor_width=net_a.width, actor_depth=net_a.depth, critic_width=net_c.width, critic_depth=net_c.depth,
            num_critics=config.num_critics, gamma=config.gamma, tau=config.tau, clip=int(config.clip),
            use_task_weights=int(config.use_task_weights), actor_lr=net_a.optimizer.lr,
            critic_lr=net_c.optimizer.lr, alpha_lr=config.temperature_optimizer_config.lr,
            actor_max_grad_norm=net_a.optimizer.max_grad_norm, critic_max_grad_norm=net_c.optimizer.max_grad_norm,
            alpha_max_grad_norm=config.temperature_optimizer_config.max_grad_norm,
            adam_eps=net_a.optimizer.adam_eps, initial_temperature=config.initial_temperature,
            log_std_min=config.actor_config.log_std_min, log_std_max=config.actor_config.log_std_max,
            batch_per_task=128, capacity=128, precision=L.PRECISIONS[precision], noise_seed=seed + 1,
        )
        eng = MTSACEngine(make_config(**kw), device=device)
        a, q = init_mtsac(T, obs_dim, act_dim, net_a.width, net_a.depth, net_c.width, net_c.depth,
                          config.num_critics, seed=seed)
        eng.set_params(L.ACTOR, a)
        eng.set_params(L.CRITIC, q)
        eng.set_params(L.CRITIC_TARGET, q)
        print("Actor Params:", eng.param_count(L.ACTOR))
        print("Critic Params:", eng.param_count(L.CRITIC))
        return MTSAC(config, env_config, seed, eng, kw)

    def _rebuild(self, **changes) -> None:
        """Re-create the engine with new batch / buffer geometry, keeping parameters, optimizer
        state and the update-noise stream.  Refused once a replay buffer lives in the engine:
        its transitions, pos/full and PCG64 stream would be lost."""
        if self._buffer is not None:
            raise ValueError(f"engine geometry change {changes} after the replay buffer was spawned "
                             "(the device buffer would be lost); keep batch_size fixed for a run")
        keep = {w: self.engine.get_params(w) for w in range(10)}
        counts = [self.engine.get_adam_count(i) for i in range(3)]
        noise = self.engine.noise_state()
        self._cfg_kwargs.update(changes)
        old = self.engine
        self.engine = MTSACEngine(make_config(**self._cfg_kwargs), device=old.device)
        old.close()
        for w, v in keep.items():
            self.engine.set_params(w, v)
        for i, c in enumerate(counts):
            self.engine.set_adam_count(i, c)
        self.engine.set_noise_state(*noise)

    # the reference's MTSAC.key (mtsac.py:134) drives both the update and the action noise; here
    # the update noise is the engine's counter stream and the action noise a numpy Generator
    def noise_key(self) -> np.ndarray:
        seed, counter = self.engine.noise_state()
        return np.array([seed & 0xFFFFFFFF, counter & 0xFFFFFFFF], np.uint32)

    def set_noise_key(self, key) -> None:
        k = np.asarray(key, np.uint64).reshape(-1)
        self.engine.set_noise_state(int(k[0]), int(k[1]))

    def rng_state(self) -> dict:
        return self._rng.bit_generator.state

    def set_rng_state(self, st: dict) -> None:
        self._rng.bit_generator.state = st

    def spawn_replay_buffer(self, env_config, config, seed: int = 1) -> MultiTaskReplayBuffer:
        T = self.num_tasks
        cap, n = config.buffer_size // T, config.batch_size // T
        assert config.batch_size % T == 0
        returns = bool(getattr(config, "returns_normalization", False))
        mode = 2 if returns else int(config.normalize_rewards)  # returns first, as buffers.py:531-538
        if (cap, n, mode) != (self._cfg_kwargs["capacity"], self._cfg_kwargs["batch_per_task"],
                              int(self._cfg_kwargs.get("normalize_rewards", 0))):
            self._rebuild(capacity=cap, batch_per_task=n, normalize_rewards=mode)
        self._buffer = MultiTaskReplayBuffer(config.buffer_size, T, env_config.observation_space,
                                             env_config.action_space, seed=seed,
                                             normalize_rewards=config.normalize_rewards,
                                             returns_normalization=returns, engine=self.engine)
        return self._buffer

    # ------------------------------------------------------------------ algorithm API
    def get_num_params(self) -> dict[str, int]:
        return {"actor_num_params": self.engine.param_count(L.ACTOR),
                "critic_num_params": self.engine.param_count(L.CRITIC)}

    def sample_action(self, observation):
        obs = np.asarray(observation, np.float32)
        eps = self._rng.standard_normal((obs.shape[0], self.engine.action_dim)).astype(np.float32)
        return self, self.engine.sample_action(obs, eps)

    def eval_action(self, observations):
        return self.engine.eval_action(np.asarray(observations, np.float32))

    def update(self, data):
        """mtsac.py:1249-1251: one gradient step on a ReplayBufferSamples batch."""
        n = np.asarray(data.rewards).shape[0] // self.num_tasks
        if n != self._cfg_kwargs["batch_per_task"]:  # raises once a buffer lives in the engine
            self._rebuild(batch_per_task=n, capacity=max(self._cfg_kwargs["capacity"], n))
        self.engine.update(tuple(data))
        return self, _DeviceLogs(self.engine)

    def update_from_buffer(self, replay_buffer, batch_size: int, want_logs: bool):
        if getattr(replay_buffer, "engine", None) is self.engine and batch_size // self.num_tasks == \
                self._cfg_kwargs["batch_per_task"]:
            self.engine.update_many(1)  # device sampling + update, no host round trip
            return self, _DeviceLogs(self.engine)
        return super().update_from_buffer(replay_buffer, batch_size, want_logs)

    def compute_weights(self, data):
        """mtsac.py:870-1170: per-task gradient-conflict metrics at evaluation time (no update).
        Per-task gradients, Gram matrix, conflict / support / interference counts on the device
        (mtrl_amd/conflict.py); the 66 log entries of the reference's dict.  The reference
        samples one (n, A) noise draw per vmapped task from a single key (mtsac.py:892, 1052);
        that structure is kept: one draw repeated for every task's rows."""
        from ....conflict import compute_weights

        T, A = self.num_tasks, self.engine.action_dim
        n = np.asarray(data.rewards).shape[0] // T
        if n != self._cfg_kwargs["batch_per_task"]:
            self._rebuild(batch_per_task=n, capacity=max(self._cfg_kwargs["capacity"], n))
        e_next = np.repeat(self._rng.standard_normal((n, A)), T, axis=0).astype(np.float32)  # row i*T + t
        e_cur = np.repeat(self._rng.standard_normal((n, A)), T, axis=0).astype(np.float32)
        return self, compute_weights(self.engine, tuple(data), e_next, e_cur)

    # ------------------------------------------------------------------ state (checkpoint)
    def state_dict(self) -> dict[str, np.ndarray]:
        """Agent pytree keyed by flax path (compat/checkpoint.py), e.g.
        ``critic/target_params/VmapQValueFunction_0/MultiHeadNetwork_0/layer_1/kernel``."""
        from ...checkpoint import agent_state

        return agent_state(self)

    def load_state_dict(self, d: Mapping) -> None:
        from ...checkpoint import load_agent_state

        if "tensor_0" in d:  # flat-vector layout of earlier checkpoints
            for w in range(10):
                self.engine.set_params(w, np.asarray(d[f"tensor_{w}"]))
            for i, c in enumerate(np.asarray(d["adam_counts"])):
                self.engine.set_adam_count(i, int(c))
            return
        load_agent_state(self, d)
