"""DrQConfig / DrQ (mtrl/rl/algorithms/drqeps.py:98-343) on the MI355X DrQ-eps engine.

The API surface the Atari experiment uses: DrQ.initialize(config, env_config, seed),
update(data) -> (self, logs), sample_action(obs, task_ids) -> (self, actions),
eval_action(obs, task_ids), get_num_params().  The device does the augmentation, the three
ImpalaDQN passes, the C51 loss, its backward, AdamW and Polyak (include/drq.h).  The random draws
the reference takes from jax.random (augmentation crops and intensities, epsilon-greedy coins and
random actions) come from a numpy Generator seeded by `seed` here: JAX's threefry is not
reproduced, so trajectories match the reference in distribution, not draw for draw."""

from __future__ import annotations

import dataclasses

import numpy as np

from ....drq import DrQEngine, DrQSettings
from ....drq_init import init_drq
from ... import types as T
from ...config.networks import ImpalaDQNConfig
from ...config.rl import AlgorithmConfig

_PAD = 4  # augmentation.py:75 (img_pad)
# compute_conflict_metrics' keys (utils.py:155-174), unprefixed in DrQ.compute_weights' dict
_CONFLICT_KEYS = ("conflict_rate", "mean_conflict_magnitude", "mean_conflict_angle", "per_task_conflict_rate",
                  "per_task_grad_magnitude", "pairwise_conflict", "pairwise_cos_sim", "pairwise_angle",
                  "avg_interference_rate", "interference_asymmetry", "per_task_interference_in",
                  "per_task_interference_out", "pairwise_interference_rate", "avg_participation_ratio",
                  "per_task_participation_ratio", "effective_rank")


@dataclasses.dataclass(frozen=True)
class DrQConfig(AlgorithmConfig):  # drqeps.py:98-109
    critic_config: ImpalaDQNConfig = ImpalaDQNConfig()
    tau: float = 0.005
    v_min: float = -10.0
    v_max: float = 10.0
    n_atoms: int = 51
    eps_start: float = 1.0
    eps_end: float = 0.01
    eps_decay_steps: int = 5_000
    num_tasks: int = 26


def _adam_settings(opt) -> tuple[float, float]:
    """(eps, weight_decay) of OptimizerConfig.spawn (config/optim.py:26-43) for the engine's
    AdamW kernel: eps defaults to 1e-5 for Adam and to optax's 1e-8 for AdamW; weight decay
    applies to AdamW only (optax.adamw's default 1e-4 when unset) -- Adam is AdamW with decay 0.
    Anything the kernel does not implement (a clip_by_global_norm link, RMSProp, SGD) raises."""
    from ...config.utils import Optimizer

    if opt.max_grad_norm is not None:
        raise NotImplementedError("DrQ engine: clip_by_global_norm (max_grad_norm) is not implemented")
    if opt.optimizer == Optimizer.Adam:
        return (opt.eps if opt.eps is not None else 1e-5), 0.0
    if opt.optimizer == Optimizer.AdamW:
        return (opt.eps if opt.eps is not None else 1e-8), (opt.weight_decay if opt.weight_decay is not None
                                                             else 1e-4)
    raise NotImplementedError(f"DrQ engine: optimizer {opt.optimizer} is not implemented (Adam / AdamW only)")


class DrQ:
    def __init__(self, engine: DrQEngine, config: DrQConfig, seed: int, batch: int):
        self.engine = engine
        self.config = config
        self.rng = np.random.default_rng(seed)
        self.step = 0
        self.batch = batch

    @staticmethod
    def initialize(config: DrQConfig, env_config, seed: int = 1, batch_size: int = 256, nstep: int = 3) -> "DrQ":
        obs_shape = tuple(getattr(env_config, "observation_space").shape)  # (C, H, W) uint8
        n_actions = int(getattr(env_config, "action_space").n)
        enc = config.critic_config.impala_config
        opt = config.critic_config.q_function_config.network_config.optimizer
        eps, weight_decay = _adam_settings(opt)
        s = DrQSettings(num_tasks=config.num_tasks, n_actions=n_actions, n_atoms=config.n_atoms, in_ch=obs_shape[0],
                        hw=obs_shape[1], scale=enc.scale, embed_dim=config.critic_config.task_embed_config.embed_dim,
                        batch=batch_size, nstep=nstep, gamma=config.gamma, v_min=config.v_min, v_max=config.v_max,
                        tau=config.tau, lr=opt.lr, eps=eps, weight_decay=weight_decay)
        eng = DrQEngine(s)
        p = init_drq(seed, num_tasks=config.num_tasks, n_actions=n_actions, n_atoms=config.n_atoms,
                     in_ch=obs_shape[0], hw=obs_shape[1], scale=enc.scale,
                     embed_dim=config.critic_config.task_embed_config.embed_dim)
        eng.set_params(0, p)
        eng.set_params(1, p)  # target = the shrink-and-perturbed params (drqeps.py:196)
        return DrQ(eng, config, seed, batch_size)

    def spawn_replay_buffer(self, env_config, config, seed: int = 1) -> "DeviceAtariReplayBuffer":
        """drqeps.py:124-137: the buffer lives on the device inside the engine (rebuilt here with
        buffer_size / num_tasks slots per task, the current parameters and optimizer state carried
        over)."""
        from mtrl_amd import _lib as L

        cap = config.buffer_size // self.config.num_tasks
        s = dataclasses.replace(self.engine.s, capacity=cap, normalize_rewards=int(config.normalize_rewards),
                                nstep=getattr(config, "nstep", self.engine.s.nstep))
        state = {w: self.engine.get_params(w) for w in (L.DRQ_PARAMS, L.DRQ_TARGET, L.DRQ_ADAM_MU, L.DRQ_ADAM_NU)}
        count = self.engine.get_step()  # Adam bias correction continues where it was
        self.engine.close()
        self.engine = DrQEngine(s)
        for w, v in state.items():
            self.engine.set_params(w, v)
        self.engine.set_step(count)
        self.engine.seed_rng(seed)
        self.engine.seed_augment(int(self.rng.integers(0, 2**63)))
        return DeviceAtariReplayBuffer(self.engine)

    def update_from_buffer(self, steps: int = 1):
        """OffPolicyAlgorithm.train's update loop (base.py:213-221) for this buffer:
        `steps` x (sample_unbalanced(batch_size) + update), rows drawn with the buffer's Generator,
        gather, augmentation and update on the device (no host batch)."""
        self.engine.sample_unbalanced_update(steps)
        return self, self.engine.logs()

    def shrink_and_perturb(self, dummy_obs=None, critic_config=None, action_dim=None, shrink_rate: float = 0.5) -> "DrQ":
        """drqeps.py:212-245: encoder leaves pulled halfway to a fresh init, the rest re-initialised,
        target = the new parameters, a fresh AdamW state.  The geometry is the engine's (the
        reference's dummy_obs / critic_config / action_dim arguments rebuild the same network)."""
        from mtrl_amd import _lib as L

        from ....drq_init import shrink_and_perturb

        s = self.engine.s
        geo = dict(num_tasks=s.num_tasks, n_actions=s.n_actions, n_atoms=s.n_atoms, in_ch=s.in_ch, hw=s.hw,
                   scale=s.scale, embed_dim=s.embed_dim, n_hidden=s.n_hidden)
        p = shrink_and_perturb(self.engine.get_params(L.DRQ_PARAMS), self.rng, shrink_rate, **geo)
        self.engine.set_params(L.DRQ_PARAMS, p)
        self.engine.set_params(L.DRQ_TARGET, p)
        zero = np.zeros_like(p)
        self.engine.set_params(L.DRQ_ADAM_MU, zero)
        self.engine.set_params(L.DRQ_ADAM_NU, zero)
        self.engine.set_step(0)
        return self

    def _metrics_engine(self, n: int) -> DrQEngine:
        """An engine of batch n (one task group) sharing the current parameters and target."""
        from mtrl_amd import _lib as L

        e = getattr(self, "_meng", None)
        if e is None or e.s.batch != n:
            if e is not None:
                e.close()
            e = self._meng = DrQEngine(dataclasses.replace(self.engine.s, batch=n, capacity=0))
        for w in (L.DRQ_PARAMS, L.DRQ_TARGET):
            e.set_params(w, self.engine.get_params(w))
        return e

    def compute_weights(self, data: T.AtariReplayBufferSamples, proj_dim: int = 10_000, chunk: int = 500_000,
                        proj_seed: int = 42):
        """drqeps.py:353-482: both observation batches augmented, rows grouped by task id (stable
        argsort), each group's C51 loss gradient on the device, project_grad's JL projection of
        every task gradient to proj_dim (the Gaussian matrix regenerated on the device from
        jax.random's threefry stream, PRNGKey(42 + block)), then vmap_cos_sim and
        compute_conflict_metrics (utils.py:49-174) on the T x proj_dim matrix."""
        from ....conflict import conflict_metrics_from_stats, matrix_stats

        c = self.config
        Tn = c.num_tasks
        obs, nobs = np.asarray(data.observations), np.asarray(data.next_observations)
        B = obs.shape[0]
        if B % Tn:
            raise ValueError(f"batch of {B} rows is not a multiple of num_tasks {Tn}")
        n = B // Tn
        co, no = self._aug_draws(B)
        cn, nn = self._aug_draws(B)
        task = np.asarray(data.task_ids).reshape(B)
        act, rew = np.asarray(data.actions).reshape(B), np.asarray(data.rewards).reshape(B)
        done = np.asarray(data.dones).reshape(B)
        order = np.argsort(task, kind="stable")
        eng = self._metrics_engine(n)
        for t in range(Tn):
            r = order[t * n:(t + 1) * n]
            eng.task_gradient((obs[r], act[r], nobs[r], done[r], rew[r], task[r]), (co[r], no[r], cn[r], nn[r]), t, Tn)
        proj = eng.project_task_gradients(Tn, proj_dim, chunk, proj_seed)
        m = conflict_metrics_from_stats(matrix_stats(proj))
        logs = {"critic_avg_cos_sim": m["avg_cos_sim"], "critic_avg_grad_magnitude": m["avg_grad_magnitude"]}
        logs.update({k: m[k] for k in _CONFLICT_KEYS})
        return self, logs

    def get_num_params(self) -> dict[str, int]:
        return {"critic_num_params": self.engine.n}

    def _aug_draws(self, n):
        crop = self.rng.integers(0, 2 * _PAD, (n, 2)).astype(np.int32)
        noise = (1.0 + 0.05 * np.clip(self.rng.standard_normal(n), -2.0, 2.0)).astype(np.float32)
        return crop, noise

    def update(self, data: T.AtariReplayBufferSamples):
        """DrQ.update (drqeps.py:337-343): augment both observation batches, _update_inner."""
        B = data.observations.shape[0]
        if B != self.batch:
            raise ValueError(f"batch of {B} rows; the engine was built for {self.batch}")
        co, no = self._aug_draws(B)
        cn, nn = self._aug_draws(B)
        self.engine.update((data.observations, np.asarray(data.actions).reshape(B), data.next_observations,
                            np.asarray(data.dones).reshape(B), np.asarray(data.rewards).reshape(B),
                            np.asarray(data.task_ids).reshape(B)), (co, no, cn, nn))
        return self, self.engine.logs()

    def _q(self, observation, task_ids):
        n = observation.shape[0]
        crop, noise = self._aug_draws(n)
        return self.engine.q_values(observation, task_ids, crop, noise)

    def sample_action(self, observation, task_ids):
        """_sample_action (drqeps.py:49-79): epsilon decays linearly over eps_decay_steps env steps."""
        c = self.config
        q = self._q(observation, task_ids)
        t = min(self.step / c.eps_decay_steps, 1.0)
        eps = c.eps_start + t * (c.eps_end - c.eps_start)
        n = q.shape[0]
        greedy = q.argmax(-1)
        coins = self.rng.uniform(size=n)
        rand = self.rng.integers(0, 18, n)  # hardcoded for Atari in the reference (drqeps.py:75)
        self.step += c.num_tasks
        return self, np.where(coins < eps, rand, greedy)

    def eval_action(self, observation, task_ids):
        """_eval_action (drqeps.py:81-97): greedy on the augmented observation."""
        return self._q(observation, task_ids).argmax(-1)

    def close(self):
        self.engine.close()
        if getattr(self, "_meng", None) is not None:
            self._meng.close()


class DeviceAtariReplayBuffer:
    """MemoryEfficientAtariMultiTaskReplayBuffer's API (buffers.py:949-1229) over the engine's
    device store: add(obs, next_obs, action, reward, truncate, done) per env step of all tasks,
    sample(batch_size) -> AtariReplayBufferSamples (a host copy of the staged batch)."""

    def __init__(self, engine: DrQEngine):
        self.engine = engine
        self.num_tasks = engine.s.num_tasks
        self.capacity = engine.s.capacity

    @property
    def pos(self) -> int:
        return self.engine.buffer_state()[0]

    @property
    def full(self) -> bool:
        return self.engine.buffer_state()[1]

    def add(self, obs, next_obs, action, reward, truncate, done) -> None:
        self.engine.buffer_add(obs, next_obs, action, reward, truncate, done)

    def _check(self, batch_size):
        if batch_size != self.engine.s.batch:
            raise ValueError(f"batch_size {batch_size}: the engine samples {self.engine.s.batch}")

    def _read(self) -> T.AtariReplayBufferSamples:
        o, a, no, tr, d, r, t = self.engine.read_batch()
        return T.AtariReplayBufferSamples(o, a, no, tr[:, None], d[:, None], r[:, None], t)

    def sample(self, batch_size: int) -> T.AtariReplayBufferSamples:
        """buffers.py:1188-1227 (batch_size % num_tasks == 0); batches other than the engine's
        (the evaluation-time metrics batch) draw their indices on the host."""
        if batch_size != self.engine.s.batch:
            o, a, no, tr, d, r, t = self.engine.sample_balanced_host(batch_size)
            return T.AtariReplayBufferSamples(o, a, no, tr[:, None], d[:, None], r[:, None], t)
        self.engine.sample()
        return self._read()

    def sample_unbalanced(self, batch_size: int) -> T.AtariReplayBufferSamples:
        """buffers.py:1230-1279: Dirichlet task proportions (what the training loop calls)."""
        self._check(batch_size)
        self.engine.sample_unbalanced()
        return self._read()
