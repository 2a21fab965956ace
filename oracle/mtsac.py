"""ORACLE (test infrastructure only) -- numpy restatement of the MTSAC gradient step.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker.  The product path
(``mtrl_amd``) never calls it; a missing HIP library is a hard error there.

Parity status: **unpinned for the update arithmetic.**  The reference's update
is JAX/flax/optax/distrax code (``mtrl/rl/algorithms/mtsac.py``) that cannot
run here (Python 3.12 syntax, jax absent) and its own tests pin
nothing on this path.  This file restates the published algorithm of the pinned
third-party versions (jax 0.5.x autodiff rules, flax 0.10.4 ``Dense``/``vmap``,
optax 0.2.4 ``adam``/``clip_by_global_norm``/``incremental_update``, distrax
0.1.5 ``Transformed``/``MultivariateNormalDiag``/``Tanh``) and anchors on the
reference call sites cited per function.  Gradients are derived by hand and
cross-checked against torch autograd in float64 (``tests/test_oracle_mtsac.py``)
-- an independent derivation, not a pin.  Known-answer pins that do exist: the
actor parameter counts (370K / 517K figure ticks, ``figures/fig1_new_mt10.svg``,
``figures/fig1_new_mt50.svg``).

Noise: the reference draws epsilon ~ N(0,1) from JAX threefry keys
(``mtsac.py:355,629``); threefry is not reproduced -- parity is defined GIVEN
injected epsilon (``eps_next`` for a' ~ pi(.|s'), ``eps_cur`` for a ~ pi(.|s)).

Every array here is float64 by default; ``dtype=np.float32`` runs the same math
in float32 (used as the CPU baseline leg of ``bench.py``).
"""

from __future__ import annotations

import dataclasses
import math

import numpy as np

LOG2 = math.log(2.0)
HALF_LOG_2PI = 0.5 * math.log(2.0 * math.pi)

LOG_KEYS = (
    "losses/qf_values",
    "losses/qf_loss",
    "metrics/critic_grad_magnitude",
    "metrics/critic_params_norm",
    "losses/actor_loss",
    "metrics/actor_grad_magnitude",
    "metrics/actor_params_norm",
    "metrics/explore_loss",
    "losses/alpha_loss",
    "alpha",
)


# ----------------------------------------------------------------------------
# configuration
# ----------------------------------------------------------------------------
@dataclasses.dataclass
class OracleConfig:
    """Hyper-parameters of ``MTSACConfig`` that the update reads.

    Defaults follow ``mtsac.py:116-127``, ``config/rl.py:16-22``,
    ``config/networks.py:6-18``, ``config/optim.py:15-43`` and the target
    scripts (``experiments/mt10_mtmhsac.py:36-51``).
    """

    num_tasks: int
    obs_dim: int  # 39 + num_tasks for Meta-World with one-hot (envs/metaworld.py:83-98)
    action_dim: int = 4
    actor_width: int = 400
    actor_depth: int = 3
    critic_width: int = 400
    critic_depth: int = 3
    num_critics: int = 2
    gamma: float = 0.99
    tau: float = 0.005
    clip: bool = False
    use_task_weights: bool = False
    log_std_min: float = -20.0
    log_std_max: float = 2.0
    actor_lr: float = 3e-4
    critic_lr: float = 3e-4
    alpha_lr: float = 3e-4
    actor_max_grad_norm: float | None = 1.0
    critic_max_grad_norm: float | None = 1.0
    alpha_max_grad_norm: float | None = None  # temperature_optimizer_config (mtsac.py:120)
    adam_b1: float = 0.9
    adam_b2: float = 0.999
    adam_eps: float = 1e-5  # config/optim.py:31-32
    initial_temperature: float = 1.0

    @property
    def target_entropy(self) -> float:  # mtsac.py:258
        return -float(self.action_dim)

    @property
    def actor_in(self) -> int:
        return self.obs_dim

    @property
    def critic_in(self) -> int:  # networks.py:61 concat(action, state)
        return self.action_dim + self.obs_dim


# ----------------------------------------------------------------------------
# parameters
# ----------------------------------------------------------------------------
def leaf_shapes(in_dim: int, width: int, depth: int, num_tasks: int, head_dim: int, ens: int | None):
    """flax leaf order of one MultiHeadNetwork (ravel_pytree / tree_flatten order).

    Keys sort as ``VmapDense_0`` < ``layer_0`` < ... and ``bias`` < ``kernel``
    (multi_head.py:34-62).  ``ens`` prepends the Ensemble axis (networks.py:214-221).
    """
    pre = () if ens is None else (ens,)
    shapes = [("head_b", pre + (num_tasks, head_dim)), ("head_W", pre + (num_tasks, width, head_dim))]
    fan = in_dim
    for i in range(depth):
        shapes.append((f"b{i}", pre + (width,)))
        shapes.append((f"W{i}", pre + (fan, width)))
        fan = width
    return shapes


def actor_leaf_shapes(cfg: OracleConfig):
    return leaf_shapes(cfg.actor_in, cfg.actor_width, cfg.actor_depth, cfg.num_tasks, 2 * cfg.action_dim, None)


def critic_leaf_shapes(cfg: OracleConfig):
    return leaf_shapes(cfg.critic_in, cfg.critic_width, cfg.critic_depth, cfg.num_tasks, 1, cfg.num_critics)


def num_params(shapes) -> int:
    return int(sum(int(np.prod(s)) for _, s in shapes))


def flatten(p: dict, shapes) -> np.ndarray:
    return np.concatenate([np.asarray(p[k]).reshape(-1) for k, _ in shapes])


def unflatten(flat: np.ndarray, shapes) -> dict:
    out, o = {}, 0
    for k, s in shapes:
        n = int(np.prod(s))
        out[k] = np.array(flat[o : o + n]).reshape(s)
        o += n
    assert o == flat.size
    return out


def init_network(rng: np.random.Generator, shapes, head_bound: float, dtype=np.float64) -> dict:
    """Init distributions of ``mtsac.py:190-243``: he_uniform kernels
    (``U(+-sqrt(6/fan_in))``, config/nn.py:192 + jax he_uniform), zero hidden
    biases (config/nn.py:196), ``uniform(head_bound)`` head kernel and bias
    (networks.py:33-34 actor 1e-3, :65-66 critic 3e-3).  Distribution only --
    JAX's threefry stream is not reproduced."""
    p = {}
    for k, s in shapes:
        if k == "head_W" or k == "head_b":
            p[k] = rng.uniform(-head_bound, head_bound, size=s).astype(dtype)
        elif k.startswith("W"):
            fan_in = s[-2]
            lim = math.sqrt(6.0 / fan_in)
            p[k] = rng.uniform(-lim, lim, size=s).astype(dtype)
        else:
            p[k] = np.zeros(s, dtype=dtype)
    return p


@dataclasses.dataclass
class AdamState:
    mu: np.ndarray
    nu: np.ndarray
    count: int = 0

    @classmethod
    def zeros(cls, n: int, dtype) -> "AdamState":
        return cls(np.zeros(n, dtype), np.zeros(n, dtype), 0)


@dataclasses.dataclass
class MTSACState:
    actor: np.ndarray  # flat, flax leaf order
    critic: np.ndarray
    critic_target: np.ndarray
    log_alpha: np.ndarray  # (T,)
    actor_opt: AdamState
    critic_opt: AdamState
    alpha_opt: AdamState

    def copy(self) -> "MTSACState":
        cp = lambda a: AdamState(a.mu.copy(), a.nu.copy(), a.count)  # noqa: E731
        return MTSACState(
            self.actor.copy(), self.critic.copy(), self.critic_target.copy(), self.log_alpha.copy(),
            cp(self.actor_opt), cp(self.critic_opt), cp(self.alpha_opt),
        )


def initialize(cfg: OracleConfig, seed: int = 1, dtype=np.float64) -> MTSACState:
    """``MTSAC.initialize`` (mtsac.py:153-284): target = params (:238-243),
    log_alpha = log(initial_temperature) (:52-58), fresh optax states."""
    rng = np.random.default_rng(seed)
    a = flatten(init_network(rng, actor_leaf_shapes(cfg), 1e-3, dtype), actor_leaf_shapes(cfg))
    c = flatten(init_network(rng, critic_leaf_shapes(cfg), 3e-3, dtype), critic_leaf_shapes(cfg))
    la = np.full(cfg.num_tasks, math.log(cfg.initial_temperature), dtype=dtype)
    return MTSACState(
        a, c, c.copy(), la,
        AdamState.zeros(a.size, dtype), AdamState.zeros(c.size, dtype), AdamState.zeros(la.size, dtype),
    )


# ----------------------------------------------------------------------------
# networks
# ----------------------------------------------------------------------------
def relu(x):
    return np.maximum(x, 0)


def task_index(x: np.ndarray, num_tasks: int) -> np.ndarray:
    """``task_idx.argmax(axis=-1)`` over the last T input columns
    (multi_head.py:27,65); numpy/jax argmax both return the first maximum."""
    return np.argmax(x[:, -num_tasks:], axis=1)


def mh_forward(p: dict, x: np.ndarray, depth: int, num_tasks: int):
    """MultiHeadNetwork.__call__ (multi_head.py:20-68): ``depth`` Dense+ReLU
    trunk layers, then every head on every row, then the row's own head.
    Computing only the selected head is the same dot product per output."""
    t = task_index(x, num_tasks)
    hs = [x]
    h = x
    for i in range(depth):
        h = relu(h @ p[f"W{i}"] + p[f"b{i}"])
        hs.append(h)
    out = np.einsum("bw,bwo->bo", h, p["head_W"][t]) + p["head_b"][t]
    return out, hs, t


def mh_backward(p: dict, hs, t, dout: np.ndarray, depth: int, need_dx: bool = False):
    """Reverse of ``mh_forward``.  relu'(0) = 0 (jax.nn.relu custom jvp)."""
    g = {k: np.zeros_like(v) for k, v in p.items()}
    h = hs[depth]
    np.add.at(g["head_W"], t, np.einsum("bw,bo->bwo", h, dout))
    np.add.at(g["head_b"], t, dout)
    dh = np.einsum("bo,bwo->bw", dout, p["head_W"][t])
    dx = None
    for i in reversed(range(depth)):
        dz = dh * (hs[i + 1] > 0)
        g[f"W{i}"] = hs[i].T @ dz
        g[f"b{i}"] = dz.sum(axis=0)
        if i > 0 or need_dx:
            dh = dz @ p[f"W{i}"].T
    if need_dx:
        dx = dh
    return g, dx


def ens_slice(p: dict, k: int) -> dict:
    return {n: v[k] for n, v in p.items()}


def critic_forward(pc: dict, x: np.ndarray, cfg: OracleConfig):
    """``Ensemble(QValueFunction)`` (networks.py:54-67, 208-222): the same input
    through each member -> (C, B, 1)."""
    outs, caches = [], []
    for k in range(cfg.num_critics):
        o, hs, t = mh_forward(ens_slice(pc, k), x, cfg.critic_depth, cfg.num_tasks)
        outs.append(o)
        caches.append((hs, t))
    return np.stack(outs), caches


def tanh_normal_sample(out: np.ndarray, eps: np.ndarray, cfg: OracleConfig):
    """ContinuousActionPolicy + TanhMultivariateNormalDiag.sample_and_log_prob
    (networks.py:37-44, distributions.py:6-13; distrax 0.1.5 Transformed over
    MultivariateNormalDiag = standard normal pushed through Shift∘DiagLinear,
    then Block(Tanh, 1)):

        ls_c = clip(ls, lo, hi);  sigma = exp(ls_c);  x = mu + sigma * eps
        a = tanh(x)
        logpi = sum_j[-eps_j^2/2 - log(2pi)/2 - log(sigma_j)]
                - sum_j 2 * (log 2 - x_j - softplus(-2 x_j))
    """
    A = cfg.action_dim
    mu, ls = out[:, :A], out[:, A:]
    ls_c = np.clip(ls, cfg.log_std_min, cfg.log_std_max)
    sigma = np.exp(ls_c)
    x = mu + sigma * eps
    a = np.tanh(x)
    base = np.sum(-0.5 * eps * eps - HALF_LOG_2PI - np.log(sigma), axis=1)
    fldj = np.sum(2.0 * (LOG2 - x - np.logaddexp(-2.0 * x, 0.0)), axis=1)
    logpi = base - fldj
    return a, logpi, (mu, ls, sigma, x, a, eps)


def clip_grad_factor(v, lo, hi):
    """d clip(v, lo, hi)/dv under jax: maximum/minimum split ties 0.5."""
    f = ((v > lo) & (v < hi)).astype(v.dtype)
    f = f + 0.5 * ((v == lo) | (v == hi)).astype(v.dtype)
    return f


def tanh_normal_backward(cache, g_a: np.ndarray, g_logpi: np.ndarray, cfg: OracleConfig):
    """Gradient of (a, logpi) w.r.t. the head output (mu, log_std).

    d logpi / d x_j = 2 tanh(x_j) (the Tanh fldj term), d a/d x = 1 - a^2,
    d x / d ls_c = sigma * eps, d logpi / d ls_c = -1 (log sigma term).
    """
    mu, ls, sigma, x, a, eps = cache
    g_x = g_a * (1.0 - a * a) + g_logpi[:, None] * 2.0 * a
    g_mu = g_x
    g_lsc = g_x * sigma * eps - g_logpi[:, None]
    g_ls = g_lsc * clip_grad_factor(ls, cfg.log_std_min, cfg.log_std_max)
    return np.concatenate([g_mu, g_ls], axis=1)


def min_grad(q: np.ndarray):
    """d min_k q_k / d q_k (jax reduce_min jvp: ties share equally)."""
    m = q.min(axis=0, keepdims=True)
    ind = (q == m).astype(q.dtype)
    return ind / ind.sum(axis=0, keepdims=True)


# ----------------------------------------------------------------------------
# optax
# ----------------------------------------------------------------------------
def global_norm(g: np.ndarray) -> float:
    return float(np.sqrt(np.sum(g.astype(np.float64) ** 2)))


def clip_by_global_norm(g: np.ndarray, max_norm: float | None):
    """optax.clip_by_global_norm (optax 0.2.4): keep if ||g|| < max else
    ``(t / ||g||) * max`` (config/optim.py:38-42)."""
    if max_norm is None:
        return g
    n = np.sqrt(np.sum(g * g))
    if n < max_norm:
        return g
    return (g / n.astype(g.dtype)) * g.dtype.type(max_norm)


def adam_step(p: np.ndarray, g: np.ndarray, st: AdamState, lr, b1, b2, eps):
    """optax.adam (0.2.4) + apply_updates (algorithms/utils.py:29-32)."""
    dt = p.dtype.type
    st.mu = dt(1 - b1) * g + dt(b1) * st.mu
    st.nu = dt(1 - b2) * (g * g) + dt(b2) * st.nu
    st.count += 1
    mu_hat = st.mu / dt(1 - b1 ** st.count)
    nu_hat = st.nu / dt(1 - b2 ** st.count)
    upd = mu_hat / (np.sqrt(nu_hat) + dt(eps))
    return p + upd * dt(-lr)


# ----------------------------------------------------------------------------
# the update
# ----------------------------------------------------------------------------
def update(cfg: OracleConfig, state: MTSACState, batch, eps_next: np.ndarray, eps_cur: np.ndarray,
           return_internals: bool = False):
    """``MTSAC._update_inner`` (mtsac.py:1173-1247): critic, then actor (with
    the UPDATED critic), then temperature.  ``batch`` is
    ``(observations, actions, next_observations, dones, rewards)``
    (types.py:49-54).  Returns ``(new_state, logs)``; ``state`` is not mutated.
    """
    s = state.copy()
    obs, act, nobs, dones, rew = [np.asarray(b) for b in batch]
    dt = s.actor.dtype.type
    T, A, C = cfg.num_tasks, cfg.action_dim, cfg.num_critics
    B = obs.shape[0]
    ash, csh = actor_leaf_shapes(cfg), critic_leaf_shapes(cfg)
    pa = unflatten(s.actor, ash)
    pc = unflatten(s.critic, csh)
    pt = unflatten(s.critic_target, csh)
    rew = rew.reshape(B, 1)
    dones = dones.reshape(B, 1)

    # alpha_vals = exp(task_ids @ log_alpha)   (mtsac.py:60-63, 1175-1177)
    task_ids = obs[:, -T:]
    alpha = np.exp(task_ids @ s.log_alpha.reshape(-1, 1))  # (B,1)
    if cfg.use_task_weights:  # extract_task_weights (mtsac.py:103-113)
        la = s.log_alpha
        e = np.exp(-la - np.max(-la))
        sm = e / e.sum()
        tw = (task_ids @ sm.reshape(-1, 1)) * dt(T)
    else:
        tw = None

    # ---------------- critic (mtsac.py:513-621) ----------------
    out_n, _, _ = mh_forward(pa, nobs, cfg.actor_depth, T)
    a_n, logpi_n, _ = tanh_normal_sample(out_n, eps_next, cfg)
    xq_n = np.concatenate([a_n, nobs], axis=1)
    q_t, _ = critic_forward(pt, xq_n, cfg)  # (C,B,1)
    min_next = q_t.min(axis=0) - alpha * logpi_n.reshape(-1, 1)
    y = rew + (dt(1) - dones) * dt(cfg.gamma) * min_next
    xq = np.concatenate([act, obs], axis=1)
    q, caches = critic_forward(pc, xq, cfg)
    if cfg.clip:  # mtsac.py:557-560
        y = np.clip(y, -5000, 5000)
        qc = np.clip(q, -5000, 5000)
        dclip = clip_grad_factor(q, -5000.0, 5000.0)
    else:
        qc = q
        dclip = np.ones_like(q)
    diff = qc - y[None]
    w = tw[None] if tw is not None else dt(1)
    sq = w * diff * diff
    qf_loss = sq.mean()
    qf_values = qc.mean()
    dq = (w * dt(2) * diff / dt(C * B)) * dclip  # d mean / d q
    gc = {}
    for k in range(C):
        hs, t = caches[k]
        g, _ = mh_backward(ens_slice(pc, k), hs, t, dq[k], cfg.critic_depth)
        for n, v in g.items():
            gc.setdefault(n, []).append(v)
    gc = flatten({n: np.stack(v) for n, v in gc.items()}, csh)
    critic_gnorm = global_norm(gc)
    gcc = clip_by_global_norm(gc, cfg.critic_max_grad_norm)
    s.critic = adam_step(s.critic, gcc, s.critic_opt, cfg.critic_lr, cfg.adam_b1, cfg.adam_b2, cfg.adam_eps)
    s.critic_target = dt(cfg.tau) * s.critic + dt(1.0 - cfg.tau) * s.critic_target  # optax.incremental_update
    critic_pnorm = global_norm(s.critic)
    pc_new = unflatten(s.critic, csh)

    # ---------------- actor (mtsac.py:623-711) ----------------
    out_c, hs_a, t_a = mh_forward(pa, obs, cfg.actor_depth, T)
    a_c, logpi_c, pcache = tanh_normal_sample(out_c, eps_cur, cfg)
    xq_pi = np.concatenate([a_c, obs], axis=1)
    q_pi, caches_pi = critic_forward(pc_new, xq_pi, cfg)
    minq = q_pi.min(axis=0)  # (B,1)
    terms = alpha * logpi_c.reshape(-1, 1) - minq
    if tw is not None:
        terms = tw * terms
    actor_loss = terms.mean()
    wb = tw if tw is not None else np.ones((B, 1), dtype=obs.dtype)
    g_logpi = (wb * alpha).reshape(-1) / dt(B)
    dminq = -wb / dt(B)  # (B,1)
    dq_pi = min_grad(q_pi) * dminq[None]
    g_a = np.zeros((B, A), dtype=obs.dtype)
    for k in range(C):
        hs, t = caches_pi[k]
        _, dx = mh_backward(ens_slice(pc_new, k), hs, t, dq_pi[k], cfg.critic_depth, need_dx=True)
        g_a += dx[:, :A]
    dout = tanh_normal_backward(pcache, g_a, g_logpi, cfg)
    ga, _ = mh_backward(pa, hs_a, t_a, dout, cfg.actor_depth)
    ga = flatten(ga, ash)
    actor_gnorm = global_norm(ga)
    gac = clip_by_global_norm(ga, cfg.actor_max_grad_norm)
    s.actor = adam_step(s.actor, gac, s.actor_opt, cfg.actor_lr, cfg.adam_b1, cfg.adam_b2, cfg.adam_eps)
    actor_pnorm = global_norm(s.actor)

    # ---------------- temperature (mtsac.py:713-731) ----------------
    lp = logpi_c.reshape(-1, 1) + dt(cfg.target_entropy)
    la_rows = task_ids @ s.log_alpha.reshape(-1, 1)
    alpha_loss = (-la_rows * lp).mean()
    g_la = (-(task_ids * lp)).sum(axis=0) / dt(B)
    g_la = clip_by_global_norm(g_la, cfg.alpha_max_grad_norm)
    s.log_alpha = adam_step(s.log_alpha, g_la, s.alpha_opt, cfg.alpha_lr, cfg.adam_b1, cfg.adam_b2, cfg.adam_eps)

    logs = {
        "losses/qf_values": float(qf_values),
        "losses/qf_loss": float(qf_loss),
        "metrics/critic_grad_magnitude": critic_gnorm,
        "metrics/critic_params_norm": critic_pnorm,
        "losses/actor_loss": float(actor_loss),
        "metrics/actor_grad_magnitude": actor_gnorm,
        "metrics/actor_params_norm": actor_pnorm,
        "metrics/explore_loss": 0.0,
        "losses/alpha_loss": float(alpha_loss),
        "alpha": float(np.exp(s.log_alpha).sum()),
    }
    if return_internals:
        internals = dict(
            a_next=a_n, logpi_next=logpi_n, q_target=q_t, y=y, q=q, critic_grad=gc,
            a_cur=a_c, logpi_cur=logpi_c, q_pi=q_pi, g_a=g_a, actor_grad=ga, alpha_grad=g_la,
            alpha_rows=alpha,
        )
        return s, logs, internals
    return s, logs


# ----------------------------------------------------------------------------
# rollout-side actions (mtsac.py:70-84) -- §8f row 1
# ----------------------------------------------------------------------------
def eval_action(cfg: OracleConfig, actor_flat: np.ndarray, obs: np.ndarray) -> np.ndarray:
    """``_eval_action``: mode() = tanh(mean) (distributions.py:15-16)."""
    pa = unflatten(actor_flat, actor_leaf_shapes(cfg))
    out, _, _ = mh_forward(pa, obs, cfg.actor_depth, cfg.num_tasks)
    return np.tanh(out[:, : cfg.action_dim])


def sample_action(cfg: OracleConfig, actor_flat: np.ndarray, obs: np.ndarray, eps: np.ndarray) -> np.ndarray:
    pa = unflatten(actor_flat, actor_leaf_shapes(cfg))
    out, _, _ = mh_forward(pa, obs, cfg.actor_depth, cfg.num_tasks)
    a, _, _ = tanh_normal_sample(out, eps, cfg)
    return a
