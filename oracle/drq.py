"""CPU restatement of the DrQ-eps (distributional dueling DQN + IMPALA CNN) update -- TEST
INFRASTRUCTURE ONLY (the checker for the HIP path in mtrl_amd/csrc/drq*.{hip,cpp}; never shipped,
never measured).  torch float64 on the CPU, gradients by autograd.

Reference (read as text; it cannot run here: jax / flax / optax absent):
  * augment / drq_image_augmentation          mtrl/nn/augmentation.py:36-117
  * ImpalaBlock / ImpalaEncoder                mtrl/nn/impala.py:13-48
  * TaskEmbedding (unit-norm rows)             mtrl/nn/task_embedding.py:5-12
  * DistributionalDense (dueling, LN)          mtrl/rl/networks.py:99-124
  * ImpalaDQN (encoder ++ embed, LN, head)     mtrl/rl/networks.py:127-149 (num_atoms: the module
    default 51 -- DrQ.initialize does not pass the config's 101, drqeps.py:165-171)
  * DrQ._update_inner (C51 projection, CE loss, AdamW, Polyak)  mtrl/rl/algorithms/drqeps.py:268-335
  * optax.adamw via OptimizerConfig.spawn (no clip: max_grad_norm None)  mtrl/config/optim.py:22-40,
    experiments/atari.py:44-52 (lr 1e-4, eps 1.5e-4, weight_decay 0.05)

Parameters travel as ONE flat vector in flax ravel_pytree order (dict keys sorted at every level:
DistributionalDense_0 < ImpalaEncoder_0 < LayerNorm_0 < TaskEmbedding_0; bias < kernel < scale),
see param_spec().  Images are NHWC float (after augment), as the reference's network sees them.

Parity: unpinned (the reference holds no fixtures for this path; JAX threefry for the augmentation
and epsilon-greedy draws is not reproduced -- crop offsets and intensity factors are inputs).
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F


@dataclass(frozen=True)
class DrQConfig:
    num_tasks: int = 26
    n_actions: int = 18
    n_atoms: int = 51
    in_ch: int = 4
    hw: int = 84
    stacks: tuple = (8, 16, 16)
    blocks: int = 2
    scale: int = 1
    embed_dim: int = 32
    n_hidden: int = 512
    gamma: float = 0.99
    nstep: int = 3
    v_min: float = -10.0
    v_max: float = 10.0
    tau: float = 0.005
    lr: float = 1e-4
    b1: float = 0.9
    b2: float = 0.999
    eps: float = 1.5e-4
    weight_decay: float = 0.05
    ln_eps: float = 1e-6


def pool_out(h: int) -> int:
    return (h + 1) // 2  # 3x3 / stride 2 / SAME


def spatial(cfg: DrQConfig):
    """[(H_in, C_in, C_out, H_out)] per IMPALA stack."""
    out, h, c = [], cfg.hw, cfg.in_ch
    for s in cfg.stacks:
        co = cfg.scale * s
        out.append((h, c, co, pool_out(h)))
        h, c = pool_out(h), co
    return out


def feat_dim(cfg: DrQConfig) -> int:
    h, _, co, ho = spatial(cfg)[-1]
    return ho * ho * co


def param_spec(cfg: DrQConfig):
    """(path, shape) in flax ravel_pytree order."""
    F_ = feat_dim(cfg) + cfg.embed_dim
    H = cfg.n_hidden * cfg.scale
    A, Z = cfg.n_actions, cfg.n_atoms
    spec = [
        ("DistributionalDense_0/Dense_0/bias", (H,)), ("DistributionalDense_0/Dense_0/kernel", (F_, H)),
        ("DistributionalDense_0/Dense_1/bias", (A * Z,)), ("DistributionalDense_0/Dense_1/kernel", (H, A * Z)),
        ("DistributionalDense_0/Dense_2/bias", (Z,)), ("DistributionalDense_0/Dense_2/kernel", (H, Z)),
        ("DistributionalDense_0/LayerNorm_0/bias", (H,)), ("DistributionalDense_0/LayerNorm_0/scale", (H,)),
    ]
    for si, (_, ci, co, _) in enumerate(spatial(cfg)):
        for k in range(1 + 2 * cfg.blocks):
            cin = ci if k == 0 else co
            spec += [(f"ImpalaEncoder_0/stack_{si}/Conv_{k}/bias", (co,)),
                     (f"ImpalaEncoder_0/stack_{si}/Conv_{k}/kernel", (3, 3, cin, co))]
    spec += [("LayerNorm_0/bias", (F_,)), ("LayerNorm_0/scale", (F_,)),
             ("TaskEmbedding_0/Embed_0/embedding", (cfg.num_tasks, cfg.embed_dim))]
    return spec


def n_params(cfg: DrQConfig) -> int:
    return sum(int(np.prod(s)) for _, s in param_spec(cfg))


def unflatten(flat, cfg: DrQConfig) -> dict:
    out, o = {}, 0
    for path, shape in param_spec(cfg):
        n = int(np.prod(shape))
        out[path] = flat[o:o + n].reshape(shape)
        o += n
    return out


def initialize(cfg: DrQConfig, seed: int = 0) -> np.ndarray:
    """Initialisers of the reference's modules (flax defaults where none is given): xavier_uniform
    for each stack's first conv and the head's Dense layers, lecun_normal for the residual convs,
    zero biases, LayerNorm scale 1, Embed variance_scaling(1, fan_in, normal).  JAX's threefry
    stream is not reproduced."""
    rng = np.random.default_rng(seed)
    parts = []
    for path, shape in param_spec(cfg):
        leaf = path.rsplit("/", 1)[1]
        if leaf == "bias":
            v = np.zeros(shape)
        elif leaf == "scale":
            v = np.ones(shape)
        elif leaf == "embedding":
            v = rng.normal(0.0, 1.0 / math.sqrt(shape[1]), shape)
        elif "Conv_" in path and not path.endswith("Conv_0/kernel"):  # residual convs: lecun_normal
            z = rng.standard_normal(shape)  # flax lecun_normal: truncated to [-2, 2], rescaled
            while (np.abs(z) > 2.0).any():
                bad = np.abs(z) > 2.0
                z[bad] = rng.standard_normal(int(bad.sum()))
            v = z / math.sqrt(shape[0] * shape[1] * shape[2]) / 0.87962566103423978
        else:  # xavier_uniform
            if len(shape) == 4:
                fan_in, fan_out = shape[0] * shape[1] * shape[2], shape[0] * shape[1] * shape[3]
            else:
                fan_in, fan_out = shape
            lim = math.sqrt(6.0 / (fan_in + fan_out))
            v = rng.uniform(-lim, lim, shape)
        parts.append(np.asarray(v, np.float64).ravel())
    return np.concatenate(parts)


# --------------------------------------------------------------------------- augmentation
def augment(obs_u8: np.ndarray, crop_xy: np.ndarray, noise: np.ndarray, pad: int = 4) -> np.ndarray:
    """augment (augmentation.py:101-117) given its random draws: uint8 NCHW -> [-1, 1] NHWC, edge
    pad by `pad`, crop at per-image offsets (x along H, y along W, in [0, 2 pad)), times the
    per-image intensity factor 1 + 0.05 clip(r, -2, 2) (`noise` = that factor)."""
    x = np.transpose(obs_u8, (0, 2, 3, 1)).astype(np.float32)
    x = (x / np.float32(255.0) - np.float32(0.5)) * np.float32(2.0)
    B, H, W, C = x.shape
    xp = np.pad(x, ((0, 0), (pad, pad), (pad, pad), (0, 0)), mode="edge")
    out = np.empty_like(x)
    for b in range(B):
        ox, oy = int(crop_xy[b, 0]), int(crop_xy[b, 1])
        out[b] = xp[b, ox:ox + H, oy:oy + W, :]
    return out * noise.astype(np.float32)[:, None, None, None]


# --------------------------------------------------------------------------- network
def _conv(x, kernel, bias):
    """flax Conv 3x3, stride 1, SAME on NHWC; kernel (3, 3, Cin, Cout)."""
    y = F.conv2d(x.permute(0, 3, 1, 2), kernel.permute(3, 2, 0, 1), bias, padding=1)
    return y.permute(0, 2, 3, 1)


def _max_pool(x):
    """nn.max_pool((3, 3), strides (2, 2), SAME): -inf padding, lo = total // 2."""
    B, H, W, C = x.shape
    ho = pool_out(H)
    total = max((ho - 1) * 2 + 3 - H, 0)
    lo, hi = total // 2, total - total // 2
    xp = F.pad(x.permute(0, 3, 1, 2), (lo, hi, lo, hi), value=-math.inf)
    return F.max_pool2d(xp, 3, 2).permute(0, 2, 3, 1)


def _layer_norm(x, scale, bias, eps):
    """flax LayerNorm (use_fast_variance): var = max(E[x^2] - E[x]^2, 0)."""
    mu = x.mean(-1, keepdim=True)
    var = torch.clamp((x * x).mean(-1, keepdim=True) - mu * mu, min=0.0)
    return (x - mu) * torch.rsqrt(var + eps) * scale + bias


def forward(p: dict, x: torch.Tensor, task_ids: torch.Tensor, cfg: DrQConfig) -> torch.Tensor:
    """ImpalaDQN.__call__ -> logits [B, A, Z]."""
    for si in range(len(cfg.stacks)):
        g = lambda k, leaf: p[f"ImpalaEncoder_0/stack_{si}/Conv_{k}/{leaf}"]
        c = _max_pool(_conv(x, g(0, "kernel"), g(0, "bias")))
        for b in range(cfg.blocks):
            r = _conv(torch.relu(c), g(1 + 2 * b, "kernel"), g(1 + 2 * b, "bias"))
            c = _conv(torch.relu(r), g(2 + 2 * b, "kernel"), g(2 + 2 * b, "bias")) + c
        x = c
    enc = torch.relu(x).reshape(x.shape[0], -1)  # NHWC flatten (h, w, c)
    emb = p["TaskEmbedding_0/Embed_0/embedding"][task_ids]
    emb = emb / (torch.linalg.norm(emb, dim=-1, keepdim=True) + 1e-8)
    h = torch.cat([enc, emb], -1)
    h = _layer_norm(h, p["LayerNorm_0/scale"], p["LayerNorm_0/bias"], cfg.ln_eps)
    d = "DistributionalDense_0/"
    h = h @ p[d + "Dense_0/kernel"] + p[d + "Dense_0/bias"]
    h = torch.relu(_layer_norm(h, p[d + "LayerNorm_0/scale"], p[d + "LayerNorm_0/bias"], cfg.ln_eps))
    adv = (h @ p[d + "Dense_1/kernel"] + p[d + "Dense_1/bias"]).reshape(-1, cfg.n_actions, cfg.n_atoms)
    val = (h @ p[d + "Dense_2/kernel"] + p[d + "Dense_2/bias"]).reshape(-1, 1, cfg.n_atoms)
    return val + (adv - adv.mean(-2, keepdim=True))


def c51_target(logits_next_online, logits_next_target, rewards, dones, cfg: DrQConfig):
    """m of drqeps.py:273-298: argmax_a of the online expected Q at s', the target net's
    distribution at that action, projected onto the support (the l == u case drops its mass, as
    the reference's two scatter-adds do)."""
    B = logits_next_online.shape[0]
    support = torch.linspace(cfg.v_min, cfg.v_max, cfg.n_atoms, dtype=logits_next_online.dtype)
    q_next = (torch.softmax(logits_next_online, -1) * support).sum(-1)
    a_next = q_next.argmax(-1)
    target_dist = torch.softmax(logits_next_target, -1)[torch.arange(B), a_next]
    tz = torch.clamp(rewards[:, None] + (cfg.gamma ** cfg.nstep) * (1 - dones[:, None]) * support, cfg.v_min, cfg.v_max)
    dz = (cfg.v_max - cfg.v_min) / (cfg.n_atoms - 1)
    b = (tz - cfg.v_min) / dz
    l, u = torch.floor(b).long(), torch.ceil(b).long()
    m = torch.zeros(B, cfg.n_atoms, dtype=b.dtype)
    m.scatter_add_(1, l, target_dist * (u.to(b.dtype) - b))
    m.scatter_add_(1, u, target_dist * (b - l.to(b.dtype)))
    return m, a_next


def _ln_abs_back(a_dy, x, scale, eps):
    """Magnitude rule of the LayerNorm backward: dx = r (g - mean g - xh mean(g xh)), g = dy s,
    so |terms| propagate as r (|g| + mean|g| + |xh| mean(|g| |xh|))."""
    mu = x.mean(-1, keepdim=True)
    r = torch.rsqrt(torch.clamp((x * x).mean(-1, keepdim=True) - mu * mu, min=0.0) + eps)
    xh = ((x - mu) * r).abs()
    g = a_dy * scale.abs()
    return r * (g + g.mean(-1, keepdim=True) + xh * (g * xh).mean(-1, keepdim=True))


def conv_error_floors(cfg: DrQConfig, params: np.ndarray, x, task_ids, actions, m) -> dict:
    """Per conv leaf, the floor an fp32 evaluation of each gradient entry is measured against
    (test infrastructure for the DrQ parity bound).

    A kernel gradient entry sums x_in[b, h+kh-1, w+kw-1, ci] * dy[b, h, w, co] over images and
    pixels; both factors carry the fp32 rounding of the step that produced them, and the entries
    of dy that come out of heavy cancellation carry more error than |dy| suggests.  So the floor
    is the same correlation of the two one-level magnitudes: A(x_in) = |x| for the image,
    conv(|x_prev|, |W|) + |b| for a conv output (window max through the pool, |a| + |b| through
    the residual add), and A(dy) = the |terms| of the step producing dy from the exact upstream
    gradient -- conv-transpose of |dy_next| with |W| under the real ReLU masks, |dc| added through
    the residual, the pool's scatter of |dc|, and the LayerNorm magnitude rule at the encoder
    output.  Deeper rounding is not magnitude-propagated (that bound grows like (sum |W|)^depth);
    a plain GEMM reduces to the tests' sum |a b| bar.  float64 torch, autograd for the exact
    upstream gradients."""
    P = unflatten(torch.as_tensor(params, dtype=torch.float64).clone().requires_grad_(True), cfg)
    B = x.shape[0]
    keep, cs = {}, {}  # conv name -> (input, A(input), output); block outputs c
    with torch.enable_grad():
        h, ah = x, x.abs()
        for si in range(len(cfg.stacks)):
            g = lambda k, leaf: P[f"ImpalaEncoder_0/stack_{si}/Conv_{k}/{leaf}"]

            def conv(xin, axin, k):
                y = _conv(xin, g(k, "kernel"), g(k, "bias"))
                y.retain_grad()
                with torch.no_grad():
                    ay = _conv(xin.detach().abs(), g(k, "kernel").abs(), g(k, "bias").abs())
                keep[f"ImpalaEncoder_0/stack_{si}/Conv_{k}"] = (xin.detach(), axin, y)
                return y, ay

            y, ay = conv(h, ah, 0)
            c = _max_pool(y)
            ac = _max_pool(ay).detach()
            c.retain_grad()
            cs[(si, -1)] = c
            for b in range(cfg.blocks):
                r, ar = conv(torch.relu(c), ac, 1 + 2 * b)
                y2, ay2 = conv(torch.relu(r), ar, 2 + 2 * b)
                ac = ay2 + c.detach().abs()
                c = y2 + c
                c.retain_grad()
                cs[(si, b)] = c
            h, ah = c, ac
        enc = torch.relu(h).reshape(B, -1)
        emb = P["TaskEmbedding_0/Embed_0/embedding"][task_ids]
        emb = emb / (torch.linalg.norm(emb, dim=-1, keepdim=True) + 1e-8)
        f0 = torch.cat([enc, emb], -1)
        f1 = _layer_norm(f0, P["LayerNorm_0/scale"], P["LayerNorm_0/bias"], cfg.ln_eps)
        f1.retain_grad()
        d = "DistributionalDense_0/"
        hh = f1 @ P[d + "Dense_0/kernel"] + P[d + "Dense_0/bias"]
        hh = torch.relu(_layer_norm(hh, P[d + "LayerNorm_0/scale"], P[d + "LayerNorm_0/bias"], cfg.ln_eps))
        adv = (hh @ P[d + "Dense_1/kernel"] + P[d + "Dense_1/bias"]).reshape(-1, cfg.n_actions, cfg.n_atoms)
        val = (hh @ P[d + "Dense_2/kernel"] + P[d + "Dense_2/bias"]).reshape(-1, 1, cfg.n_atoms)
        lg = (val + adv - adv.mean(-2, keepdim=True))[torch.arange(B), actions]
        (-(m * torch.log_softmax(lg, -1)).sum(-1).mean()).backward()
    with torch.no_grad():
        def conv_t(name, a):  # conv-transpose of a magnitude with |W|
            w = P[name + "/kernel"].detach().abs().permute(3, 2, 0, 1)
            return torch.nn.grad.conv2d_input((a.shape[0], w.shape[1], a.shape[1], a.shape[2]), w,
                                              a.permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)

        a_df0 = _ln_abs_back(f1.grad.abs(), f0.detach(), P["LayerNorm_0/scale"].detach(), cfg.ln_eps)
        a_dc = a_df0[:, :enc.shape[1]].reshape(h.shape) * (h.detach() > 0)
        A = {}
        for si in reversed(range(len(cfg.stacks))):
            pre = f"ImpalaEncoder_0/stack_{si}/Conv_"
            for b in reversed(range(cfg.blocks)):
                A[pre + str(2 + 2 * b)] = a_dc  # the block output's gradient is the conv's
                dc = cs[(si, b)].grad.abs()
                A[pre + str(1 + 2 * b)] = conv_t(pre + str(2 + 2 * b), dc) * (keep[pre + str(2 + 2 * b)][0] > 0)
                dr = keep[pre + str(1 + 2 * b)][2].grad.abs()
                a_dc = dc + conv_t(pre + str(1 + 2 * b), dr) * (keep[pre + str(1 + 2 * b)][0] > 0)
            with torch.enable_grad():  # the pool's scatter-add of |dc| (windows overlap)
                y0 = keep[pre + "0"][2].detach().clone().requires_grad_(True)
                (_max_pool(y0) * cs[(si, -1)].grad.abs()).sum().backward()
            A[pre + "0"] = y0.grad
            if si > 0:
                a_dc = conv_t(pre + "0", keep[pre + "0"][2].grad.abs())
        out = {}
        for name, (_, axin, _) in keep.items():
            xa, dy = axin.permute(0, 3, 1, 2), A[name].permute(0, 3, 1, 2)
            w = torch.nn.grad.conv2d_weight(xa, (dy.shape[1], xa.shape[1], 3, 3), dy, padding=1)
            out[name + "/kernel"] = w.permute(2, 3, 1, 0).reshape(-1).numpy()
            out[name + "/bias"] = dy.sum((0, 2, 3)).numpy()
        return out


@dataclass
class DrQState:
    params: np.ndarray
    target: np.ndarray
    mu: np.ndarray
    nu: np.ndarray
    count: int = 0


def init_state(cfg: DrQConfig, seed: int = 0) -> DrQState:
    p = initialize(cfg, seed)
    return DrQState(p.copy(), p.copy(), np.zeros_like(p), np.zeros_like(p), 0)


def update(cfg: DrQConfig, st: DrQState, batch, return_internals: bool = False, dtype=torch.float64):
    """One DrQ._update_inner step (drqeps.py:268-335) on an augmented batch
    (obs NHWC float, actions int, next_obs NHWC float, dones, rewards, task_ids).
    Returns the new state and the LogDict (mean online logit, loss, grad / pre-update param norms).
    dtype=torch.float32 only for the bench's CPU baseline (the reference computes in fp32)."""
    obs, actions, next_obs, dones, rewards, task_ids = batch
    t = lambda a: torch.as_tensor(np.asarray(a)).to(dtype)
    ti = torch.as_tensor(np.asarray(task_ids, np.int64))
    pt = t(st.params).clone().requires_grad_(True)
    with torch.no_grad():
        P = unflatten(t(st.params), cfg)
        T = unflatten(t(st.target), cfg)
        ln_on = forward(P, t(next_obs), ti, cfg)
        ln_tg = forward(T, t(next_obs), ti, cfg)
        m, a_next = c51_target(ln_on, ln_tg, t(rewards), t(dones), cfg)
    B = obs.shape[0]
    logits = forward(unflatten(pt, cfg), t(obs), ti, cfg)[torch.arange(B), torch.as_tensor(np.asarray(actions, np.int64))]
    loss = -(m * torch.log_softmax(logits, -1)).sum(-1).mean()
    loss.backward()
    g = pt.grad.detach().numpy().astype(np.float64)
    # optax.adamw: mu, nu, bias correction, u = -lr (mu_hat / (sqrt(nu_hat) + eps) + wd p)
    count = st.count + 1
    mu = (1 - cfg.b1) * g + cfg.b1 * st.mu
    nu = (1 - cfg.b2) * g * g + cfg.b2 * st.nu
    mh = mu / (1 - cfg.b1 ** count)
    nh = nu / (1 - cfg.b2 ** count)
    p_new = st.params - cfg.lr * (mh / (np.sqrt(nh) + cfg.eps) + cfg.weight_decay * st.params)
    tgt = cfg.tau * p_new + (1 - cfg.tau) * st.target
    logs = {
        "losses/online_logits": float(logits.detach().mean()),
        "metrics/critic_grad_magnitude": float(np.linalg.norm(g)),
        "metrics/critic_params_norm": float(np.linalg.norm(st.params)),
        "losses/critic_loss": float(loss.detach()),
    }
    new = DrQState(p_new, tgt, mu, nu, count)
    if return_internals:
        floors = conv_error_floors(cfg, st.params, torch.as_tensor(np.asarray(obs), dtype=torch.float64), ti,
                                   torch.as_tensor(np.asarray(actions, np.int64)), m.double())
        return new, logs, {"grad": g, "m": m.double().numpy(), "a_next": a_next.numpy(), "conv_abs": floors,
                           "batch": batch}
    return new, logs
