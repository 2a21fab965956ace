"""Independent float64 torch-autograd restatement of the MTSAC losses.

Test helper only: it re-derives the loss functions of ``mtrl/rl/algorithms/mtsac.py``
(critic ``:538-566``, actor ``:631-675``, temperature ``:718-721``) with torch
autograd, so the oracle's hand-written backward passes can be checked against
an independent differentiation.
"""

from __future__ import annotations

import math

import numpy as np
import torch

from oracle import mtsac as om


def _t(x):
    return torch.as_tensor(np.asarray(x), dtype=torch.float64)


def _mh(p, x, depth, T):
    t = torch.argmax(x[:, -T:], dim=1)
    h = x
    for i in range(depth):
        h = torch.relu(h @ p[f"W{i}"] + p[f"b{i}"])
    all_heads = torch.einsum("bw,two->bto", h, p["head_W"]) + p["head_b"][None]
    return all_heads[torch.arange(x.shape[0]), t]


def _params(flat, shapes, requires_grad=False):
    d = om.unflatten(np.asarray(flat, dtype=np.float64), shapes)
    return {k: _t(v).requires_grad_(requires_grad) for k, v in d.items()}


def _sample(out, eps, cfg):
    A = cfg.action_dim
    mu, ls = out[:, :A], out[:, A:]
    ls = torch.clamp(ls, cfg.log_std_min, cfg.log_std_max)
    sigma = torch.exp(ls)
    x = mu + sigma * eps
    a = torch.tanh(x)
    base = (-0.5 * eps**2 - 0.5 * math.log(2 * math.pi) - torch.log(sigma)).sum(1)
    fldj = (2.0 * (math.log(2.0) - x - torch.nn.functional.softplus(-2.0 * x))).sum(1)
    return a, base - fldj


def grads(cfg: om.OracleConfig, state: om.MTSACState, critic_after, batch, eps_next, eps_cur):
    """Return (critic_grad, actor_grad, alpha_grad, qf_loss, actor_loss, alpha_loss)."""
    obs, act, nobs, dones, rew = [_t(b) for b in batch]
    B = obs.shape[0]
    T, C = cfg.num_tasks, cfg.num_critics
    rew, dones = rew.reshape(B, 1), dones.reshape(B, 1)
    ash, csh = om.actor_leaf_shapes(cfg), om.critic_leaf_shapes(cfg)
    la = _t(state.log_alpha)
    tids = obs[:, -T:]
    alpha = torch.exp(tids @ la.reshape(-1, 1))
    w = (tids @ torch.softmax(-la, 0).reshape(-1, 1)) * T if cfg.use_task_weights else torch.ones_like(alpha)

    pa = _params(state.actor, ash)
    pt = _params(state.critic_target, csh)
    pc = _params(state.critic, csh, requires_grad=True)
    with torch.no_grad():
        a_n, lp_n = _sample(_mh(pa, nobs, cfg.actor_depth, T), _t(eps_next), cfg)
        xq_n = torch.cat([a_n, nobs], 1)
        qt = torch.stack([_mh({k: v[c] for k, v in pt.items()}, xq_n, cfg.critic_depth, T) for c in range(C)])
        y = rew + (1 - dones) * cfg.gamma * (qt.min(0).values - alpha * lp_n.reshape(-1, 1))
    xq = torch.cat([act, obs], 1)
    q = torch.stack([_mh({k: v[c] for k, v in pc.items()}, xq, cfg.critic_depth, T) for c in range(C)])
    if cfg.clip:
        y = torch.clamp(y, -5000, 5000)
        q = torch.clamp(q, -5000, 5000)
    qf_loss = (w[None] * (q - y[None]) ** 2).mean()
    qf_loss.backward()
    gc = np.concatenate([pc[k].grad.numpy().reshape(-1) for k, _ in csh])

    pa = _params(state.actor, ash, requires_grad=True)
    pcn = _params(critic_after, csh)
    a_c, lp_c = _sample(_mh(pa, obs, cfg.actor_depth, T), _t(eps_cur), cfg)
    xq_pi = torch.cat([a_c, obs], 1)
    qpi = torch.stack([_mh({k: v[c] for k, v in pcn.items()}, xq_pi, cfg.critic_depth, T) for c in range(C)])
    actor_loss = (w * (alpha * lp_c.reshape(-1, 1) - qpi.min(0).values)).mean()
    actor_loss.backward()
    ga = np.concatenate([pa[k].grad.numpy().reshape(-1) for k, _ in ash])

    lav = la.clone().requires_grad_(True)
    alpha_loss = (-(tids @ lav.reshape(-1, 1)) * (lp_c.detach().reshape(-1, 1) + cfg.target_entropy)).mean()
    alpha_loss.backward()
    return gc, ga, lav.grad.numpy(), float(qf_loss), float(actor_loss), float(alpha_loss)
