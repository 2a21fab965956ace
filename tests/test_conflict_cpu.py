"""Gradient-conflict metrics on CPU: the oracle's per-task gradients against finite differences
of each task's own loss (mtrl/rl/algorithms/mtsac.py:1009-1026, 1055-1074), and the host-side
T x T algebra of mtrl_amd/conflict.py against the oracle's literal restatement of
compute_gram_metrics / compute_support_metrics / compute_conflict_metrics (mtsac.py:733-867,
algorithms/utils.py:49-174), fed with the statistics the device kernels produce (computed here
in numpy from the same float32 gradient matrix)."""

from __future__ import annotations

import numpy as np
import pytest

from helpers import synthetic_batch, synthetic_eps
from mtrl_amd import conflict as mc
from oracle import conflict as oc
from oracle import mtsac as om


def _task_losses(cfg, st, batch, en, ec):
    """Per-task critic and actor losses as functions of flat params (forward only)."""
    obs, act, nobs, dones, rew = batch
    T = cfg.num_tasks
    tasks = np.argmax(obs[:, -T:], axis=1)
    alpha = np.exp(obs[:, -T:] @ st.log_alpha.reshape(-1, 1))
    ash, csh = om.actor_leaf_shapes(cfg), om.critic_leaf_shapes(cfg)

    def critic_loss(t, critic_flat):
        r = np.flatnonzero(tasks == t)
        pa, pc, pt = om.unflatten(st.actor, ash), om.unflatten(critic_flat, csh), om.unflatten(st.critic_target, csh)
        out, _, _ = om.mh_forward(pa, obs[r], cfg.actor_depth, T)
        a_n, lp, _ = om.tanh_normal_sample(out, en[r], cfg)
        qt, _ = om.critic_forward(pt, np.concatenate([a_n, nobs[r]], 1), cfg)
        y = rew[r] + (1 - dones[r]) * cfg.gamma * (qt.min(0) - alpha[r] * lp.reshape(-1, 1))
        q, _ = om.critic_forward(pc, np.concatenate([act[r], obs[r]], 1), cfg)
        return ((q - y[None]) ** 2).mean()

    def actor_loss(t, actor_flat):
        r = np.flatnonzero(tasks == t)
        pa, pc = om.unflatten(actor_flat, ash), om.unflatten(st.critic, csh)
        out, _, _ = om.mh_forward(pa, obs[r], cfg.actor_depth, T)
        a, lp, _ = om.tanh_normal_sample(out, ec[r], cfg)
        q, _ = om.critic_forward(pc, np.concatenate([a, obs[r]], 1), cfg)
        return (alpha[r] * lp.reshape(-1, 1) - q.min(0)).mean()

    return critic_loss, actor_loss


def test_task_grads_match_finite_differences():
    T, W, n = 3, 12, 4
    cfg = om.OracleConfig(num_tasks=T, obs_dim=39 + T, actor_width=W, critic_width=W)
    st = om.initialize(cfg, seed=3)
    st.log_alpha = np.array([0.1, -0.2, 0.3])
    batch = synthetic_batch(T, n * T, seed=4)
    en, ec = synthetic_eps(n * T, seed=5)
    Gc, Ga = oc.task_grads(cfg, st, batch, en, ec)
    assert Gc.shape == (T, st.critic.size) and Ga.shape == (T, st.actor.size)
    cl, al = _task_losses(cfg, st, batch, en, ec)
    rng = np.random.default_rng(0)
    h = 1e-6
    for G, base, loss in ((Gc, st.critic, cl), (Ga, st.actor, al)):
        for t in range(T):
            idx = np.concatenate([rng.choice(base.size, 40, replace=False), np.flatnonzero(G[t])[:10]])
            for k in idx:
                p, m = base.copy(), base.copy()
                p[k] += h
                m[k] -= h
                fd = (loss(t, p) - loss(t, m)) / (2 * h)
                assert abs(fd - G[t, k]) <= 1e-6 * max(1.0, abs(fd)), (t, k, fd, G[t, k])


def test_task_grads_sum_to_the_batch_gradient():
    """Means over tasks compose: sum_t (n/B) grad(loss_t) is the whole-batch actor gradient of
    the update with the same critic (the oracle's update uses the updated critic, so compare
    against a fresh update with critic_lr = 0 and no Polyak motion of the critic)."""
    T, W, n = 4, 10, 3
    cfg = om.OracleConfig(num_tasks=T, obs_dim=39 + T, actor_width=W, critic_width=W, critic_lr=0.0)
    st = om.initialize(cfg, seed=7)
    batch = synthetic_batch(T, n * T, seed=8)
    en, ec = synthetic_eps(n * T, seed=9)
    _, Ga = oc.task_grads(cfg, st, batch, en, ec)
    _, _, internals = om.update(cfg, st, batch, en, ec, return_internals=True)
    np.testing.assert_allclose(Ga.sum(axis=0) * n / (n * T), internals["actor_grad"], rtol=1e-10, atol=1e-14)


def _device_stats(G32: np.ndarray, q=0.8, eps=1e-3, tau=1.0) -> dict:
    """What conflict.hip computes, from a float32 gradient matrix."""
    T, P = G32.shape
    G64 = G32.astype(np.float64)
    lo, hi, lw, hw = mc.quantile_ranks(P, q)
    s = np.sort(np.abs(G32), axis=1)
    thr = (s[:, lo] * lw + s[:, hi] * hw).astype(np.float32)
    sup = np.abs(G32) >= thr[:, None]
    prod = G32[:, None, :] * G32[None, :, :]
    conf = prod < 0
    joint = sup[:, None, :] & sup[None, :, :]
    nz, lg = np.abs(G32) < eps, np.abs(G32) > tau
    return {"gram": G64 @ G64.T, "l1": np.abs(G64).sum(1), "conflict": conf.sum(-1), "intersection": joint.sum(-1),
            "genuine": (joint & conf).sum(-1), "mismatch": (nz[:, None, :] & lg[None, :, :]).sum(-1),
            "near_zero": nz.sum(1), "threshold": thr, "P": P}


def _grad_matrix(T, P, seed):
    rng = np.random.default_rng(seed)
    G = rng.standard_normal((T, P)) * rng.choice([1e-4, 1e-2, 1.0, 3.0], size=(T, P), p=[0.3, 0.3, 0.3, 0.1])
    G[:, rng.choice(P, P // 10, replace=False)] = 0.0  # dead units / other tasks' heads
    G[0, :7] = [1e-4, -1e-4, 2.0, -2.0, 0.0, 5e-4, -0.9]
    return G.astype(np.float32)


@pytest.mark.parametrize("T,P", [(3, 501), (10, 2000), (50, 900)])
def test_host_metrics_match_oracle(T, P):
    G32 = _grad_matrix(T, P, T + P)
    got = mc.metrics_from_stats(_device_stats(G32))
    want = oc.network_metrics(G32.astype(np.float64))
    assert set(got) == set(want) | set()
    for k, v in want.items():
        g = np.asarray(got[k], np.float64)
        w = np.asarray(v, np.float64)
        assert g.shape == w.shape, (k, g.shape, w.shape)
        np.testing.assert_allclose(g, w, rtol=2e-5, atol=1e-6, err_msg=k)


def test_quantile_ranks_follow_jnp_quantile():
    rng = np.random.default_rng(1)
    for P in (2, 5, 17, 1000, 12345):
        x = np.abs(rng.standard_normal(P)).astype(np.float32)
        lo, hi, lw, hw = mc.quantile_ranks(P, 0.8)
        s = np.sort(x)
        assert np.float32(s[lo] * lw + s[hi] * hw) == oc.quantile_f32(x, 0.8)
