"""ORACLE (test infrastructure only) -- numpy restatement of ``MTSAC.compute_weights``.

Only ``tests/`` may import this module, as the checker of ``mtrl_amd.conflict`` and the
engine's per-task gradient pass; the product path never calls it.

Restates, per network:
  * the per-task gradients of ``compute_weights`` (mtrl/rl/algorithms/mtsac.py:870-1090, MSE
    critic branch :1000-1048, actor :1051-1090): tasks split by ``split_data_by_tasks``
    (:313-327, a stable argsort of the task ids), each task's loss a mean over ITS rows, the
    critic's "next" actions sampled from pi(.|s) of the observations (:1000-1004), scored by the
    target critic at s' (:1005-1007); gradients flattened in flax ravel order (:1040-1042);
  * ``compute_gram_metrics`` (:733-771) and ``compute_support_metrics`` (:774-867) with the
    reference's T x T x P broadcasting;
  * ``vmap_cos_sim``, ``compute_sparsity_mismatch``, ``compute_participation_ratio``,
    ``compute_effective_rank``, ``compute_conflict_metrics`` (algorithms/utils.py:49-174).

Parity status: unpinned (as oracle/mtsac.py -- the reference needs jax; its tests pin nothing
here).  Noise is injected per row ([B][A], rows in the batch's order); the reference draws one
(n, A) sample per vmapped task with the same key, which a caller reproduces by repeating it.
"""

from __future__ import annotations

import numpy as np

from . import mtsac as om


def task_grads(cfg: om.OracleConfig, state: om.MTSACState, batch, eps_next: np.ndarray, eps_cur: np.ndarray):
    """(critic [T][Pc], actor [T][Pa]) per-task gradients, float64."""
    obs, act, nobs, dones, rew = [np.asarray(b, np.float64) for b in batch]
    T, A, C = cfg.num_tasks, cfg.action_dim, cfg.num_critics
    B = obs.shape[0]
    ash, csh = om.actor_leaf_shapes(cfg), om.critic_leaf_shapes(cfg)
    pa, pc, pt = om.unflatten(state.actor, ash), om.unflatten(state.critic, csh), om.unflatten(state.critic_target, csh)
    rew, dones = rew.reshape(B, 1), dones.reshape(B, 1)
    task_ids = obs[:, -T:]
    tasks = np.argmax(task_ids, axis=1)
    alpha = np.exp(task_ids @ state.log_alpha.reshape(-1, 1))
    if cfg.use_task_weights:
        la = state.log_alpha
        e = np.exp(-la - np.max(-la))
        tw = (task_ids @ (e / e.sum()).reshape(-1, 1)) * T
    else:
        tw = np.ones((B, 1))
    Gc = np.zeros((T, om.num_params(csh)))
    Ga = np.zeros((T, om.num_params(ash)))
    for t in range(T):
        r = np.flatnonzero(tasks == t)  # split_data_by_tasks: stable order inside the task
        n = r.size
        o, a_, no, d, rw, al, w = obs[r], act[r], nobs[r], dones[r], rew[r], alpha[r], tw[r]
        # critic (mtsac.py:1000-1026): next actions from pi(.|s) -- the reference's quirk
        out, _, _ = om.mh_forward(pa, o, cfg.actor_depth, T)
        a_n, lp_n, _ = om.tanh_normal_sample(out, eps_next[r], cfg)
        q_t, _ = om.critic_forward(pt, np.concatenate([a_n, no], axis=1), cfg)
        y = rw + (1.0 - d) * cfg.gamma * (q_t.min(axis=0) - al * lp_n.reshape(-1, 1))
        q, caches = om.critic_forward(pc, np.concatenate([a_, o], axis=1), cfg)
        if cfg.clip:
            y = np.clip(y, -5000, 5000)
            qc, dclip = np.clip(q, -5000, 5000), om.clip_grad_factor(q, -5000.0, 5000.0)
        else:
            qc, dclip = q, np.ones_like(q)
        dq = w[None] * 2.0 * (qc - y[None]) / (C * n) * dclip
        g = {}
        for k in range(C):
            hs, tt = caches[k]
            gk, _ = om.mh_backward(om.ens_slice(pc, k), hs, tt, dq[k], cfg.critic_depth)
            for nm, v in gk.items():
                g.setdefault(nm, []).append(v)
        Gc[t] = om.flatten({nm: np.stack(v) for nm, v in g.items()}, csh)
        # actor (mtsac.py:1055-1080): the current critic, mean over the task's rows
        out, hs_a, t_a = om.mh_forward(pa, o, cfg.actor_depth, T)
        a_c, lp_c, pcache = om.tanh_normal_sample(out, eps_cur[r], cfg)
        q_pi, caches_pi = om.critic_forward(pc, np.concatenate([a_c, o], axis=1), cfg)
        g_logpi = (w * al).reshape(-1) / n
        dq_pi = om.min_grad(q_pi) * (-w / n)[None]
        g_a = np.zeros((n, A))
        for k in range(C):
            hs, tt = caches_pi[k]
            _, dx = om.mh_backward(om.ens_slice(pc, k), hs, tt, dq_pi[k], cfg.critic_depth, need_dx=True)
            g_a += dx[:, :A]
        dout = om.tanh_normal_backward(pcache, g_a, g_logpi, cfg)
        ga, _ = om.mh_backward(pa, hs_a, t_a, dout, cfg.actor_depth)
        Ga[t] = om.flatten(ga, ash)
    return Gc, Ga


# ---------------------------------------------------------------------------- metrics
def vmap_cos_sim(grads: np.ndarray, T: int):
    """utils.py:49-70 (shape (1, T, T) as the reference's vmap with out_axes=-1)."""
    norms = np.linalg.norm(grads, axis=1)
    cos = np.stack([np.sum(grads[i] * grads, axis=1) / (norms[i] * norms + 1e-8) for i in range(T)], axis=-1)[None]
    mask = np.triu(np.ones((T, T)), k=1)
    return (mask * cos).sum() / (mask.sum() + 1e-8), cos


def compute_sparsity_mismatch(G, eps=1e-3, tau=1.0):
    T = G.shape[0]
    nz, lg = np.abs(G) < eps, np.abs(G) > tau
    mismatch = nz[:, None, :] & lg[None, :, :]
    return mismatch.sum(axis=-1) / np.maximum(nz.sum(axis=1), 1)[:, None] * (1 - np.eye(T))


def compute_participation_ratio(G):
    return np.abs(G).sum(axis=1) ** 2 / (G.shape[1] * np.maximum((G ** 2).sum(axis=1), 1e-10))


def compute_effective_rank(G):
    sv = np.linalg.svd(G @ G.T, compute_uv=False)
    d = sv / max(sv.sum(), 1e-10)
    return np.exp(-(d * np.log(d + 1e-10)).sum())


def compute_conflict_metrics(cos, G, eps=1e-3, tau=1.0):
    T = G.shape[0]
    off = 1 - np.eye(T)
    cm = (cos < 0).astype(np.float64)
    n_off = T * (T - 1)
    mags = np.linalg.norm(G, axis=1)
    outer = mags[:, None] * mags[None, :]
    conf_mag = np.where((cm * off).astype(bool), np.abs(cos) * outer, 0.0)
    angles = np.degrees(np.arccos(np.clip(cos, -1.0, 1.0)))
    ir = compute_sparsity_mismatch(G, eps, tau)
    pr = compute_participation_ratio(G)
    return {
        "conflict_rate": (cm * off).sum() / n_off,
        "mean_conflict_magnitude": (conf_mag * off).sum() / n_off,
        "mean_conflict_angle": (angles * off).sum() / n_off,
        "per_task_conflict_rate": (cm * off).sum(axis=1) / (T - 1),
        "per_task_grad_magnitude": mags,
        "pairwise_conflict": cm,
        "pairwise_cos_sim": cos,
        "pairwise_angle": angles,
        "avg_interference_rate": (ir * off).sum() / n_off,
        "interference_asymmetry": (np.abs(ir - ir.T) * off).sum() / n_off,
        "per_task_interference_in": (ir * off).sum(axis=0) / (T - 1),
        "per_task_interference_out": (ir * off).sum(axis=1) / (T - 1),
        "pairwise_interference_rate": ir,
        "avg_participation_ratio": pr.mean(),
        "per_task_participation_ratio": pr,
        "effective_rank": compute_effective_rank(G),
    }


def compute_gram_metrics(G, T):
    gram = G @ G.T
    norms = np.sqrt(np.diag(gram))
    cg = gram / (np.outer(norms, norms) + 1e-8)
    mask = 1.0 - np.eye(T)
    n = T * (T - 1)
    mean = (gram * mask).sum() / n
    return {"gram": gram, "cosine_from_gram": cg, "avg_cosine_gram": (cg * mask).sum() / n, "gram_diag": np.diag(gram),
            "gram_off_diag_mean": mean, "gram_off_diag_std": np.sqrt((((gram - mean) ** 2) * mask).sum() / n)}


def quantile_f32(x: np.ndarray, q: float) -> np.float32:
    """jnp.quantile(x, q) ('linear', x64 off): float32 index arithmetic and interpolation."""
    n = x.size
    pos = np.float32(q) * np.float32(n - 1)
    lo, hi = np.floor(pos), np.ceil(pos)
    hw = np.float32(pos - lo)
    s = np.sort(x.astype(np.float32))
    return np.float32(s[int(lo)] * (np.float32(1) - hw) + s[int(hi)] * hw)


def compute_support_metrics(G, T, support_percentile=0.8):
    Gf = G.astype(np.float32)
    thr = np.array([quantile_f32(np.abs(Gf[t]), support_percentile) for t in range(T)], np.float32)[:, None]
    sup = np.abs(Gf) >= thr
    si, sj = sup[:, None, :], sup[None, :, :]
    inter = (si & sj).sum(axis=-1).astype(np.float64)
    union = (si | sj).sum(axis=-1).astype(np.float64)
    jac = inter / (union + 1e-8)
    mask = 1.0 - np.eye(T)
    n = T * (T - 1)
    sc = (Gf[:, None, :] * Gf[None, :, :]) < 0
    joint = si & sj
    genuine = (joint & sc).sum(axis=-1).astype(np.float64)
    ghost = (~joint & sc).sum(axis=-1).astype(np.float64)
    tot = genuine + ghost + 1e-8
    size = sup.sum(axis=-1).astype(np.float64)
    return {"thresholds": thr[:, 0], "supports": sup, "pairwise_jaccard": jac, "avg_jaccard": (jac * mask).sum() / n,
            "genuine_conflict_count": genuine, "ghost_conflict_count": ghost, "genuine_conflict_rate": genuine / tot,
            "ghost_conflict_rate": ghost / tot, "avg_genuine_conflict_rate": (genuine / tot * mask).sum() / n,
            "avg_ghost_conflict_rate": (ghost / tot * mask).sum() / n,
            "ghost_to_genuine_ratio": ghost.sum() / (genuine.sum() + 1e-8), "per_task_support_size": size,
            "avg_support_size": size.mean()}


def network_metrics(G: np.ndarray, support_percentile=0.8, eps=1e-3, tau=1.0) -> dict:
    """One network's entries of compute_weights' log dict (mtsac.py:1040-1048, 1093-1170),
    keyed without the critic_ / actor_ prefix."""
    T = G.shape[0]
    avg_cos, cos = vmap_cos_sim(G, T)
    cm = compute_conflict_metrics(cos, G, eps, tau)
    gm = compute_gram_metrics(G, T)
    sm = compute_support_metrics(G, T, support_percentile)
    out = {"avg_cos_sim": avg_cos, "avg_grad_magnitude": np.linalg.norm(G, axis=1).mean()}
    out.update(cm)
    out.update({"avg_cosine_gram": gm["avg_cosine_gram"], "gram_diag": gm["gram_diag"],
                "gram_off_diag_mean": gm["gram_off_diag_mean"], "gram_off_diag_std": gm["gram_off_diag_std"],
                "pairwise_gram": gm["gram"], "pairwise_cosine_gram": gm["cosine_from_gram"],
                "avg_jaccard": sm["avg_jaccard"], "pairwise_jaccard": sm["pairwise_jaccard"],
                "avg_genuine_conflict_rate": sm["avg_genuine_conflict_rate"],
                "avg_ghost_conflict_rate": sm["avg_ghost_conflict_rate"],
                "ghost_to_genuine_ratio": sm["ghost_to_genuine_ratio"],
                "per_task_support_size": sm["per_task_support_size"], "avg_support_size": sm["avg_support_size"],
                "pairwise_genuine_conflict_rate": sm["genuine_conflict_rate"],
                "pairwise_ghost_conflict_rate": sm["ghost_conflict_rate"]})
    return out
