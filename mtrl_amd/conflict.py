"""Eval-time gradient-conflict metrics of ``MTSAC.compute_weights`` on the HIP engine.

Reference: ``mtrl/rl/algorithms/mtsac.py:870-1170`` (``compute_weights``, ``compute_gram_metrics``
:733-771, ``compute_support_metrics`` :774-867) and ``mtrl/rl/algorithms/utils.py:49-174``
(``vmap_cos_sim``, ``compute_sparsity_mismatch``, ``compute_participation_ratio``,
``compute_effective_rank``, ``compute_conflict_metrics``).

Every O(T^2 P) reduction over the T x P per-task gradient matrix runs on the GPU
(``mtsac_task_gradients`` / ``_select`` / ``_stats``, conflict.hip): Gram matrix, sign-conflict
counts, support intersections, genuine conflicts, sparsity mismatch, L1 norms and the two order
statistics of each task's support quantile.  What is left here is the reference's T x T algebra,
restated on those statistics (float64, returned as float32 like the reference's float32 arrays).
Log keys, shapes and formulas follow ``compute_weights``'s return dict (mtsac.py:1093-1170).
"""

from __future__ import annotations

import numpy as np

CRITIC, ACTOR = 0, 1


def quantile_ranks(P: int, q: float):
    """``jnp.quantile(..., method='linear')`` index arithmetic (x64 off: float32):
    position q (P - 1), floor / ceil ranks and their weights."""
    pos = np.float32(q) * np.float32(P - 1)
    low, high = np.floor(pos), np.ceil(pos)
    hw = np.float32(pos - low)
    lw = np.float32(1.0) - hw
    low = int(min(max(low, 0), P - 1))
    high = int(min(max(high, 0), P - 1))
    return low, high, lw, hw


def network_stats(engine, which: int, support_percentile: float = 0.8, eps: float = 1e-3, tau: float = 1.0) -> dict:
    """Device statistics of one network's per-task gradients (after ``engine.task_gradients``)."""
    T = engine.T_l
    P = engine.task_gradient_size(which)
    low, high, lw, hw = quantile_ranks(P, support_percentile)
    v = engine.task_gradient_select(which, np.tile([low, high], (T, 1)))
    thr = (v[:, 0] * lw + v[:, 1] * hw).astype(np.float32)  # low_value * low_weight + high_value * high_weight
    st = engine.task_gradient_stats(which, thr, eps, tau)
    st["threshold"] = thr
    st["P"] = P
    return st


def conflict_metrics_from_stats(st: dict) -> dict:
    """vmap_cos_sim + compute_conflict_metrics (utils.py:49-174) from the Gram matrix, L1 norms,
    near-zero counts and sparsity-mismatch counts of a [T][P] gradient matrix (float64)."""
    gram = np.asarray(st["gram"], np.float64)
    T = gram.shape[0]
    P = int(st["P"])
    eye = np.eye(T)
    off = 1.0 - eye
    n_pairs = T * (T - 1)
    norms = np.sqrt(np.maximum(np.diag(gram), 0.0))

    # vmap_cos_sim (utils.py:49-70): cos[0, j, i] = g_i . g_j / (|g_i| |g_j| + 1e-8), upper-triangle mean
    cos = gram / (np.outer(norms, norms) + 1e-8)
    cos_sim_mat = cos.T[None]
    triu = np.triu(np.ones((T, T)), k=1)
    avg_cos_sim = (triu * cos_sim_mat).sum() / (triu.sum() + 1e-8)

    # compute_conflict_metrics (utils.py:116-174)
    conflict_mask = (cos_sim_mat < 0).astype(np.float64)
    conflict_rate = (conflict_mask * off).sum() / n_pairs
    outer_mag = norms[:, None] * norms[None, :]
    conflict_magnitude = np.where((conflict_mask * off).astype(bool), np.abs(cos_sim_mat) * outer_mag, 0.0)
    mean_conflict_magnitude = (conflict_magnitude * off).sum() / n_pairs
    angles = np.degrees(np.arccos(np.clip(cos_sim_mat, -1.0, 1.0)))
    mean_conflict_angle = (angles * off).sum() / n_pairs
    per_task_conflict_rate = (conflict_mask * off).sum(axis=1) / (T - 1)
    near_zero = np.maximum(np.asarray(st["near_zero"], np.float64), 1.0)
    interference = np.asarray(st["mismatch"], np.float64) / near_zero[:, None] * off
    avg_interference_rate = (interference * off).sum() / n_pairs
    asymmetry = (np.abs(interference - interference.T) * off).sum() / n_pairs
    per_task_in = (interference * off).sum(axis=0) / (T - 1)
    per_task_out = (interference * off).sum(axis=1) / (T - 1)
    l1 = np.asarray(st["l1"], np.float64)
    participation = l1 ** 2 / (P * np.maximum(np.diag(gram), 1e-10))
    sv = np.linalg.svd(gram, compute_uv=False)
    sv_dist = sv / max(sv.sum(), 1e-10)
    effective_rank = float(np.exp(-(sv_dist * np.log(sv_dist + 1e-10)).sum()))
    f = np.float32
    return {
        "avg_cos_sim": f(avg_cos_sim),
        "avg_grad_magnitude": f(norms.mean()),
        "conflict_rate": f(conflict_rate),
        "mean_conflict_magnitude": f(mean_conflict_magnitude),
        "mean_conflict_angle": f(mean_conflict_angle),
        "per_task_conflict_rate": per_task_conflict_rate.astype(f),
        "per_task_grad_magnitude": norms.astype(f),
        "pairwise_conflict": conflict_mask.astype(f),
        "pairwise_cos_sim": cos_sim_mat.astype(f),
        "pairwise_angle": angles.astype(f),
        "avg_interference_rate": f(avg_interference_rate),
        "interference_asymmetry": f(asymmetry),
        "per_task_interference_in": per_task_in.astype(f),
        "per_task_interference_out": per_task_out.astype(f),
        "pairwise_interference_rate": interference.astype(f),
        "avg_participation_ratio": f(participation.mean()),
        "per_task_participation_ratio": participation.astype(f),
        "effective_rank": f(effective_rank),
    }


def matrix_stats(flat: np.ndarray, eps: float = 1e-3, tau: float = 1.0) -> dict:
    """The statistics conflict_metrics_from_stats takes, from a small [T][P] matrix on the host
    (DrQ's projected gradients, T x 10 000)."""
    g = np.asarray(flat, np.float64)
    a = np.abs(np.asarray(flat, np.float32))
    near = (a < np.float32(eps)).astype(np.float64)
    large = (a > np.float32(tau)).astype(np.float64)
    return {"gram": g @ g.T, "l1": a.astype(np.float64).sum(1), "near_zero": near.sum(1), "mismatch": near @ large.T,
            "P": g.shape[1]}


def metrics_from_stats(st: dict) -> dict:
    """The reference's per-network metrics from the device statistics."""
    out = conflict_metrics_from_stats(st)
    gram = np.asarray(st["gram"], np.float64)
    T = gram.shape[0]
    off = 1.0 - np.eye(T)
    n_pairs = T * (T - 1)
    norms = np.sqrt(np.maximum(np.diag(gram), 0.0))

    # compute_gram_metrics (mtsac.py:733-771)
    cosine_from_gram = gram / (np.outer(norms, norms) + 1e-8)
    avg_cosine_gram = (cosine_from_gram * off).sum() / n_pairs
    gram_off_mean = (gram * off).sum() / n_pairs
    gram_off_std = np.sqrt((((gram - gram_off_mean) ** 2) * off).sum() / n_pairs)

    # compute_support_metrics (mtsac.py:774-867)
    inter = np.asarray(st["intersection"], np.float64)
    size = np.diag(inter).copy()
    union = size[:, None] + size[None, :] - inter
    jaccard = inter / (union + 1e-8)
    avg_jaccard = (jaccard * off).sum() / n_pairs
    genuine = np.asarray(st["genuine"], np.float64)
    ghost = np.asarray(st["conflict"], np.float64) - genuine
    total = genuine + ghost + 1e-8
    genuine_rate, ghost_rate = genuine / total, ghost / total
    f = np.float32
    return {
        **out,
        "avg_cosine_gram": f(avg_cosine_gram),
        "gram_diag": np.diag(gram).astype(f),
        "gram_off_diag_mean": f(gram_off_mean),
        "gram_off_diag_std": f(gram_off_std),
        "pairwise_gram": gram.astype(f),
        "pairwise_cosine_gram": cosine_from_gram.astype(f),
        "avg_jaccard": f(avg_jaccard),
        "pairwise_jaccard": jaccard.astype(f),
        "avg_genuine_conflict_rate": f((genuine_rate * off).sum() / n_pairs),
        "avg_ghost_conflict_rate": f((ghost_rate * off).sum() / n_pairs),
        "ghost_to_genuine_ratio": f(ghost.sum() / (genuine.sum() + 1e-8)),
        "per_task_support_size": size.astype(f),
        "avg_support_size": f(size.mean()),
        "pairwise_genuine_conflict_rate": genuine_rate.astype(f),
        "pairwise_ghost_conflict_rate": ghost_rate.astype(f),
    }


# compute_weights' log keys (mtsac.py:1093-1170) -> the per-network metric they carry
_KEYS = ("avg_cos_sim", "avg_grad_magnitude", "conflict_rate", "mean_conflict_magnitude", "mean_conflict_angle",
         "per_task_conflict_rate", "per_task_grad_magnitude", "pairwise_conflict", "pairwise_cos_sim",
         "pairwise_angle", "avg_interference_rate", "interference_asymmetry", "per_task_interference_in",
         "per_task_interference_out", "pairwise_interference_rate", "avg_participation_ratio",
         "per_task_participation_ratio", "effective_rank", "avg_cosine_gram", "gram_diag", "gram_off_diag_mean",
         "gram_off_diag_std", "pairwise_gram", "pairwise_cosine_gram", "avg_jaccard", "pairwise_jaccard",
         "avg_genuine_conflict_rate", "avg_ghost_conflict_rate", "ghost_to_genuine_ratio", "per_task_support_size",
         "avg_support_size", "pairwise_genuine_conflict_rate", "pairwise_ghost_conflict_rate")


def compute_weights(engine, batch=None, eps_next=None, eps_cur=None, support_percentile: float = 0.8,
                    eps: float = 1e-3, tau: float = 1.0) -> dict:
    """``MTSAC.compute_weights`` logs: per-task gradients on the device, then every metric.
    ``batch`` = (obs, actions, next_obs, dones, rewards) rows interleaved i*T + t (None: sample
    on the device); eps_next / eps_cur: injected [B][A] noise or None."""
    engine.task_gradients(batch, eps_next, eps_cur)
    logs = {}
    for net, which in (("critic", CRITIC), ("actor", ACTOR)):
        m = metrics_from_stats(network_stats(engine, which, support_percentile, eps, tau))
        for k in _KEYS:
            logs[f"{net}_{k}"] = m[k]
    return logs
