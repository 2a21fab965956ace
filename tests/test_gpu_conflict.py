"""Gradient-conflict metrics on the GPU (MTSAC.compute_weights, mtrl/rl/algorithms/mtsac.py:870-1170).

* the engine's per-task gradients (mtsac_task_gradients) against the float64 oracle
  (oracle/conflict.py), both precisions, with task weights and clip;
* the device statistics (mtsac_task_gradient_select / _stats, conflict.hip) against numpy on
  the SAME float32 matrix: order statistics and every count exact, the Gram matrix and L1 norms
  to fp32-accumulation accuracy;
* compute_weights end to end (mtrl_amd/conflict.py) against the oracle's literal metrics on the
  engine's own gradients, every log key and shape;
* a full-size run (MT10/W400, B = 1280) and the unsharded-only contract.
"""

from __future__ import annotations

import numpy as np
import pytest

from helpers import synthetic_batch, synthetic_eps
from oracle import conflict as oc
from oracle import mtsac as om

pytestmark = pytest.mark.gpu


def _setup(T, W, n, precision, clip=False, tw=False, depth=3, seed=21):
    from mtrl_amd import _lib as L
    from mtrl_amd.engine import MTSACEngine, make_config

    cfg = om.OracleConfig(num_tasks=T, obs_dim=39 + T, actor_width=W, critic_width=W, actor_depth=depth,
                          critic_depth=depth, clip=clip, use_task_weights=tw)
    st = om.initialize(cfg, seed=seed)
    st.log_alpha = np.random.default_rng(seed).uniform(-0.3, 0.3, T)
    st.critic_target = st.critic + np.random.default_rng(seed + 1).normal(0, 1e-3, st.critic.size)
    for k in ("actor", "critic", "critic_target", "log_alpha"):
        setattr(st, k, getattr(st, k).astype(np.float32).astype(np.float64))
    e = MTSACEngine(make_config(num_tasks=T, task_count=T, obs_dim=39 + T, actor_width=W, critic_width=W,
                                actor_depth=depth, critic_depth=depth, batch_per_task=n, capacity=max(n, 64),
                                clip=int(clip), use_task_weights=int(tw), precision=precision))
    e.set_params(L.ACTOR, st.actor)
    e.set_params(L.CRITIC, st.critic)
    e.set_params(L.CRITIC_TARGET, st.critic_target)
    e.set_params(L.LOG_ALPHA, st.log_alpha)
    B = n * T
    batch = synthetic_batch(T, B, seed=seed + 2, dtype=np.float32)
    en, ec = synthetic_eps(B, seed=seed + 3, dtype=np.float32)
    return cfg, st, e, batch, en, ec


@pytest.mark.parametrize("precision", [0, 1], ids=["fp32", "split3"])
@pytest.mark.parametrize("T,W,n,clip,tw", [(3, 32, 4, False, False), (5, 64, 8, True, True), (10, 128, 16, False, False)],
                         ids=["t3", "t5_clip_tw", "t10"])
def test_task_gradients_match_oracle(T, W, n, clip, tw, precision):
    cfg, st, e, batch, en, ec = _setup(T, W, n, precision, clip, tw)
    e.task_gradients(batch, en, ec)
    Gc, Ga = oc.task_grads(cfg, st, [b.astype(np.float64) for b in batch], en.astype(np.float64),
                           ec.astype(np.float64))
    for which, want in ((0, Gc), (1, Ga)):
        got = e.get_task_gradients(which).astype(np.float64)
        assert got.shape == want.shape
        for t in range(T):
            scale = np.abs(want[t]).max()
            err = np.abs(got[t] - want[t]).max()
            assert err <= 1e-5 * scale, (which, t, err, scale)
    e.close()


def _numpy_stats(G32, thr, eps, tau):
    G64 = G32.astype(np.float64)
    sup = np.abs(G32) >= thr[:, None]
    conf = (G32[:, None, :] * G32[None, :, :]) < 0
    joint = sup[:, None, :] & sup[None, :, :]
    nz, lg = np.abs(G32) < eps, np.abs(G32) > tau
    return {"gram": G64 @ G64.T, "l1": np.abs(G64).sum(1), "conflict": conf.sum(-1), "intersection": joint.sum(-1),
            "genuine": (joint & conf).sum(-1), "mismatch": (nz[:, None, :] & lg[None, :, :]).sum(-1),
            "near_zero": nz.sum(1)}


@pytest.mark.parametrize("T", [3, 10, 50])
def test_device_statistics_exact(T):
    from mtrl_amd import conflict as mc

    W = 32 if T == 50 else 64
    cfg, st, e, *_ = _setup(T, W, 2, 1)
    P = e.task_gradient_size(0)
    rng = np.random.default_rng(T)
    G = (rng.standard_normal((T, P)) * rng.choice([1e-4, 1e-2, 1.0, 3.0], size=(T, P))).astype(np.float32)
    G[:, rng.choice(P, P // 7, replace=False)] = 0.0
    G[0, :4] = [np.float32(1e-30), np.float32(-1e-30), 2.0, -2.0]
    e.set_task_gradients(0, G)
    lo, hi, lw, hw = mc.quantile_ranks(P, 0.8)
    ranks = np.tile([lo, hi], (T, 1))
    v = e.task_gradient_select(0, ranks)
    s = np.sort(np.abs(G), axis=1)
    np.testing.assert_array_equal(v[:, 0], s[:, lo])
    np.testing.assert_array_equal(v[:, 1], s[:, hi])
    v2 = e.task_gradient_select(0, np.tile([0, P - 1], (T, 1)))  # extremes
    np.testing.assert_array_equal(v2, np.stack([s[:, 0], s[:, -1]], 1))
    thr = (v[:, 0] * lw + v[:, 1] * hw).astype(np.float32)
    got = e.task_gradient_stats(0, thr, 1e-3, 1.0)
    want = _numpy_stats(G, thr, 1e-3, 1.0)
    for k in ("conflict", "intersection", "genuine", "mismatch", "near_zero"):
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    np.testing.assert_allclose(got["gram"], want["gram"], rtol=2e-6, atol=1e-6 * np.abs(want["gram"]).max())
    np.testing.assert_allclose(got["l1"], want["l1"], rtol=2e-6)
    e.close()


def test_compute_weights_matches_oracle_metrics():
    from mtrl_amd import conflict as mc

    T, W, n = 6, 64, 8
    cfg, st, e, batch, en, ec = _setup(T, W, n, 1)
    logs = mc.compute_weights(e, batch, en, ec)
    for net, which in (("critic", 0), ("actor", 1)):
        G = e.get_task_gradients(which).astype(np.float64)
        want = oc.network_metrics(G)
        for k, v in want.items():
            g = np.asarray(logs[f"{net}_{k}"], np.float64)
            assert g.shape == np.shape(v), (net, k, g.shape, np.shape(v))
            np.testing.assert_allclose(g, v, rtol=2e-5, atol=1e-6, err_msg=f"{net}_{k}")
    assert len(logs) == 66  # compute_weights' 66 keys (mtsac.py:1093-1170)
    e.close()


def test_full_size_mt10_w400_device_sampled():
    from mtrl_amd import conflict as mc
    from mtrl_amd import _lib as L
    from mtrl_amd.engine import MTSACEngine, make_config
    from mtrl_amd.init import init_mtsac

    T, W = 10, 400
    e = MTSACEngine(make_config(num_tasks=T, task_count=T, obs_dim=39 + T, actor_width=W, critic_width=W,
                                batch_per_task=128, capacity=1000, precision=1))
    a, q = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=1)
    e.set_params(L.ACTOR, a)
    e.set_params(L.CRITIC, q)
    e.set_params(L.CRITIC_TARGET, q)
    e.buffer_fill_synthetic(7)
    e.seed_rng(1)
    logs = mc.compute_weights(e)  # device batch + device noise
    assert logs["critic_pairwise_gram"].shape == (T, T) and logs["actor_pairwise_cos_sim"].shape == (1, T, T)
    assert all(np.all(np.isfinite(v)) for v in logs.values())
    assert 0 < logs["critic_avg_support_size"] <= e.task_gradient_size(0)
    e.close()


def test_sharded_engine_refuses():
    from mtrl_amd.engine import MTSACEngine, make_config
    from mtrl_amd._lib import MTSACError

    e = MTSACEngine(make_config(num_tasks=4, task_begin=2, task_count=2, obs_dim=43, actor_width=32, critic_width=32,
                                batch_per_task=4, capacity=64, precision=1))
    with pytest.raises(MTSACError):
        e.task_gradients()
    e.close()
