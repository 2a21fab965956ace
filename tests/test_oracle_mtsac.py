"""The oracle's hand-derived MTSAC backward passes vs an independent torch
autograd derivation (float64), plus the known-answer parameter counts."""

import numpy as np
import pytest

from helpers import synthetic_batch, synthetic_eps
from oracle import mtsac as om


@pytest.mark.parametrize("clip,tw,depth", [(False, False, 3), (True, False, 3), (False, True, 2)])
def test_grads_match_autograd(clip, tw, depth):
    import torch_ref

    T, B = 3, 12
    cfg = om.OracleConfig(num_tasks=T, obs_dim=39 + T, actor_width=16, critic_width=24, clip=clip,
                          use_task_weights=tw, actor_depth=depth, critic_depth=depth)
    st = om.initialize(cfg, seed=3)
    st.log_alpha = np.array([0.1, -0.2, 0.3])
    batch = synthetic_batch(T, B, seed=1)
    en, ec = synthetic_eps(B)
    new, logs, it = om.update(cfg, st, batch, en, ec, return_internals=True)
    gc, ga, gl, ql, al, alo = torch_ref.grads(cfg, st, new.critic, batch, en, ec)
    rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()  # noqa: E731
    assert rel(it["critic_grad"], gc) < 1e-12
    assert rel(it["actor_grad"], ga) < 1e-12
    assert rel(it["alpha_grad"], gl) < 1e-12
    assert abs(logs["losses/qf_loss"] - ql) < 1e-12 * abs(ql)
    assert abs(logs["losses/actor_loss"] - al) < 1e-12 * abs(al)
    assert abs(logs["losses/alpha_loss"] - alo) < 1e-12 + 1e-12 * abs(alo)


def test_finite_difference_critic_grad():
    T, B = 2, 8
    cfg = om.OracleConfig(num_tasks=T, obs_dim=39 + T, actor_width=8, critic_width=8)
    st = om.initialize(cfg, seed=1)
    batch = synthetic_batch(T, B, seed=2)
    en, ec = synthetic_eps(B)
    _, _, it = om.update(cfg, st, batch, en, ec, return_internals=True)
    g = it["critic_grad"]
    rng = np.random.default_rng(0)
    for i in rng.choice(g.size, 12, replace=False):
        for sgn in (1,):
            h = 1e-6
            s1, s2 = st.copy(), st.copy()
            s1.critic[i] += h
            s2.critic[i] -= h
            # target params stay at the original values (stop-gradient through y)
            s1.critic_target = st.critic_target.copy(); s2.critic_target = st.critic_target.copy()
            l1 = om.update(cfg, s1, batch, en, ec)[1]["losses/qf_loss"]
            l2 = om.update(cfg, s2, batch, en, ec)[1]["losses/qf_loss"]
            fd = (l1 - l2) / (2 * h)
            assert abs(fd - g[i]) < 1e-5 * max(1.0, abs(g[i])), (i, fd, g[i])


def test_known_answer_actor_param_counts():
    """figures/fig1_new_mt10.svg '370K', figures/fig1_new_mt50.svg '517K' (W=400)."""
    for T, want in ((10, 372_880), (50, 517_200)):
        cfg = om.OracleConfig(num_tasks=T, obs_dim=39 + T)
        assert om.num_params(om.actor_leaf_shapes(cfg)) == want
    # SURVEY.md §8a a13 counts
    cfg = om.OracleConfig(num_tasks=50, obs_dim=89, actor_width=2048, critic_width=2048)
    assert om.num_params(om.actor_leaf_shapes(cfg)) == 9_396_624
    assert om.num_params(om.critic_leaf_shapes(cfg)) == 17_375_332  # both ensemble members


def test_golden_fixture_reproduces():
    """tests/golden/update_small.npz was written by tests/golden/make_golden.py from this oracle."""
    import pathlib

    p = pathlib.Path(__file__).parent / "golden" / "update_small.npz"
    z = np.load(p, allow_pickle=False)
    cfg = om.OracleConfig(num_tasks=int(z["T"]), obs_dim=int(z["D"]), actor_width=int(z["W"]),
                          critic_width=int(z["W"]))
    st = om.initialize(cfg, seed=int(z["seed"]))
    batch = tuple(z[k] for k in ("obs", "act", "nobs", "done", "rew"))
    new, logs = om.update(cfg, st, batch, z["eps_next"], z["eps_cur"])
    got = np.array([logs[k] for k in om.LOG_KEYS])
    np.testing.assert_allclose(got, z["logs"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(new.actor, z["actor_after"], rtol=1e-12, atol=1e-15)
