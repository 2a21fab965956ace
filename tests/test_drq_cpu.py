"""DrQ-eps path on CPU: the oracle's pieces against independent restatements (max-pool SAME
padding, C51 projection mass, LayerNorm), the product-side parameter layout (mtrl_amd/drq_init.py)
against the oracle's flax ravel order, and the compat API surface (mtrl.rl.algorithms.DrQConfig,
experiments/atari.py's config tree)."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import drq as od


def test_param_layout_matches_oracle():
    from mtrl_amd.drq_init import init_drq, param_spec

    cfg = od.DrQConfig()
    assert param_spec() == od.param_spec(cfg)
    assert od.n_params(cfg) == 1535697 == init_drq(3).size
    small = od.DrQConfig(hw=20, n_hidden=64, scale=1)
    assert param_spec(hw=20, n_hidden=64) == od.param_spec(small)


def test_max_pool_same_padding():
    x = torch.arange(2 * 5 * 5 * 3, dtype=torch.float64).reshape(2, 5, 5, 3) * ((-1) ** torch.arange(150).reshape(2, 5, 5, 3))
    y = od._max_pool(x)
    assert y.shape == (2, 3, 3, 3)
    # SAME for 5 -> 3 with k 3 / s 2: total pad 2, lo 1: window rows of output 0 are -1..1
    xn = x.numpy()
    for b in range(2):
        for oy in range(3):
            for ox in range(3):
                ys, xs = slice(max(2 * oy - 1, 0), 2 * oy + 2), slice(max(2 * ox - 1, 0), 2 * ox + 2)
                np.testing.assert_array_equal(y[b, oy, ox].numpy(), xn[b, ys, xs].reshape(-1, 3).max(0))


def test_c51_projection_conserves_mass_off_the_grid():
    cfg = od.DrQConfig()
    B = 6
    lo = torch.randn(B, cfg.n_actions, cfg.n_atoms, dtype=torch.float64)
    lt = torch.randn(B, cfg.n_actions, cfg.n_atoms, dtype=torch.float64)
    rew = torch.tensor([0.013, -0.17, 0.21, 0.5, 0.0, 0.05], dtype=torch.float64)
    done = torch.tensor([0.0, 0.0, 0.0, 1.0, 1.0, 0.0], dtype=torch.float64)
    m, _ = od.c51_target(lo, lt, rew, done, cfg)
    s = m.sum(-1).numpy()
    # unclipped off-grid targets keep their mass; a terminal reward on an atom (0.0 -> b = 25
    # exactly) drops it, as the reference's two scatter-adds do (l == u: (u - b) = (b - l) = 0)
    np.testing.assert_allclose(s[[0, 1, 2, 3, 5]], 1.0, rtol=1e-12)
    assert abs(s[4]) < 1e-15


def test_compat_config_tree():
    import mtrl  # noqa: F401
    from mtrl.config.networks import ImpalaDQNConfig, QValueFunctionConfig
    from mtrl.config.nn import ImpalaEncoderConfig, VanillaNetworkConfig
    from mtrl.config.optim import OptimizerConfig
    from mtrl.config.rl import DrQTrainingConfig
    from mtrl.config.utils import Optimizer
    from mtrl.envs import AtariConfig
    from mtrl.rl.algorithms import DrQ, DrQConfig, get_algorithm_for_config

    c = DrQConfig(num_tasks=26, gamma=0.99, critic_config=ImpalaDQNConfig(
        impala_config=ImpalaEncoderConfig(scale=1),
        q_function_config=QValueFunctionConfig(use_classification=True, num_atoms=101, network_config=VanillaNetworkConfig(
            optimizer=OptimizerConfig(lr=1e-4, optimizer=Optimizer.AdamW, eps=1.5e-4, weight_decay=0.05)))))
    assert get_algorithm_for_config(c) is DrQ
    assert (c.n_atoms, c.v_min, c.v_max, c.tau, c.eps_decay_steps) == (51, -10.0, 10.0, 0.005, 5000)
    t = DrQTrainingConfig(total_steps=26 * 100_000, normalize_rewards=True, buffer_size=26 * 100_000)
    assert (t.batch_size, t.nstep, t.replay_ratio) == (256, 3, 2)
    env = AtariConfig()
    assert env.observation_space.shape == (4, 84, 84) and env.action_space.n == 18


def test_residual_convs_use_truncated_lecun_normal():
    """flax Conv's default kernel init (impala.py:27,29): truncated normal on [-2, 2] std units,
    variance 1 / fan_in."""
    from mtrl_amd.drq_init import truncated_lecun_normal

    fan = 3 * 3 * 16
    v = truncated_lecun_normal(np.random.default_rng(0), (200_000,), fan)
    lim = 2.0 / np.sqrt(fan) / 0.87962566103423978
    assert np.abs(v).max() <= lim and np.abs(v).max() > 0.99 * lim
    assert abs(v.var() * fan - 1.0) < 0.01


def test_optimizer_settings_follow_optimizer_config_spawn():
    """config/optim.py:26-43: Adam gets eps 1e-5 and no decay, AdamW optax's defaults unless set;
    what the AdamW kernel cannot run (a clip link, RMSProp) is refused, not silently replaced."""
    import mtrl  # noqa: F401
    from mtrl.config.optim import OptimizerConfig
    from mtrl.config.utils import Optimizer
    from mtrl_amd.compat.rl.algorithms.drqeps import _adam_settings

    assert _adam_settings(OptimizerConfig()) == (1e-5, 0.0)
    assert _adam_settings(OptimizerConfig(eps=1e-3, weight_decay=0.5)) == (1e-3, 0.0)
    assert _adam_settings(OptimizerConfig(optimizer=Optimizer.AdamW)) == (1e-8, 1e-4)
    assert _adam_settings(OptimizerConfig(optimizer=Optimizer.AdamW, eps=1.5e-4, weight_decay=0.05)) == (1.5e-4, 0.05)
    for bad in (OptimizerConfig(max_grad_norm=1.0), OptimizerConfig(optimizer=Optimizer.RMSProp)):
        with pytest.raises(NotImplementedError):
            _adam_settings(bad)


@pytest.mark.parametrize("kind", [0, 1], ids=["memory_efficient", "atari"])
def test_unbalanced_rows_reproduce_reference_draws(kind):
    """The host half of sample_unbalanced (mtrl_amd.drq.unbalanced_rows): the same Generator calls
    as buffers.py:1235-1257 / 906-925, so gathering the restated buffer at its (slot, task) rows
    gives the restatement's own batch, through the fill and the (wrapping) guard window."""
    from mtrl_amd.drq import unbalanced_rows
    from oracle.atari_buffer import AtariBuffer

    T, cap, B = 6, 17, 31
    ref = AtariBuffer(cap, T, (4, 4, 4), seed=3, kind=kind)
    rng = np.random.default_rng(1)
    host = np.random.default_rng(3)
    for step in range(50):
        o = rng.integers(0, 256, (T, 4, 4, 4), dtype=np.uint8)
        ref.add(o, rng.integers(0, 256, (T, 4, 4, 4), dtype=np.uint8), rng.integers(0, 18, T), rng.standard_normal(T),
                np.zeros(T), (rng.random(T) < 0.1) * 1.0)
        if ref.pos == 0 and not ref.full:
            continue
        slots, tasks = unbalanced_rows(host, T, B, ref.pos, ref.full, cap, 3, kind)
        want = ref.sample_unbalanced(B)
        np.testing.assert_array_equal(ref.obs[slots, tasks], want[0])
        nxt = ref.next_obs[slots, tasks] if kind == 1 else ref.obs[(slots + 3) % cap, tasks]
        np.testing.assert_array_equal(nxt, want[2])
        np.testing.assert_array_equal(tasks, want[6])
        assert host.bit_generator.state == ref.rng.bit_generator.state
    assert ref.full


def test_shrink_and_perturb_mixes_only_the_encoder():
    from mtrl_amd.drq_init import init_drq, param_spec, shrink_and_perturb

    geo = dict(num_tasks=3, hw=20, n_hidden=64)
    p = init_drq(1, **geo)
    q = shrink_and_perturb(p, np.random.default_rng(5), 0.5, **geo)
    fresh = shrink_and_perturb(np.zeros_like(p), np.random.default_rng(5), 0.5, **geo)
    assert q.dtype == np.float32 and q.shape == p.shape
    o = 0
    for path, shape in param_spec(**geo):
        n = int(np.prod(shape))
        a, b, f = p[o:o + n], q[o:o + n], fresh[o:o + n]
        if path.startswith("ImpalaEncoder_0"):
            np.testing.assert_array_equal(b, a * np.float32(0.5) + (f * 2) * np.float32(0.5))
        else:
            np.testing.assert_array_equal(b, f)
        o += n


def test_threefry_known_answers():
    """threefry2x32_20 against the Random123 known-answer vectors (the ones jax's own random tests
    use): this pins the bit stream of the compute_weights projection (oracle/jl_projection.py)."""
    from oracle.jl_projection import normal, threefry2x32

    for key, ctr, want in (((0, 0), (0, 0), (0x6B200159, 0x99BA4EFE)),
                           ((0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF), (0x1CB996FC, 0xBB002BE7)),
                           ((0x13198A2E, 0x03707344), (0x243F6A88, 0x85A308D3), (0xC4923A9C, 0x483DF7A0))):
        x0, x1 = threefry2x32(key[0], key[1], np.array([ctr[0]], np.uint32), np.array([ctr[1]], np.uint32))
        assert (int(x0[0]), int(x1[0])) == want
    z = normal(42, np.arange(400_000)).astype(np.float64)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01 and np.abs(z).max() < 6


def test_matrix_stats_match_their_definitions():
    """The host statistics of DrQ's projected gradients against utils.py:73-113's broadcast forms."""
    from mtrl_amd.conflict import matrix_stats

    rng = np.random.default_rng(0)
    g = (rng.standard_normal((5, 300)) * rng.choice([1e-4, 1e-2, 3.0], (5, 300))).astype(np.float32)
    st = matrix_stats(g)
    near, large = np.abs(g) < 1e-3, np.abs(g) > 1.0
    np.testing.assert_array_equal(st["mismatch"], (near[:, None, :] & large[None, :, :]).sum(-1))
    np.testing.assert_array_equal(st["near_zero"], near.sum(1))
    np.testing.assert_allclose(st["gram"], g.astype(np.float64) @ g.T.astype(np.float64))
    np.testing.assert_allclose(st["l1"], np.abs(g).sum(1), rtol=1e-6)
