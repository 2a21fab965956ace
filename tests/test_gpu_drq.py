"""DrQ-eps update on the GPU (include/drq.h, mtrl_amd/csrc/drq*.{hip,cpp}) against the float64
restatement oracle/drq.py (DrQ.update / _update_inner, mtrl/rl/algorithms/drqeps.py:268-343):
augmentation bit-exact inputs, one update -> logs within 1e-5 relative, the gradient leaf by leaf,
AdamW moments and the Polyak target; a small geometry and the reference's own (84 x 84, scale 1,
hidden 512); determinism.  Parity unpinned (no reference fixtures; see oracle/drq.py)."""

from __future__ import annotations

import numpy as np
import pytest

from oracle import drq as od

pytestmark = pytest.mark.gpu


def _batch(cfg, B, seed):
    rng = np.random.default_rng(seed)
    obs = rng.integers(0, 256, (B, cfg.in_ch, cfg.hw, cfg.hw), dtype=np.uint8)
    nobs = rng.integers(0, 256, (B, cfg.in_ch, cfg.hw, cfg.hw), dtype=np.uint8)
    act = rng.integers(0, cfg.n_actions, B).astype(np.int32)
    done = (rng.random(B) < 0.2).astype(np.float32)
    rew = np.round(rng.standard_normal(B) * 2, 3).astype(np.float32)
    task = rng.integers(0, cfg.num_tasks, B).astype(np.int32)
    co, cn = rng.integers(0, 8, (B, 2)).astype(np.int32), rng.integers(0, 8, (B, 2)).astype(np.int32)
    no = (1 + 0.05 * np.clip(rng.standard_normal(B), -2, 2)).astype(np.float32)
    nn = (1 + 0.05 * np.clip(rng.standard_normal(B), -2, 2)).astype(np.float32)
    return (obs, act, nobs, done, rew, task), (co, no, cn, nn)


def _engine(cfg, B):
    from mtrl_amd.drq import DrQEngine, DrQSettings

    s = DrQSettings(num_tasks=cfg.num_tasks, n_actions=cfg.n_actions, n_atoms=cfg.n_atoms, in_ch=cfg.in_ch, hw=cfg.hw,
                    scale=cfg.scale, embed_dim=cfg.embed_dim, n_hidden=cfg.n_hidden, batch=B)
    return DrQEngine(s)


def _run_both(cfg, B, seed):
    from mtrl_amd import _lib as L

    st = od.init_state(cfg, seed)
    st.params = st.params.astype(np.float32).astype(np.float64)
    st.target = (st.params + np.random.default_rng(seed + 9).normal(0, 1e-3, st.params.size)).astype(np.float32).astype(np.float64)
    batch, aug = _batch(cfg, B, seed + 1)
    e = _engine(cfg, B)
    e.set_params(L.DRQ_PARAMS, st.params)
    e.set_params(L.DRQ_TARGET, st.target)
    e.update(batch, aug)
    got = e.logs()
    obs, act, nobs, done, rew, task = batch
    co, no, cn, nn = aug
    ob = od.augment(obs, co, no)
    nb = od.augment(nobs, cn, nn)
    new, want, internals = od.update(cfg, st, (ob, act, nb, done, rew, task), return_internals=True)
    return e, st, new, got, want, internals


# A conv weight-gradient entry sums B x H x W products (1.8e6 at 84 x 84, batch 256) with heavy
# cancellation.  Two bars per conv leaf (kernel and bias):
#  * elementwise against the entry's rounding floor (oracle conv_error_floors: the |terms| of the
#    sum, each factor at its one-level magnitude), as the GEMM tests hold C to sum |a b|;
#  * the leaf's error norm against that of a plain PyTorch fp32 evaluation of the same update
#    (oracle.drq.update in float32): the device is as accurate as an fp32 reference.
# Calibrated on PyTorch fp32 (CPU) at batch 256 over 4 seeds: elementwise ratios up to 9e-5.
CONV_FLOOR_TOL = 3e-4
CONV_VS_FP32_REF = 4.0


@pytest.mark.parametrize("hw,hidden,B,mfma", [(20, 64, 8, 0), (84, 512, 16, 0), (84, 512, 256, 0), (20, 64, 8, 7),
                                               (84, 512, 16, 7)],
                         ids=["small", "reference_geometry", "reference_geometry_b256", "small_mfma",
                              "reference_geometry_mfma"])
def test_update_matches_oracle(hw, hidden, B, mfma):
    """b256 is the benched configuration (bench.py --workload atari_drq): the single 3B-image
    encoder pass, the split-K dense layers at M = 256..768 and the segment-table partial sums of
    all 15 convs run at the bench's own sizes.  mfma: the experimental f32-MFMA convolutions
    (mtsac_debug_drq_mfma(7); measured slower, off by default) at the two smaller geometries -- at
    b256 their stack-0 Conv_0 bias error norm is 8x the PyTorch fp32 reference's (profiles/r4d_drq_tests.log),
    above this test's 4x bar though inside the elementwise floors."""
    import torch

    from mtrl_amd import _lib as L

    lib = L.load()
    old = lib.mtsac_debug_drq_mfma(mfma)
    try:
        cfg = od.DrQConfig(hw=hw, n_hidden=hidden)
        e, st, new, got, want, internals = _run_both(cfg, B, seed=hw + B)
    finally:
        lib.mtsac_debug_drq_mfma(old)
    for k, v in want.items():
        assert abs(got[k] - v) <= 1e-5 * max(1.0, abs(v)), (k, got[k], v)
    g_gpu = e.get_params(L.DRQ_GRAD).astype(np.float64)
    g_ref = internals["grad"]
    floors = internals["conv_abs"]
    _, _, ref32 = od.update(cfg, st, internals["batch"], return_internals=True, dtype=torch.float32)
    g32 = ref32["grad"]
    o, worst, norm_ratio = 0, {}, {}
    for path, shape in od.param_spec(cfg):
        n = int(np.prod(shape))
        a, b, c = g_gpu[o:o + n], g_ref[o:o + n], g32[o:o + n]
        o += n
        if path in floors:
            err = np.abs(a - b)
            worst[path] = float((err / (floors[path] + 1e-30)).max())
            assert (err <= CONV_FLOOR_TOL * floors[path] + 1e-12).all(), (path, worst[path])
            e_dev, e_ref = np.linalg.norm(a - b), np.linalg.norm(c - b)
            norm_ratio[path] = e_dev / max(e_ref, 1e-30)
            assert e_dev <= CONV_VS_FP32_REF * e_ref + 1e-7 * np.linalg.norm(b), (path, e_dev, e_ref)
            continue
        scale = np.abs(b).max() + 1e-12
        assert np.abs(a - b).max() <= 1e-4 * scale + 1e-9, (path, float(np.abs(a - b).max()), float(scale))
    assert len(worst) == 2 * 5 * len(cfg.stacks)
    print(f"conv |err| / floor worst {max(worst.values()):.2e} ({max(worst, key=worst.get)}); "
          f"|err| vs fp32 reference worst {max(norm_ratio.values()):.2f} ({max(norm_ratio, key=norm_ratio.get)})")
    # first AdamW step from zero moments: mu = (1 - b1) g, nu = (1 - b2) g^2 of the device's own
    # gradient (held to the oracle above, leaf by leaf)
    mu = e.get_params(L.DRQ_ADAM_MU).astype(np.float64)
    nu = e.get_params(L.DRQ_ADAM_NU).astype(np.float64)
    c1, c2 = (float(np.float32(1) - np.float32(b)) for b in (cfg.b1, cfg.b2))  # fp32 constants, as optax
    np.testing.assert_allclose(mu, c1 * g_gpu, rtol=1e-6, atol=1e-12)
    np.testing.assert_allclose(nu, c2 * g_gpu * g_gpu, rtol=1e-6, atol=1e-20)
    tgt = e.get_params(L.DRQ_TARGET).astype(np.float64)
    np.testing.assert_allclose(tgt, new.target, rtol=1e-6, atol=1e-6)
    p = e.get_params(L.DRQ_PARAMS).astype(np.float64)
    dp_gpu, dp_ref = p - st.params, new.params - st.params
    assert np.median(np.abs(dp_gpu - dp_ref)) < 1e-7
    e.close()


@pytest.mark.parametrize("hw,B", [(20, 8), (84, 16), (84, 256)], ids=["small", "reference_geometry", "b256"])
def test_row_tile_convs_match_the_pixel_kernels(hw, B):
    """Round 6: the row-tile conv kernels (forward, data grad, weight grad; drq.hip conv_rows_kernel /
    conv_wgrad_rows_kernel) against the kernels they replaced (mtsac_debug_drq_legacy(7)) on one update.
    The forward and the data grad keep the per-output summation order, so the loss, the logits and
    every dense-layer gradient are bitwise equal; the weight grads sum the same products in another
    order (row tiles, a pixel-group tree), so the conv leaves agree to fp32 rounding of their
    Sum|terms| (both are held to the float64 oracle in test_update_matches_oracle)."""
    from mtrl_amd import _lib as L

    lib = L.load()
    cfg = od.DrQConfig(hw=hw, n_hidden=64 if hw == 20 else 512)
    st = od.init_state(cfg, 5)
    batch, aug = _batch(cfg, B, 6)
    out = {}
    old = lib.mtsac_debug_drq_legacy(-1)
    try:
        for mask in (7 | 16, 16):  # 16: no split2h MFMA convs in either arm (their own test below)
            lib.mtsac_debug_drq_legacy(mask)
            e = _engine(cfg, B)
            e.set_params(L.DRQ_PARAMS, st.params)
            e.set_params(L.DRQ_TARGET, st.params)
            e.update(batch, aug)
            e.synchronize()
            out[mask] = (e.logs(), e.get_params(L.DRQ_GRAD))
            e.close()
    finally:
        lib.mtsac_debug_drq_legacy(old)
    (l_old, g_old), (l_new, g_new) = out[7 | 16], out[16]
    for k in ("losses/online_logits", "losses/critic_loss"):
        assert l_old[k] == l_new[k], (k, l_old, l_new)
    o = 0
    for path, shape in od.param_spec(cfg):
        n = int(np.prod(shape))
        a, b = g_new[o:o + n], g_old[o:o + n]
        o += n
        if "Conv" in path:
            scale = float(np.abs(b).max()) + 1e-30
            assert np.abs(a - b).max() <= 2e-5 * scale, (path, float(np.abs(a - b).max()), scale)
        else:
            np.testing.assert_array_equal(a, b, err_msg=path)


@pytest.mark.parametrize("hw,B", [(20, 8), (84, 16), (84, 256)], ids=["small", "reference_geometry", "b256"])
def test_split2h_convs_match_the_fp32_kernels(hw, B):
    """Round 6: the 8- and 16-channel conv forwards and data grads on split2h MFMA (drq.hip
    conv_h2_kernel; the default for 16 input channels at W <= 32, here forced everywhere) against the
    fp32 VALU kernels (mtsac_debug_drq_legacy(16)) on one update: losses within 1e-5 relative, every gradient leaf within 1e-4 of its largest entry (conv
    leaves 1e-3: a conv bias gradient is a sum over B x H x W pixels with heavy cancellation, where
    two fp32-accurate summation orders differ by up to ~3e-4 of the leaf max at b256).  The strict bar
    is test_update_matches_oracle's, which holds the default (split2h) path to the float64 oracle:
    elementwise Sum|terms| floors and the error norm <= 4x a PyTorch fp32 evaluation's."""
    from mtrl_amd import _lib as L

    lib = L.load()
    cfg = od.DrQConfig(hw=hw, n_hidden=64 if hw == 20 else 512)
    st = od.init_state(cfg, 7)
    batch, aug = _batch(cfg, B, 8)
    out = {}
    old = lib.mtsac_debug_drq_legacy(-1)
    try:
        for mask in (16, 32):  # 32: the split2h convs at every shape they support (default: 16 ch, W <= 32)
            lib.mtsac_debug_drq_legacy(mask)
            e = _engine(cfg, B)
            e.set_params(L.DRQ_PARAMS, st.params)
            e.set_params(L.DRQ_TARGET, st.params)
            e.update(batch, aug)
            e.synchronize()
            out[mask] = (e.logs(), e.get_params(L.DRQ_GRAD).astype(np.float64))
            e.close()
    finally:
        lib.mtsac_debug_drq_legacy(old)
    (l32, g32), (lh, gh) = out[16], out[32]
    for k, v in l32.items():
        assert abs(lh[k] - v) <= 1e-5 * max(1.0, abs(v)), (k, lh[k], v)
    o = 0
    for path, shape in od.param_spec(cfg):
        n = int(np.prod(shape))
        a, b = gh[o:o + n], g32[o:o + n]
        o += n
        scale = float(np.abs(b).max()) + 1e-30
        tol = 1e-3 if "Conv" in path else 1e-4
        assert np.abs(a - b).max() <= tol * scale, (path, float(np.abs(a - b).max()), scale)


@pytest.mark.parametrize("kind", [0, 1, 2], ids=["forward", "data_grad", "weight_grad"])
def test_conv_bench_entry_runs(kind):
    """mtsac_debug_drq_conv_bench (the per-kernel sweep in tools/drq_conv_bench.py) on one shape."""
    import ctypes

    from mtrl_amd import _lib as L

    us = ctypes.c_double(0.0)
    assert L.load().mtsac_debug_drq_conv_bench(kind, 16, 21, 21, 16, 16, 3, ctypes.byref(us)) == 0
    assert us.value > 0.0


def test_deterministic():
    from mtrl_amd import _lib as L

    cfg = od.DrQConfig(hw=20, n_hidden=64)
    outs = []
    for _ in range(2):
        st = od.init_state(cfg, 3)
        batch, aug = _batch(cfg, 8, 4)
        e = _engine(cfg, 8)
        e.set_params(L.DRQ_PARAMS, st.params)
        e.set_params(L.DRQ_TARGET, st.params)
        e.update(batch, aug)
        e.update_resident(2)
        e.synchronize()
        outs.append((e.get_params(L.DRQ_PARAMS), e.logs()))
        e.close()
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1]


def test_q_values_match_oracle():
    import torch

    from mtrl_amd import _lib as L

    cfg = od.DrQConfig(hw=84, n_hidden=512)
    st = od.init_state(cfg, 5)
    e = _engine(cfg, 16)
    e.set_params(L.DRQ_PARAMS, st.params)
    (obs, _, _, _, _, task), (co, no, _, _) = _batch(cfg, 11, 6)
    q = e.q_values(obs, task, co, no)
    with torch.no_grad():
        lg = od.forward(od.unflatten(torch.as_tensor(st.params.astype(np.float32).astype(np.float64)), cfg),
                        torch.as_tensor(od.augment(obs, co, no).astype(np.float64)), torch.as_tensor(task.astype(np.int64)), cfg)
        sup = torch.linspace(cfg.v_min, cfg.v_max, cfg.n_atoms, dtype=torch.float64)
        want = (torch.softmax(lg, -1) * sup).sum(-1).numpy()
    np.testing.assert_allclose(q, want, rtol=1e-5, atol=1e-5)
    e.close()


def test_compat_drq_api():
    import mtrl  # noqa: F401
    from mtrl.envs import AtariConfig
    from mtrl.rl.algorithms import DrQ, DrQConfig
    from mtrl_amd.compat.types import AtariReplayBufferSamples

    agent = DrQ.initialize(DrQConfig(num_tasks=26), AtariConfig(), seed=1, batch_size=32)
    assert agent.get_num_params()["critic_num_params"] == 1535697
    rng = np.random.default_rng(0)
    obs = rng.integers(0, 256, (26, 4, 84, 84), dtype=np.uint8)
    agent, a = agent.sample_action(obs, np.arange(26))
    assert a.shape == (26,) and a.min() >= 0 and a.max() < 18 and agent.step == 26
    g = agent.eval_action(obs, np.arange(26))
    assert g.shape == (26,)
    data = AtariReplayBufferSamples(rng.integers(0, 256, (32, 4, 84, 84), dtype=np.uint8), rng.integers(0, 18, (32, 1)),
                                    rng.integers(0, 256, (32, 4, 84, 84), dtype=np.uint8), np.zeros((32, 1)),
                                    np.zeros((32, 1)), rng.standard_normal((32, 1)), np.arange(32) % 26)
    agent, logs = agent.update(data)
    assert set(logs) == {"losses/online_logits", "metrics/critic_grad_magnitude", "metrics/critic_params_norm",
                         "losses/critic_loss"}
    assert all(np.isfinite(v) for v in logs.values())
    agent.close()


def _same_batch(got, want, where):
    names = ("obs", "actions", "next_obs", "truncations", "dones", "rewards", "task_ids")
    for nm, g, w in zip(names, got, want):
        w = np.asarray(w)
        if w.dtype == np.float64:  # AtariMultiTaskReplayBuffer returns float64 rewards; the update takes float32
            w = w.astype(np.float32)
        np.testing.assert_array_equal(np.asarray(g).reshape(w.shape).astype(w.dtype), w, err_msg=f"{nm} at {where}")


_KINDS = pytest.mark.parametrize("kind", [0, 1], ids=["memory_efficient", "atari"])


@_KINDS
@pytest.mark.parametrize("normalize", [False, True], ids=["raw", "normalized"])
def test_device_buffer_matches_reference_buffer(normalize, kind):
    """MemoryEfficientAtariMultiTaskReplayBuffer (buffers.py:949-1229, kind 0) and
    AtariMultiTaskReplayBuffer (buffers.py:710-947, kind 1) on the device against their numpy
    restatement: n-step aggregation with episode ends, the guard window once full (both the plain
    and the wrapping case), the PCG64 index stream, reward normalisation -- bit for bit."""
    from mtrl_amd.drq import DrQEngine, DrQSettings
    from oracle.atari_buffer import AtariBuffer

    T, n, cap, hw = 4, 3, 23, 20
    B = T * n
    ref = AtariBuffer(cap, T, (4, hw, hw), seed=11, nstep=3, gamma=0.99, normalize_rewards=normalize, kind=kind)
    e = DrQEngine(DrQSettings(num_tasks=T, hw=hw, n_hidden=64, batch=B, capacity=cap, normalize_rewards=int(normalize),
                              buffer_kind=kind))
    e.seed_rng(11)
    rng = np.random.default_rng(5)
    checks = 0
    for step in range(70):
        o = rng.integers(0, 256, (T, 4, hw, hw), dtype=np.uint8)
        no = rng.integers(0, 256, (T, 4, hw, hw), dtype=np.uint8)
        a = rng.integers(0, 18, T).astype(np.int32)
        r = np.round(rng.standard_normal(T) * 3, 2).astype(np.float32)
        tr = (rng.random(T) < 0.05).astype(np.float32)
        d = (rng.random(T) < 0.15).astype(np.float32)
        ref.add(o, no, a, r, tr, d)
        e.buffer_add(o, no, a, r, tr, d)
        assert e.buffer_state() == (ref.pos, ref.full)
        if ref.pos > 0 or ref.full:
            if step % 3 == 0:
                want = ref.sample(B)
                e.sample()
                _same_batch(e.read_batch(), want, f"step {step}")
                checks += 1
            elif step % 3 == 1:  # another batch size: indices on the host, same stream (base.py:280)
                _same_batch(e.sample_balanced_host(T * 5), ref.sample(T * 5), f"step {step} (host indices)")
    assert ref.full and checks > 15
    e.close()


@_KINDS
@pytest.mark.parametrize("normalize", [False, True], ids=["raw", "normalized"])
def test_unbalanced_sample_matches_reference_buffer(normalize, kind):
    """sample_unbalanced (buffers.py:1230-1279, the one OffPolicyAlgorithm.train calls) against the
    numpy restatement bit for bit, batch not a multiple of the task count, interleaved with the
    balanced device sampler on the same Generator stream (host <-> device hand-over of the state)."""
    from mtrl_amd.drq import DrQEngine, DrQSettings
    from oracle.atari_buffer import AtariBuffer

    T, cap, hw, B = 5, 29, 20, 23
    ref = AtariBuffer(cap, T, (4, hw, hw), seed=7, nstep=3, gamma=0.99, normalize_rewards=normalize, kind=kind)
    e = DrQEngine(DrQSettings(num_tasks=T, hw=hw, n_hidden=64, batch=B, capacity=cap, normalize_rewards=int(normalize),
                              buffer_kind=kind))
    e.seed_rng(7)
    rng = np.random.default_rng(9)
    checks = 0
    for step in range(80):
        o = rng.integers(0, 256, (T, 4, hw, hw), dtype=np.uint8)
        no = rng.integers(0, 256, (T, 4, hw, hw), dtype=np.uint8)
        a = rng.integers(0, 18, T).astype(np.int32)
        r = np.round(rng.standard_normal(T) * 3, 2).astype(np.float32)
        tr = (rng.random(T) < 0.05).astype(np.float32)
        d = (rng.random(T) < 0.15).astype(np.float32)
        ref.add(o, no, a, r, tr, d)
        e.buffer_add(o, no, a, r, tr, d)
        if ref.pos > 0 or ref.full:
            if step % 2 == 0:
                want = ref.sample_unbalanced(B)
                e.sample_unbalanced()
            elif step % 7 == 1:  # the balanced sampler needs batch % T == 0: draw its indices only
                want = None
                ref.sample_indices(3)
                e2 = e.get_rng_state()
                g = np.random.Generator(np.random.PCG64())
                g.bit_generator.state = e2
                if kind == 1:
                    g.integers(0, max(ref.pos if not ref.full else cap, 3), size=(3,))
                else:
                    g.integers(0, max(ref.pos - 3, 1) if not ref.full else cap - 9, size=(3,))
                e.set_rng_state(g.bit_generator.state)
            else:
                continue
            if want is not None:
                _same_batch(e.read_batch(), want, f"step {step}")
                checks += 1
    assert ref.full and checks > 25
    assert e.get_rng_state() == ref.rng.bit_generator.state
    e.close()


def test_sample_rows_rejects_out_of_range():
    from mtrl_amd import _lib as L
    from mtrl_amd.drq import DrQEngine, DrQSettings

    e = DrQEngine(DrQSettings(num_tasks=2, hw=20, n_hidden=64, batch=4, capacity=12))
    tasks = np.zeros(4, np.int32)
    for slots, tk in ((np.array([0, 1, 12, 2], np.int64), tasks), (np.array([0, 1, -1, 2], np.int64), tasks),
                      (np.zeros(4, np.int64), np.array([0, 2, 0, 0], np.int32))):
        assert e.lib.drq_sample_rows(e.h, slots.ctypes.data, tk.ctypes.data) == -22
        assert b"out of range" in e.lib.drq_last_error()
    with pytest.raises(L.MTSACError, match="empty buffer"):
        e.sample_unbalanced()
    e.close()


def test_sample_update_runs():
    from mtrl_amd import _lib as L
    from mtrl_amd.drq import DrQEngine, DrQSettings

    cfg = od.DrQConfig(hw=20, n_hidden=64)
    T, B = 26, 26 * 2
    e = DrQEngine(DrQSettings(hw=20, n_hidden=64, batch=B, capacity=40))
    e.set_params(L.DRQ_PARAMS, od.initialize(cfg, 1))
    e.set_params(L.DRQ_TARGET, od.initialize(cfg, 1))
    e.seed_rng(3)
    rng = np.random.default_rng(0)
    for _ in range(20):
        o = rng.integers(0, 256, (T, 4, 20, 20), dtype=np.uint8)
        e.buffer_add(o, o, rng.integers(0, 18, T), rng.standard_normal(T), np.zeros(T), np.zeros(T))
    e.sample_update(3)
    e.synchronize()
    logs = e.logs()
    assert all(np.isfinite(v) for v in logs.values())
    e.seed_augment(5)
    e.sample_unbalanced_update(70)  # > one 64-step row upload
    e.synchronize()
    assert all(np.isfinite(v) for v in e.logs().values())
    e.close()


def test_compat_device_buffer_and_fast_path():
    import mtrl  # noqa: F401
    from mtrl.config.rl import DrQTrainingConfig
    from mtrl.envs import AtariConfig
    from mtrl.rl.algorithms import DrQ, DrQConfig

    agent = DrQ.initialize(DrQConfig(num_tasks=26), AtariConfig(), seed=1, batch_size=52)
    buf = agent.spawn_replay_buffer(AtariConfig(), DrQTrainingConfig(total_steps=100, buffer_size=26 * 30), seed=1)
    rng = np.random.default_rng(0)
    for _ in range(12):
        o = rng.integers(0, 256, (26, 4, 84, 84), dtype=np.uint8)
        buf.add(o, o, rng.integers(0, 18, 26), rng.standard_normal(26), np.zeros(26), np.zeros(26))
    assert buf.pos == 10 and not buf.full  # 12 steps, 3-step returns
    data = buf.sample(52)
    assert data.observations.shape == (52, 4, 84, 84) and data.rewards.shape == (52, 1)
    agent, logs = agent.update(data)
    ub = buf.sample_unbalanced(52)
    assert ub.observations.shape == (52, 4, 84, 84) and np.all(np.diff(ub.task_ids) >= 0)
    agent, logs2 = agent.update_from_buffer(2)
    assert all(np.isfinite(v) for v in list(logs.values()) + list(logs2.values()))
    agent.close()


def test_compat_shrink_and_perturb():
    """drqeps.py:212-245 through the engine: encoder leaves halfway to a fresh draw, the rest fresh,
    target = params, AdamW state reset (the next update's moments are those of a first step)."""
    import mtrl  # noqa: F401
    from mtrl.envs import AtariConfig
    from mtrl.rl.algorithms import DrQ, DrQConfig
    from mtrl_amd import _lib as L
    from mtrl_amd.compat.types import AtariReplayBufferSamples

    agent = DrQ.initialize(DrQConfig(num_tasks=26), AtariConfig(), seed=2, batch_size=26)
    rng = np.random.default_rng(0)
    data = AtariReplayBufferSamples(rng.integers(0, 256, (26, 4, 84, 84), dtype=np.uint8), rng.integers(0, 18, (26, 1)),
                                    rng.integers(0, 256, (26, 4, 84, 84), dtype=np.uint8), np.zeros((26, 1)),
                                    np.zeros((26, 1)), rng.standard_normal((26, 1)), np.arange(26))
    agent, _ = agent.update(data)
    before = agent.engine.get_params(L.DRQ_PARAMS)
    agent = agent.shrink_and_perturb()
    p = agent.engine.get_params(L.DRQ_PARAMS)
    assert not np.array_equal(p, before)
    np.testing.assert_array_equal(agent.engine.get_params(L.DRQ_TARGET), p)
    assert not agent.engine.get_params(L.DRQ_ADAM_MU).any() and not agent.engine.get_params(L.DRQ_ADAM_NU).any()
    agent, logs = agent.update(data)
    g = agent.engine.get_params(L.DRQ_GRAD)
    np.testing.assert_allclose(agent.engine.get_params(L.DRQ_ADAM_MU), 0.1 * g, rtol=1e-6, atol=1e-12)
    assert all(np.isfinite(v) for v in logs.values())
    agent.close()


def test_task_gradients_and_projection_match_oracle():
    """compute_weights' device half (drqeps.py:385-460): each group's gradient lands in flax order
    (== the update path's gradient of the same rows), and project_grad's JL projection with the
    Gaussian blocks regenerated from threefry matches the numpy restatement (several blocks + a
    remainder, float64 reference; tolerance 1e-5 of each row's scale: fp32 sums of 1e5 terms)."""
    from mtrl_amd import _lib as L
    from oracle import jl_projection as jl

    cfg = od.DrQConfig(hw=20, n_hidden=64)
    st = od.init_state(cfg, 4)
    n, T = 6, 3
    e = _engine(cfg, n)
    e.set_params(L.DRQ_PARAMS, st.params)
    e.set_params(L.DRQ_TARGET, st.params)
    grads = []
    for t in range(T):
        batch, aug = _batch(cfg, n, 20 + t)
        e.task_gradient(batch, aug, t, T)
        grads.append(e.get_task_gradient(t))
    # the same rows through the update path give the same gradient (DRQ_GRAD, host-side reorder)
    e2 = _engine(cfg, n)
    e2.set_params(L.DRQ_PARAMS, st.params)
    e2.set_params(L.DRQ_TARGET, st.params)
    batch, aug = _batch(cfg, n, 22)
    e2.update(batch, aug)
    np.testing.assert_array_equal(e2.get_params(L.DRQ_GRAD), grads[2])
    e2.close()
    G = np.stack(grads)
    P = G.shape[1]
    for D, chunk, seed in ((64, 20_000, 42), (37, P // 2 + 5, 7)):
        got = e.project_task_gradients(T, D, chunk, seed)
        want = jl.project(G, D, chunk, seed)
        scale = np.linalg.norm(G, axis=1, keepdims=True) / np.sqrt(D)
        assert np.max(np.abs(got - want) / scale) < 1e-5, (D, chunk)
    e.close()


def test_compat_compute_weights():
    """DrQ.compute_weights at the reference geometry (26 tasks, 1.5 M parameters, proj_dim 10 000):
    the reference's 18 keys, shapes, and the T x T algebra consistent with the pairwise matrices."""
    import mtrl  # noqa: F401
    from mtrl.config.rl import DrQTrainingConfig
    from mtrl.envs import AtariConfig
    from mtrl.rl.algorithms import DrQ, DrQConfig

    agent = DrQ.initialize(DrQConfig(num_tasks=26), AtariConfig(), seed=1, batch_size=52)
    buf = agent.spawn_replay_buffer(AtariConfig(), DrQTrainingConfig(total_steps=100, buffer_size=26 * 40), seed=1)
    rng = np.random.default_rng(0)
    for _ in range(20):
        o = rng.integers(0, 256, (26, 4, 84, 84), dtype=np.uint8)
        buf.add(o, o, rng.integers(0, 18, 26), rng.standard_normal(26), np.zeros(26), (rng.random(26) < 0.1) * 1.0)
    data = buf.sample(26 * 4)  # the metrics batch (base.py:280), 4 rows per task
    assert data.observations.shape == (104, 4, 84, 84)
    agent, logs = agent.compute_weights(data)
    assert len(logs) == 18 and logs["pairwise_cos_sim"].shape == (1, 26, 26)  # vmap_cos_sim's leading axis
    cos = logs["pairwise_cos_sim"][0].astype(np.float64)
    np.testing.assert_allclose(cos, cos.T, atol=1e-6)
    np.testing.assert_allclose(np.diag(cos), 1.0, atol=1e-5)
    triu = np.triu(np.ones((26, 26)), 1)
    np.testing.assert_allclose(logs["critic_avg_cos_sim"], (triu * cos).sum() / triu.sum(), rtol=1e-5)
    assert abs(logs["critic_avg_grad_magnitude"] - logs["per_task_grad_magnitude"].mean()) < 1e-5 * \
        logs["critic_avg_grad_magnitude"]
    assert all(np.all(np.isfinite(v)) for v in logs.values())
    agent.close()
