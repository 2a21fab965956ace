"""GPU parity of the individual device kernels (fp32 MFMA GEMM, index stream, gather).

All calls go through libmtsac.so.  GEMMs are checked against a float64 numpy
product of the same fp32 inputs (the "plain fp32 reference of the same op");
the index stream and the gather are checked BIT-EXACT against the oracle, whose
PCG64 restatement is itself pinned to ``numpy.random.default_rng`` (the
reference's dependency; tests/test_oracle_pcg64.py).
"""

from __future__ import annotations

import numpy as np
import pytest

from oracle.buffer import MultiTaskReplayBufferOracle
from oracle.pcg64 import PCG64State

pytestmark = pytest.mark.gpu

NN, NT, TN = 0, 1, 2
STORE, BIAS_RELU, MASK = 0, 1, 2


def _ref(kind, A, B, M, N, K):
    A64, B64 = A.astype(np.float64), B.astype(np.float64)
    if kind == NN:
        return A64[:M, :K] @ B64[:K, :N], np.abs(A64[:M, :K]) @ np.abs(B64[:K, :N])
    if kind == NT:
        return A64[:M, :K] @ B64[:N, :K].T, np.abs(A64[:M, :K]) @ np.abs(B64[:N, :K]).T
    return A64[:K, :M].T @ B64[:K, :N], np.abs(A64[:K, :M]).T @ np.abs(B64[:K, :N])


@pytest.mark.parametrize("precision", [0, 1])
@pytest.mark.parametrize("kind", [NN, NT, TN])
@pytest.mark.parametrize("shape", [(200, 136, 93), (128, 128, 32), (64, 400, 400), (257, 132, 260), (8, 4, 4)])
def test_gemm_store(kind, shape, precision):
    """precision 0: f32-input MFMA; 1: 3-way bf16 split (fp32-accurate).  Error bound vs a
    float64 product of the same fp32 inputs: |err| <= 2e-6 (f32) / 4e-6 (split) x sum|a*b|."""
    from mtrl_amd.engine import debug_gemm

    M, N, K = shape
    rng = np.random.default_rng(0)
    Kp = (K + 3) // 4 * 4
    if kind == NN:
        A = np.zeros((M, Kp), np.float32); A[:, :K] = rng.standard_normal((M, K))
        B = rng.standard_normal((K, N)).astype(np.float32)
    elif kind == NT:
        A = np.zeros((M, Kp), np.float32); A[:, :K] = rng.standard_normal((M, K))
        B = np.zeros((N, Kp), np.float32); B[:, :K] = rng.standard_normal((N, K))
    else:
        Mp = (M + 3) // 4 * 4
        A = np.zeros((K, Mp), np.float32); A[:, :M] = rng.standard_normal((K, M))
        B = rng.standard_normal((K, N)).astype(np.float32)
    C0 = np.full((M, N), 7.0, np.float32)
    C, db = debug_gemm(kind, STORE, A, B, C0, M, N, K, want_db=(kind == TN), precision=precision)
    ref, mag = _ref(kind, A, B, M, N, K)
    err = np.abs(C - ref)
    tol = 2e-6 if precision == 0 else 4e-6
    assert np.all(err <= tol * mag + 1e-30), float((err / mag).max())
    if kind == TN:
        np.testing.assert_allclose(db[0], B[:K, :N].astype(np.float64).sum(0), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("precision", [0, 1])
def test_gemm_epilogues_batched(precision):
    from functools import partial

    from mtrl_amd.engine import debug_gemm as _dg

    debug_gemm = partial(_dg, precision=precision)

    rng = np.random.default_rng(1)
    M, N, K, E = 300, 200, 96, 2
    A = rng.standard_normal((M, K)).astype(np.float32)
    B = rng.standard_normal((E, K, N)).astype(np.float32)
    bias = rng.standard_normal((E, N)).astype(np.float32)
    C, _ = debug_gemm(NN, BIAS_RELU, A, B, np.zeros((E, M, N), np.float32), M, N, K, batch=E, a_shared=True,
                      bias=bias)
    for e in range(E):
        ref = np.maximum(A.astype(np.float64) @ B[e] + bias[e], 0)
        np.testing.assert_allclose(C[e], ref, rtol=1e-5, atol=1e-4)
    # relu-mask epilogue on NT: C = (dY W^T) * (H > 0)
    dY = rng.standard_normal((E, M, N)).astype(np.float32)
    W = rng.standard_normal((E, K, N)).astype(np.float32)  # stored [N=K][K=N] for the NT product
    H = rng.standard_normal((E, M, K)).astype(np.float32)
    C, _ = debug_gemm(NT, MASK, dY, W, np.zeros((E, M, K), np.float32), M, K, N, batch=E, mask=H)
    for e in range(E):
        ref = (dY[e].astype(np.float64) @ W[e].T.astype(np.float64)) * (H[e] > 0)
        np.testing.assert_allclose(C[e], ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("precision", [0, 1])
@pytest.mark.parametrize("splits", [2, 5, 16])
@pytest.mark.parametrize("shape", [(93, 300, 6400, 2), (64, 130, 1000, 1), (7, 8, 33, 1)])
def test_gemm_splitk_weight_grad(shape, splits, precision):
    """Split-K TN (weight gradient of a narrow layer over a long batch): partial slabs reduced in
    slice order, db column sums from the same slices; same bound as the unsplit GEMM."""
    from mtrl_amd.engine import debug_gemm

    M, N, K, E = shape
    rng = np.random.default_rng(3)
    Mp = (M + 3) // 4 * 4
    A = np.zeros((E, K, Mp), np.float32)
    A[..., :M] = rng.standard_normal((E, K, M))
    B = rng.standard_normal((E, K, N)).astype(np.float32)
    C, db = debug_gemm(TN, STORE, A, B, np.zeros((E, M, N), np.float32), M, N, K, batch=E, want_db=True,
                       precision=precision, splits=splits)
    tol = 2e-6 if precision == 0 else 4e-6
    for e in range(E):
        ref, mag = _ref(TN, A[e], B[e], M, N, K)
        err = np.abs(C[e] - ref)
        assert np.all(err <= tol * mag + 1e-30), float((err / mag).max())
        np.testing.assert_allclose(db[e], B[e].astype(np.float64).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("precision", [0, 1])
def test_gemm_nt_bias_relu(precision):
    """Trunk forward against a pre-transposed weight: relu(A W^T_stored^T + b) on the NT kernel."""
    from mtrl_amd.engine import debug_gemm

    rng = np.random.default_rng(4)
    M, N, K, E = 300, 200, 96, 2
    A = rng.standard_normal((E, M, K)).astype(np.float32)
    Wt = rng.standard_normal((E, N, K)).astype(np.float32)
    bias = rng.standard_normal((E, N)).astype(np.float32)
    C, _ = debug_gemm(NT, BIAS_RELU, A, Wt, np.zeros((E, M, N), np.float32), M, N, K, batch=E, bias=bias,
                      precision=precision)
    for e in range(E):
        ref = np.maximum(A[e].astype(np.float64) @ Wt[e].T.astype(np.float64) + bias[e], 0)
        np.testing.assert_allclose(C[e], ref, rtol=1e-5, atol=1e-4)


def _small_engine(T=3, n=4, cap=50, D=None, normalize=False, **kw):
    from mtrl_amd.engine import MTSACEngine, make_config

    D = D if D is not None else 39 + T
    cfg = make_config(num_tasks=T, task_count=T, obs_dim=D, batch_per_task=n, capacity=cap, actor_width=16,
                      critic_width=16, normalize_rewards=1 if normalize else 0, **kw)
    return MTSACEngine(cfg)


@pytest.mark.parametrize("n", [1, 3, 4, 128])
@pytest.mark.parametrize("seed", [0, 1, 42])
def test_index_stream_bit_exact(n, seed):
    cap = 100_000 if n == 128 else 5000
    eng = _small_engine(T=2, n=n, cap=cap)
    eng.buffer_fill_synthetic(3)  # valid one-hot rows everywhere
    eng.seed_rng(seed)
    ref = PCG64State.from_seed(seed)
    # sizes before full (pos < n gives high = n), mid-fill, and full
    for pos, full in [(0, False), (1, False), (n, False), (777 % cap, False), (0, True), (0, True), (13, True)]:
        eng.set_buffer_state(pos, full)
        high = max(cap if full else pos, n)
        idx, _ = eng.sample()
        want = ref.integers(high, n)
        np.testing.assert_array_equal(idx, want)
        assert eng.get_rng_state() == ref.to_numpy_state()
    eng.close()


def _fill(eng_or_oracle_pairs, cap, T, D, A, seed=5, slots=None):
    rng = np.random.default_rng(seed)
    slots = cap if slots is None else slots
    F = D - T
    obs = np.zeros((slots, T, D), np.float32)
    obs[:, :, :F] = rng.standard_normal((slots, T, F))
    obs[:, np.arange(T), F + np.arange(T)] = 1.0
    nobs = obs.copy()
    nobs[:, :, :F] = rng.standard_normal((slots, T, F))
    act = rng.uniform(-1, 1, (slots, T, A)).astype(np.float32)
    rew = rng.uniform(0, 10, (slots, T)).astype(np.float32)
    done = (rng.uniform(size=(slots, T)) < 0.1).astype(np.float32)
    return obs, nobs, act, rew, done


@pytest.mark.parametrize("normalize", [False, True])
def test_gather_bit_exact(normalize):
    T, n, cap, A = 3, 8, 64, 4
    D = 39 + T
    eng = _small_engine(T=T, n=n, cap=cap, normalize=normalize)
    orc = MultiTaskReplayBufferOracle(cap * T, T, D, A, seed=7, normalize_rewards=normalize)
    eng.seed_rng(7)
    obs, nobs, act, rew, done = _fill(None, cap, T, D, A, slots=40)
    for s in range(40):  # buffer_add path (advances pos, tracks reward stats)
        eng.buffer_add(obs[s], nobs[s], act[s], rew[s], done[s])
        orc.add(obs[s], nobs[s], act[s], rew[s], done[s])
    assert eng.buffer_state() == (orc.pos, orc.full)
    for _ in range(3):
        idx, got = eng.sample()
        want_idx = orc.sample_indices(n * T)
        np.testing.assert_array_equal(idx, want_idx)
        want = orc.gather(want_idx)
        for g, w in zip(got, want):
            np.testing.assert_array_equal(g.reshape(w.shape), w.astype(np.float32))
    # bulk write path + wrap-around semantics (buffers.py:337-343)
    eng.buffer_write(0, obs[:32].reshape(-1, D), nobs[:32].reshape(-1, D), act[:32].reshape(-1, A),
                     rew[:32].reshape(-1), done[:32].reshape(-1))
    o2, n2, a2, r2, d2 = eng.buffer_read(0, 32)
    np.testing.assert_array_equal(o2, obs[:32]); np.testing.assert_array_equal(n2, nobs[:32])
    np.testing.assert_array_equal(a2, act[:32]); np.testing.assert_array_equal(r2, rew[:32])
    np.testing.assert_array_equal(d2, done[:32])
    eng.close()


def test_buffer_add_wraps_like_reference():
    """tests/test_rl_buffers.py:21-35 semantics, on the multi-task device buffer."""
    T, cap, A = 2, 4, 4
    D = 39 + T
    eng = _small_engine(T=T, n=1, cap=cap)
    obs, nobs, act, rew, done = _fill(None, cap, T, D, A, slots=cap + 2)
    for s in range(cap):
        eng.buffer_add(obs[s], nobs[s], act[s], rew[s], done[s])
    assert eng.buffer_state() == (0, True)
    for s in range(2):
        eng.buffer_add(obs[cap + s], nobs[cap + s], act[cap + s], rew[cap + s], done[cap + s])
    assert eng.buffer_state() == (2, True)
    o, _, _, _, _ = eng.buffer_read(0, 2)
    np.testing.assert_array_equal(o, obs[cap:cap + 2])
    eng.close()


def test_bad_one_hot_is_reported():
    from mtrl_amd._lib import MTSACError

    T, n, cap, A = 2, 2, 8, 4
    D = 39 + T
    eng = _small_engine(T=T, n=n, cap=cap)
    obs, nobs, act, rew, done = _fill(None, cap, T, D, A)
    obs[:, 0, D - T:] = 0.0  # task 0 rows lose their one-hot
    eng.buffer_write(0, obs.reshape(-1, D), nobs.reshape(-1, D), act.reshape(-1, A), rew.reshape(-1),
                     done.reshape(-1))
    eng.set_buffer_state(0, True)
    with pytest.raises(MTSACError):
        eng.sample()
    eng.close()


def test_return_normalisation_matches_reference():
    """returns_normalization=True (buffers.py:347-422, 531-533): per-episode discounted returns
    (terminal, and truncated with the mean-reward bootstrap) tracked on the host, the per-task
    denominator applied in the device gather; batches bit for bit against the restatement, the
    checkpoint carrying returns_min / returns_max."""
    from mtrl_amd.compat.rl.buffers import MultiTaskReplayBuffer
    from mtrl_amd.engine import MTSACEngine, make_config

    T, n, cap, A = 3, 8, 64, 4
    D = 39 + T
    eng = MTSACEngine(make_config(num_tasks=T, task_count=T, obs_dim=D, batch_per_task=n, capacity=cap,
                                  actor_width=16, critic_width=16, normalize_rewards=2))
    buf = MultiTaskReplayBuffer(cap * T, T, seed=7, returns_normalization=True, engine=eng)
    orc = MultiTaskReplayBufferOracle(cap * T, T, D, A, seed=7, returns_normalization=True)
    obs, nobs, act, _, _ = _fill(None, cap, T, D, A, slots=60)
    rng = np.random.default_rng(3)
    checks = 0
    for s in range(60):
        rew = rng.normal(2.0, 3.0, T)  # float64, as an env hands them over
        term = rng.uniform(size=T) < 0.08
        trunc = (rng.uniform(size=T) < 0.05) & ~term
        done = (term | trunc).astype(np.float32)
        kw = {"terminal": term, "truncated": trunc} if s % 2 else {}
        buf.add(obs[s], nobs[s], act[s], rew, done, **kw)
        orc.add(obs[s], nobs[s], act[s], rew, done, **kw)
        if s % 5 == 4 and s >= n:  # only written slots (the engine rejects rows without a task one-hot)
            got = buf.sample(n * T)
            want = orc.sample(n * T)
            for g, w in zip(got, want):
                np.testing.assert_array_equal(np.asarray(g).reshape(w.shape), w.astype(np.float32))
            checks += 1
    assert checks == 11 and np.isfinite(orc._returns_max).all()
    np.testing.assert_array_equal(buf.return_denominator(), orc.return_denominator())
    ck = buf.checkpoint()
    np.testing.assert_array_equal(ck["data"]["returns_min"], orc._returns_min)
    np.testing.assert_array_equal(ck["data"]["returns_max"], orc._returns_max)
    eng.close()


@pytest.mark.parametrize("persist", [False, True], ids=["reference_dict", "persisted_stream"])
def test_buffer_resume_from_checkpoint_dict(persist):
    """a run interrupted after some samples is checkpointed and resumed into a fresh
    device buffer spawned with the same seed.  With the reference's checkpoint dict (rng_state None:
    numpy 2.2's Generator.__getstate__, mtrl/rl/buffers.py:323) the resumed buffer's next batches are
    the oracle's after the same load -- the fresh default_rng(seed) stream, as a resumed reference run
    draws them -- bit for bit; with persist_rng_state the interrupted stream continues instead."""
    from mtrl_amd.compat.rl.buffers import MultiTaskReplayBuffer
    from mtrl_amd.engine import MTSACEngine, make_config

    T, n, cap, A = 3, 8, 64, 4
    D = 39 + T

    def engine():
        return MTSACEngine(make_config(num_tasks=T, task_count=T, obs_dim=D, batch_per_task=n, capacity=cap,
                                       actor_width=16, critic_width=16))

    e1 = engine()
    buf = MultiTaskReplayBuffer(cap * T, T, seed=1, engine=e1)
    buf.persist_rng_state = persist
    orc = MultiTaskReplayBufferOracle(cap * T, T, D, A, seed=1)
    obs, nobs, act, rew, done = _fill(None, cap, T, D, A, slots=40)
    for s in range(40):
        buf.add(obs[s], nobs[s], act[s], rew[s], done[s])
        orc.add(obs[s], nobs[s], act[s], rew[s], done[s])
    for _ in range(3):  # the interrupted run advances its stream
        buf.sample(n * T)
        orc.sample(n * T)
    ck = buf.checkpoint()
    assert (ck["rng_state"] is None) != persist
    e1.close()
    e2 = engine()
    buf2 = MultiTaskReplayBuffer(cap * T, T, seed=1, engine=e2)  # spawn_replay_buffer(seed) on resume
    buf2.load_checkpoint(ck)
    ref = MultiTaskReplayBufferOracle(cap * T, T, D, A, seed=1)
    ref.load_checkpoint({"data": {k: np.asarray(v) for k, v in ck["data"].items()}, "rng_state": ck["rng_state"]})
    cont = orc  # persisted: the uninterrupted stream
    for _ in range(3):
        got = buf2.sample(n * T)
        want = (cont if persist else ref).sample(n * T)
        for g, w in zip(got, want):
            np.testing.assert_array_equal(np.asarray(g).reshape(w.shape), w.astype(np.float32))
    e2.close()
