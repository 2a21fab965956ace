"""Oracle MultiTaskReplayBuffer: the reference's own test semantics
(tests/test_rl_buffers.py:21-62 -- full/pos wrap) restated for the multi-task
buffer, plus the sample layout of buffers.py:520-549 (row = i*T + t)."""

import numpy as np

from oracle.buffer import MultiTaskReplayBufferOracle


def _add(buf, value):
    T = buf.num_tasks
    obs = np.full((T, 3), value, np.float32)
    buf.add(obs, obs + 1, np.full((T, 2), -value, np.float32), np.full(T, value, np.float32),
            np.full(T, int(value) % 2, np.float32))


def test_full_flag_after_single_transitions():
    buf = MultiTaskReplayBufferOracle(4 * 2, 2, 3, 2, seed=0)
    for i in range(buf.capacity):
        _add(buf, float(i))
    assert buf.full is True and buf.pos == 0


def test_wrap_keeps_full_and_advances_pos():
    buf = MultiTaskReplayBufferOracle(5 * 2, 2, 3, 2, seed=0)
    for i in range(7):
        _add(buf, float(i))
    assert buf.full is True and buf.pos == 2
    assert buf.obs[0, 0, 0] == 5.0 and buf.obs[1, 1, 0] == 6.0


def test_sample_layout_and_stream():
    T, cap = 3, 10
    buf = MultiTaskReplayBufferOracle(cap * T, T, 3, 2, seed=42)
    for i in range(cap):
        _add(buf, float(i))
    obs, act, nobs, done, rew = buf.sample(4 * T)
    idx = np.random.default_rng(42).integers(0, cap, size=4)
    assert obs.shape == (12, 3) and rew.shape == (12, 1) and done.shape == (12, 1)
    np.testing.assert_array_equal(obs[:, 0], np.repeat(idx, T).astype(np.float32))
    np.testing.assert_array_equal(nobs[:, 0], np.repeat(idx, T).astype(np.float32) + 1)


def test_high_uses_n_before_filled():
    T = 2
    buf = MultiTaskReplayBufferOracle(100 * T, T, 3, 2, seed=1)
    _add(buf, 1.0)
    idx = buf.sample_indices(8 * T)
    np.testing.assert_array_equal(idx, np.random.default_rng(1).integers(0, 8, size=8))


def test_reward_normalization_float64():
    T = 2
    buf = MultiTaskReplayBufferOracle(10 * T, T, 3, 2, seed=1, normalize_rewards=True)
    for v in (1.0, 3.0, 2.0):
        _add(buf, v)
    _, _, _, _, rew = buf.gather(np.array([0, 1, 2]))
    np.testing.assert_allclose(rew[:, 0], np.repeat([0.0, 1.0, 0.5], T), rtol=1e-7)
