"""Replay-buffer checkpoint interop with the reference dict (CPU).

The reference saves ``"rng_state": self._rng.__getstate__()`` (mtrl/rl/buffers.py:323, as JSON by
mtrl/checkpoint.py:66) and restores with ``self._rng.__setstate__(ckpt["rng_state"])`` (:335).  Under
the pinned numpy (2.2.4; 2.2.6 here, same Generator) that value is ``None`` and ``__setstate__(None)``
leaves the stream alone, so a resumed reference run draws its indices from the fresh
``default_rng(seed)`` that ``spawn_replay_buffer`` made (base.py:148).  Pinned here:
  * those numpy facts themselves;
  * the oracle restatement (oracle/buffer.py) against numpy's own stream after a load;
  * the compat buffer's host logic (mtrl_amd/compat/rl/buffers.py) on a stub engine: a reference
    checkpoint (rng_state None) loads without touching the stream, a dict sets it, and checkpoint()
    writes None unless persist_rng_state is set;
  * the npz checkpoint manager's round trip of both forms.
The device side (the engine's PCG64 after such a load) is tests/test_gpu_trainer.py's resume case.
"""

from __future__ import annotations

import numpy as np

from oracle.buffer import MultiTaskReplayBufferOracle


def _filled(seed, T=3, cap=16, D=8, A=4, slots=11):
    b = MultiTaskReplayBufferOracle(cap * T, T, D, A, seed=seed)
    rng = np.random.default_rng(99)
    for _ in range(slots):
        b.add(rng.standard_normal((T, D)), rng.standard_normal((T, D)), rng.uniform(-1, 1, (T, A)),
              rng.uniform(0, 10, T), np.zeros(T))
    return b


def test_numpy_generator_state_is_none_and_setstate_none_keeps_the_stream():
    g = np.random.default_rng(1)
    assert g.__getstate__() is None  # what buffers.py:323 stores under numpy 2.2
    first = g.integers(0, 1000, 5)
    g.__setstate__(None)  # buffers.py:335 with a reference checkpoint: the stream continues
    np.testing.assert_array_equal(np.concatenate([first, g.integers(0, 1000, 5)]),
                                  np.random.default_rng(1).integers(0, 1000, 10))
    g2 = np.random.default_rng(5)
    g2.__setstate__(np.random.default_rng(7).bit_generator.state)  # a state dict sets the stream
    np.testing.assert_array_equal(g2.integers(0, 1000, 5), np.random.default_rng(7).integers(0, 1000, 5))


def test_oracle_resume_from_reference_checkpoint_draws_the_fresh_stream():
    src = _filled(seed=1)
    src.sample(3 * 4)  # the interrupted run has advanced its stream
    ck = src.checkpoint()
    assert ck["rng_state"] is None
    dst = MultiTaskReplayBufferOracle(16 * 3, 3, 8, 4, seed=1)  # spawn_replay_buffer(seed=1)
    dst.load_checkpoint(ck)
    high = max(dst.pos if not dst.full else dst.capacity, 4)
    want = np.random.default_rng(1).integers(0, high, size=4)  # buffers.py:523-527 on the fresh stream
    np.testing.assert_array_equal(dst.sample_indices(12), want)
    np.testing.assert_array_equal(dst.obs, src.obs)
    assert (dst.pos, dst.full) == (src.pos, src.full)


def test_oracle_load_with_state_dict_continues_that_stream():
    src = _filled(seed=1)
    ck = src.checkpoint()
    g = np.random.default_rng(7)
    g.integers(0, 5, 3)
    ck["rng_state"] = g.bit_generator.state
    dst = MultiTaskReplayBufferOracle(16 * 3, 3, 8, 4, seed=1)
    dst.load_checkpoint(ck)
    high = max(dst.pos, 4)
    np.testing.assert_array_equal(dst.sample_indices(12), g.integers(0, high, size=4))


class _StubEngine:
    """The slice of MTSACEngine the compat buffer calls, recording the stream calls."""

    class config:
        normalize_rewards = 0

    def __init__(self, T, cap, D, A):
        self.T, self.cap, self.D, self.A = T, cap, D, A
        self.calls = []
        self.state = (0, False)

    def seed_rng(self, seed):
        self.calls.append(("seed", seed))

    def set_rng_state(self, st):
        self.calls.append(("set", st))

    def get_rng_state(self):
        return np.random.default_rng(3).bit_generator.state

    def buffer_write(self, slot, *arrays):
        self.calls.append(("write", slot, arrays[0].shape))

    def buffer_read(self, slot, count):
        T, D, A = self.T, self.D, self.A
        return (np.zeros((count, T, D), np.float32), np.zeros((count, T, D), np.float32),
                np.zeros((count, T, A), np.float32), np.zeros((count, T), np.float32), np.zeros((count, T), np.float32))

    def set_buffer_state(self, pos, full):
        self.state = (pos, full)

    def buffer_state(self):
        return self.state


def test_compat_buffer_loads_a_reference_checkpoint_dict():
    from mtrl_amd.compat.rl.buffers import MultiTaskReplayBuffer

    T, cap, D, A = 3, 16, 8, 4
    ref = _filled(seed=1, T=T, cap=cap, D=D, A=A)
    ck = ref.checkpoint()  # {"data": ..., "rng_state": None}: what the reference writes
    eng = _StubEngine(T, cap, D, A)
    buf = MultiTaskReplayBuffer(cap * T, T, seed=1, engine=eng)
    buf.load_checkpoint(ck)
    assert ("seed", 1) in eng.calls and not any(c[0] == "set" for c in eng.calls)  # stream untouched
    assert eng.state == (ref.pos, ref.full)
    # a state dict (numpy's legacy __setstate__ form, or persist_rng_state checkpoints) sets it
    st = np.random.default_rng(7).bit_generator.state
    buf.load_checkpoint({**ck, "rng_state": st})
    assert eng.calls[-1] == ("set", st)


def test_compat_buffer_checkpoint_writes_none_unless_persisting():
    from mtrl_amd.compat.rl.buffers import MultiTaskReplayBuffer

    eng = _StubEngine(2, 4, 6, 4)
    buf = MultiTaskReplayBuffer(8, 2, seed=0, engine=eng)
    assert buf.checkpoint()["rng_state"] is None
    buf.persist_rng_state = True
    assert buf.checkpoint()["rng_state"] == np.random.default_rng(3).bit_generator.state


def test_npz_manager_round_trips_both_rng_forms(tmp_path):
    from mtrl_amd.compat.experiment import NpzCheckpointManager
    from mtrl_amd.compat.rl.buffers import MultiTaskReplayBuffer

    class _Agent:
        def state_dict(self):
            return {"x": np.arange(3.0)}

        def load_state_dict(self, d):
            self.d = d

    for persist in (False, True):
        eng = _StubEngine(2, 4, 6, 4)
        buf = MultiTaskReplayBuffer(8, 2, seed=0, engine=eng)
        buf.persist_rng_state = persist
        m = NpzCheckpointManager(tmp_path / f"p{int(persist)}")
        m.save(5, _Agent(), buffer=buf, metadata={"step": 5})
        _, bck = m.restore(5, _Agent(), buffer=buf)
        want = np.random.default_rng(3).bit_generator.state if persist else None
        assert bck["rng_state"] == want
