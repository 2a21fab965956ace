"""The drop-in trainer API (mtrl.experiment / mtrl.rl, base.py:121-359 loop order) on the
device engine, driven by a synthetic gymnasium-shaped vector env."""

from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _experiment(tmp_path, T=3, total=600, resume=False, checkpoint=True):
    from fake_env import FakeMetaworldConfig
    from mtrl.config.networks import ContinuousActionPolicyConfig, QValueFunctionConfig
    from mtrl.config.nn import MultiHeadConfig
    from mtrl.config.optim import OptimizerConfig
    from mtrl.config.rl import OffPolicyTrainingConfig
    from mtrl.experiment import Experiment
    from mtrl.rl.algorithms import MTSACConfig

    return Experiment(
        exp_name="fake_mtmhsac", seed=1, data_dir=tmp_path,
        env=FakeMetaworldConfig(env_id="MT10" if T == 10 else "MT50", terminate_on_success=False)
        if T in (10, 50) else FakeMetaworldConfig(env_id="MT10"),
        algorithm=MTSACConfig(
            num_tasks=T, gamma=0.99,
            actor_config=ContinuousActionPolicyConfig(network_config=MultiHeadConfig(
                num_tasks=T, width=64, optimizer=OptimizerConfig(max_grad_norm=1.0))),
            critic_config=QValueFunctionConfig(network_config=MultiHeadConfig(
                num_tasks=T, width=64, optimizer=OptimizerConfig(max_grad_norm=1.0))),
            num_critics=2),
        training_config=OffPolicyTrainingConfig(total_steps=total, buffer_size=200 * T, batch_size=16 * T,
                                                warmstart_steps=20, evaluation_frequency=10),
        checkpoint=checkpoint, resume=resume,
    )


def test_experiment_runs_and_resumes(tmp_path):
    from fake_env import FakeMTVecEnv
    from mtrl_amd import _lib as L

    T = 10
    exp = _experiment(tmp_path, T=T, total=T * 60)
    agent = exp.run(envs=FakeMTVecEnv(T, max_steps=7))
    assert agent.get_num_params()["actor_num_params"] == agent.engine.param_count(L.ACTOR)
    buf = agent._last_buffer
    assert buf.pos == 60 % 200 and buf.full is False
    logs = agent.engine.logs()
    assert all(np.isfinite(v) for v in logs.values())
    assert agent.engine.get_adam_count(0) == 60 - 21  # one update per step once global_step > warmstart
    ck = sorted((tmp_path / "fake_mtmhsac_1" / "checkpoints").glob("ckpt_*.npz"))
    assert ck, "evaluation points save checkpoints"
    # resume restores agent tensors, Adam state, buffer contents and the PCG64 stream
    exp2 = _experiment(tmp_path, T=T, total=T * 60, resume=True)
    from mtrl_amd.compat.experiment import NpzCheckpointManager

    m = NpzCheckpointManager(tmp_path / "fake_mtmhsac_1" / "checkpoints")
    import mtrl.rl.algorithms as A

    a2 = A.MTSAC.initialize(exp2.algorithm, exp2.env, seed=1)
    rb2 = a2.spawn_replay_buffer(exp2.env, exp2.training_config, 1)
    meta, bck = m.restore(m.latest_step(), a2, rb2)
    rb2.load_checkpoint(bck)
    assert meta["step"] > 20 and bck["data"]["obs"].shape == (200, T, 39 + T)
    assert a2.engine.get_adam_count(1) > 0


def test_update_with_host_batch_and_actions(tmp_path):
    from fake_env import FakeMTVecEnv
    from mtrl.rl.algorithms import MTSAC
    from mtrl.types import ReplayBufferSamples

    T = 10
    exp = _experiment(tmp_path, T=T, checkpoint=False)
    agent = MTSAC.initialize(exp.algorithm, exp.env, seed=3)
    env = FakeMTVecEnv(T)
    obs, _ = env.reset()
    agent, act = agent.sample_action(obs)
    assert act.shape == (T, 4) and np.all(np.abs(act) <= 1)
    ev = agent.eval_action(obs)
    assert ev.shape == (T, 4)
    rng = np.random.default_rng(0)
    B = 16 * T
    o = np.zeros((B, 39 + T), np.float32)
    o[:, :39] = rng.standard_normal((B, 39))
    o[np.arange(B), 39 + np.arange(B) % T] = 1
    batch = ReplayBufferSamples(o, rng.uniform(-1, 1, (B, 4)).astype(np.float32), o.copy(),
                                np.zeros((B, 1), np.float32), rng.uniform(0, 10, (B, 1)).astype(np.float32))
    agent, logs = agent.update(batch)
    assert set(logs) == {"losses/qf_values", "losses/qf_loss", "metrics/critic_grad_magnitude",
                         "metrics/critic_params_norm", "losses/actor_loss", "metrics/actor_grad_magnitude",
                         "metrics/actor_params_norm", "metrics/explore_loss", "losses/alpha_loss", "alpha"}
    assert np.isfinite(logs["losses/qf_loss"])


def test_flax_named_checkpoint_resumes_bitwise(tmp_path):
    """Save the agent by flax path (compat/checkpoint.py) after 2 updates, restore into a
    fresh engine; the next update on identical batch + noise gives identical logs and state."""
    from mtrl.rl.algorithms import MTSAC
    from mtrl_amd import _lib as L
    from mtrl_amd.compat.experiment import NpzCheckpointManager

    T = 10
    exp = _experiment(tmp_path, T=T, checkpoint=False)
    agent = MTSAC.initialize(exp.algorithm, exp.env, seed=3)
    rng = np.random.default_rng(5)
    B = 16 * T

    def batch():
        o = np.zeros((B, 39 + T), np.float32)
        o[:, :39] = rng.standard_normal((B, 39))
        o[np.arange(B), 39 + np.arange(B) % T] = 1
        n = o.copy()
        n[:, :39] = rng.standard_normal((B, 39))
        return (o, rng.uniform(-1, 1, (B, 4)).astype(np.float32), n, np.zeros((B, 1), np.float32),
                rng.uniform(0, 10, (B, 1)).astype(np.float32))

    def eps():
        return rng.standard_normal((B, 4)).astype(np.float32)

    from mtrl.types import ReplayBufferSamples

    agent.update(ReplayBufferSamples(*batch()))  # sizes the engine for B
    for _ in range(2):
        agent.engine.update(batch(), eps(), eps())
    m = NpzCheckpointManager(tmp_path / "ck")
    m.save(2, agent, metadata={"step": 2})
    with np.load(tmp_path / "ck" / "ckpt_2.npz") as z:
        assert "agent/critic/target_params/params/VmapQValueFunction_0/MultiHeadNetwork_0/layer_2/kernel" in z.files
    a2 = MTSAC.initialize(exp.algorithm, exp.env, seed=11)
    a2.update(ReplayBufferSamples(*batch()))
    meta, _ = m.restore(m.latest_step(), a2)
    assert meta == {"step": 2}
    np.testing.assert_array_equal(a2.noise_key(), agent.noise_key())  # update-noise stream position
    assert a2.rng_state() == agent.rng_state()  # action-noise Generator
    b, en, ec = batch(), eps(), eps()
    agent.engine.update(b, en, ec)
    a2.engine.update(b, en, ec)
    assert agent.engine.logs() == a2.engine.logs()
    for w in range(10):
        np.testing.assert_array_equal(agent.engine.get_params(w), a2.engine.get_params(w))
    assert [agent.engine.get_adam_count(i) for i in range(3)] == [a2.engine.get_adam_count(i) for i in range(3)]
    assert agent.engine.param_count(L.CRITIC) == a2.engine.param_count(L.CRITIC)
