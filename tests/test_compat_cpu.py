"""CPU checks of the drop-in import surface (no device calls)."""

import pathlib
import re

import pytest

REF = pathlib.Path("/root/reference/experiments")


@pytest.mark.parametrize("script", ["mt10_mtmhsac.py", "mt50_mtmhsac_v2.py",
                                    "width_scaling/mt10_mtmhsac_v2_2048.py",
                                    "width_scaling/mt50_mtmhsac_v2_2048.py"])
def test_reference_scripts_mtrl_imports_resolve(script):
    """Every ``from mtrl... import ...`` line of the target scripts resolves here."""
    p = REF / script
    if not p.exists():
        pytest.skip("reference tree not mounted")
    lines = [l.strip() for l in p.read_text().splitlines() if re.match(r"\s*from mtrl", l)]
    assert lines
    ns: dict = {}
    for l in lines:
        exec(l, ns)  # noqa: S102 - import statements only


def test_config_surface_and_defaults():
    from mtrl.config.networks import ContinuousActionPolicyConfig, QValueFunctionConfig
    from mtrl.config.nn import MultiHeadConfig
    from mtrl.config.optim import OptimizerConfig
    from mtrl.config.rl import OffPolicyTrainingConfig
    from mtrl.envs import MetaworldConfig
    from mtrl.rl.algorithms import MTSACConfig, get_algorithm_for_config
    from mtrl.rl.algorithms.mtsac import MTSAC

    cfg = MTSACConfig(
        num_tasks=50, gamma=0.99,
        actor_config=ContinuousActionPolicyConfig(
            network_config=MultiHeadConfig(width=2048, num_tasks=50, optimizer=OptimizerConfig(max_grad_norm=1.0))),
        critic_config=QValueFunctionConfig(
            network_config=MultiHeadConfig(width=2048, num_tasks=50, optimizer=OptimizerConfig(max_grad_norm=1.0))),
        num_critics=2, use_task_weights=False)
    assert get_algorithm_for_config(cfg) is MTSAC
    assert (cfg.tau, cfg.initial_temperature, cfg.temperature_optimizer_config.max_grad_norm) == (0.005, 1.0, None)
    tc = OffPolicyTrainingConfig(total_steps=int(1e8), buffer_size=100_000 * 50, batch_size=128 * 50,
                                 evaluation_frequency=1_000_000 // 500)
    assert tc.warmstart_steps == 4000
    env = MetaworldConfig(env_id="MT50", terminate_on_success=False, reward_func_version="v2")
    assert env.observation_space.shape == (89,) and env.action_space.shape == (4,)
    with pytest.raises(ValueError):
        get_algorithm_for_config(object())
