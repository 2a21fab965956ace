"""``mtrl`` import surface for the reference's experiment scripts.

Aliases the reference's module paths to the MI355X host mirror in
``mtrl_amd.compat`` (e.g. ``mtrl.config.nn`` -> ``mtrl_amd.compat.config.nn``), so
``experiments/mt10_mtmhsac.py`` and ``experiments/mt50_mtmhsac_v2.py`` import unchanged.
"""

import importlib
import sys

_ALIASES = (
    "config", "config.nn", "config.networks", "config.optim", "config.rl", "config.utils",
    "envs", "envs.base", "envs.metaworld", "rl", "rl.buffers", "rl.algorithms", "rl.algorithms.base",
    "rl.algorithms.mtsac", "types", "experiment",
)

for _name in _ALIASES:
    sys.modules[f"{__name__}.{_name}"] = importlib.import_module(f"mtrl_amd.compat.{_name}")

config = sys.modules[f"{__name__}.config"]
envs = sys.modules[f"{__name__}.envs"]
rl = sys.modules[f"{__name__}.rl"]
types = sys.modules[f"{__name__}.types"]
experiment = sys.modules[f"{__name__}.experiment"]
