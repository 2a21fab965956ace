"""CPU-side checks of the C-ABI library: it loads, and exports every function
declared in include/*.h (no compute calls -- there is no GPU here)."""

import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parent.parent


def _declared():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names |= set(re.findall(r"\b((?:mtsac|drq)_[a-z0-9_]+)\s*\(", text))
    return names


def test_library_exports_every_declared_symbol():
    from mtrl_amd import _lib

    lib = _lib.load()
    declared = _declared()
    assert len(declared) >= 30
    missing = [n for n in sorted(declared) if not hasattr(lib, n)]
    assert not missing, missing
    assert set(_lib.SIGNATURES) == declared
    assert lib.mtsac_abi_version() == 1


def test_default_config_matches_reference_defaults():
    from mtrl_amd.engine import default_config

    c = default_config(50)
    # mtsac.py:116-127, config/optim.py:15-43, config/networks.py:6-18, config/nn.py:8-31
    assert (c.num_tasks, c.obs_dim, c.action_dim, c.actor_width, c.actor_depth, c.num_critics) == (50, 89, 4, 400, 3, 2)
    assert abs(c.gamma - 0.99) < 1e-7 and abs(c.tau - 0.005) < 1e-9 and abs(c.adam_eps - 1e-5) < 1e-12
    assert (c.log_std_min, c.log_std_max, c.batch_per_task, c.capacity) == (-20.0, 2.0, 128, 100000)


def test_missing_library_fails_loudly(tmp_path):
    import pytest

    from mtrl_amd import _lib

    with pytest.raises(_lib.MTSACLibraryError):
        _lib.load(tmp_path / "nope.so")
