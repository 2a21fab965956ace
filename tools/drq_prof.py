"""Resident-batch DrQ-eps updates for rocprofv3 --kernel-trace --stats (batch 256)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd.drq import DrQEngine, DrQSettings  # noqa: E402

B = 256
rng = np.random.default_rng(0)
n = DrQEngine(DrQSettings(batch=B))
p = (rng.standard_normal(n.n) * 0.02).astype(np.float32)
n.set_params(L.DRQ_PARAMS, p)
n.set_params(L.DRQ_TARGET, p)
obs = rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8)
batch = (obs, rng.integers(0, 18, B), obs[::-1].copy(), np.zeros(B), rng.standard_normal(B), np.arange(B) % 26)
aug = (rng.integers(0, 8, (B, 2)), np.ones(B), rng.integers(0, 8, (B, 2)), np.ones(B))
n.update(batch, aug)
n.update_resident(10)
n.synchronize()
n.close()
