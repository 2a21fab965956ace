"""DrQ conv channel-group sweep: resident-batch update time for forced forward / data-grad groups
(mtsac_debug_drq_groups).  usage: python tools/drq_group_sweep.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd.drq import DrQEngine, DrQSettings  # noqa: E402
from mtrl_amd.drq_init import init_drq  # noqa: E402

B = 256
rng = np.random.default_rng(0)
obs = rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8)
nobs = rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8)
act = rng.integers(0, 18, B).astype(np.int32)
done = (rng.random(B) < 0.05).astype(np.float32)
rew = rng.standard_normal(B).astype(np.float32)
task = (np.arange(B) % 26).astype(np.int32)
co, cn = rng.integers(0, 8, (B, 2)).astype(np.int32), rng.integers(0, 8, (B, 2)).astype(np.int32)
no = (1 + 0.05 * np.clip(rng.standard_normal(B), -2, 2)).astype(np.float32)
nn = (1 + 0.05 * np.clip(rng.standard_normal(B), -2, 2)).astype(np.float32)
lib = L.load()
e = DrQEngine(DrQSettings(batch=B))
p0 = init_drq(seed=0)
e.set_params(L.DRQ_PARAMS, p0)
e.set_params(L.DRQ_TARGET, p0)
e.update((obs, act, nobs, done, rew, task), (co, no, cn, nn))
out = {}
for f, b in [(0, 0), (4, 0), (8, 0), (16, 0), (0, 8), (0, 16), (4, 4), (8, 4), (0, 0)]:
    lib.mtsac_debug_drq_groups(f, b)
    e.update_resident(20)
    e.synchronize()
    t0 = time.perf_counter()
    e.update_resident(200)
    e.synchronize()
    out[f"fwd{f}_bwd{b}"] = round(1e3 * (time.perf_counter() - t0) / 200, 4)
    print(f, b, out[f"fwd{f}_bwd{b}"], flush=True)
lib.mtsac_debug_drq_groups(0, 0)
print(json.dumps(out))
