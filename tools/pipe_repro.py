"""Race hunt ("Lanes and hardware queues"): K fresh child processes, started
with GPU_MAX_HW_QUEUES=16 and the 5-lane form (MTSAC_LANES=1), each compare 4 whole steps with 4
pipelined steps at MT10/W400 bitwise; prints the mismatch count.  usage: pipe_repro.py K [ENV=VAL ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = """
import sys
sys.path.insert(0, {root!r})
import numpy as np
from mtrl_amd import _lib as L
from mtrl_amd.engine import MTSACEngine, make_config
from mtrl_amd.init import init_mtsac
T, tc, W, prec = 10, 10, 400, 1
outs = []
for pipe in (0, 1):
    e = MTSACEngine(make_config(num_tasks=T, task_begin=0, task_count=tc, obs_dim=39 + T, actor_width=W,
                                critic_width=W, batch_per_task=128, capacity=512, precision=prec))
    assert e.lib.mtsac_debug_lane_mode(e._h) == 0
    a, c = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=4, task_begin=0, task_count=tc)
    e.set_params(L.ACTOR, a); e.set_params(L.CRITIC, c); e.set_params(L.CRITIC_TARGET, c)
    e.buffer_fill_synthetic(77); e.seed_rng(5); e.enable_graph(False)
    e.lib.mtsac_debug_set_pipeline(e._h, pipe)
    e.update_many(4)
    outs.append((e.logs(), e.get_params(L.ACTOR), e.get_params(L.CRITIC)))
    e.close()
a, b = outs
assert a[0] == b[0], (a[0], b[0])
np.testing.assert_array_equal(a[1], b[1]); np.testing.assert_array_equal(a[2], b[2])
print("ok")
"""
K = int(sys.argv[1])
extra = dict(kv.split("=", 1) for kv in sys.argv[2:])
env = dict(os.environ, GPU_MAX_HW_QUEUES="16", MTSAC_LANES="1", **extra)
bad = 0
for k in range(K):
    r = subprocess.run([sys.executable, "-u", "-c", CHILD.format(root=ROOT)], capture_output=True, text=True,
                       timeout=200, env=env)
    ok = r.returncode == 0 and "ok" in r.stdout
    bad += 0 if ok else 1
    if not ok:
        print("  mismatch:", (r.stderr.strip().splitlines() or ["?"])[-1][:300], flush=True)
print(f"{extra}: {bad} of {K} runs mismatched", flush=True)
