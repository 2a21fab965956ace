"""Time MTSAC.compute_weights (gradient-conflict metrics) at a workload's full size on the device:
per-task gradients, order statistics, pair statistics, host finish.
usage: python tools/conflict_bench.py [T] [W] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd import conflict as mc  # noqa: E402
from mtrl_amd.engine import MTSACEngine, make_config  # noqa: E402
from mtrl_amd.init import init_mtsac  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 50
W = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
e = MTSACEngine(make_config(num_tasks=T, task_count=T, obs_dim=39 + T, actor_width=W, critic_width=W,
                            batch_per_task=128, capacity=1000, precision=1))
a, q = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=1)
e.set_params(L.ACTOR, a)
e.set_params(L.CRITIC, q)
e.set_params(L.CRITIC_TARGET, q)
e.buffer_fill_synthetic(7)
e.seed_rng(1)
mc.compute_weights(e)  # warm-up (allocates the [T][P] matrices)
for r in range(reps):
    t0 = time.perf_counter()
    e.task_gradients()
    e.synchronize()
    t1 = time.perf_counter()
    stats = [mc.network_stats(e, w) for w in (0, 1)]
    t2 = time.perf_counter()
    logs = {k: v for w, s in zip(("critic", "actor"), stats) for k, v in mc.metrics_from_stats(s).items()}
    t3 = time.perf_counter()
    print(f"T={T} W={W}: per-task gradients {1e3 * (t1 - t0):.1f} ms, device statistics {1e3 * (t2 - t1):.1f} ms, "
          f"host finish {1e3 * (t3 - t2):.1f} ms; P critic {e.task_gradient_size(0)}, actor {e.task_gradient_size(1)}",
          flush=True)
print("critic avg cos", float(logs["avg_cos_sim"]), "support", float(logs["avg_support_size"]))
