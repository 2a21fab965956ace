"""MT10 / W = 400 (BASELINE configs[1]): eager vs graph step time, then untimed eager steps for a
rocprofv3 kernel trace (tools/step_timeline.py: wall vs busy union per step = the launch gaps).
usage: c1_timeline.py [T W [precision]]  (precision: 1 split3, 2 bf16, 3 split2h = the default)"""
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd.engine import MTSACEngine, make_config  # noqa: E402
from mtrl_amd.init import init_mtsac  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 10
W = int(sys.argv[2]) if len(sys.argv) > 2 else 400
PREC = int(sys.argv[3]) if len(sys.argv) > 3 else 3
cfg = make_config(num_tasks=T, task_begin=0, task_count=T, obs_dim=39 + T, actor_width=W, critic_width=W,
                  batch_per_task=128, capacity=20_000, clip=0, precision=PREC)
eng = MTSACEngine(cfg, device=0)
actor, critic = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=1, task_begin=0, task_count=T)
eng.set_params(L.ACTOR, actor)
eng.set_params(L.CRITIC, critic)
eng.set_params(L.CRITIC_TARGET, critic)
eng.buffer_fill_synthetic(1234)
eng.seed_rng(1)
for mode in ("eager", "graph", "eager"):
    eng.enable_graph(mode == "graph")
    eng.update_many(20)
    eng.synchronize()
    t0 = time.perf_counter()
    eng.update_many(400)
    eng.synchronize()
    print(f"T={T} W={W} {mode}: {(time.perf_counter() - t0) / 400 * 1e6:.1f} us/step", flush=True)
eng.enable_graph(False)
eng.update_many(12)
eng.synchronize()
eng.close()
