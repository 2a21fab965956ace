"""Step time of one task shard on one GPU: what a rank of an N-GPU job computes (no all-reduce).
usage: python tools/shard_step.py [T_local ...]"""
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd.engine import MTSACEngine, make_config  # noqa: E402
from mtrl_amd.init import init_mtsac  # noqa: E402

T, W = 50, 2048
for tl in [int(x) for x in (sys.argv[1:] or ["50", "25", "13", "7"])]:
    cfg = make_config(num_tasks=T, task_begin=0, task_count=tl, obs_dim=39 + T, actor_width=W, critic_width=W,
                      batch_per_task=128, capacity=100_000, clip=1, precision=1)
    eng = MTSACEngine(cfg, device=0)
    actor, critic = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=1, task_begin=0, task_count=tl)
    eng.set_params(L.ACTOR, actor)
    eng.set_params(L.CRITIC, critic)
    eng.set_params(L.CRITIC_TARGET, critic)
    eng.buffer_fill_synthetic(1234)
    eng.seed_rng(1)
    res = {}
    for mode in ("eager", "graph"):
        eng.enable_graph(mode == "graph")
        eng.update_many(3)
        eng.synchronize()
        t0 = time.perf_counter()
        eng.update_many(20)
        eng.synchronize()
        res[mode] = (time.perf_counter() - t0) / 20 * 1e3
    print(f"T_local={tl:3d} B={128 * tl:5d}: eager {res['eager']:.3f} ms/step, graph {res['graph']:.3f} ms/step", flush=True)
    eng.close()
