"""A/B of engine-wide switches on whole S3 (or shard) steps in ONE process: for each variant, a fresh
engine, 5 warm-up steps, then the mean of 3 x 20 timed device-sampled steps (graph replay or eager).
usage: python tools/step_ab.py [--tl 50] [--prec 3] [--eager] VARIANT...   VARIANT = name:geo[:K=V,K=V]
  geo: mtsac_debug_x3p_geo (-1 auto, 2 = 256x128 k16, 3 = 256x256 k16); K=V: environment variables set
  while the variant's engine is created (switches the engine reads at create)"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd.engine import MTSACEngine, make_config  # noqa: E402
from mtrl_amd.init import init_mtsac  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tl", type=int, default=50)
ap.add_argument("--prec", type=int, default=3)
ap.add_argument("--eager", action="store_true")
ap.add_argument("variants", nargs="+")
a = ap.parse_args()
T, W = 50, 2048
lib = L.load()
res = {}
for rnd in range(2):
    for v in a.variants:
        name, geo, *envs = v.split(":")
        lib.mtsac_debug_x3p_geo(int(geo))
        kv = dict(x.split("=", 1) for x in (envs[0].split(",") if envs and envs[0] else []))
        old = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        eng = MTSACEngine(make_config(num_tasks=T, task_begin=0, task_count=a.tl, obs_dim=39 + T, actor_width=W,
                                      critic_width=W, batch_per_task=128, capacity=10_000, precision=a.prec))
        ac, cr = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=1, task_begin=0, task_count=a.tl)
        for k, o in old.items():
            if o is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = o
        eng.set_params(L.ACTOR, ac)
        eng.set_params(L.CRITIC, cr)
        eng.set_params(L.CRITIC_TARGET, cr)
        eng.buffer_fill_synthetic(3)
        eng.seed_rng(1)
        eng.enable_graph(not a.eager)
        eng.update_many(5)
        eng.synchronize()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            eng.update_many(20)
            eng.synchronize()
            ts.append((time.perf_counter() - t0) / 20 * 1e3)
        eng.close()
        res.setdefault(name, []).append(min(ts))
        print(f"round {rnd} {name}: {min(ts):.3f} ms/step ({', '.join(f'{x:.3f}' for x in ts)})", flush=True)
lib.mtsac_debug_x3p_geo(-1)
for k, v in res.items():
    print(f"{k}: best {min(v):.3f} ms/step")
