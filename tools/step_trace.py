"""Eager pipelined steps (no serialisation) of one config for a rocprofv3 kernel trace read by
tools/step_timeline.py.  usage: step_trace.py T_local [T W precision]"""
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd.engine import MTSACEngine, make_config  # noqa: E402
from mtrl_amd.init import init_mtsac  # noqa: E402

tl = int(sys.argv[1]) if len(sys.argv) > 1 else 10
T = int(sys.argv[2]) if len(sys.argv) > 2 else 10
W = int(sys.argv[3]) if len(sys.argv) > 3 else 400
prec = int(sys.argv[4]) if len(sys.argv) > 4 else 1
cfg = make_config(num_tasks=T, task_begin=0, task_count=tl, obs_dim=39 + T, actor_width=W, critic_width=W,
                  batch_per_task=128, capacity=20_000, clip=1, precision=prec)
eng = MTSACEngine(cfg, device=0)
actor, critic = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=1, task_begin=0, task_count=tl)
eng.set_params(L.ACTOR, actor)
eng.set_params(L.CRITIC, critic)
eng.set_params(L.CRITIC_TARGET, critic)
eng.buffer_fill_synthetic(1234)
eng.seed_rng(1)
eng.enable_graph(False)
eng.update_many(20)
eng.synchronize()
eng.update_many(12)
eng.synchronize()
eng.close()
