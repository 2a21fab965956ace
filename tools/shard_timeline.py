"""Eager, pipelined steps of the 7-task MT50 shard with a 1-rank RCCL communicator, for a
rocprofv3 kernel trace: the bucketed all-reduces run on their own stream (lane 4) at the points
the N-GPU job issues them, so the per-stream timeline (tools/step_timeline.py ... full) shows what
overlaps them.  One rank cannot time the xGMI transfer itself."""
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd.engine import MTSACEngine, make_config  # noqa: E402
from mtrl_amd.init import init_mtsac  # noqa: E402

tl, T, W = 7, 50, 2048
cfg = make_config(num_tasks=T, task_begin=0, task_count=tl, obs_dim=39 + T, actor_width=W, critic_width=W,
                  batch_per_task=128, capacity=20_000, clip=1, precision=1)
eng = MTSACEngine(cfg, device=0)
actor, critic = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=1, task_begin=0, task_count=tl)
eng.set_params(L.ACTOR, actor)
eng.set_params(L.CRITIC, critic)
eng.set_params(L.CRITIC_TARGET, critic)
eng.comm_init(MTSACEngine.comm_unique_id(), 1, 0, timeout_s=120)
eng.buffer_fill_synthetic(1234)
eng.seed_rng(1)
eng.enable_graph(False)
eng.update_many(3)
eng.synchronize()
eng.update_many(8)
eng.synchronize()
print("comm ranks", eng.comm_nranks())
eng.close()
