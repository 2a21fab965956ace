"""What one rank of an N-GPU MT50/W2048 job steps in, on ONE GPU: the rank's task shard (the
slowest rank's tasks: 25 / 13 / 7 for N = 2 / 4 / 8) with the modelled trunk all-reduce
(mtsac_debug_set_collective_model: at every RCCL point a delay of 2 (N - 1) / N x bucket bytes over an
assumed bus bandwidth, on the collective stream, held by 8 workgroups), whole vs pipelined steps.
usage: python tools/shard_model.py [GBPS ...] [split3|split2h|bf16]   (default 0 300 150; 0 = no collective)"""
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd.engine import MTSACEngine, make_config  # noqa: E402
from mtrl_amd.init import init_mtsac  # noqa: E402

T, W = 50, 2048
PREC = {"split3": 1, "bf16": 2, "split2h": 3}
prec = next((PREC[a] for a in sys.argv[1:] if a in PREC), 1)
gbps_list = [float(x) for x in ([a for a in sys.argv[1:] if a not in PREC] or ["0", "300", "150"])]
only = [int(x) for x in __import__("os").environ.get("SHARD_N", "8,4,2").split(",")]  # SHARD_N=8: that N only
for nr, tl in ((8, 7), (4, 13), (2, 25)):
    if nr not in only:
        continue
    cfg = make_config(num_tasks=T, task_begin=0, task_count=tl, obs_dim=39 + T, actor_width=W, critic_width=W,
                      batch_per_task=128, capacity=20_000, clip=0, precision=prec)
    eng = MTSACEngine(cfg, device=0)
    actor, critic = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=1, task_begin=0, task_count=tl)
    eng.set_params(L.ACTOR, actor)
    eng.set_params(L.CRITIC, critic)
    eng.set_params(L.CRITIC_TARGET, critic)
    eng.buffer_fill_synthetic(1234)
    eng.seed_rng(1)
    eng.enable_graph(False)
    for gbps in gbps_list:
        L.check(eng.lib.mtsac_debug_set_collective_model(eng._h, nr if gbps > 0 else 1, gbps, 0))
        res = {}
        for pipe in (0, 1):
            eng.lib.mtsac_debug_set_pipeline(eng._h, pipe)
            eng.update_many(4)
            eng.synchronize()
            t0 = time.perf_counter()
            eng.update_many(30)
            eng.synchronize()
            res[pipe] = (time.perf_counter() - t0) / 30 * 1e3
        print(f"N={nr} T_local={tl:2d} bus {gbps:5.0f} GB/s: whole {res[0]:.3f} ms/step, pipelined {res[1]:.3f} ms/step",
              flush=True)
    eng.close()
