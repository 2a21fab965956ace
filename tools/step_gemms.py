"""Per-launch GEMM timeline of one MT50 width-2048 step (timing mode, single stream).
usage: python tools/step_gemms.py [precision (1 = split3)] [T_local (default 50: unsharded)]"""
import ctypes
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd.engine import MTSACEngine, make_config  # noqa: E402
from mtrl_amd.init import init_mtsac  # noqa: E402

prec = int(sys.argv[1]) if len(sys.argv) > 1 else 1
T, W = 50, 2048
TL = int(sys.argv[2]) if len(sys.argv) > 2 else T
cfg = make_config(num_tasks=T, task_begin=0, task_count=TL, obs_dim=39 + T, actor_width=W, critic_width=W,
                  batch_per_task=128, capacity=100_000, clip=1, precision=prec)
eng = MTSACEngine(cfg, device=0)
actor, critic = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=1, task_begin=0, task_count=TL)
eng.set_params(L.ACTOR, actor)
eng.set_params(L.CRITIC, critic)
eng.set_params(L.CRITIC_TARGET, critic)
eng.buffer_fill_synthetic(1234)
eng.seed_rng(1)
eng.enable_graph(False)
eng.update_many(3)
eng.synchronize()
eng.set_timing(True, serial=True)
eng.update_many(1)
eng.synchronize()
lib = L.load()
n = lib.mtsac_debug_timed_launch(eng._h, -1, None, None)
dims = (ctypes.c_int32 * 5)()
ms = ctypes.c_double()
tot = 0.0
kinds = ["fwd", "dgrad", "wgrad", "in-fwd", "in-wgrad"]
for i in range(n):
    L.check(lib.mtsac_debug_timed_launch(eng._h, i, dims, ctypes.byref(ms)))
    f, M, N, K, E = list(dims)
    fl = 2.0 * M * N * K * E
    tot += ms.value
    print(f"{i:3d} {kinds[f]:8s} M={M:5d} N={N:5d} K={K:5d} E={E} {ms.value * 1e3:8.1f} us {fl / (ms.value * 1e-3) / 1e12:7.1f} TF/s")
print(f"total GEMM {tot:.3f} ms")
