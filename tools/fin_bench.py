"""Split-K with and without the in-launch finish, at task-shard shapes (microbench, HIP events).
x3f: forward (bias+ReLU, planes out) and data grad shapes at 896 / 1664 rows; x3p: k-major weight
grads W x W over K = 896 / 1664 rows, split-K 2 (+ reduce) vs in-launch reduce vs 256x128 tiles unsplit."""
import ctypes
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402

lib = L.load()
ms = ctypes.c_double()
for M in (896, 1664):
    for outs, nm in ((1, "planes"), (2, "fp32")):
        r = []
        for fin in (0, 4096):
            L.check(lib.mtsac_debug_gemm_fwd_bench(1, 1 | (outs << 8) | 2048 | fin, 2, M, 2048, 2048, 20, ctypes.byref(ms)))
            r.append(ms.value * 1e3)
        print(f"x3f fwd M={M:5d} E=2 {nm:6s}: split+finish {r[0]:7.1f} us, in-launch {r[1]:7.1f} us", flush=True)
for K in (896, 1664):
    r = []
    for geo, epi in ((-1, 0 | (3 << 8) | (255 << 16)), (-1, 0 | (3 << 8) | (255 << 16) | 4096), (1, 0 | (3 << 8))):
        lib.mtsac_debug_x3p_geo(geo)
        L.check(lib.mtsac_debug_gemm_x3p_bench(epi, 2, 2048, 2048, K, 20, ctypes.byref(ms)))
        r.append(ms.value * 1e3)
    lib.mtsac_debug_x3p_geo(-1)
    print(f"x3p wgrad K={K:5d} E=2: split+reduce {r[0]:7.1f} us, in-launch {r[1]:7.1f} us, 256x128 unsplit {r[2]:7.1f} us",
          flush=True)
