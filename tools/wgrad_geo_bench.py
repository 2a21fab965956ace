"""k-major weight-grad GEMM (dW = H^T dZ, W x W, K = rows) by x3p geometry, auto split-K
(microbench, HIP events): 256x256 k16 (geo 3, the default), 256x128 k32 (geo 1), 256x128 k16 (geo 2)."""
import ctypes
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402

lib = L.load()
ms = ctypes.c_double()
for W in (2048, 400):
    for E in (2, 1):
        for K in ((896, 1664, 3200, 6400) if W == 2048 else (1280, 6400)):
            r = []
            for geo in (3, 1, 2, 4):
                lib.mtsac_debug_x3p_geo(geo)
                L.check(lib.mtsac_debug_gemm_x3p_bench(0 | (3 << 8) | (255 << 16), E, W, W, K, 20, ctypes.byref(ms)))
                r.append(ms.value * 1e3)
            lib.mtsac_debug_x3p_geo(-1)
            print(f"wgrad W={W} E={E} K={K:5d}: geo3 {r[0]:7.1f}  geo1 {r[1]:7.1f}  geo2 {r[2]:7.1f}  geo4 {r[3]:7.1f} us",
                  flush=True)
