"""Ablations of the split GEMM (gemm_x3): skip loads / MFMA / split, NT and TN at step shapes + 4096^3."""
import ctypes
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402

lib = L.load()
shapes = [("NT-E2", 1, 1, 6400, 2048, 2048, 2), ("TN-E2", 2, 0, 2048, 2048, 6400, 2), ("NT-4k", 1, 0, 4096, 4096, 4096, 1),
          ("NT-6144", 1, 0, 6144, 4096, 4096, 1)]
for dbg in (0, 1, 2, 4, 5, 3):
    lib.mtsac_debug_x3p_geo(255 | (dbg << 16))
    for name, kind, epi, M, N, K, E in shapes:
        ms = ctypes.c_double()
        L.check(lib.mtsac_debug_gemm_bench(1, kind, epi, E, M, N, K, 10, ctypes.byref(ms)))
        tf = 2.0 * M * N * K * E / (ms.value * 1e-3) / 1e12
        print(f"dbg={dbg} {name:7s}: {ms.value*1e3:8.1f} us  {tf:6.1f} TF/s", flush=True)
lib.mtsac_debug_x3p_geo(-1)
