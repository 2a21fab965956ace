"""Microbenchmark of the engine's GEMM kernels at the MT50/W2048 shapes (mtsac_debug_gemm_bench)."""
import ctypes
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402

lib = L.load()
prec = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1").split(",")]
shapes = [("NN", 0, 1, 6400, 2048, 2048, 1), ("NN-E2", 0, 1, 6400, 2048, 2048, 2), ("NT", 1, 2, 6400, 2048, 2048, 1),
          ("NT-E2", 1, 2, 6400, 2048, 2048, 2), ("TN", 2, 0, 2048, 2048, 6400, 1), ("TN-E2", 2, 0, 2048, 2048, 6400, 2),
          ("NN-l0", 0, 1, 6400, 2048, 93, 2)]
for p in prec:
    for name, kind, epi, M, N, K, E in shapes:
        ms = ctypes.c_double()
        L.check(lib.mtsac_debug_gemm_bench(p, kind, epi, E, M, N, K, 10, ctypes.byref(ms)))
        tf = 2.0 * M * N * K * E / (ms.value * 1e-3) / 1e12
        print(f"prec={p} {name:6s} M={M} N={N} K={K} E={E}: {ms.value*1e3:8.1f} us  {tf:6.1f} TF/s", flush=True)
