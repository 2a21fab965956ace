"""Ablations of the plane GEMM (gemm_x3p) at the step's shapes: dbg bits 1 = no refill DMA in the
K-loop, 2 = no MFMA, 8 = refill issued up front, 64 = no balanced launch; geometries 3 = 256x256,
5 = 224x256, 255 = auto."""
import ctypes
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402

lib = L.load()
# (name, epi, layout bits: 1 = A k-major, 2 = B k-major, M, N, K, E)
cases = [("fwd-E1", 1, 2, 6400, 2048, 2048, 1), ("fwd-E2", 1, 2, 6400, 2048, 2048, 2),
         ("dgrad-E1", 2, 0, 6400, 2048, 2048, 1), ("wgrad-E1", 0, 3, 2048, 2048, 6400, 1)]
dbgs = [int(d) for d in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,8").split(",")]
geos = [int(g) for g in (sys.argv[2] if len(sys.argv) > 2 else "3").split(",")]  # 255 = auto
for geo in geos:
    for dbg in dbgs:
        lib.mtsac_debug_x3p_geo(geo | (dbg << 8))
        for name, epi, lay, M, N, K, E in cases:
            ms = ctypes.c_double()
            L.check(lib.mtsac_debug_gemm_x3p_bench(epi | (lay << 8), E, M, N, K, 10, ctypes.byref(ms)))
            print(f"geo{geo} dbg{dbg:2d} {name:9s} {ms.value*1e3:8.1f} us {2.0*M*N*K*E/(ms.value*1e-3)/1e12:7.1f} TF/s",
                  flush=True)
lib.mtsac_debug_x3p_geo(-1)
