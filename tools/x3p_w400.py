"""Weight-grad GEMM of the W = 400 trunk (M = N = 400, K = 1280 rows, k-major planes): gemm_x3p
geometry x split-K sweep (launch + split-K reduction, HIP events over 20 launches)."""
import ctypes, sys
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L
lib = L.load()
for E in (2, 1):
    for geo in (0, 4, 1, 2, 3):
        lib.mtsac_debug_x3p_geo(geo)
        for sp in (1, 2, 3, 4, 5, 6, 8, 10):
            ms = ctypes.c_double()
            L.check(lib.mtsac_debug_gemm_x3p_bench(0 | (3 << 8) | (sp << 16), E, 400, 400, 1280, 20, ctypes.byref(ms)))
            print(f"E{E} geo{geo} splits{sp:2d} {ms.value*1e3:7.1f} us", flush=True)
lib.mtsac_debug_x3p_geo(-1)
