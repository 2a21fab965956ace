import ctypes, sys
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L
lib = L.load()
# (name, epi, layout bits: 1 = A k-major, 2 = B k-major, M, N, K, E)
cases = []
for lay, nm in [(0, "rr"), (2, "rk"), (1, "kr"), (3, "kk")]:
    cases += [(f"fwd-{nm}-E2", 1, lay, 6400, 2048, 2048, 2), (f"fwd-{nm}-E1", 1, lay, 6400, 2048, 2048, 1),
              (f"wg-{nm}-E2", 0, lay, 2048, 2048, 6400, 2), (f"sq4k-{nm}", 0, lay, 4096, 4096, 4096, 1),
              (f"fwd-{nm}-M896", 1, lay, 896, 2048, 2048, 2)]
for geo in [int(g) for g in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4").split(",")]:
    lib.mtsac_debug_x3p_geo(geo)
    for name, epi, lay, M, N, K, E in cases:
        ms = ctypes.c_double()
        L.check(lib.mtsac_debug_gemm_x3p_bench(epi | (lay << 8), E, M, N, K, 10, ctypes.byref(ms)))
        print(f"geo{geo & 255} dbg{geo >> 8} {name:7s} {ms.value*1e3:8.1f} us {2.0*M*N*K*E/(ms.value*1e-3)/1e12:7.1f} TF/s", flush=True)
lib.mtsac_debug_x3p_geo(-1)
