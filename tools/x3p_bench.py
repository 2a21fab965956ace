import ctypes, sys
sys.path.insert(0, ".")
from mtrl_amd import _lib as L
lib = L.load()
# (name, epi, layout bits: 1 = A k-major, 2 = B k-major, M, N, K, E)
cases = [("NT-E2", 1, 0, 6400, 2048, 2048, 2), ("NT-E1", 2, 0, 6400, 2048, 2048, 1),
         ("TN-E2", 0, 3, 2048, 2048, 6400, 2), ("TN-E1", 0, 3, 2048, 2048, 6400, 1),
         ("NT-4k", 0, 0, 4096, 4096, 4096, 1), ("TN-4k", 0, 3, 4096, 4096, 4096, 1),
         ("NT-M3200", 1, 0, 3200, 2048, 2048, 2), ("NT-M1600", 1, 0, 1600, 2048, 2048, 2),
         ("NT-M800", 1, 0, 800, 2048, 2048, 2), ("NT-M768E1", 1, 0, 768, 2048, 2048, 1)]
for geo in [int(g) for g in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4").split(",")]:
    lib.mtsac_debug_x3p_geo(geo)
    for name, epi, lay, M, N, K, E in cases:
        ms = ctypes.c_double()
        L.check(lib.mtsac_debug_gemm_x3p_bench(epi | (lay << 8), E, M, N, K, 10, ctypes.byref(ms)))
        print(f"geo{geo & 255} dbg{geo >> 8} {name:7s} {ms.value*1e3:8.1f} us {2.0*M*N*K*E/(ms.value*1e-3)/1e12:7.1f} TF/s", flush=True)
lib.mtsac_debug_x3p_geo(-1)
