import ctypes, sys
sys.path.insert(0, ".")
from mtrl_amd import _lib as L
lib = L.load()
for geo in (0, 1, 1 | 256, 1 | 512, 0 | 256, 0 | 512):
    lib.mtsac_debug_x3p_geo(geo)
    for name, epi, M, N, K, E in [("NN-E2", 1, 6400, 2048, 2048, 2), ("TN", 0, 2048, 2048, 6400, 1),
                                  ("4096^3", 0, 4096, 4096, 4096, 1), ("8192^3", 0, 8192, 8192, 8192, 1)]:
        ms = ctypes.c_double()
        L.check(lib.mtsac_debug_gemm_x3p_bench(epi, E, M, N, K, 10, ctypes.byref(ms)))
        print(f"geo{geo & 255} dbg{geo >> 8} {name:7s} {ms.value*1e3:8.1f} us {2.0*M*N*K*E/(ms.value*1e-3)/1e12:7.1f} TF/s", flush=True)
