"""Time the trunk-forward plane GEMM at the bench shapes: gemm_x3p (current) vs gemm_x3f (new).
usage: python tools/x3f_bench.py [iters]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtrl_amd import _lib as L

lib = L.load()
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for (E, M, N, K) in [(1, 6400, 2048, 2048), (2, 6400, 2048, 2048), (2, 6400, 2048, 128), (1, 12800, 2048, 2048)]:
    for epi in (1, 2, 1 | 256, 1 | 512):  # bits 8-9: outputs 0 fp32 + planes, 1 planes only, 2 fp32 only
        row = []
        for which in (0, 1):
            ms = ctypes.c_double()
            rc = lib.mtsac_debug_gemm_fwd_bench(which, epi, E, M, N, K, iters, ctypes.byref(ms))
            tf = 2.0 * M * N * K * E / (ms.value * 1e-3) / 1e12 if rc == 0 else 0.0
            row.append(f"{['x3p', 'x3f'][which]} {ms.value * 1e3:8.1f} us {tf:6.1f} TF ({tf / 416.67:.3f})" if rc == 0
                       else f"{['x3p', 'x3f'][which]} rc={rc}")
        print(f"E={E} M={M} N={N} K={K} epi={epi}: " + " | ".join(row), flush=True)
