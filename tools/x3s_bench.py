"""Time the small-row-count trunk-forward plane GEMM: gemm_x3p (previous path, split-K) vs gemm_x3s.
usage: python tools/x3s_bench.py [iters]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtrl_amd import _lib as L

lib = L.load()
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for (E, M, N, K) in [(1, 896, 2048, 2048), (2, 896, 2048, 2048), (1, 768, 2048, 2048), (1, 1280, 2048, 2048),
                     (2, 1280, 2048, 2048), (1, 3200, 2048, 2048), (1, 1280, 400, 416), (2, 1280, 400, 416)]:
    for epi in (1 | 256, 1 | 512):  # bits 8-9: outputs 1 planes only, 2 fp32 only
        row = []
        for which in (0, -1):
            ms = ctypes.c_double()
            rc = lib.mtsac_debug_gemm_fwd_bench(which, epi, E, M, N, K, iters, ctypes.byref(ms))
            name = "x3p" if which == 0 else "x3s"
            tf = 2.0 * M * N * K * E / (ms.value * 1e-3) / 1e12 if rc == 0 else 0.0
            row.append(f"{name} {ms.value * 1e3:8.1f} us {tf:6.1f} TF ({tf / 416.67:.3f})" if rc == 0 else f"{name} rc={rc}")
        print(f"E={E} M={M} N={N} K={K} epi={epi} TI={lib.mtsac_debug_x3s_ti(M, N, E)}: " + " | ".join(row), flush=True)
