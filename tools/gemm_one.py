"""Run one forward-shaped plane GEMM `iters` times (for rocprofv3 PMC passes).
usage: python tools/gemm_one.py which epi E M N K iters   (which 0 = gemm_x3p, 1 = gemm_x3f)"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtrl_amd import _lib as L

which, epi, E, M, N, K, iters = (int(x) for x in sys.argv[1:8])
ms = ctypes.c_double()
L.check(L.load().mtsac_debug_gemm_fwd_bench(which, epi, E, M, N, K, iters, ctypes.byref(ms)))
print(f"{ms.value * 1e3:.1f} us/launch, {2.0 * M * N * K * E / (ms.value * 1e-3) / 1e12:.1f} TF/s", flush=True)
