"""Would a feature-major trunk run the S3 forward faster?  Times, split2h, E = 2:
  x3f_fwd   : today's forward, gemm_x3f, row-major activations x W^T planes (6400 x 2048 x 2048),
              bias+ReLU, planes out
  x3p_fm    : the feature-major forward Y^T = W . X^T on gemm_x3p with BOTH operands k-major
              (2048 x 6400 x 2048), bias+ReLU, planes out
  x3p_fm_st : the same GEMM with an fp32 store epilogue
  x3p_wgrad : today's weight grad shape (2048 x 2048 x 6400, k-major both, fp32 out)
usage: python tools/fm_forward_probe.py [iters]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtrl_amd import _lib as L

lib = L.load()
lib.mtsac_debug_gemm_x3p_bench.argtypes = [ctypes.c_int] * 6 + [ctypes.POINTER(ctypes.c_double)]
lib.mtsac_debug_gemm_fwd_bench.argtypes = [ctypes.c_int] * 7 + [ctypes.POINTER(ctypes.c_double)]
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
E, PEAK = 2, 833.33
H2, POUT = 1 << 13, 1 << 14
cases = [
    ("x3f_fwd", lambda ms: lib.mtsac_debug_gemm_fwd_bench(1, 1 | 256 | 8192 | 16384, E, 6400, 2048, 2048, iters, ms), 6400, 2048, 2048),
    ("x3p_fm", lambda ms: lib.mtsac_debug_gemm_x3p_bench(1 | (3 << 8) | H2 | POUT, E, 2048, 6400, 2048, iters, ms), 2048, 6400, 2048),
    ("x3p_fm_st", lambda ms: lib.mtsac_debug_gemm_x3p_bench(0 | (3 << 8) | H2, E, 2048, 6400, 2048, iters, ms), 2048, 6400, 2048),
    ("x3p_wgrad", lambda ms: lib.mtsac_debug_gemm_x3p_bench(0 | (3 << 8) | H2, E, 2048, 2048, 6400, iters, ms), 2048, 2048, 6400),
]
for rep in range(2):
    for name, fn, M, N, K in cases:
        ms = ctypes.c_double()
        L.check(fn(ctypes.byref(ms)))
        tf = 2.0 * M * N * K * E / (ms.value * 1e-3) / 1e12
        print(f"{name:10s} {M}x{N}x{K}: {ms.value * 1e3:7.1f} us {tf:6.1f} TF ({tf / PEAK:.3f} of the split2h peak)", flush=True)
