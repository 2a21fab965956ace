"""Where the split2h input-layer forward's time goes (S3: E = 2, 6400 x 2048, K = in_dim padded to 128,
planes out): gemm_x3f at that shape with ablations -- 0 full, 3 no operand reloads, 128 no epilogue
stores, 131 neither (MFMA + LDS + barriers + the epilogue's LDS staging and arithmetic only) -- and
the hidden-layer shape (K = 2048) for comparison.  Ablated results are wrong; only the time matters.
usage: python tools/x3f_input_probe.py [iters]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtrl_amd import _lib as L

lib = L.load()
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
E, M, N = 2, 6400, 2048
for K in (128, 2048):
    for rep in range(2):
        for abl in (0, 3, 128, 131):
            ms = ctypes.c_double()
            # 1 = bias+ReLU, 256 = planes only, 8192 = split2h, 16384 = B in the fragment layout
            L.check(lib.mtsac_debug_gemm_fwd_bench(2 + abl, 1 | 256 | 8192 | 16384, E, M, N, K, iters, ctypes.byref(ms)))
            out_mb = E * M * N * 4 / 1e6
            print(f"K {K:5d} abl {abl:3d}: {ms.value * 1e3:7.1f} us  ({out_mb / (ms.value * 1e-3) / 1e6:5.2f} TB/s of "
                  f"plane writes, {2.0 * M * N * K * E / (ms.value * 1e-3) / 1e12:6.1f} TF)", flush=True)
