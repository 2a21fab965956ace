"""gemm_x3f + split-K against gemm_x3p + split-K at task-shard row counts (N = K = 2048):
forward (bias+ReLU; x3p writes fp32 + planes as the engine's k-major path does, x3f planes only)
and data grad (ReLU mask).  usage: python tools/x3f_split_bench.py [iters]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtrl_amd import _lib as L

lib = L.load()
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N = K = 2048
SPLIT = 2048
for M in (768, 896, 1280, 1792):
    for E in (1, 2):
        for name, epi_x3p, epi_x3f in (("fwd", 1, 1 | 256), ("dgrad", 2, 2 | 256)):
            out = []
            for which, epi in ((0, epi_x3p), (1, epi_x3f)):
                ms = ctypes.c_double()
                rc = lib.mtsac_debug_gemm_fwd_bench(which, epi | SPLIT, E, M, N, K, iters, ctypes.byref(ms))
                if rc != 0:
                    out.append(f"rc {rc}")
                    continue
                tf = 2.0 * M * N * K * E / (ms.value * 1e-3) / 1e12
                out.append(f"{ms.value * 1e3:7.1f} us {tf:6.1f} TF")
            print(f"M {M:5d} E {E} {name:5s}: x3p {out[0]}   x3f {out[1]}", flush=True)
