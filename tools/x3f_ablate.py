"""gemm_x3f ablations at the bench shape (E=2, 6400 x 2048 x 2048, bias+ReLU, planes out):
0 full kernel, 1 no A refills, 2 no B reloads, 3 neither, 4 s_setprio 1 for waves 4-7,
64 B read as contiguous 1-KB blocks (TA pattern probe).
Ablated results are wrong; only the time matters.  usage: python tools/x3f_ablate.py [iters]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtrl_amd import _lib as L

lib = L.load()
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
E, M, N, K = 2, int(os.environ.get("X3F_M", "6400")), 2048, 2048  # X3F_M=1280 + ablations 300x: C2's 80-row bf16 tile
bf16 = os.environ.get("X3F_BF16") == "1"  # precision bf16 at the 400-row tile (peak 2500 TF)
h2 = os.environ.get("X3F_H2") == "1"  # precision split2h (3 fp16 products, peak 833 TF)
frag = os.environ.get("X3F_FRAG") == "1"  # B planes in the fragment layout (the engine's weight planes at S3)
peak = 2500.0 if bf16 else 833.33 if h2 else 416.67
for rep in range(2):
    for abl in [int(a) for a in os.environ.get("X3F_ABL", "0 1 2 3 4 64").split()]:
        ms = ctypes.c_double()
        L.check(lib.mtsac_debug_gemm_fwd_bench(2 + abl, 1 | 256 | (1024 if bf16 else 0) | (8192 if h2 else 0) | (16384 if frag else 0), E, M, N, K, iters,
                                               ctypes.byref(ms)))
        tf = 2.0 * M * N * K * E / (ms.value * 1e-3) / 1e12
        print(f"{'bf16 ' if bf16 else 'split2h ' if h2 else ''}{'frag ' if frag else ''}abl {abl}: {ms.value * 1e3:7.1f} us {tf:6.1f} TF ({tf / peak:.3f})", flush=True)
