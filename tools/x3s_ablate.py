"""gemm_x3s ablations at the 7-task shard shape (M 896, N 2048, K 2048): full kernel, without the
operand loads after the prologue, without the MFMAs.  Ablated results are wrong; only time matters.
usage: python tools/x3s_ablate.py [iters]   (X3S_SHAPE="M N K" for another shape, e.g. MT10/W400's
"1280 400 400"; X3S_H2=1: precision split2h)"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtrl_amd import _lib as L

lib = L.load()
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
M, N, K = (int(x) for x in os.environ.get("X3S_SHAPE", "896 2048 2048").split())
h2 = 8192 if os.environ.get("X3S_H2") == "1" else 0
for E in (1, 2):
    for which, name in ((-1, "full"), (-2, "no loads"), (-3, "no MFMA")):
        ms = ctypes.c_double()
        rc = lib.mtsac_debug_gemm_fwd_bench(which, 1 | 256 | h2, E, M, N, K, iters, ctypes.byref(ms))
        print(f"E={E} {name:9s} rc={rc} {ms.value * 1e3:8.1f} us", flush=True)
