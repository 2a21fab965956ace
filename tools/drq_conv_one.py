"""One DrQ conv pass, iters launches (for rocprofv3 --pmc passes): drq_conv_one.py kind B H ci co iters [legacy]
(kind 0 forward, 1 data grad, 2 weight grad; legacy = mtsac_debug_drq_legacy mask, default 0)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402

kind, B, H, ci, co, it = (int(v) for v in sys.argv[1:7])
lib = L.load()
lib.mtsac_debug_drq_legacy(int(sys.argv[7]) if len(sys.argv) > 7 else 0)
us = ctypes.c_double()
assert lib.mtsac_debug_drq_conv_bench(kind, B, H, H, ci, co, it, ctypes.byref(us)) == 0
print(f"kind {kind} B {B} {H}x{H} {ci}->{co}: {us.value:.1f} us per launch")
