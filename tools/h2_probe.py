"""split2h vs split3 gemm_x3f per-launch time at the S3 shapes (tools for DESIGN section 3)."""
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import ctypes

from mtrl_amd import _lib as L

lib = L.load()
shapes = [("s3_fwd_e2", 2, 6400, 2048, 2048, 1 | 256), ("s3_actor_fwd_e1", 1, 12832, 2048, 2048, 1 | 256),
          ("s3_dgrad_e2", 2, 6400, 2048, 2048, 2 | 256), ("s3_fwd_e1", 1, 6400, 2048, 2048, 1 | 256)]
for name, E, M, N, K, epi in shapes:
    row = []
    for tag, bits in (("split3", 0), ("split2h", 8192), ("bf16", 1024)):
        ms = ctypes.c_double()
        rc = lib.mtsac_debug_gemm_fwd_bench(1, epi | bits, E, M, N, K, 20, ctypes.byref(ms))
        tf = 2.0 * E * M * N * K / (ms.value * 1e-3) / 1e12 if rc == 0 else 0.0
        row.append(f"{tag} {ms.value * 1e3:8.1f} us {tf:6.1f} TF (rc {rc})")
    print(f"{name:16s} " + " | ".join(row), flush=True)
