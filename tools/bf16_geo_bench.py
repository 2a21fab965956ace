"""Precision bf16 (one plane, one MFMA per product) forward-shaped GEMM at MT10 / MT50 row counts:
gemm_x3f (A through LDS, B straight to registers; its cost-model row tile) against gemm_x3p with
both operands staged through LDS (B k-major), by geometry (microbench, HIP events)."""
import ctypes
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402

lib = L.load()
ms = ctypes.c_double()
for M, E in ((1280, 2), (1280, 1), (2560, 1), (6400, 2)):
    r = {}
    L.check(lib.mtsac_debug_gemm_fwd_bench(1, 1 | (1 << 8) | 1024, E, M, 2048, 2048, 20, ctypes.byref(ms)))
    r["x3f"] = ms.value * 1e3
    for geo in (0, 1, 2, 3, 4):
        lib.mtsac_debug_x3p_geo(geo)
        for sp in (0, 2048):
            rc = lib.mtsac_debug_gemm_fwd_bench(0, 1 | (1 << 8) | 1024 | sp, E, M, 2048, 2048, 20, ctypes.byref(ms))
            r[f"x3p g{geo}{'s' if sp else ''}"] = ms.value * 1e3 if rc == 0 else None
        lib.mtsac_debug_x3p_geo(-1)
    fl = 2.0 * M * 2048 * 2048 * E
    print(f"bf16 fwd M={M} E={E}: " + ", ".join(f"{k} {v:.1f}us ({fl / v / 1e6 / 2500:.2f})" for k, v in r.items() if v),
          flush=True)
