"""Every split-K form of gemm_x3f (separate finishing pass / in-launch finish, split or not) against
float64 on the shard shapes, printing the rows and columns of any bad output (the check that located
the late-wave failures of the round-5 staggered schedule).
usage: python tools/x3f_stg_check.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402

lib = L.load()
for (E, M, N, K, epi, m16, h2) in [(2, 896, 2048, 2048, 1, False, True), (2, 6400, 2048, 2048, 1, False, True),
                                   (2, 896, 2048, 2048, 1, False, False), (2, 768, 2048, 2048, 2, True, True)]:
    rng = np.random.default_rng(M + 3 * K + epi)
    A = rng.standard_normal((E, M, K)).astype(np.float32)
    B = (rng.standard_normal((E, N, K)) / np.sqrt(K)).astype(np.float32)
    bias = rng.standard_normal((E, N)).astype(np.float32) * 0.1
    mask = np.maximum(rng.standard_normal((E, M, N)), 0).astype(np.float32)
    acc = np.einsum("emk,enk->emn", A.astype(np.float64), B.astype(np.float64))
    want = np.maximum(acc + bias[:, None, :], 0) if epi == 1 else np.where(mask > 0, acc, 0.0)
    p = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data  # noqa: E731
    for fin in (0, 4096):
        for split in (2048, 0):
            C = np.zeros((E, M, N), np.float32)
            Cs = np.zeros((E, M, N), np.float32)
            rc = lib.mtsac_debug_gemm_x3f(epi | (256 if m16 else 0) | split | fin | (8192 if h2 else 0), E, M, N, K,
                                          p(A), p(B), C.ctypes.data, p(bias), p(mask), Cs.ctypes.data)
            if rc != 0:
                print(f"E{E} M{M} epi{epi} h2={h2} fin={fin} split={split}: rc {rc}")
                continue
            err = np.abs(C - want)
            bad = ~np.isfinite(C) | (err > 1e-3 * (1 + np.abs(want)))
            rows = np.unique(np.nonzero(bad)[1])
            cols = np.unique(np.nonzero(bad)[2])
            print(f"E{E} M{M} epi{epi} h2={h2} fin={fin} split={split}: bad {int(bad.sum())} "
                  f"rows {rows[:10]} ({rows.size}) cols {cols[:10]} ({cols.size}) max err {float(np.nanmax(err)):.3e}",
                  flush=True)
