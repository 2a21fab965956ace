"""DrQ update at several batch sizes against the float64 oracle: per-leaf relative error of the
gradient (diagnostics for the batch-dependent paths).  usage: python tools/drq_diag.py B..."""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))), "tests"))
from oracle import drq as od  # noqa: E402
from test_gpu_drq import _run_both  # noqa: E402

from mtrl_amd import _lib as L  # noqa: E402

cfg = od.DrQConfig(hw=84, n_hidden=512)
for B in [int(x) for x in sys.argv[1:]]:
    e, st, new, got, want, internals = _run_both(cfg, B, seed=84 + B)
    print(f"B={B}", {k: (round(got[k], 6), round(want[k], 6)) for k in want}, flush=True)
    g_gpu = e.get_params(L.DRQ_GRAD).astype(np.float64)
    g_ref = internals["grad"]
    o = 0
    for path, shape in od.param_spec(cfg):
        n = int(np.prod(shape))
        a, b = g_gpu[o:o + n], g_ref[o:o + n]
        o += n
        rel = np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)
        if rel > 1e-5:
            print(f"  {path:55s} rel {rel:.2e}  |ref| {np.linalg.norm(b):.3e}", flush=True)
    e.close()
