"""Per-launch time of every DrQ conv pass at the benched geometry (batch 256, 84x84, IMPALA scale 1):
the default per-shape choice, the VALU kernels' per-shape choice (mask 16: no split2h MFMA) and the
pre-round-6 kernels (mask 7), in one process (mtsac_debug_drq_conv_bench / mtsac_debug_drq_legacy).
usage: drq_conv_bench.py [iters] [--wg-sweep]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402

lib = L.load()
it = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 20
B = 256
# (images, H, ci, co): forward over 3B images, backward passes over B
shapes = [(3 * B, 84, 4, 8), (3 * B, 42, 8, 8), (3 * B, 42, 8, 16), (3 * B, 21, 16, 16), (3 * B, 11, 16, 16)]
names = ("forward", "data_grad", "weight_grad")
us = ctypes.c_double()
print(f"{'pass':12s} {'B':>4s} {'HxW':>6s} {'ci->co':>7s} {'default':>8s} {'VALU us':>8s} {'legacy us':>9s}  GFMA/s(default)")
for kind in (0, 1, 2):
    for nb, h, ci, co in shapes:
        b = nb if kind == 0 else B
        row = []
        for legacy in (0, 16, 7):
            lib.mtsac_debug_drq_legacy(legacy)
            rc = lib.mtsac_debug_drq_conv_bench(kind, b, h, h, ci, co, it, ctypes.byref(us))
            assert rc == 0, rc
            row.append(us.value)
        lib.mtsac_debug_drq_legacy(0)
        fma = b * h * h * 9 * ci * co
        print(f"{names[kind]:12s} {b:4d} {h:3d}x{h:<3d} {ci:3d}->{co:<3d} {row[0]:8.1f} {row[1]:8.1f} {row[2]:9.1f}  {fma / row[0] / 1e3:8.0f}", flush=True)
if "--wg-sweep" in sys.argv:  # the row-tile weight grad's grid cap
    old = lib.mtsac_debug_drq_wgrad_blocks(-1)
    for nb, h, ci, co in shapes:
        row = []
        for cap in (128, 256, 512, 1024, 2048):
            lib.mtsac_debug_drq_wgrad_blocks(cap)
            assert lib.mtsac_debug_drq_conv_bench(2, B, h, h, ci, co, it, ctypes.byref(us)) == 0
            row.append(f"{cap}:{us.value:.1f}")
        print(f"weight_grad grid caps {h}x{h} {ci}->{co}: " + " ".join(row), flush=True)
    lib.mtsac_debug_drq_wgrad_blocks(old)
