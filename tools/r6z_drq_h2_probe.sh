set -o pipefail
O=gpurun_out/r6z; mkdir -p $O
timeout -k 10 300 python -u tools/drq_conv_bench.py 20 > $O/conv_bench.txt 2>&1 || exit 1
python - >> $O/conv_bench.txt 2>&1 <<'PY'
import ctypes, sys
sys.path.insert(0, '.')
from mtrl_amd import _lib as L
lib = L.load(); us = ctypes.c_double()
print("split2h forced everywhere (mask 32):")
lib.mtsac_debug_drq_legacy(32)
for kind in (0, 1):
    for nb, h, ci, co in [(768, 42, 8, 8), (768, 42, 8, 16), (768, 21, 16, 16), (768, 11, 16, 16)]:
        b = nb if kind == 0 else 256
        assert lib.mtsac_debug_drq_conv_bench(kind, b, h, h, ci, co, 20, ctypes.byref(us)) == 0
        print(kind, b, h, ci, co, round(us.value, 1))
PY
echo done
