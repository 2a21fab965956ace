# c2_deep_ab.sh TAG -- the bf16 kernels' deep B ring: parity (x3f + full-batch tests), the C2 80-row tile
# alone (tools/x3f_ablate.py, ablation 3000 = the full kernel), and MT10/W2048 bf16 bench runs against
# mtrl_amd/libmtsac_ab.so (built with -DX3F_DEEP_B=0), alternating
set -o pipefail
O=gpurun_out/${1:-c2deep}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3f.py tests/test_gpu_fullbatch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
X3F_M=1280 X3F_BF16=1 X3F_FRAG=1 X3F_ABL="3000 3002" timeout -k 10 120 python tools/x3f_ablate.py 50 > $O/ablate_new.txt 2>&1 || exit 1
MTSAC_LIB=mtrl_amd/libmtsac_ab.so X3F_M=1280 X3F_BF16=1 X3F_FRAG=1 X3F_ABL="3000 3002" timeout -k 10 120 python tools/x3f_ablate.py 50 > $O/ablate_old.txt 2>&1 || exit 1
B="python bench.py --workload mt10_w2048 --precision bf16 --no-cpu-baseline --steps 100"
for i in 1 2 3; do
  timeout -k 10 200 $B > $O/new_$i.json 2>/dev/null || exit 1
  MTSAC_LIB=mtrl_amd/libmtsac_ab.so timeout -k 10 200 $B > $O/old_$i.json 2>/dev/null || exit 1
done
echo done
