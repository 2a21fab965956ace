# s3_deep3_ab.sh TAG -- the split2h 208-row three-buffer B ring: parity (x3f + full-batch tests), the S3
# forward alone (tools/x3f_ablate.py ablation 0) and the S3 bench, each against mtrl_amd/libmtsac_ab.so
# (-DX3F_DEEP3=0), alternating
set -o pipefail
O=gpurun_out/${1:-deep3}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3f.py tests/test_gpu_fullbatch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
X3F_H2=1 X3F_FRAG=1 X3F_ABL="0" timeout -k 10 120 python tools/x3f_ablate.py 30 > $O/ablate_new.txt 2>&1 || exit 1
MTSAC_LIB=mtrl_amd/libmtsac_ab.so X3F_H2=1 X3F_FRAG=1 X3F_ABL="0" timeout -k 10 120 python tools/x3f_ablate.py 30 > $O/ablate_old.txt 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/new_$i.json 2>/dev/null || exit 1
  MTSAC_LIB=mtrl_amd/libmtsac_ab.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/old_$i.json 2>/dev/null || exit 1
done
echo done
