# r6v_drq_dense_ab.sh TAG: the DrQ oracle tests with the dense layers on gemm_x3 (MTSAC_DRQ_DENSE=x3),
# then a same-box bench A/B (gemm_f32 default vs x3), alternating three times
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
MTSAC_DRQ_DENSE=x3 timeout -k 10 600 python -u -m pytest tests/test_gpu_drq.py -m gpu -x -q --timeout 300 --timeout-method thread -k "update_matches_oracle or deterministic or row_tile" > $O/tests_x3.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 --workload atari_drq > $O/f32_$i.json 2>/dev/null || exit 1
  MTSAC_DRQ_DENSE=x3 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 --workload atari_drq > $O/x3_$i.json 2>/dev/null || exit 1
done
echo done
