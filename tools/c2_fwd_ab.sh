# c2_fwd_ab.sh TAG -- MT10/W2048 bf16 (configs[2]): trunk forward / data grads on gemm_x3f (default) vs
# gemm_x3p at a fixed geometry (MTSAC_X3F_MIN_TILES above any grid, MTSAC_BFRAG=0), whole bench runs
set -o pipefail
O=gpurun_out/${1:-c2fwd}; mkdir -p $O
B="python bench.py --workload mt10_w2048 --precision bf16 --no-cpu-baseline --steps 100"
for i in 1 2; do
  timeout -k 10 200 $B > $O/base_$i.json 2>/dev/null || exit 1
  for g in 2 3 0 4; do
    MTSAC_X3F_MIN_TILES=1000000 MTSAC_BFRAG=0 MTSAC_X3P_GEO=$g timeout -k 10 200 $B > $O/x3p_g${g}_$i.json 2>/dev/null || exit 1
  done
done
echo done
