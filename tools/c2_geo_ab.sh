# c2_geo_ab.sh TAG -- MT10/W2048 bf16 (configs[2]) with the weight-grad geometry forced (MTSAC_X3P_GEO:
# 0 128x128 k32, 1 256x128 k32 two stages, 2 256x128 k16 (the default pick), 3 256x256 k16), alternating
set -o pipefail
O=gpurun_out/${1:-c2geo}; mkdir -p $O
B="python bench.py --workload mt10_w2048 --precision bf16 --no-cpu-baseline --steps 100"
for i in 1 2; do
  timeout -k 10 200 $B > $O/base_$i.json 2>/dev/null || exit 1
  for g in 0 1 3; do
    MTSAC_X3P_GEO=$g timeout -k 10 200 $B > $O/g${g}_$i.json 2>/dev/null || exit 1
  done
done
echo done
