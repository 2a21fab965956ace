# c2_env_ab.sh TAG -- MT10/W2048 bf16 (configs[2]) bench with and without an environment switch
# (here MTSAC_X3F_ORDER=1: row tiles fastest inside an XCD's run), alternating, 3 rounds
set -o pipefail
O=gpurun_out/${1:-c2ab}; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --workload mt10_w2048 --precision bf16 --no-cpu-baseline --steps 100 > $O/base_$i.json 2>/dev/null || exit 1
  MTSAC_X3F_ORDER=1 timeout -k 10 200 python bench.py --workload mt10_w2048 --precision bf16 --no-cpu-baseline --steps 100 > $O/order1_$i.json 2>/dev/null || exit 1
done
echo done
