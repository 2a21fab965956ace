# cfg_and_fin.sh TAG -- bench lines of the other configs (tools/gpu_configs.sh), the 7-task shard model,
# and MT10/W400 (configs[1]) with the in-launch split-K finish (MTSAC_SPLITK_FIN=1) against the default
set -o pipefail
O=gpurun_out/${1:-cfgfin}; mkdir -p $O
bash tools/gpu_configs.sh ${1:-cfgfin} || exit 1
SHARD_N=8 timeout -k 10 200 python tools/shard_model.py 0 300 150 split2h > $O/shard_model.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload mt10_w400 --no-cpu-baseline --steps 200 > $O/c1_base_$i.json 2>/dev/null || exit 1
  MTSAC_SPLITK_FIN=1 timeout -k 10 200 python bench.py --workload mt10_w400 --no-cpu-baseline --steps 200 > $O/c1_fin_$i.json 2>/dev/null || exit 1
done
echo done
