# cfg_final.sh TAG -- bench lines of the other configs (tools/gpu_configs.sh) and the 7-task shard model
# on the current tree
set -o pipefail
O=gpurun_out/${1:-cfgfinal}; mkdir -p $O
bash tools/gpu_configs.sh ${1:-cfgfinal} || exit 1
SHARD_N=8 timeout -k 10 200 python tools/shard_model.py 0 300 150 split2h > $O/shard_model.txt 2>&1 || exit 1
echo done
