# gpu_r4z2.sh -- round-4 final evidence, part 2: rocprofv3 kernel stats + PMC traffic of the default
# bench (tools/profile_round.sh), the other configs' bench lines, the task-shard model
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile_round.sh r4z_prof split2h || exit 1
bash tools/gpu_configs.sh r4z_cfg || exit 1
timeout -k 10 400 python -u tools/shard_model.py 0 300 150 split2h > gpurun_out/r4z_cfg/shard_model.txt 2>&1 || exit 1
echo done
